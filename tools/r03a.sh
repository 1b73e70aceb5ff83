#!/bin/bash
# round 3 (a): float64 solver accumulation in the fp32 build -- parity sweep over tolerances, fp64 sanity, bench
set -o pipefail
O=gpurun_out/r03a; mkdir -p $O
export FM_TRAJ_CACHE=traj_cache
for tol in 0 1e-9 1e-10 1e-12; do
  timeout -k 10 240 python -u tools/parity_sweep.py --prec fp32 --tol $tol --tag f32_tol$tol >> $O/sweep.jsonl 2>> $O/sweep.err || { echo "SWEEP FAILED tol $tol"; tail -20 $O/sweep.err; exit 1; }
done
timeout -k 10 240 python -u tools/parity_sweep.py --prec fp64 --tag f64 >> $O/sweep.jsonl 2>> $O/sweep.err || { echo "SWEEP FAILED fp64"; tail -20 $O/sweep.err; exit 1; }
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail $O/bench.err; exit 1; }
cat $O/bench.json
