#!/bin/bash
# round 3 (m): fp32 Newton tolerance: MuJoCo's 1e-8 and 1e-9 against the 1e-7 default -- parity and cost
set -o pipefail
O=gpurun_out/r03m; mkdir -p $O
export FM_TRAJ_CACHE=traj_cache
for tol in 1e-8 1e-9; do
  timeout -k 10 300 python -u tools/parity_sweep.py --prec fp32 --tol $tol --tag tol$tol >> $O/sweep.jsonl 2>> $O/sweep.err || { echo "SWEEP FAILED"; tail -20 $O/sweep.err; exit 1; }
done
cat $O/sweep.jsonl
for tol in 1e-8 1e-9; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --fp64-steps 0 --solver-tolerance $tol > $O/bench_tol$tol.json 2> $O/bench.err || { echo "BENCH FAILED"; tail $O/bench.err; exit 1; }
  cat $O/bench_tol$tol.json
done
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --fp64-steps 0 > $O/bench_default.json 2>> $O/bench.err || { echo "BENCH FAILED"; tail $O/bench.err; exit 1; }
cat $O/bench_default.json
