#!/bin/bash
# round 3 (f): float64 narrowphase in the fp32 build (default now); compile-time (4,16) fp32 scene with the dense
# matrix-core Cholesky vs the sparse LDS one vs the runtime-dims kernel; behaviour of the saved policies; GPU suite
set -o pipefail
O=gpurun_out/r03f; mkdir -p $O
export FM_TRAJ_CACHE=traj_cache
T416=4,16,150,3,PauseIKToggleEnv
timeout -k 10 300 python -u tools/parity_sweep.py --prec fp32 --tag main >> $O/sweep.jsonl 2>> $O/sweep.err || { echo "SWEEP FAILED"; tail -20 $O/sweep.err; exit 1; }
timeout -k 10 300 python -u tools/parity_sweep.py --prec fp32 --tag fixed416_dense --traj $T416 >> $O/sweep.jsonl 2>> $O/sweep.err || { echo "SWEEP 416 FAILED"; tail -20 $O/sweep.err; exit 1; }
FM_CHOL_LDS=2 timeout -k 10 300 python -u tools/parity_sweep.py --prec fp32 --tag fixed416_sparse --traj $T416 >> $O/sweep.jsonl 2>> $O/sweep.err || { echo "SWEEP 416s FAILED"; tail -20 $O/sweep.err; exit 1; }
cat $O/sweep.jsonl
timeout -k 10 300 python bench.py --workload config5 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || { echo "BENCH c5 FAILED"; tail $O/bench_c5.err; exit 1; }
cat $O/bench_c5.json
FM_CHOL_LDS=2 timeout -k 10 300 python bench.py --workload config5 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_c5_sparse.json 2> $O/bench_c5s.err || { echo "BENCH c5 sparse FAILED"; tail $O/bench_c5s.err; exit 1; }
cat $O/bench_c5_sparse.json
timeout -k 10 300 python -u tools/phase_profile.py --steps 3 --arms 4 --objects 16 --env-class PauseIKToggleEnv --preroll 60 > $O/phase_4x16_fixed.json 2> $O/phase.err || { echo "PHASE416 FAILED"; tail $O/phase.err; exit 1; }
cat $O/phase_4x16_fixed.json
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail $O/bench.err; exit 1; }
cat $O/bench.json
for run in r666unuv xfwgqibb y6lp1j7k; do
  timeout -k 10 400 python -u tools/behaviour.py policy $run --arenas 512 --precision fp32 > $O/beh_$run.json 2>> $O/beh.err || { echo "BEH $run FAILED"; tail $O/beh.err; exit 1; }
  cat $O/beh_$run.json
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; echo "tests rc $?"; tail -15 $O/tests.log
