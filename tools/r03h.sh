#!/bin/bash
# round 3 (h): fp32 Newton direction refined with a float64 residual (register Cholesky scenes); dense blocked
# Cholesky v2 (padded stride, matrix-core panel and trailing update) for (4,16); sweep, benches, profile, GPU suite
set -o pipefail
O=gpurun_out/r03h; mkdir -p $O
export FM_TRAJ_CACHE=traj_cache
T416=4,16,150,3,PauseIKToggleEnv
timeout -k 10 300 python -u tools/parity_sweep.py --prec fp32 --tag refine >> $O/sweep.jsonl 2>> $O/sweep.err || { echo "SWEEP FAILED"; tail -20 $O/sweep.err; exit 1; }
timeout -k 10 300 python -u tools/parity_sweep.py --prec fp32 --tag dense2 --traj $T416 >> $O/sweep.jsonl 2>> $O/sweep.err || { echo "SWEEP 416 FAILED"; tail -20 $O/sweep.err; exit 1; }
FM_CHOL_LDS=2 timeout -k 10 300 python -u tools/parity_sweep.py --prec fp32 --tag sparse --traj $T416 >> $O/sweep.jsonl 2>> $O/sweep.err || { echo "SWEEP 416s FAILED"; tail -20 $O/sweep.err; exit 1; }
timeout -k 10 300 python -u tools/parity_sweep.py --prec fp64 --tag f64 >> $O/sweep.jsonl 2>> $O/sweep.err || { echo "SWEEP f64 FAILED"; tail -20 $O/sweep.err; exit 1; }
cat $O/sweep.jsonl
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python -u tools/phase_profile.py --steps 3 --arms 4 --objects 16 --env-class PauseIKToggleEnv --preroll 60 > $O/phase_4x16_pause.json 2> $O/phase.err || { echo "PHASE416 FAILED"; tail $O/phase.err; exit 1; }
cat $O/phase_4x16_pause.json
timeout -k 10 300 python bench.py --workload config5 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || { echo "BENCH c5 FAILED"; tail $O/bench_c5.err; exit 1; }
cat $O/bench_c5.json
timeout -k 10 300 python -u tools/phase_profile.py --steps 10 > $O/phase_2x4_fp32.json 2>> $O/phase.err || { echo "PHASE FAILED"; tail $O/phase.err; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; echo "tests rc $?"; tail -15 $O/tests.log
