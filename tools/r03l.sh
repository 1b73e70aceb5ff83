#!/bin/bash
# round 3 (l): cached midphase for (2,8), (2,10), (4,16): parity identical to r03i, config 3 / 5 benches, phase
# profiles, GPU suite
set -o pipefail
O=gpurun_out/r03l; mkdir -p $O
export FM_TRAJ_CACHE=traj_cache
timeout -k 10 300 python -u tools/parity_sweep.py --prec fp32 --tag mc --traj 2,8,300,5 2,10,250,9 4,16,150,3,PauseIKToggleEnv >> $O/sweep.jsonl 2>> $O/sweep.err || { echo "SWEEP FAILED"; tail -20 $O/sweep.err; exit 1; }
timeout -k 10 300 python -u tools/parity_sweep.py --prec fp64 --tag mc64 --traj 2,8,300,5 2,10,250,9 >> $O/sweep.jsonl 2>> $O/sweep.err || { echo "SWEEP64 FAILED"; tail -20 $O/sweep.err; exit 1; }
cat $O/sweep.jsonl
timeout -k 10 300 python bench.py --workload config5 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_config5.json 2> $O/bench_c5.err || { echo "BENCH c5 FAILED"; tail $O/bench_c5.err; exit 1; }
cat $O/bench_config5.json
timeout -k 10 300 python -u tools/phase_profile.py --steps 3 --arms 4 --objects 16 --env-class PauseIKToggleEnv --preroll 60 > $O/phase_fp32_4x16.json 2> $O/phase.err || { echo "PHASE416 FAILED"; tail $O/phase.err; exit 1; }
timeout -k 10 300 python -u tools/phase_profile.py --steps 5 --arms 2 --objects 8 > $O/phase_fp32_2x8.json 2>> $O/phase.err || { echo "PHASE28 FAILED"; tail $O/phase.err; exit 1; }
timeout -k 10 400 python bench.py --workload config3 --no-cpu-baseline > $O/bench_config3.json 2> $O/bench_c3.err || { echo "BENCH c3 FAILED"; tail $O/bench_c3.err; exit 1; }
cat $O/bench_config3.json
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; echo "tests rc $?"; tail -12 $O/tests.log
