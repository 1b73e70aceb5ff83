#!/bin/bash
# round 3 (c): physics pinned by the reference runs (pyramid position stiffness, post-teleport stage) + float64
# solver accumulation: parity sweep, misses, bench, behavioural statistics, GPU test suite
set -o pipefail
O=gpurun_out/r03c; mkdir -p $O
export FM_TRAJ_CACHE=traj_cache
timeout -k 10 300 python -u tools/parity_sweep.py --prec fp32 --tag f32 >> $O/sweep.jsonl 2>> $O/sweep.err || { echo "SWEEP FAILED"; tail -20 $O/sweep.err; exit 1; }
timeout -k 10 300 python -u tools/parity_sweep.py --prec fp64 --tag f64 >> $O/sweep.jsonl 2>> $O/sweep.err || { echo "SWEEP64 FAILED"; tail -20 $O/sweep.err; exit 1; }
FACTORYSIM_LIB=factory_marl_amd/lib_int64.so timeout -k 10 300 python -u tools/parity_sweep.py --prec fp32 --tag int64 >> $O/sweep.jsonl 2>> $O/sweep.err || { echo "SWEEP int64 FAILED"; tail -20 $O/sweep.err; exit 1; }
timeout -k 10 300 python -u tools/miss_report.py --tag base > $O/miss.jsonl 2> $O/miss.err || { echo "MISS FAILED"; tail -20 $O/miss.err; exit 1; }
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python -u tools/behaviour.py base 2 --arenas 1000 --episodes 100 > $O/beh_base2.json 2> $O/beh.err || { echo "BEH2 FAILED"; tail $O/beh.err; exit 1; }
cat $O/beh_base2.json
timeout -k 10 300 python -u tools/behaviour.py policy rk5rxnav --arenas 1000 --precision fp32 > $O/beh_rk5.json 2>> $O/beh.err || { echo "BEH rk5 FAILED"; tail $O/beh.err; exit 1; }
timeout -k 10 300 python -u tools/behaviour.py base 4 --arenas 256 --episodes 20 > $O/beh_base4.json 2>> $O/beh.err || { echo "BEH4 FAILED"; tail $O/beh.err; exit 1; }
cat $O/beh_base4.json
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; echo "tests rc $?"; tail -15 $O/tests.log
