#!/bin/bash
# round 3 (i): fp64 IK-kernel regression hunt (parallel box-box SAT vs serial), refinement off
set -o pipefail
O=gpurun_out/r03i; mkdir -p $O
timeout -k 10 300 python -u -m pytest "tests/test_gpu_parity.py::test_teacher_forced_ik_classes_fp64[PauseIKToggleEnv]" -q -x --timeout 200 --timeout-method thread > $O/ik_default.log 2>&1; echo "default rc $?"; grep -E "passed|failed" $O/ik_default.log
FM_SERIAL_BOXBOX=1 timeout -k 10 300 python -u -m pytest "tests/test_gpu_parity.py::test_teacher_forced_ik_classes_fp64[PauseIKToggleEnv]" -q -x --timeout 200 --timeout-method thread > $O/ik_serial.log 2>&1; echo "serial rc $?"; grep -E "passed|failed" $O/ik_serial.log
export FM_TRAJ_CACHE=traj_cache
timeout -k 10 300 python -u tools/parity_sweep.py --prec fp32 --tag base >> $O/sweep.jsonl 2>> $O/sweep.err || { echo "SWEEP FAILED"; tail -20 $O/sweep.err; exit 1; }
cat $O/sweep.jsonl
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail $O/bench.err; exit 1; }
cat $O/bench.json
