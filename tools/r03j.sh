#!/bin/bash
# round 3 (j): register Cholesky restored (refinement removed): fp64 IK classes, then the whole GPU suite
set -o pipefail
O=gpurun_out/r03j; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -k "ik_classes_fp64 or ik_timing" --timeout 200 --timeout-method thread > $O/ik.log 2>&1; echo "ik rc $?"; grep -E "passed|failed|fp64 " $O/ik.log | tail -12
FM_SERIAL_BOXBOX=1 timeout -k 10 300 python -u -m pytest "tests/test_gpu_parity.py::test_teacher_forced_ik_classes_fp64[PauseIKToggleEnv]" -q --timeout 200 --timeout-method thread > $O/ik_serial.log 2>&1; echo "serial rc $?"; grep -E "passed|failed|fp64 " $O/ik_serial.log | tail -3
