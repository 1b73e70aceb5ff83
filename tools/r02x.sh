#!/bin/bash
# fp32 parity tests with the float-restatement floor, then the full measurement set on the current kernel
set -o pipefail
O=gpurun_out/r02x
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "fp32" -x -v -s --timeout 300 --timeout-method thread > $O/fp32_tests.log 2>&1 || { echo "FP32 TESTS FAILED"; tail -40 $O/fp32_tests.log; exit 1; }
grep -E "within|restatement|passed|failed" $O/fp32_tests.log
bash tools/r02_measure.sh r02x
