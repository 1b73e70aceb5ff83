#!/bin/bash
# IK env classes on the GPU: parity tests, then the whole GPU suite, then the bench
set -o pipefail
O=gpurun_out/r02g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -s -k "ik_classes" > $O/tests_ik.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|fp64 |assert" $O/tests_ik.log | head -40
[ $rc -eq 0 ] || { echo "IK TESTS FAILED rc=$rc"; exit 1; }
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_all.log 2>&1 || { echo "GPU SUITE FAILED"; tail -30 $O/tests_all.log; exit 1; }
tail -2 $O/tests_all.log
timeout -k 10 300 python bench.py --no-cpu-baseline --fp64-steps 0 > $O/bench.json 2> $O/bench.err || { echo BENCH FAILED; tail $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
echo R02G_OK
