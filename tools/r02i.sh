#!/bin/bash
set -o pipefail
O=gpurun_out/r02i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ppo.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|mean return|assert" $O/tests.log | head -20
[ $rc -eq 0 ] || { echo "PPO TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
timeout -k 10 400 python bench.py --workload config3 > $O/bench3.json 2> $O/bench3.err || { echo BENCH3 FAILED; tail $O/bench3.err; exit 1; }
cat $O/bench3.json
echo R02I_OK
