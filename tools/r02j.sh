#!/bin/bash
set -o pipefail
O=gpurun_out/r02j
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -s > $O/tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|fp32 \(4|dropped" $O/tests.log | tail -40
[ $rc -eq 0 ] || { echo "GPU SUITE FAILED"; tail -30 $O/tests.log; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --fp64-steps 0 > $O/bench.json 2> $O/bench.err || { echo BENCH FAILED; tail $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
timeout -k 10 400 python bench.py --workload config3 > $O/bench3.json 2> $O/bench3.err || { echo BENCH3 FAILED; tail $O/bench3.err; exit 1; }
cut -c1-250 $O/bench3.json; grep -o '"diagnostics.*' $O/bench3.json
echo R02J_OK
