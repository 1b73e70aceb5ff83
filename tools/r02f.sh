#!/bin/bash
set -o pipefail
O=gpurun_out/r02f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -s > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|Error|fp32|fp64" $O/tests.log | tail -40
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH FAILED; tail $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
echo R02F_OK
