#!/bin/bash
# final round-2 check of the committed tree: full GPU suite (oracle checker rebuilt with the faster collision /
# envelope Cholesky), smoke, default bench with the CPU-baseline leg
set -o pipefail
O=gpurun_out/${R02Z_TAG:-r02z}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { echo "GPU SUITE FAILED"; tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
timeout -k 10 120 python __graft_entry__.py smoke > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH FAILED; tail $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['traffic'], d['cpu_baseline'])"
echo R02Z_OK
