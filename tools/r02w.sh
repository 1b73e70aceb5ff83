#!/bin/bash
# fresh-container rebuild check: full GPU suite, smoke, default bench (driver's command), rocprofv3 kernel stats
set -o pipefail
O=gpurun_out/r02w
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { echo "GPU SUITE FAILED"; tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log
timeout -k 10 120 python __graft_entry__.py smoke > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail $O/smoke.log; exit 1; }
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH FAILED; tail $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --fp64-steps 0 > $O/prof.log 2>&1 || { echo PROF FAILED; tail $O/prof.log; exit 1; }
echo R02W_OK
