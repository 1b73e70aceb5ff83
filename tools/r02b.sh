#!/bin/bash
# force-termination ballot fix check + which dofs set the fp32 error
set -o pipefail
O=gpurun_out/r02b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python tools/parity_sweep.py --prec fp64 --tag ballotfix > $O/sweep64.jsonl 2> $O/sweep.err || { echo SWEEP FAILED; tail $O/sweep.err; exit 1; }
cut -c1-400 $O/sweep64.jsonl
timeout -k 10 300 python tools/worst_dofs.py --prec fp32 > $O/worst32.jsonl 2> $O/worst.err || { echo WORST FAILED; tail $O/worst.err; exit 1; }
grep hist $O/worst32.jsonl
echo R02B_OK
