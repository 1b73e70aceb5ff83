#!/bin/bash
set -o pipefail
O=gpurun_out/r02d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1; echo "tests rc=$?"; tail -3 $O/tests.log
timeout -k 10 300 python tools/parity_sweep.py --prec fp32 --tag zshift > $O/sweep32.jsonl 2> $O/sweep.err || { echo SWEEP FAILED; tail $O/sweep.err; exit 1; }
cut -c1-300 $O/sweep32.jsonl
timeout -k 10 300 python tools/worst_dofs.py --prec fp32 > $O/worst32.jsonl 2> $O/worst.err || { echo WORST FAILED; tail $O/worst.err; exit 1; }
grep hist $O/worst32.jsonl
echo R02C_OK
