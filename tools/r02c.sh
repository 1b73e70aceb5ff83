#!/bin/bash
# float64 master state for the fp32 build: parity sweeps fp32/fp64, worst dofs, tests, bench
set -o pipefail
O=gpurun_out/r02c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1; echo "tests rc=$?"; tail -3 $O/tests.log
timeout -k 10 300 python tools/parity_sweep.py --prec fp32 --tag master64 > $O/sweep32.jsonl 2> $O/sweep.err || { echo SWEEP FAILED; tail $O/sweep.err; exit 1; }
cut -c1-300 $O/sweep32.jsonl
timeout -k 10 300 python tools/parity_sweep.py --prec fp64 --tag master64 > $O/sweep64.jsonl 2>> $O/sweep.err || { echo SWEEP FAILED; tail $O/sweep.err; exit 1; }
cut -c1-300 $O/sweep64.jsonl
timeout -k 10 300 python tools/worst_dofs.py --prec fp32 > $O/worst32.jsonl 2> $O/worst.err || { echo WORST FAILED; tail $O/worst.err; exit 1; }
grep hist $O/worst32.jsonl
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo BENCH FAILED; tail $O/bench.err; exit 1; }
cut -c1-600 $O/bench.json
echo R02C_OK
