#!/bin/bash
# Round-2 GPU iteration: full GPU suite on the IK-split kernel, headline bench, 1000-episode flag divergence.
set -o pipefail
O=gpurun_out/r02n
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { echo "GPU SUITE FAILED"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline --fp64-steps 0 > $O/bench.json 2> $O/bench.err || { echo BENCH FAILED; tail $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
OMP_NUM_THREADS=1 timeout -k 10 1000 python -u tools/flag_divergence.py --episodes 1000 --workers 16 > $O/flagdiv.json 2> $O/flagdiv.err || { echo FLAGDIV FAILED; tail $O/flagdiv.err; exit 1; }
cat $O/flagdiv.json
echo R02N_OK
