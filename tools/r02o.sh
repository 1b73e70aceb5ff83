#!/bin/bash
# Round-2 GPU iteration: rendering tests, then a sample image for the record.
set -o pipefail
O=gpurun_out/r02o
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_render.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "RENDER TESTS FAILED"; tail -40 $O/tests.log; exit 1; }
tail -4 $O/tests.log
timeout -k 10 200 python -u tools/render_demo.py --out $O/render_demo.png > $O/demo.log 2>&1 || { echo DEMO FAILED; tail $O/demo.log; exit 1; }
cat $O/demo.log
echo R02O_OK
