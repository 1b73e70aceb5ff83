#!/bin/bash
# longest-first dispatch order (lpt_order_kernel): GPU suite, then A/B benches with FACTORYSIM_NO_LPT=1
set -o pipefail
O=gpurun_out/r02l
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { echo "GPU SUITE FAILED"; tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
for r in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --fp64-steps 0 > $O/lpt_$r.json 2> $O/lpt_$r.err || { echo "BENCH LPT FAILED"; tail $O/lpt_$r.err; exit 1; }
  FACTORYSIM_NO_LPT=1 timeout -k 10 200 python bench.py --no-cpu-baseline --fp64-steps 0 > $O/plain_$r.json 2> $O/plain_$r.err || { echo "BENCH PLAIN FAILED"; tail $O/plain_$r.err; exit 1; }
  python -c "import json; a=json.load(open('$O/lpt_$r.json')); b=json.load(open('$O/plain_$r.json')); print('config2 lpt', a['value'], a['roofline']['kernel_ms_avg'], 'plain', b['value'], b['roofline']['kernel_ms_avg'])"
done
for wl in config3 config5; do
  timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline > $O/lpt_$wl.json 2> $O/lpt_$wl.err || { echo "BENCH $wl LPT FAILED"; tail $O/lpt_$wl.err; exit 1; }
  FACTORYSIM_NO_LPT=1 timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline > $O/plain_$wl.json 2> $O/plain_$wl.err || { echo "BENCH $wl PLAIN FAILED"; tail $O/plain_$wl.err; exit 1; }
  python -c "import json; a=json.load(open('$O/lpt_$wl.json')); b=json.load(open('$O/plain_$wl.json')); print('$wl lpt', a['value'], 'plain', b['value'])"
done
echo R02L_OK
