#!/bin/bash
# round 3 (end): the GPU suite on lib_wip.so (fused Newton warmstart passes + two-pass arrowhead Cholesky of the
# bordered scenes, built from branch wip-r03-fusion), config 2 / config 3 benches of both libraries, then the GPU
# suite on the product library
set -o pipefail
O=gpurun_out/r03v2; mkdir -p $O
W=factory_marl_amd/lib_wip.so
FACTORYSIM_LIB=$W timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/tests_wip.log 2>&1; echo "wip tests rc $?"; tail -3 $O/tests_wip.log
FACTORYSIM_LIB=$W timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/bench_wip.json 2> $O/bench_wip.err || { echo "BENCH WIP FAILED"; tail $O/bench_wip.err; exit 1; }
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail $O/bench.err; exit 1; }
FACTORYSIM_LIB=$W timeout -k 10 300 python bench.py --workload config3 --steps 8 --warmup 2 --no-cpu-baseline > $O/bench_config3_wip.json 2> $O/bench_c3w.err || { echo "BENCH C3W FAILED"; tail $O/bench_c3w.err; exit 1; }
timeout -k 10 300 python bench.py --workload config3 --steps 8 --warmup 2 --no-cpu-baseline > $O/bench_config3.json 2> $O/bench_c3.err || { echo "BENCH C3 FAILED"; tail $O/bench_c3.err; exit 1; }
python -c "
import json
for f in ('bench_wip', 'bench', 'bench_config3_wip', 'bench_config3'):
    d = json.load(open('$O/' + f + '.json')); print(f, d['value'], d.get('fp64_value', {}).get('value'))
"
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; echo "product tests rc $?"; tail -3 $O/tests.log
