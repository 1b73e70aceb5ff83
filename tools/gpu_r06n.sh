# round-6 product check: the full GPU test suite, then config 2 and config 3 benches of the product library
set -o pipefail
O=gpurun_out/r06n; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/c2.json 2> $O/c2.err || exit 1
python -c "import json; d=json.load(open('$O/c2.json')); print('c2', d['value'], d['roofline']['kernel_ms_avg'], d.get('fp64', {}).get('value'))"
timeout -k 10 300 python bench.py --workload config3 --steps 12 --warmup 2 --preroll 100 --ppo-epochs 1 --no-cpu-baseline > $O/c3.json 2> $O/c3.err || exit 1
python -c "import json; d=json.load(open('$O/c3.json')); print('c3', d['value'], d['kernel_ms_avg'])"
