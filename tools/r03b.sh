#!/bin/bash
# round 3 (b): where the remaining fp32 misses are; float64 integration / IEEE div-sqrt variants
set -o pipefail
O=gpurun_out/r03b; mkdir -p $O
export FM_TRAJ_CACHE=traj_cache
timeout -k 10 240 python -u tools/miss_report.py --tag base > $O/miss.jsonl 2> $O/miss.err || { echo "MISS FAILED"; tail -20 $O/miss.err; exit 1; }
for v in int64 ieee; do
  FACTORYSIM_LIB=factory_marl_amd/lib_$v.so timeout -k 10 240 python -u tools/parity_sweep.py --prec fp32 --tag $v >> $O/sweep.jsonl 2>> $O/sweep.err || { echo "SWEEP FAILED $v"; tail -20 $O/sweep.err; exit 1; }
  FACTORYSIM_LIB=factory_marl_amd/lib_$v.so timeout -k 10 240 python -u tools/miss_report.py --tag $v >> $O/miss.jsonl 2>> $O/miss.err || { echo "MISS FAILED"; tail -20 $O/miss.err; exit 1; }
  FACTORYSIM_LIB=factory_marl_amd/lib_$v.so timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --fp64-steps 0 > $O/bench_$v.json 2> $O/bench_$v.err || { echo "BENCH FAILED"; tail $O/bench_$v.err; exit 1; }
done
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --fp64-steps 0 > $O/bench_base.json 2> $O/bench_base.err || { echo "BENCH FAILED"; tail $O/bench_base.err; exit 1; }
grep -h '"value"' $O/bench_*.json | python -c "import sys,json; [print(json.loads(l)['value']) for l in sys.stdin]"
