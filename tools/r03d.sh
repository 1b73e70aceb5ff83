#!/bin/bash
# round 3 (d): contact impedance / R in float64 for the fp32 build; precision variants (IEEE div/sqrt, float64
# implicit solve) on the parity sweep; behavioural statistics; GPU test suite
set -o pipefail
O=gpurun_out/r03d; mkdir -p $O
export FM_TRAJ_CACHE=traj_cache
for v in main ieee int64; do
  L=factory_marl_amd/libfactorysim.so; [ $v != main ] && L=factory_marl_amd/lib_$v.so
  FACTORYSIM_LIB=$L timeout -k 10 300 python -u tools/parity_sweep.py --prec fp32 --tag $v >> $O/sweep.jsonl 2>> $O/sweep.err || { echo "SWEEP $v FAILED"; tail -20 $O/sweep.err; exit 1; }
done
timeout -k 10 300 python -u tools/parity_sweep.py --prec fp64 --tag f64 >> $O/sweep.jsonl 2>> $O/sweep.err || { echo "SWEEP64 FAILED"; tail -20 $O/sweep.err; exit 1; }
T416=4,16,150,3,PauseIKToggleEnv
timeout -k 10 300 python -u tools/parity_sweep.py --prec fp32 --tag dense416 --traj $T416 >> $O/sweep.jsonl 2>> $O/sweep.err || { echo "SWEEP dense416 FAILED"; tail -20 $O/sweep.err; exit 1; }
FM_CHOL_LDS=2 timeout -k 10 300 python -u tools/parity_sweep.py --prec fp32 --tag sparse416 --traj $T416 >> $O/sweep.jsonl 2>> $O/sweep.err || { echo "SWEEP sparse416 FAILED"; tail -20 $O/sweep.err; exit 1; }
timeout -k 10 300 python -u tools/parity_sweep.py --prec fp64 --tag f64_416 --traj $T416 >> $O/sweep.jsonl 2>> $O/sweep.err || { echo "SWEEP f64_416 FAILED"; tail -20 $O/sweep.err; exit 1; }
timeout -k 10 300 python bench.py --workload config5 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || { echo "BENCH c5 FAILED"; tail $O/bench_c5.err; exit 1; }
cat $O/bench_c5.json
FM_CHOL_LDS=2 timeout -k 10 300 python bench.py --workload config5 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_c5_sparse.json 2> $O/bench_c5s.err || { echo "BENCH c5 sparse FAILED"; tail $O/bench_c5s.err; exit 1; }
cat $O/bench_c5_sparse.json
timeout -k 10 300 python -u tools/miss_report.py --tag main > $O/miss.jsonl 2> $O/miss.err || { echo "MISS FAILED"; tail -20 $O/miss.err; exit 1; }
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 400 python -u tools/behaviour.py base 2 --arenas 1000 --episodes 10 > $O/beh_base2.json 2> $O/beh.err || { echo "BEH2 FAILED"; tail $O/beh.err; exit 1; }
cat $O/beh_base2.json
timeout -k 10 400 python -u tools/behaviour.py policy rk5rxnav --arenas 1000 --precision fp32 > $O/beh_rk5.json 2>> $O/beh.err || { echo "BEH rk5 FAILED"; tail $O/beh.err; exit 1; }
cat $O/beh_rk5.json
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; echo "tests rc $?"; tail -15 $O/tests.log
