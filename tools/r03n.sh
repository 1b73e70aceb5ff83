#!/bin/bash
# round 3 (n): fp32 default Newton tolerance 1e-8 (MuJoCo's); cached-midphase margin 4 / 2 / 1 cm on config 5 and
# (2,8); GPU suite
set -o pipefail
O=gpurun_out/r03n; mkdir -p $O
export FM_TRAJ_CACHE=traj_cache
timeout -k 10 300 python -u tools/parity_sweep.py --prec fp32 --tag tol1e-8default >> $O/sweep.jsonl 2>> $O/sweep.err || { echo "SWEEP FAILED"; tail -20 $O/sweep.err; exit 1; }
cat $O/sweep.jsonl
for v in main mc2 mc1; do
  L=factory_marl_amd/libfactorysim.so; [ $v != main ] && L=factory_marl_amd/lib_$v.so
  FACTORYSIM_LIB=$L timeout -k 10 300 python bench.py --workload config5 --steps 10 --warmup 3 --no-cpu-baseline --solver-tolerance 1e-8 > $O/bench_c5_$v.json 2> $O/bench_c5.err || { echo "BENCH c5 $v FAILED"; tail $O/bench_c5.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_c5_$v.json')); print('$v c5', d['value'])"
  FACTORYSIM_LIB=$L timeout -k 10 300 python -u tools/phase_profile.py --steps 5 --arms 2 --objects 8 > $O/phase_2x8_$v.json 2>> $O/phase.err || { echo "PHASE28 FAILED"; tail $O/phase.err; exit 1; }
  python -c "import json; d=json.load(open('$O/phase_2x8_$v.json')); print('$v 2x8', d['_total_us_per_arena_substep'], d['_collision_total_us_per_arena_substep'])"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; echo "tests rc $?"; tail -8 $O/tests.log
