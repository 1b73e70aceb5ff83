#!/bin/bash
# round 3 (o): dense Cholesky skips zero tiles; 1 cm midphase margin; midphase cache at (2,4) too; parity (must equal
# r03n), config 2 / 5, phase profiles, suite
set -o pipefail
O=gpurun_out/r03o; mkdir -p $O
export FM_TRAJ_CACHE=traj_cache
timeout -k 10 300 python -u tools/parity_sweep.py --prec fp32 --tag skip --traj 2,4,96,7 2,4,300,21 2,8,300,5 2,10,250,9 4,16,150,3,PauseIKToggleEnv >> $O/sweep.jsonl 2>> $O/sweep.err || { echo "SWEEP FAILED"; tail -20 $O/sweep.err; exit 1; }
timeout -k 10 300 python -u tools/parity_sweep.py --prec fp64 --tag f64 >> $O/sweep.jsonl 2>> $O/sweep.err || { echo "SWEEP64 FAILED"; tail -20 $O/sweep.err; exit 1; }
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print('c2', d['value'], d['fp64_value']['value'])"
timeout -k 10 300 python -u tools/phase_profile.py --steps 10 > $O/phase_fp32.json 2> $O/phase.err || { echo "PHASE FAILED"; tail $O/phase.err; exit 1; }
python -c "import json; d=json.load(open('$O/phase_fp32.json')); print({k:(v['us_per_arena_substep'] if isinstance(v,dict) else v) for k,v in d.items() if k.startswith('coll') or k.startswith('_')})"
cat $O/sweep.jsonl
timeout -k 10 300 python bench.py --workload config5 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_config5.json 2> $O/bench_c5.err || { echo "BENCH c5 FAILED"; tail $O/bench_c5.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_config5.json')); print('c5', d['value'], d['diagnostics'])"
timeout -k 10 300 python -u tools/phase_profile.py --steps 3 --arms 4 --objects 16 --env-class PauseIKToggleEnv --preroll 60 > $O/phase_fp32_4x16.json 2> $O/phase.err || { echo "PHASE416 FAILED"; tail $O/phase.err; exit 1; }
python -c "import json; d=json.load(open('$O/phase_fp32_4x16.json')); print({k:(v['us_per_arena_substep'] if isinstance(v,dict) else v) for k,v in d.items() if k.startswith('chol') or k.startswith('_')})"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; echo "tests rc $?"; tail -8 $O/tests.log
