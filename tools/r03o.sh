#!/bin/bash
# round 3 (o): dense Cholesky skips zero tiles; 1 cm midphase margin; (4,16) parity, config 5, phase profile, suite
set -o pipefail
O=gpurun_out/r03o; mkdir -p $O
export FM_TRAJ_CACHE=traj_cache
timeout -k 10 300 python -u tools/parity_sweep.py --prec fp32 --tag skip --traj 4,16,150,3,PauseIKToggleEnv 2,8,300,5 >> $O/sweep.jsonl 2>> $O/sweep.err || { echo "SWEEP FAILED"; tail -20 $O/sweep.err; exit 1; }
cat $O/sweep.jsonl
timeout -k 10 300 python bench.py --workload config5 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_config5.json 2> $O/bench_c5.err || { echo "BENCH c5 FAILED"; tail $O/bench_c5.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_config5.json')); print('c5', d['value'], d['diagnostics'])"
timeout -k 10 300 python -u tools/phase_profile.py --steps 3 --arms 4 --objects 16 --env-class PauseIKToggleEnv --preroll 60 > $O/phase_fp32_4x16.json 2> $O/phase.err || { echo "PHASE416 FAILED"; tail $O/phase.err; exit 1; }
python -c "import json; d=json.load(open('$O/phase_fp32_4x16.json')); print({k:(v['us_per_arena_substep'] if isinstance(v,dict) else v) for k,v in d.items() if k.startswith('chol') or k.startswith('_')})"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; echo "tests rc $?"; tail -8 $O/tests.log
