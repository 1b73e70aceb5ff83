#!/bin/bash
# round 3 (s): expansion owner by prefix-max scan: parity identical, narrowphase split, bench, GPU suite
set -o pipefail
O=gpurun_out/r03s; mkdir -p $O
export FM_TRAJ_CACHE=traj_cache
timeout -k 10 300 python -u tools/parity_sweep.py --prec fp32 --tag scan --traj 2,4,96,7 2,4,300,21 2,8,300,5 2,10,250,9 4,16,150,3,PauseIKToggleEnv >> $O/sweep.jsonl 2>> $O/sweep.err || { echo "SWEEP FAILED"; tail -20 $O/sweep.err; exit 1; }
timeout -k 10 300 python -u tools/parity_sweep.py --prec fp64 --tag f64 >> $O/sweep.jsonl 2>> $O/sweep.err || { echo "SWEEP64 FAILED"; tail -20 $O/sweep.err; exit 1; }
python -c "
import json
for l in open('$O/sweep.jsonl'):
    r=json.loads(l); print(r['tag'], r['traj'], r['within'], '%.3e' % r['worst'], r['int_bad'], r['flag_bad'], r['missing_steps'][:8])
"
timeout -k 10 300 python -u tools/phase_profile.py --steps 10 > $O/phase_fp32.json 2> $O/phase.err || { echo "PHASE FAILED"; tail $O/phase.err; exit 1; }
python -c "import json; d=json.load(open('$O/phase_fp32.json')); print({k:(v['us_per_arena_substep'] if isinstance(v,dict) else v) for k,v in d.items() if k.startswith('coll') or k.startswith('_')})"
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print('c2', d['value'], d['fp64_value']['value'])"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; echo "tests rc $?"; tail -4 $O/tests.log
