#!/bin/bash
# round 3 final: parity sweep of the final kernels (fp32 against the 1e-12 and the MuJoCo-tolerance oracle, fp64),
# then the GPU suite verbose
set -o pipefail
O=gpurun_out/r03fin2; mkdir -p $O
export FM_TRAJ_CACHE=traj_cache
timeout -k 10 400 python -u tools/parity_sweep.py --prec fp32 --tag final --traj 2,4,96,7 2,4,300,21 2,8,300,5 2,10,250,9 4,16,150,3,PauseIKToggleEnv > $O/sweep.jsonl 2> $O/sweep.err || { echo "SWEEP FAILED"; tail -20 $O/sweep.err; exit 1; }
timeout -k 10 300 python -u tools/parity_sweep.py --prec fp32 --tag final_vs_tol8 --traj 2,4,300,21,,1e-8 2,8,300,5,,1e-8 2,10,250,9,,1e-8 >> $O/sweep.jsonl 2>> $O/sweep.err || { echo "SWEEP8 FAILED"; tail -20 $O/sweep.err; exit 1; }
timeout -k 10 300 python -u tools/parity_sweep.py --prec fp64 --tag final_f64 >> $O/sweep.jsonl 2>> $O/sweep.err || { echo "SWEEP64 FAILED"; tail -20 $O/sweep.err; exit 1; }
python -c "
import json
for l in open('$O/sweep.jsonl'):
    r=json.loads(l); print(r['tag'], r['traj'], r['within'], '%.3e' % r['worst'], r['int_bad'], r['flag_bad'], r['missing_steps'][:8])
"
[ -n "$SKIP_TESTS" ] || timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; echo "tests rc $?"; tail -4 $O/tests.log
