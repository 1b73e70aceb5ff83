#!/bin/bash
# round 3 (u): the GPU kernel against oracle outputs at MuJoCo's Newton tolerance (1e-8) from the same states
set -o pipefail
O=gpurun_out/r03u; mkdir -p $O
export FM_TRAJ_CACHE=traj_cache
T="2,4,96,7,,1e-8 2,4,300,21,,1e-8 2,8,300,5,,1e-8 2,10,250,9,,1e-8"
timeout -k 10 300 python -u tools/parity_sweep.py --prec fp32 --tag vs_tol8 --traj $T > $O/sweep.jsonl 2> $O/sweep.err || { echo "SWEEP FAILED"; tail -20 $O/sweep.err; exit 1; }
timeout -k 10 300 python -u tools/parity_sweep.py --prec fp64 --tol 1e-8 --tag f64_vs_tol8 --traj $T >> $O/sweep.jsonl 2>> $O/sweep.err || { echo "SWEEP64 FAILED"; tail -20 $O/sweep.err; exit 1; }
python -c "
import json
for l in open('$O/sweep.jsonl'):
    r=json.loads(l); print(r['tag'], r['traj'], r['within'], '%.3e' % r['worst'], r['int_bad'], r['flag_bad'], r['missing_steps'][:8])
"
