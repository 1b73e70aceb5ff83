#!/bin/bash
# fp32 parity after the master state + z-shifted frame: solver tolerance / IEEE div-sqrt variants
set -o pipefail
O=gpurun_out/r02e
mkdir -p $O
export TMPDIR=/tmp
S=$O/sweep.jsonl
run() { timeout -k 10 240 "$@" >> $S 2>> $O/sweep.err || { echo "SWEEP FAILED: $*"; tail -5 $O/sweep.err; exit 1; }; }
run env FM_NO_NOISE_GUARD=1 python tools/parity_sweep.py --prec fp32 --tol 1e-10 --tag tight
run env FM_NO_NOISE_GUARD=1 python tools/parity_sweep.py --prec fp32 --tol 1e-12 --iters 200 --tag tighter
run env FACTORYSIM_LIB=factory_marl_amd/lib_ieee.so python tools/parity_sweep.py --prec fp32 --tag ieee
run env FACTORYSIM_LIB=factory_marl_amd/lib_ieee.so FM_NO_NOISE_GUARD=1 python tools/parity_sweep.py --prec fp32 --tol 1e-10 --tag ieee_tight
python -c "
import json
for l in open('$S'):
    d=json.loads(l); print(d['tag'], d['traj'], d['within'], '%.2e'%d['median'], '%.2e'%d['worst'], d['missing_steps'][:20])"
echo R02E_OK
