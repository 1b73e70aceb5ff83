#!/bin/bash
# scheduler-strategy variants of the (2,4) kernel: bit-identity of results, then the headline bench for each
set -o pipefail
O=gpurun_out/r02y
mkdir -p $O
export TMPDIR=/tmp
for v in main maxilp bias0; do
  if [ $v = main ]; then L=factory_marl_amd/libfactorysim.so; else L=factory_marl_amd/lib_$v.so; fi
  FACTORYSIM_LIB=$L timeout -k 10 120 python tools/variant_obs.py $O/obs_$v.npy > $O/obs_$v.log 2>&1 || { echo "OBS $v FAILED"; tail $O/obs_$v.log; exit 1; }
done
python -c "
import numpy as np
a=np.load('$O/obs_main.npy')
for v in ['maxilp','bias0']:
    b=np.load('$O/obs_'+v+'.npy'); print(v, 'bit-identical' if np.array_equal(a,b) else 'DIFFERS')
"
for v in main maxilp bias0 main; do
  if [ $v = main ]; then L=factory_marl_amd/libfactorysim.so; else L=factory_marl_amd/lib_$v.so; fi
  FACTORYSIM_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --fp64-steps 0 > $O/bench_$v.json 2> $O/bench_$v.err || { echo "BENCH $v FAILED"; tail $O/bench_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$v.json')); print('$v', d['value'], d['roofline']['kernel_ms_avg'])"
done
echo R02Y_OK
