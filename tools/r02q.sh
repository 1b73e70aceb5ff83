#!/bin/bash
# bordered register Cholesky for (2,8) / (2,10): parity, phase profile, config-3 bench
set -o pipefail
O=gpurun_out/r02q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -v -s --timeout 400 --timeout-method thread -k "other_scenes or other_configs or long_fp64" > $O/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "fp32 \(|PASS|FAIL" $O/tests.log; tail -30 $O/tests.log; exit 1; }
grep -E "fp32 \(|passed|failed" $O/tests.log
for k in 8 10; do
timeout -k 10 170 python tools/phase_profile.py --objects $k --arenas 4096 --preroll 100 > $O/phase_2x$k.json 2> $O/p$k.err || { echo P$k FAILED; tail $O/p$k.err; exit 1; }
python - $k <<'PY'
import json,sys
d=json.load(open(f"gpurun_out/r02q/phase_2x{sys.argv[1]}.json"))
print(" ".join(f"{k}={v['us_per_arena_substep']:.1f}" if isinstance(v,dict) else f"{k}={v}" for k,v in d.items()))
PY
done
timeout -k 10 400 python bench.py --workload config3 > $O/bench3.json 2> $O/bench3.err || { echo BENCH3 FAILED; tail $O/bench3.err; exit 1; }
cut -c1-250 $O/bench3.json
echo R02Q_OK
