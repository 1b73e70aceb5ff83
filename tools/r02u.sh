#!/bin/bash
set -o pipefail
O=gpurun_out/r02u
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -v -s --timeout 400 --timeout-method thread -k "other_configs or long_fp64 or config5 or other_scenes" > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
grep -E "fp32 \(|passed|failed" $O/tests.log
timeout -k 10 170 python tools/phase_profile.py --arms 4 --objects 16 --arenas 2048 --preroll 60 --steps 4 > $O/phase_4x16.json 2> $O/p.err || { echo P FAILED; tail $O/p.err; exit 1; }
python - <<'PY'
import json
d=json.load(open("gpurun_out/r02u/phase_4x16.json"))
print(" ".join(f"{k}={v['us_per_arena_substep']:.1f}" if isinstance(v,dict) else f"{k}={v}" for k,v in d.items()))
PY
timeout -k 10 300 python bench.py --workload config5 > $O/bench5.json 2> $O/bench5.err || { echo BENCH5 FAILED; tail $O/bench5.err; exit 1; }
cut -c1-200 $O/bench5.json
echo R02T_OK
