#!/bin/bash
# fp64 sparse register Cholesky: full GPU suite, fp64 phase profile, headline bench with the fp64 leg
set -o pipefail
O=gpurun_out/r02v
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { echo "GPU SUITE FAILED"; tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log
timeout -k 10 170 python tools/phase_profile.py --precision fp64 > $O/phase_fp64.json 2> $O/p.err || { echo P FAILED; tail $O/p.err; exit 1; }
python - <<'PY'
import json
d=json.load(open("gpurun_out/r02v/phase_fp64.json"))
print(" ".join(f"{k}={v['us_per_arena_substep']:.1f}" if isinstance(v,dict) else f"{k}={v}" for k,v in d.items()))
PY
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo BENCH FAILED; tail $O/bench.err; exit 1; }
cut -c1-200 $O/bench.json; grep -o '"fp64_value": {"value": [0-9.]*' $O/bench.json
echo R02V_OK
