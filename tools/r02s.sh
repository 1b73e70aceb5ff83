#!/bin/bash
# sparse LDS Cholesky: full GPU suite, (4,16) and fp64 (2,8) phase profiles
set -o pipefail
O=gpurun_out/r02s
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 400 --timeout-method thread > $O/tests.log 2>&1 || { echo "GPU SUITE FAILED"; grep -E "fp32 \(|PASS|FAIL" $O/tests.log | tail -30; tail -30 $O/tests.log; exit 1; }
grep -E "fp32 \(|passed|failed" $O/tests.log
timeout -k 10 170 python tools/phase_profile.py --arms 4 --objects 16 --arenas 2048 --preroll 60 --steps 4 > $O/phase_4x16.json 2> $O/p.err || { echo P FAILED; tail $O/p.err; exit 1; }
timeout -k 10 170 python tools/phase_profile.py --objects 8 --arenas 4096 --preroll 60 --steps 4 --precision fp64 > $O/phase_2x8_fp64.json 2> $O/p2.err || { echo P2 FAILED; tail $O/p2.err; exit 1; }
python - <<'PY'
import json
for f in ("phase_4x16","phase_2x8_fp64"):
    d=json.load(open(f"gpurun_out/r02s/{f}.json"))
    print(f, " ".join(f"{k}={v['us_per_arena_substep']:.1f}" if isinstance(v,dict) else f"{k}={v}" for k,v in d.items()))
PY
timeout -k 10 300 python bench.py --workload config5 > $O/bench5.json 2> $O/bench5.err || { echo BENCH5 FAILED; tail $O/bench5.err; exit 1; }
cut -c1-200 $O/bench5.json; grep -o '"kernel_ms_avg.*' $O/bench5.json
echo R02S_OK
