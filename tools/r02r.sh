#!/bin/bash
# (4,16) runtime-dims scene phase profile (config 5 physics)
set -o pipefail
O=gpurun_out/r02r
mkdir -p $O
timeout -k 10 170 python tools/phase_profile.py --arms 4 --objects 16 --arenas 2048 --preroll 60 --steps 4 > $O/phase_4x16.json 2> $O/p.err || { echo P FAILED; tail $O/p.err; exit 1; }
python - <<'PY'
import json
d=json.load(open("gpurun_out/r02r/phase_4x16.json"))
print(" ".join(f"{k}={v['us_per_arena_substep']:.1f}" if isinstance(v,dict) else f"{k}={v}" for k,v in d.items()))
PY
