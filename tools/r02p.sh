#!/bin/bash
# phase profiles of the larger fixed scenes (config 3 / the reference runs' K)
set -o pipefail
O=gpurun_out/r02p
mkdir -p $O
timeout -k 10 200 python tools/phase_profile.py --objects 8 --arenas 8192 > $O/phase_2x8.json 2> $O/p8.err || { echo P8 FAILED; tail $O/p8.err; exit 1; }
timeout -k 10 200 python tools/phase_profile.py --objects 10 --arenas 8192 > $O/phase_2x10.json 2> $O/p10.err || { echo P10 FAILED; tail $O/p10.err; exit 1; }
python - <<'PY'
import json
for s in ("2x8","2x10"):
    d=json.load(open(f"gpurun_out/r02p/phase_{s}.json"))
    print(s, " ".join(f"{k}={v['us_per_arena_substep']:.1f}" if isinstance(v,dict) else f"{k}={v}" for k,v in d.items()))
PY
