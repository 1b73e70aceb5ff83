#!/bin/bash
# round 3: sub-phase split of rows + setup (lib_split1) and gradient + line search (lib_split2), (2,4) fp32
set -o pipefail
O=gpurun_out/r03sp; mkdir -p $O
for v in split1 split2; do
  FACTORYSIM_LIB=factory_marl_amd/lib_$v.so timeout -k 10 200 python tools/phase_profile.py --precision fp32 > $O/phase_$v.json 2>> $O/phase.err || { echo "PHASE $v FAILED"; tail $O/phase.err; exit 1; }
done
python - << 'PY'
import json
for f in ("phase_split1", "phase_split2"):
    d = json.load(open(f"gpurun_out/r03sp/{f}.json"))
    print(f, " ".join(f"{k}={v['us_per_arena_substep']:.2f}" for k, v in d.items() if isinstance(v, dict)))
PY
