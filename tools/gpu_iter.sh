#!/bin/bash
# One GPU iteration (run on the box via gpurun): parity tests, phase profile, short bench.
# usage: bash tools/gpu_iter.sh TAG [tests|notests]
set -o pipefail
TAG=${1:-iter}
mkdir -p gpurun_out
if [ "${2:-tests}" = "tests" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -2 gpurun_out/${TAG}_tests.log
fi
timeout -k 10 200 python tools/phase_profile.py --precision fp32 > gpurun_out/${TAG}_phase.json 2> gpurun_out/${TAG}_phase.err || { echo "PHASE FAILED"; tail gpurun_out/${TAG}_phase.err; exit 1; }
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "BENCH FAILED"; tail gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
python - "$TAG" << 'PY'
import json,sys
d=json.load(open(f"gpurun_out/{sys.argv[1]}_phase.json"))
print(" ".join(f"{k}={v['us_per_arena_substep']:.1f}" if isinstance(v,dict) else f"{k}={v}" for k,v in d.items()))
PY
