#!/bin/bash
# round 3 (z): arm kinematics + RNE as chain scans, the arms 9x9 solves over 9 lanes, belt diagonal by wave sum -- switch A/B (timing of each setting), phase profiles, bench,
# then the GPU suite
set -o pipefail
O=gpurun_out/r03z; mkdir -p $O
timeout -k 10 300 python -u tools/switch_probe.py "" "FM_SERIAL_FK=1" "FM_SERIAL_SPD9=1" "FM_SERIAL_FK=1 FM_SERIAL_SPD9=1" > $O/switch_probe.log 2>&1 || { echo "PROBE FAILED"; tail -20 $O/switch_probe.log; exit 1; }
tail -1 $O/switch_probe.log
timeout -k 10 200 python tools/phase_profile.py --precision fp32 > $O/phase_fp32.json 2> $O/phase.err || { echo "PHASE FAILED"; tail $O/phase.err; exit 1; }
FM_SERIAL_FK=1 FM_SERIAL_SPD9=1 timeout -k 10 200 python tools/phase_profile.py --precision fp32 > $O/phase_fp32_prev.json 2>> $O/phase.err || { echo "PHASE2 FAILED"; tail $O/phase.err; exit 1; }
python - << 'PY'
import json
for f in ("phase_fp32", "phase_fp32_prev"):
    d = json.load(open(f"gpurun_out/r03z/{f}.json"))
    print(f, " ".join(f"{k}={v['us_per_arena_substep']:.2f}" for k, v in d.items() if isinstance(v, dict)))
PY
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail $O/bench.err; exit 1; }
FM_SERIAL_FK=1 FM_SERIAL_SPD9=1 timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/bench_prev.json 2> $O/bench2.err || { echo "BENCH2 FAILED"; tail $O/bench2.err; exit 1; }
python -c "
import json
for f in ('bench', 'bench_prev'):
    d = json.load(open('$O/' + f + '.json')); print(f, d['value'], d['fp64_value']['value'])
"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; echo "tests rc $?"; tail -4 $O/tests.log
