#!/bin/bash
# round 3: fused Newton warmstart passes (switch A/B: bit-identity + timing), two-pass arrowhead Cholesky of the
# bordered scenes ((2,8) phase profile and config 3 A/B), bench; then the parity sweep and the GPU suite (r03fin2.sh)
set -o pipefail
O=gpurun_out/r03fz; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u tools/switch_probe.py --precisions fp32,fp64 "" "FM_TWO_PASS_SETUP=1" > $O/switch_probe.log 2>&1 || { echo "PROBE FAILED"; tail -20 $O/switch_probe.log; exit 1; }
tail -1 $O/switch_probe.log
timeout -k 10 200 python -u tools/phase_profile.py --steps 5 --arms 2 --objects 8 > $O/phase_2x8.json 2> $O/phase.err || { echo "PHASE FAILED"; tail $O/phase.err; exit 1; }
FM_NO_ARROW=1 timeout -k 10 200 python -u tools/phase_profile.py --steps 5 --arms 2 --objects 8 > $O/phase_2x8_noarrow.json 2>> $O/phase.err || { echo "PHASE2 FAILED"; tail $O/phase.err; exit 1; }
python - << 'PY'
import json
for f in ("phase_2x8", "phase_2x8_noarrow"):
    d = json.load(open(f"gpurun_out/r03fz/{f}.json"))
    print(f, " ".join(f"{k}={v['us_per_arena_substep']:.2f}" for k, v in d.items() if isinstance(v, dict)))
PY
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail $O/bench.err; exit 1; }
timeout -k 10 300 python bench.py --workload config3 --steps 8 --warmup 2 --no-cpu-baseline > $O/bench_config3.json 2> $O/bench_c3.err || { echo "BENCH C3 FAILED"; tail $O/bench_c3.err; exit 1; }
FM_NO_ARROW=1 timeout -k 10 300 python bench.py --workload config3 --steps 8 --warmup 2 --no-cpu-baseline > $O/bench_config3_noarrow.json 2> $O/bench_c3b.err || { echo "BENCH C3b FAILED"; tail $O/bench_c3b.err; exit 1; }
python -c "
import json
for f in ('bench', 'bench_config3', 'bench_config3_noarrow'):
    d = json.load(open('$O/' + f + '.json')); print(f, d['value'], d.get('fp64_value', {}).get('value'))
"
SKIP_TESTS=1 bash tools/r03fin2.sh
