#!/bin/bash
# register-operand MFMA Hessian contact term ((2,4) fp32): parity tests, A/B bench vs FM_HESS_ATOMICS=1, phase profile
set -o pipefail
O=gpurun_out/r02n2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "fp32 or full_size or fp64" -x -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "within|FAIL|Error" $O/tests.log | head; tail -20 $O/tests.log; exit 1; }
grep -E "fp32 teacher|float restatement|passed|failed" $O/tests.log
for r in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --fp64-steps 0 > $O/mfma_$r.json 2> $O/mfma_$r.err || { echo "BENCH MFMA FAILED"; tail $O/mfma_$r.err; exit 1; }
  FM_HESS_ATOMICS=1 timeout -k 10 200 python bench.py --no-cpu-baseline --fp64-steps 0 > $O/atom_$r.json 2> $O/atom_$r.err || { echo "BENCH ATOM FAILED"; tail $O/atom_$r.err; exit 1; }
  python -c "import json; a=json.load(open('$O/mfma_$r.json')); b=json.load(open('$O/atom_$r.json')); print('mfma', a['value'], a['roofline']['kernel_ms_avg'], 'atomics', b['value'], b['roofline']['kernel_ms_avg'])"
done
timeout -k 10 200 python tools/phase_profile.py --precision fp32 > $O/phase_fp32.json 2> $O/phase.err || { echo PHASE FAILED; tail $O/phase.err; exit 1; }
python -c "import json; d=json.load(open('$O/phase_fp32.json')); print({k: v['us_per_arena_substep'] for k, v in d.items() if isinstance(v, dict)}, d['_total_us_per_arena_substep'])"
echo R02N2_OK
