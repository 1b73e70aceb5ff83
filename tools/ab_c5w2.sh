# A/B: config 5 ((4,16) PauseIKToggle fp32) product vs two waves per SIMD with the collision lists, the coupled system
# and the phase clocks in the global block (FM_GL416=1: 32.0 KB of LDS, 5 arenas per CU instead of 4), then that
# variant's (4,16) parity tests
set -o pipefail
O=gpurun_out/r06o; mkdir -p $O
for i in 1 2; do
  for v in prod c5w2; do
    L=factory_marl_amd/libfactorysim.so; [ $v = c5w2 ] && L=factory_marl_amd/libfactorysim_c5w2.so
    FACTORYSIM_LIB=$L timeout -k 10 300 python bench.py --workload config5 --steps 10 --warmup 2 --no-cpu-baseline > $O/c5_${v}_$i.json 2> $O/c5_${v}_$i.err || exit 1
    python -c "import json; d=json.load(open('$O/c5_${v}_$i.json')); print('$v', $i, d['value'], d['roofline']['kernel_ms_avg'])"
  done
done
FACTORYSIM_LIB=factory_marl_amd/libfactorysim_c5w2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -s --timeout 300 --timeout-method thread -k "4x16 or config5" > $O/tests_c5w2.log 2>&1 || exit 1
tail -1 $O/tests_c5w2.log
