# A/B batch: (a) the (2,10) scene with the phase clocks in the global block (libfactorysim.so: 180 VGPRs spilled in
# the fp32 AllFullRL kernel) vs in LDS (libfactorysim_next.so: 893); (b) config 5 product vs two waves per SIMD
# (libfactorysim_c5w2.so), then the c5w2 (4,16) parity tests
set -o pipefail
O=gpurun_out/r06r; mkdir -p $O
for i in 1 2; do
  for v in profgl proflds; do
    L=factory_marl_amd/libfactorysim.so; [ $v = proflds ] && L=factory_marl_amd/libfactorysim_next.so
    FACTORYSIM_LIB=$L timeout -k 10 300 python bench.py --objects 10 --arenas 16384 --steps 10 --warmup 2 --preroll 100 --fp64-steps 0 --no-cpu-baseline > $O/s210_${v}_$i.json 2> $O/s210_${v}_$i.err || exit 1
    python -c "import json; d=json.load(open('$O/s210_${v}_$i.json')); print('s210', '$v', $i, d['value'], d['roofline']['kernel_ms_avg'])"
  done
done
for i in 1 2; do
  for v in prod c5w2; do
    L=factory_marl_amd/libfactorysim.so; [ $v = c5w2 ] && L=factory_marl_amd/libfactorysim_c5w2.so
    FACTORYSIM_LIB=$L timeout -k 10 300 python bench.py --workload config5 --steps 10 --warmup 2 --no-cpu-baseline > $O/c5_${v}_$i.json 2> $O/c5_${v}_$i.err || exit 1
    python -c "import json; d=json.load(open('$O/c5_${v}_$i.json')); print('c5', '$v', $i, d['value'], d['roofline']['kernel_ms_avg'])"
  done
done
FACTORYSIM_LIB=factory_marl_amd/libfactorysim_c5w2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -s --timeout 300 --timeout-method thread -k "4x16 or config5" > $O/tests_c5w2.log 2>&1 || exit 1
tail -1 $O/tests_c5w2.log
