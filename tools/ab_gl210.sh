# A/B: the (2,10) scene (16384 arenas, random policy) product vs the fp32 (2,10) collision lists + coupled system in the global block
# (FM_GL210=1: 8 arenas per CU instead of 5), then that variant's (2,10) parity tests
set -o pipefail
O=gpurun_out/r06m; mkdir -p $O
for i in 1 2; do
  for v in prod gl210; do
    L=factory_marl_amd/libfactorysim.so; [ $v = gl210 ] && L=factory_marl_amd/libfactorysim_gl210.so
    FACTORYSIM_LIB=$L timeout -k 10 300 python bench.py --objects 10 --arenas 16384 --steps 10 --warmup 2 --preroll 100 --fp64-steps 0 --no-cpu-baseline > $O/s210_${v}_$i.json 2> $O/s210_${v}_$i.err || exit 1
    python -c "import json; d=json.load(open('$O/s210_${v}_$i.json')); print('$v', $i, d['value'], d['roofline']['kernel_ms_avg'])"
  done
done
FACTORYSIM_LIB=factory_marl_amd/libfactorysim_gl210.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -s --timeout 300 --timeout-method thread -k "(fp32_ik_classes and 2-10) or fp64_other_configs or long_fp64 or fp32_other_scenes or mujoco_tolerance" > $O/tests_gl210.log 2>&1 || exit 1
tail -1 $O/tests_gl210.log
