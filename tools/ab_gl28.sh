set -o pipefail
O=gpurun_out/r06k; mkdir -p $O
for i in 1 2; do
  for v in prod gl28; do
    L=factory_marl_amd/libfactorysim.so; [ $v = gl28 ] && L=factory_marl_amd/libfactorysim_gl28.so
    FACTORYSIM_LIB=$L timeout -k 10 300 python bench.py --workload config3 --steps 12 --warmup 2 --preroll 100 --ppo-epochs 1 --no-cpu-baseline > $O/c3_${v}_$i.json 2> $O/c3_${v}_$i.err || exit 1
    python -c "import json; d=json.load(open('$O/c3_${v}_$i.json')); print('$v', $i, d['value'], d['kernel_ms_avg'])"
  done
done
FACTORYSIM_LIB=factory_marl_amd/libfactorysim_gl28.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -s --timeout 300 --timeout-method thread -k "fp64_other_configs or long_fp64 or fp32_other_scenes or mujoco_tolerance" > $O/tests_gl28.log 2>&1 || exit 1
tail -1 $O/tests_gl28.log
