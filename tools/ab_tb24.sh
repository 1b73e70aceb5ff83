set -o pipefail
O=gpurun_out/r06l; mkdir -p $O
for i in 1 2; do
  for v in prod tb24; do
    L=factory_marl_amd/libfactorysim.so; [ $v = tb24 ] && L=factory_marl_amd/libfactorysim_tb24.so
    FACTORYSIM_LIB=$L timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --fp64-steps 30 > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err || exit 1
    python -c "import json; d=json.load(open('$O/b_${v}_$i.json')); print('$v', $i, d['value'], d['roofline']['kernel_ms_avg'], 'fp64', d['fp64_value']['value'])"
  done
done
FACTORYSIM_LIB=factory_marl_amd/libfactorysim_tb24.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -s --timeout 300 --timeout-method thread -k "teacher_forced_fp32 or test_teacher_forced_fp64 or above_64 or ik_classes_fp64 or long_fp64" > $O/tests_tb24.log 2>&1 || exit 1
tail -1 $O/tests_tb24.log
