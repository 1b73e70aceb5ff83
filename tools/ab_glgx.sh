# A/B: config 2 (fp32 and the fp64 leg) product vs the fp64 (2,4) geom centres in the global block (FM_GL_GX=1:
# 22.7 -> 18.7 KB, 7 -> 8 fp64 arenas per CU), then that variant's fp64 (2,4) parity tests
set -o pipefail
O=gpurun_out/r06t; mkdir -p $O
for i in 1 2; do
  for v in prod glgx; do
    L=factory_marl_amd/libfactorysim.so; [ $v = glgx ] && L=factory_marl_amd/libfactorysim_glgx.so
    FACTORYSIM_LIB=$L timeout -k 10 300 python bench.py --steps 10 --warmup 2 --fp64-steps 40 --no-cpu-baseline > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err || exit 1
    python -c "import json; d=json.load(open('$O/b_${v}_$i.json')); print('$v', $i, d['value'], 'fp64', d['fp64_value']['value'], d['fp64_value']['kernel_ms_avg'])"
  done
done
FACTORYSIM_LIB=factory_marl_amd/libfactorysim_glgx.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -s --timeout 300 --timeout-method thread -k "fp64 and not 4x16 and not other_configs and not long_fp64" > $O/tests_glgx.log 2>&1 || exit 1
tail -1 $O/tests_glgx.log
