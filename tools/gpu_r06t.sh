# smoke() on cuda:0, then the fp64 geom-centre A/B (tools/ab_glgx.sh)
set -o pipefail
mkdir -p gpurun_out/r06t
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06t/smoke.log 2>&1 || { tail -20 gpurun_out/r06t/smoke.log; exit 1; }
tail -1 gpurun_out/r06t/smoke.log
bash tools/ab_glgx.sh
