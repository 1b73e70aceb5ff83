#!/bin/bash
# Measurement run on the GPU box (via gpurun): full bench line (with the CPU baseline), rocprofv3 kernel
# trace + stats, the two PMC passes for HBM traffic (FETCH_SIZE and WRITE_SIZE cannot share a pass), and the
# fp32 / fp64 phase profiles.  usage: bash tools/gpu_measure.sh TAG
set -o pipefail
TAG=${1:-meas}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/ktrace.log 2>&1 || { echo "KTRACE FAILED"; tail $O/ktrace.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/pmc_fetch.log 2>&1 || { echo "PMC FETCH FAILED"; tail $O/pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/pmc_write.log 2>&1 || { echo "PMC WRITE FAILED"; tail $O/pmc_write.log; exit 1; }
timeout -k 10 200 python tools/phase_profile.py --precision fp32 > $O/phase_fp32.json 2> $O/phase_fp32.err || { echo "PHASE32 FAILED"; exit 1; }
timeout -k 10 300 python tools/phase_profile.py --precision fp64 > $O/phase_fp64.json 2> $O/phase_fp64.err || { echo "PHASE64 FAILED"; exit 1; }
echo MEASURE_OK
