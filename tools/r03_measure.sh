#!/bin/bash
# Round-3 measurement set: default bench (with the CPU baseline leg), config 3 / 5 benches, rocprofv3
# kernel stats + PMC passes on the headline, phase profiles.  usage: bash tools/r03_measure.sh TAG
set -o pipefail
TAG=${1:-r03m}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python bench.py --workload config5 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_config5.json 2> $O/bench_c5.err || { echo "BENCH c5 FAILED"; tail $O/bench_c5.err; exit 1; }
cat $O/bench_config5.json
timeout -k 10 400 python bench.py --workload config3 --no-cpu-baseline > $O/bench_config3.json 2> $O/bench_c3.err || { echo "BENCH c3 FAILED"; tail $O/bench_c3.err; exit 1; }
cat $O/bench_config3.json
P="--steps 3 --warmup 1 --no-cpu-baseline --fp64-steps 0 --preroll 200"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --fp64-steps 0 > $O/ktrace.log 2>&1 || { echo "KTRACE FAILED"; tail $O/ktrace.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -- python3 bench.py $P > $O/pmc_fetch.log 2>&1 || { echo "PMC FETCH FAILED"; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -- python3 bench.py $P > $O/pmc_write.log 2>&1 || { echo "PMC WRITE FAILED"; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $O/pmc_sq -- python3 bench.py $P > $O/pmc_sq.log 2>&1 || { echo "PMC SQ FAILED"; exit 1; }
timeout -k 10 200 python tools/phase_profile.py --precision fp32 > $O/phase_fp32.json 2> $O/phase.err || { echo "PHASE FAILED"; tail $O/phase.err; exit 1; }
timeout -k 10 200 python tools/phase_profile.py --precision fp64 > $O/phase_fp64.json 2>> $O/phase.err || { echo "PHASE64 FAILED"; tail $O/phase.err; exit 1; }
timeout -k 10 300 python -u tools/phase_profile.py --steps 3 --arms 4 --objects 16 --env-class PauseIKToggleEnv --preroll 60 > $O/phase_fp32_4x16.json 2>> $O/phase.err || { echo "PHASE416 FAILED"; tail $O/phase.err; exit 1; }
timeout -k 10 300 python -u tools/phase_profile.py --steps 5 --arms 2 --objects 8 > $O/phase_fp32_2x8.json 2>> $O/phase.err || { echo "PHASE28 FAILED"; tail $O/phase.err; exit 1; }
timeout -k 10 400 python bench.py --workload config4 --steps 4 --warmup 1 --preroll 10 --no-cpu-baseline > $O/bench_config4_1gpu.json 2> $O/bench_c4.err || { echo "BENCH c4 FAILED"; tail $O/bench_c4.err; exit 1; }
cat $O/bench_config4_1gpu.json
find $O -name "*kernel_stats.csv" | head -3
echo MEASURE_OK
