#!/bin/bash
# Round-2 measurement set for the current kernel: rocprofv3 kernel stats, PMC traffic / SQ / VALU passes,
# phase profiles.  usage: bash tools/r02_measure.sh TAG
set -o pipefail
TAG=${1:-r02m}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
P="--steps 3 --warmup 1 --no-cpu-baseline --fp64-steps 0 --preroll 200"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --fp64-steps 0 > $O/ktrace.log 2>&1 || { echo "KTRACE FAILED"; tail $O/ktrace.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -- python3 bench.py $P > $O/pmc_fetch.log 2>&1 || { echo "PMC FETCH FAILED"; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -- python3 bench.py $P > $O/pmc_write.log 2>&1 || { echo "PMC WRITE FAILED"; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $O/pmc_sq -- python3 bench.py $P > $O/pmc_sq.log 2>&1 || { echo "PMC SQ FAILED"; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d $O/pmc_valu -- python3 bench.py $P > $O/pmc_valu.log 2>&1 || { echo "PMC VALU FAILED"; exit 1; }
timeout -k 10 200 python tools/phase_profile.py --precision fp32 > $O/phase_fp32.json 2> $O/phase_fp32.err || { echo "PHASE FAILED"; tail $O/phase_fp32.err; exit 1; }
timeout -k 10 200 python tools/phase_profile.py --precision fp64 > $O/phase_fp64.json 2> $O/phase_fp64.err || { echo "PHASE64 FAILED"; tail $O/phase_fp64.err; exit 1; }
find $O -name "*kernel_stats.csv" | head -3
echo MEASURE_OK
