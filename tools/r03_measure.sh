#!/bin/bash
# Round-3 measurement set: default bench (with the CPU baseline leg), config 3 / 5 benches, rocprofv3
# kernel stats + PMC passes (HBM traffic, SQ waits, VALU work) on the headline, phase profiles.  usage: bash tools/r03_measure.sh TAG
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
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d $O/pmc_valu -- python3 bench.py $P > $O/pmc_valu.log 2>&1 || { echo "PMC VALU FAILED"; exit 1; }
F=$(find $O/pmc_fetch -name "*counter_collection.csv" | head -1); W=$(find $O/pmc_write -name "*counter_collection.csv" | head -1)
V=$(find $O/pmc_valu -name "*counter_collection.csv" | head -1); S=$(find $O/pmc_sq -name "*counter_collection.csv" | head -1)
python tools/pmc_traffic.py $F $W --arenas 4096 --out $O/pmc_traffic.json || { echo "TRAFFIC FAILED"; exit 1; }
python tools/pmc_valu.py $V --arenas 4096 --last 3 --out $O/pmc_valu.json || { echo "VALU FAILED"; exit 1; }
python - $S $O/pmc_sq_summary.json << 'PY'
import csv, json, sys
from collections import defaultdict
tot = defaultdict(float); name = None
for r in csv.DictReader(open(sys.argv[1])):
    if "step_kernel" in r["Kernel_Name"]:
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); name = r["Kernel_Name"]
c = dict(tot)
out = {"kernel": name, "source": "rocprofv3 --pmc, summed over the bench launches", "counters": c,
       "wait_any_frac_of_wave_cycles": c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"],
       "wait_inst_any_frac": c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"],
       "active_inst_frac": c["SQ_ACTIVE_INST_ANY"] / c["SQ_WAVE_CYCLES"],
       "lds_bank_conflict_frac_of_lds_active": c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"],
       "valu_per_lds": c["SQ_INSTS_VALU"] / c["SQ_INSTS_LDS"]}
json.dump(out, open(sys.argv[2], "w"), indent=1); print(json.dumps({k: v for k, v in out.items() if k != "counters"}))
PY
timeout -k 10 200 python tools/phase_profile.py --precision fp32 > $O/phase_fp32.json 2> $O/phase.err || { echo "PHASE FAILED"; tail $O/phase.err; exit 1; }
timeout -k 10 200 python tools/phase_profile.py --precision fp64 > $O/phase_fp64.json 2>> $O/phase.err || { echo "PHASE64 FAILED"; tail $O/phase.err; exit 1; }
timeout -k 10 300 python -u tools/phase_profile.py --steps 3 --arms 4 --objects 16 --env-class PauseIKToggleEnv --preroll 60 > $O/phase_fp32_4x16.json 2>> $O/phase.err || { echo "PHASE416 FAILED"; tail $O/phase.err; exit 1; }
timeout -k 10 300 python -u tools/phase_profile.py --steps 5 --arms 2 --objects 8 > $O/phase_fp32_2x8.json 2>> $O/phase.err || { echo "PHASE28 FAILED"; tail $O/phase.err; exit 1; }
timeout -k 10 400 python bench.py --workload config4 --steps 4 --warmup 1 --preroll 10 --no-cpu-baseline > $O/bench_config4_1gpu.json 2> $O/bench_c4.err || { echo "BENCH c4 FAILED"; tail $O/bench_c4.err; exit 1; }
cat $O/bench_config4_1gpu.json
find $O -name "*kernel_stats.csv" | head -3
echo MEASURE_OK
