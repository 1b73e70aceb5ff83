#!/bin/bash
# Round-2 first GPU call: parity tests, parity sweeps over builds / solver settings, bench, rocprof stats, PMC.
set -o pipefail
O=gpurun_out/r02a
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/counters_list.txt 2>&1 || true
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1
echo "tests rc=$?"; tail -3 $O/tests.log
S=$O/sweep.jsonl
run() { timeout -k 10 240 "$@" >> $S 2>> $O/sweep.err || { echo "SWEEP FAILED: $*"; tail -5 $O/sweep.err; exit 1; }; }
run python tools/parity_sweep.py --prec fp64 --tag main
run python tools/parity_sweep.py --prec fp32 --tag main
run env FM_NO_NOISE_GUARD=1 python tools/parity_sweep.py --prec fp32 --tol 1e-10 --tag main_tight
run env FACTORYSIM_LIB=factory_marl_amd/lib_ieee.so python tools/parity_sweep.py --prec fp32 --tag ieee --traj 2,4,96,7 2,4,300,21 2,8,300,5
run env FACTORYSIM_LIB=factory_marl_amd/lib_ieee.so FM_NO_NOISE_GUARD=1 python tools/parity_sweep.py --prec fp32 --tol 1e-10 --tag ieee_tight --traj 2,4,96,7 2,4,300,21 2,8,300,5
run env FACTORYSIM_LIB=factory_marl_amd/lib_f64noslp.so python tools/parity_sweep.py --prec fp64 --tag f64noslp --traj 2,4,96,7 2,4,300,21
run env FACTORYSIM_LIB=factory_marl_amd/lib_f64rl.so python tools/parity_sweep.py --prec fp64 --tag f64rl --traj 2,4,96,7 2,4,300,21
cat $S | python -c "import json,sys; [print({k:v for k,v in json.loads(l).items() if k in ('tag','prec','traj','within','median','worst','int_bad','flag_bad','max_cubes')}) for l in sys.stdin]"
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 200 python tools/phase_profile.py --precision fp32 > $O/phase_fp32.json 2> $O/phase_fp32.err || { echo "PHASE FAILED"; tail $O/phase_fp32.err; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --fp64-steps 0 > $O/ktrace.log 2>&1 || { echo "KTRACE FAILED"; tail $O/ktrace.log; exit 1; }
P="--steps 3 --warmup 1 --no-cpu-baseline --fp64-steps 0"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -- python3 bench.py $P > $O/pmc_fetch.log 2>&1 || { echo "PMC FETCH FAILED"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -- python3 bench.py $P > $O/pmc_write.log 2>&1 || { echo "PMC WRITE FAILED"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $O/pmc_sq -- python3 bench.py $P > $O/pmc_sq.log 2>&1 || { echo "PMC SQ FAILED"; exit 1; }
if grep -q SQ_INSTS_VALU_FMA_F32 $O/counters_list.txt; then
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d $O/pmc_valu -- python3 bench.py $P > $O/pmc_valu.log 2>&1 || { echo "PMC VALU FAILED"; exit 1; }
fi
echo R02A_OK
