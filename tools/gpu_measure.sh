#!/bin/bash
# GPU-box measurement runner (via gpurun).  Every step runs under its own time limit; the first failing step ends
# the run (no GPU step after a failure).  Output under gpurun_out/TAG/.
#
# usage: bash tools/gpu_measure.sh TAG STEP [STEP ...]
#   LIB=path        library for the steps (FACTORYSIM_LIB; default factory_marl_amd/libfactorysim.so)
#   SWEEP="specs"   parity-sweep trajectories (A,K,T,seed[,EnvClass[,oracle_tol]]; default: the four long ones)
#   SFX=name        suffix for the output files of the steps (A/B runs of two libraries in one TAG)
#   TOL=x           Newton tolerance of the sweeps' GPU env (0 = the precision's default)
# steps:
#   tests       pytest -m gpu (verbose, prints kept)          sweep32 / sweep64   parity sweep fp32 / fp64
#   bench       default bench line (with the CPU baseline)    quick               bench, 30 steps, no CPU leg
#   c3 c4 c5    config 3 / 4 (one GPU) / 5 benches             ktrace              rocprofv3 kernel trace + stats
#   ktrace3 pmc3 / ktrace5 pmc5   config 3 / 5 kernel stats (+ PMC passes)
#   pmc         PMC passes (FETCH, WRITE, SQ, VALU) + summaries
#   phase       phase profiles (2,4) fp32 / fp64, (2,8), (4,16)     phase24   (2,4) fp32 only
#   pmcsq       the SQ counter pass alone (waits, LDS bank conflicts)      pmcic   instruction-cache counters
#   flags       1000-episode flag-divergence study (fp32, fp64)
set -o pipefail
TAG=${1:?tag}
shift
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
export FM_TRAJ_CACHE=${FM_TRAJ_CACHE:-traj_cache}
[ -n "$LIB" ] && export FACTORYSIM_LIB=$LIB
S=${SFX:+_$SFX}
SWEEP=${SWEEP:-"2,4,96,7 2,4,300,21 2,8,300,5 2,10,250,9"}
P="--steps 3 --warmup 1 --no-cpu-baseline --fp64-steps 0 --preroll 200"

fail() { echo "$1 FAILED (rc $2)"; [ -n "$3" ] && tail -20 "$3"; exit 1; }

for step in "$@"; do
  echo "== $step$S $(date +%T)"
  case $step in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $O/tests$S.log 2>&1 \
        || fail tests $? $O/tests$S.log
      tail -2 $O/tests$S.log ;;
    sweep32|sweep64)
      pr=fp${step#sweep}
      timeout -k 10 600 python -u tools/parity_sweep.py --prec $pr --tag $step$S --verbose-tol 1e-4 --tol ${TOL:-0} --traj $SWEEP \
        > $O/$step$S.log 2> $O/$step$S.err || fail $step $? $O/$step$S.err
      grep '^{' $O/$step$S.log > $O/$step$S.jsonl
      python -c "
import json
for l in open('$O/$step$S.jsonl'):
    r = json.loads(l); print(r['prec'], r['traj'], r['within'], '%.3e' % r['worst'], r['int_bad'], r['flag_bad'], r['missing_steps'][:10], 'resets', r['resets_compared'], r['reset_bad'], '%.1e' % r['reset_worst'])
" ;;
    bench)
      timeout -k 10 400 python bench.py > $O/bench$S.json 2> $O/bench$S.err || fail bench $? $O/bench$S.err
      cat $O/bench$S.json ;;
    quick)
      timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/quick$S.json 2> $O/quick$S.err \
        || fail quick $? $O/quick$S.err
      cat $O/quick$S.json ;;
    c3)
      timeout -k 10 400 python bench.py --workload config3 --no-cpu-baseline > $O/bench_config3$S.json 2> $O/c3$S.err \
        || fail c3 $? $O/c3$S.err
      cat $O/bench_config3$S.json ;;
    c4)
      timeout -k 10 400 python bench.py --workload config4 --steps 4 --warmup 1 --preroll 10 --no-cpu-baseline \
        > $O/bench_config4_1gpu$S.json 2> $O/c4$S.err || fail c4 $? $O/c4$S.err
      cat $O/bench_config4_1gpu$S.json ;;
    c5)
      timeout -k 10 300 python bench.py --workload config5 --steps 10 --warmup 3 --no-cpu-baseline \
        > $O/bench_config5$S.json 2> $O/c5$S.err || fail c5 $? $O/c5$S.err
      cat $O/bench_config5$S.json ;;
    ktrace)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace$S -- python3 bench.py --steps 20 \
        --warmup 2 --no-cpu-baseline --fp64-steps 0 > $O/ktrace$S.log 2>&1 || fail ktrace $? $O/ktrace$S.log
      find $O/ktrace$S -name "*kernel_stats.csv" | head -1 | xargs -r head -4 ;;
    pmc)
      timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch$S -- python3 bench.py $P \
        > $O/pmc_fetch$S.log 2>&1 || fail pmc_fetch $? $O/pmc_fetch$S.log
      timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write$S -- python3 bench.py $P \
        > $O/pmc_write$S.log 2>&1 || fail pmc_write $? $O/pmc_write$S.log
      timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU \
        SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $O/pmc_sq$S -- python3 bench.py $P \
        > $O/pmc_sq$S.log 2>&1 || fail pmc_sq $? $O/pmc_sq$S.log
      timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 \
        SQ_INSTS_VALU_TRANS_F32 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d $O/pmc_valu$S -- python3 \
        bench.py $P > $O/pmc_valu$S.log 2>&1 || fail pmc_valu $? $O/pmc_valu$S.log
      timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 \
        SQ_INSTS_VALU_TRANS_F64 SQ_WAVES --output-format csv -d $O/pmc_valu64$S -- python3 \
        bench.py $P > $O/pmc_valu64$S.log 2>&1 || fail pmc_valu64 $? $O/pmc_valu64$S.log
      F=$(find $O/pmc_fetch$S -name "*counter_collection.csv" | head -1)
      W=$(find $O/pmc_write$S -name "*counter_collection.csv" | head -1)
      V=$(find $O/pmc_valu$S -name "*counter_collection.csv" | head -1)
      V64=$(find $O/pmc_valu64$S -name "*counter_collection.csv" | head -1)
      Q=$(find $O/pmc_sq$S -name "*counter_collection.csv" | head -1)
      python tools/pmc_traffic.py $F $W --arenas 4096 --out $O/pmc_traffic$S.json || fail traffic $?
      python tools/pmc_valu.py $V --f64 $V64 --arenas 4096 --last 3 --out $O/pmc_valu$S.json || fail valu $?
      python tools/pmc_sq.py $Q $O/pmc_sq_summary$S.json || fail sq $? ;;
    ktrace5|pmc5)
      # config 5's kernel ((4,16) PauseIKToggleEnv fp32, 4096 arenas on one GPU): kernel stats, then the PMC passes
      P5="--workload config5 --steps 3 --warmup 1 --no-cpu-baseline"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace5$S -- python3 bench.py \
        --workload config5 --steps 8 --warmup 2 --no-cpu-baseline > $O/ktrace5$S.log 2>&1 || fail ktrace5 $? $O/ktrace5$S.log
      find $O/ktrace5$S -name "*kernel_stats.csv" | head -1 | xargs -r head -4
      if [ $step = pmc5 ]; then
        timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc5_fetch$S -- python3 bench.py $P5 \
          > $O/pmc5_fetch$S.log 2>&1 || fail pmc5_fetch $? $O/pmc5_fetch$S.log
        timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc5_write$S -- python3 bench.py $P5 \
          > $O/pmc5_write$S.log 2>&1 || fail pmc5_write $? $O/pmc5_write$S.log
        timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU \
          SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $O/pmc5_sq$S -- python3 bench.py $P5 \
          > $O/pmc5_sq$S.log 2>&1 || fail pmc5_sq $? $O/pmc5_sq$S.log
        timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 \
          SQ_INSTS_VALU_TRANS_F32 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d $O/pmc5_valu$S -- python3 \
          bench.py $P5 > $O/pmc5_valu$S.log 2>&1 || fail pmc5_valu $? $O/pmc5_valu$S.log
        timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 \
          SQ_INSTS_VALU_TRANS_F64 SQ_WAVES --output-format csv -d $O/pmc5_valu64$S -- python3 \
          bench.py $P5 > $O/pmc5_valu64$S.log 2>&1 || fail pmc5_valu64 $? $O/pmc5_valu64$S.log
        python tools/pmc_traffic.py $(find $O/pmc5_fetch$S -name "*counter_collection.csv" | head -1) \
          $(find $O/pmc5_write$S -name "*counter_collection.csv" | head -1) --arenas 4096 --arms 4 --objects 16 \
          --out $O/pmc5_traffic$S.json || fail traffic5 $?
        python tools/pmc_valu.py $(find $O/pmc5_valu$S -name "*counter_collection.csv" | head -1) \
          --f64 $(find $O/pmc5_valu64$S -name "*counter_collection.csv" | head -1) --arenas 4096 --arms 4 --objects 16 \
          --last 2 --out $O/pmc5_valu$S.json || fail valu5 $?
        python tools/pmc_sq.py $(find $O/pmc5_sq$S -name "*counter_collection.csv" | head -1) $O/pmc5_sq_summary$S.json \
          || fail sq5 $?
      fi ;;
    ktrace3|pmc3)
      # config 3's kernel ((2,8) AllFullRL fp32, 16384 arenas on one GPU, PPO rollout): kernel stats, then the PMC passes
      P3="--workload config3 --steps 3 --warmup 1 --preroll 50 --ppo-epochs 1 --no-cpu-baseline"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace3$S -- python3 bench.py \
        --workload config3 --steps 8 --warmup 2 --no-cpu-baseline > $O/ktrace3$S.log 2>&1 || fail ktrace3 $? $O/ktrace3$S.log
      find $O/ktrace3$S -name "*kernel_stats.csv" | head -1 | xargs -r head -4
      if [ $step = pmc3 ]; then
        timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc3_fetch$S -- python3 bench.py $P3 \
          > $O/pmc3_fetch$S.log 2>&1 || fail pmc3_fetch $? $O/pmc3_fetch$S.log
        timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc3_write$S -- python3 bench.py $P3 \
          > $O/pmc3_write$S.log 2>&1 || fail pmc3_write $? $O/pmc3_write$S.log
        timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU \
          SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $O/pmc3_sq$S -- python3 bench.py $P3 \
          > $O/pmc3_sq$S.log 2>&1 || fail pmc3_sq $? $O/pmc3_sq$S.log
        timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 \
          SQ_INSTS_VALU_TRANS_F32 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d $O/pmc3_valu$S -- python3 \
          bench.py $P3 > $O/pmc3_valu$S.log 2>&1 || fail pmc3_valu $? $O/pmc3_valu$S.log
        timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 \
          SQ_INSTS_VALU_TRANS_F64 SQ_WAVES --output-format csv -d $O/pmc3_valu64$S -- python3 \
          bench.py $P3 > $O/pmc3_valu64$S.log 2>&1 || fail pmc3_valu64 $? $O/pmc3_valu64$S.log
        python tools/pmc_traffic.py $(find $O/pmc3_fetch$S -name "*counter_collection.csv" | head -1) \
          $(find $O/pmc3_write$S -name "*counter_collection.csv" | head -1) --arenas 16384 --arms 2 --objects 8 \
          --out $O/pmc3_traffic$S.json || fail traffic3 $?
        python tools/pmc_valu.py $(find $O/pmc3_valu$S -name "*counter_collection.csv" | head -1) \
          --f64 $(find $O/pmc3_valu64$S -name "*counter_collection.csv" | head -1) --arenas 16384 --arms 2 --objects 8 \
          --last 3 --out $O/pmc3_valu$S.json || fail valu3 $?
        python tools/pmc_sq.py $(find $O/pmc3_sq$S -name "*counter_collection.csv" | head -1) $O/pmc3_sq_summary$S.json \
          || fail sq3 $?
      fi ;;
    phase24)
      timeout -k 10 200 python tools/phase_profile.py --precision fp32 > $O/phase_fp32$S.json 2> $O/phase$S.err \
        || fail phase24 $? $O/phase$S.err ;;
    pmcsq)
      timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU \
        SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $O/pmc_sq$S -- python3 bench.py $P \
        > $O/pmc_sq$S.log 2>&1 || fail pmc_sq $? $O/pmc_sq$S.log
      python tools/pmc_sq.py $(find $O/pmc_sq$S -name "*counter_collection.csv" | head -1) $O/pmc_sq_summary$S.json \
        || fail sq $? ;;
    pmcic)
      timeout -s KILL 150 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE \
        SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --output-format csv -d $O/pmc_ic$S -- python3 bench.py $P \
        > $O/pmc_ic$S.log 2>&1 || fail pmc_ic $? $O/pmc_ic$S.log
      python tools/pmc_sq.py $(find $O/pmc_ic$S -name "*counter_collection.csv" | head -1) $O/pmc_ic_summary$S.json \
        || fail ic $? ;;
    phase)
      timeout -k 10 200 python tools/phase_profile.py --precision fp32 > $O/phase_fp32$S.json 2> $O/phase$S.err \
        || fail phase32 $? $O/phase$S.err
      timeout -k 10 200 python tools/phase_profile.py --precision fp64 > $O/phase_fp64$S.json 2>> $O/phase$S.err \
        || fail phase64 $? $O/phase$S.err
      timeout -k 10 200 python -u tools/phase_profile.py --steps 5 --arms 2 --objects 8 > $O/phase_fp32_2x8$S.json \
        2>> $O/phase$S.err || fail phase28 $? $O/phase$S.err
      timeout -k 10 300 python -u tools/phase_profile.py --steps 3 --arms 4 --objects 16 --env-class PauseIKToggleEnv \
        --preroll 60 > $O/phase_fp32_4x16$S.json 2>> $O/phase$S.err || fail phase416 $? $O/phase$S.err ;;
    flags)
      timeout -k 10 900 python -u tools/flag_divergence.py --episodes 1000 --workers 16 --prec fp32 fp64 \
        > $O/flags$S.jsonl 2> $O/flags$S.err || fail flags $? $O/flags$S.err
      cat $O/flags$S.jsonl ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo MEASURE_OK
