#!/bin/bash
# round 3 (g): wave-parallel box-box SAT (A/B against the serial one: identical results), Newton tolerance study
# for the fp32 build, phase profile and bench
set -o pipefail
O=gpurun_out/r03g; mkdir -p $O
export FM_TRAJ_CACHE=traj_cache
timeout -k 10 300 python -u tools/parity_sweep.py --prec fp32 --tag par >> $O/sweep.jsonl 2>> $O/sweep.err || { echo "SWEEP FAILED"; tail -20 $O/sweep.err; exit 1; }
FM_SERIAL_BOXBOX=1 timeout -k 10 300 python -u tools/parity_sweep.py --prec fp32 --tag serial >> $O/sweep.jsonl 2>> $O/sweep.err || { echo "SWEEP serial FAILED"; tail -20 $O/sweep.err; exit 1; }
timeout -k 10 300 python -u tools/parity_sweep.py --prec fp64 --tag f64 >> $O/sweep.jsonl 2>> $O/sweep.err || { echo "SWEEP f64 FAILED"; tail -20 $O/sweep.err; exit 1; }
for tol in 1e-10 1e-12; do
  timeout -k 10 300 python -u tools/parity_sweep.py --prec fp32 --tol $tol --tag tol$tol >> $O/sweep.jsonl 2>> $O/sweep.err || { echo "SWEEP tol FAILED"; tail -20 $O/sweep.err; exit 1; }
done
cat $O/sweep.jsonl
timeout -k 10 300 python -u tools/phase_profile.py --steps 10 > $O/phase_2x4_fp32.json 2> $O/phase.err || { echo "PHASE FAILED"; tail $O/phase.err; exit 1; }
cat $O/phase_2x4_fp32.json
FM_SERIAL_BOXBOX=1 timeout -k 10 300 python -u tools/phase_profile.py --steps 10 > $O/phase_2x4_fp32_serialbb.json 2>> $O/phase.err || { echo "PHASE FAILED"; tail $O/phase.err; exit 1; }
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "BENCH FAILED"; tail $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python -u tools/phase_profile.py --steps 3 --arms 4 --objects 16 --env-class PauseIKToggleEnv --preroll 60 > $O/phase_4x16_pause.json 2>> $O/phase.err || { echo "PHASE416 FAILED"; tail $O/phase.err; exit 1; }
cat $O/phase_4x16_pause.json
timeout -k 10 300 python -u tools/phase_profile.py --steps 3 --arms 4 --objects 16 --preroll 60 > $O/phase_4x16_allfull.json 2>> $O/phase.err || { echo "PHASE416a FAILED"; tail $O/phase.err; exit 1; }
cat $O/phase_4x16_allfull.json
