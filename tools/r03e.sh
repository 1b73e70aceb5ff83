#!/bin/bash
# round 3 (e): phase profiles with the collision sub-phases: (2,4) fp32 / fp64, (4,16) PauseIKToggle fp32 with the
# dense matrix-core Cholesky and with the sparse LDS one
set -o pipefail
O=gpurun_out/r03e; mkdir -p $O
timeout -k 10 300 python -u tools/phase_profile.py --steps 10 > $O/phase_2x4_fp32.json 2> $O/phase.err || { echo "PHASE FAILED"; tail $O/phase.err; exit 1; }
cat $O/phase_2x4_fp32.json
timeout -k 10 300 python -u tools/phase_profile.py --steps 10 --precision fp64 > $O/phase_2x4_fp64.json 2>> $O/phase.err || { echo "PHASE64 FAILED"; tail $O/phase.err; exit 1; }
timeout -k 10 300 python -u tools/phase_profile.py --steps 3 --arms 4 --objects 16 --env-class PauseIKToggleEnv --preroll 60 > $O/phase_4x16_dense.json 2>> $O/phase.err || { echo "PHASE416 FAILED"; tail $O/phase.err; exit 1; }
cat $O/phase_4x16_dense.json
FM_CHOL_LDS=2 timeout -k 10 300 python -u tools/phase_profile.py --steps 3 --arms 4 --objects 16 --env-class PauseIKToggleEnv --preroll 60 > $O/phase_4x16_sparse.json 2>> $O/phase.err || { echo "PHASE416s FAILED"; tail $O/phase.err; exit 1; }
cat $O/phase_4x16_sparse.json
# float64 narrowphase variant (fp32 build): parity sweep, phase profile, GPU physics pins
export FM_TRAJ_CACHE=traj_cache
FACTORYSIM_LIB=factory_marl_amd/lib_npf64.so timeout -k 10 300 python -u tools/parity_sweep.py --prec fp32 --tag npf64 >> $O/sweep.jsonl 2>> $O/sweep.err || { echo "SWEEP npf64 FAILED"; tail -20 $O/sweep.err; exit 1; }
FACTORYSIM_LIB=factory_marl_amd/lib_npf64.so timeout -k 10 300 python -u tools/parity_sweep.py --prec fp32 --tag npf64 --traj 4,16,150,3,PauseIKToggleEnv >> $O/sweep.jsonl 2>> $O/sweep.err || { echo "SWEEP npf64 416 FAILED"; tail -20 $O/sweep.err; exit 1; }
cat $O/sweep.jsonl
FACTORYSIM_LIB=factory_marl_amd/lib_npf64.so timeout -k 10 300 python -u tools/phase_profile.py --steps 10 > $O/phase_2x4_fp32_npf64.json 2>> $O/phase.err || { echo "PHASE npf64 FAILED"; tail $O/phase.err; exit 1; }
cat $O/phase_2x4_fp32_npf64.json
FACTORYSIM_LIB=factory_marl_amd/lib_npf64.so timeout -k 10 300 python -u -m pytest tests/test_gpu_physics_pins.py -q --timeout 200 --timeout-method thread > $O/pins.log 2>&1; echo "pins rc $?"; tail -5 $O/pins.log
