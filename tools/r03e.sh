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
