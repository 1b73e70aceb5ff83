# last check of the shipped build (FM_GL_GX=1): the GPU suite, then the default bench line
set -o pipefail
bash tools/gpu_measure.sh r06u tests bench
