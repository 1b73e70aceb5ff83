#!/bin/bash
# Experiment builds of the product library (CPU, cross-compiled for gfx950) next to the real one:
#   tools/build_variant.sh NAME SCENES [make VAR=value ...]
# e.g. tools/build_variant.sh ieee "2_4 2_8" FASTFP=        (fp32 with IEEE div/sqrt and denormals)
#      tools/build_variant.sh f64noslp 2_4 F64FLAGS=-fno-slp-vectorize
# -> factory_marl_amd/lib_NAME.so, loaded with FACTORYSIM_LIB=factory_marl_amd/lib_NAME.so
set -e
NAME=$1; SCENES=$2; shift 2
cd "$(dirname "$0")/../factory_marl_amd/csrc"
make -s -j8 OBJDIR=build_$NAME OUT=../lib_$NAME.so SCENES="$SCENES" "$@" 2>&1 | grep -E "error|Error" || true
test -f ../lib_$NAME.so && echo "built factory_marl_amd/lib_$NAME.so"
