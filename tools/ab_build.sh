#!/bin/bash
# Build a C-ABI library variant with extra compile flags for one source (A/B experiments):
#   tools/ab_build.sh <name> <source-stem> [-DFLAG=...]...   -> build/ab_<name>.so
set -e
NAME=$1; STEM=$2; shift 2
make -s all >/dev/null
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Iinclude -Ibuild -Wno-unused-result"
case $STEM in synth|synth_frame|backward|dense) HIPFLAGS="$HIPFLAGS -fno-slp-vectorize";; esac
/opt/rocm/bin/hipcc $HIPFLAGS "$@" -c ddsp_pytorch_amd/csrc/$STEM.hip -o build/ab_${NAME}_$STEM.o
OBJS=$(ls build/*.o | grep -v "/ab_" | grep -v "/$STEM.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o build/ab_$NAME.so $OBJS build/ab_${NAME}_$STEM.o
echo built build/ab_$NAME.so
