#!/bin/bash
# Build C-ABI library variants from edited copies of ONE source (A/B experiments, never shipped):
#   tools/ab_src.sh <stem> <name>=<path to the variant's .hip> ...   -> build/ab_<name>.so
set -e
STEM=$1; shift
make -s all >/dev/null
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Iinclude -Ibuild -Iddsp_pytorch_amd/csrc -Wno-unused-result"
case $STEM in synth|synth_frame|backward) HIPFLAGS="$HIPFLAGS -fno-slp-vectorize";; esac
OBJS=$(ls build/*.o | grep -v "/ab_" | grep -v "/$STEM.o")
for nv in "$@"; do
  NAME=${nv%%=*}; SRC=${nv#*=}
  /opt/rocm/bin/hipcc $HIPFLAGS -c $SRC -o build/ab_${NAME}_$STEM.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o build/ab_$NAME.so $OBJS build/ab_${NAME}_$STEM.o
  echo built build/ab_$NAME.so
done
