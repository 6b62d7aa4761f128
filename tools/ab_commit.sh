#!/bin/bash
# Build a C-ABI library variant whose <stem>.hip (and the csrc headers) come from another commit,
# linked with HEAD's other objects (same-box A/B of one kernel across history):
#   tools/ab_commit.sh <name> <commit> [stem=synth_frame] [-DFLAG=...]...   -> build/ab_<name>.so
# The entry points of <stem>.hip must have the same C signatures at <commit> as at HEAD.
set -e
NAME=$1; COMMIT=$2; STEM=${3:-synth_frame}; shift 3 || shift $#
make -s all >/dev/null
SRC=build/ab_src_$NAME
rm -rf $SRC && mkdir -p $SRC/csrc $SRC/include
for f in $(git ls-tree --name-only $COMMIT ddsp_pytorch_amd/csrc/); do
  case $f in *.h|*.hip) git show $COMMIT:$f > $SRC/csrc/$(basename $f);; esac
done
git show $COMMIT:include/ddsp_hip.h > $SRC/include/ddsp_hip.h
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I$SRC/include -Ibuild -Wno-unused-result"
case $STEM in synth|synth_frame|backward) HIPFLAGS="$HIPFLAGS -fno-slp-vectorize";; esac
/opt/rocm/bin/hipcc $HIPFLAGS "$@" -c $SRC/csrc/$STEM.hip -o build/ab_${NAME}_$STEM.o
OBJS=$(ls build/*.o | grep -v "/ab_" | grep -v "/$STEM.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o build/ab_$NAME.so $OBJS build/ab_${NAME}_$STEM.o
echo built build/ab_$NAME.so
