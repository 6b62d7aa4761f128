#!/bin/bash
# Same-box A/B of two library variants (build/ab_<a>.so, build/ab_<b>.so): bench step and kernel averages.
mkdir -p gpurun_out
export TMPDIR=/tmp
A=$1; B=$2
bash tools/ab_bench.sh $A $B $A $B || exit 1
cat gpurun_out/ab_bench.log
bash tools/ab_prof.sh fused "synth_frame_kernel<true, false, false>" $A $B || exit 1
