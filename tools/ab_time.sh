#!/bin/bash
# A/B timing of C-ABI library variants on one GPU box (run via gpurun from the repo root):
#   [AB_SCRIPT=tools/exp_bwd.py] tools/ab_time.sh <name>...
# times build/ab_<name>.so for each name, twice, in order; each variant loads through
# DDSP_HIP_LIB into its own process running AB_SCRIPT (default tools/exp_synth_time.py).
mkdir -p gpurun_out
: > gpurun_out/ab.log
for rep in 1 2; do
  for v in "$@"; do
    DDSP_HIP_LIB=$PWD/build/ab_$v.so timeout -k 10 60 python ${AB_SCRIPT:-tools/exp_synth_time.py} >> gpurun_out/ab.log 2>&1 || exit 1
    echo "$v" >> gpurun_out/ab.log
  done
done
