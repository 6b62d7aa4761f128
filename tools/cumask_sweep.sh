#!/bin/bash
# One process per CU-mask configuration of tools/exp_cumask.py (run via gpurun from the repo root):
#   bash tools/cumask_sweep.sh [mode ...]      (modes: plain, <k>:block, <k>:xcd; default sweep below)
mkdir -p gpurun_out; : > gpurun_out/cumask.log
for m in ${@:-plain 48:block 56:block 64:block 72:block 80:block}; do
  timeout -k 10 60 python -u tools/exp_cumask.py $m >> gpurun_out/cumask.log 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/cumask.log
