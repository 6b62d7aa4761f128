#!/bin/bash
# Kernel-trace profile of bench.py's train-step leg (rocprofv3 --kernel-trace --stats), run via gpurun from
# the repo root:  bash tools/train_prof.sh <tag>  ->  gpurun_out/prof_train_<tag>/
TAG=${1:-train}
ROOT=$(pwd)
export TMPDIR=/tmp
mkdir -p $ROOT/gpurun_out
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/prof_train_$TAG -o t \
  -- python3 $ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-decoder-leg --no-loss-leg --no-model-train-leg \
  --no-pipelined-leg --no-op-leg --no-uncached-leg > $ROOT/gpurun_out/prof_train_$TAG.log 2>&1 || exit 1
python3 $ROOT/tools/kstats.py $ROOT/gpurun_out/prof_train_$TAG/t_kernel_stats.csv | head -24
