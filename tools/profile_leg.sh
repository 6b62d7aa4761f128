#!/bin/bash
# rocprofv3 kernel trace + stats of one bench.py leg (run via gpurun from the repo root):
#   tools/profile_leg.sh <tag> <bench.py args...>
# e.g. tools/profile_leg.sh train --no-decoder-leg --no-loss-leg --no-model-train-leg --no-op-leg
# -> gpurun_out/prof_<tag>/trace_kernel_stats.csv
set -e
TAG=$1; shift
ROOT=$(pwd)
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/prof_$TAG -o trace \
  -- python3 $ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > $ROOT/gpurun_out/prof_${TAG}.log 2>&1
echo "profile $TAG done"
