#!/bin/bash
# Kernel-trace + PMC profile of bench.py on the GPU box (run via gpurun from the repo root).
#   tools/profile.sh <tag>
# Writes gpurun_out/prof_<tag>/ (kernel trace + stats) and gpurun_out/pmc_<tag>_{fetch,write}/
# (FETCH_SIZE / WRITE_SIZE in separate passes, as MI355X_MICROARCH.md prescribes).
set -e
TAG=${1:-r01}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
export TMPDIR=/tmp
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --no-decoder-leg --no-train-leg --no-loss-leg --no-model-train-leg --no-pipelined-leg --no-realtime-leg"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o trace \
  -- python3 $ROOT/bench.py $ARGS > $OUT/prof_${TAG}_bench.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_${TAG}_fetch -o fetch \
  -- python3 $ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-decoder-leg --no-train-leg --no-loss-leg --no-model-train-leg --no-pipelined-leg --no-realtime-leg > $OUT/pmc_${TAG}_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_${TAG}_write -o write \
  -- python3 $ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-decoder-leg --no-train-leg --no-loss-leg --no-model-train-leg --no-pipelined-leg --no-realtime-leg > $OUT/pmc_${TAG}_write.log 2>&1
echo profile done
