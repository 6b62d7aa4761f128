#!/bin/bash
# bench.py (short legs) + rocprofv3 kernel stats of the timed step, on the GPU box:
#   bash tools/bench_prof.sh <tag> [bench args...]
TAG=${1:-bp}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS="--no-train-leg --no-loss-leg --no-model-train-leg --no-decoder-leg --no-op-leg --cpu-reps 1 $*"
timeout -k 10 300 python bench.py $ARGS > gpurun_out/bench_$TAG.log 2>&1 || exit 1
tail -1 gpurun_out/bench_$TAG.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernel_ms'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d.get('uncached_ir'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rp_$TAG -o t -- python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-uncached-leg --no-train-leg --no-loss-leg --no-model-train-leg --no-decoder-leg --no-op-leg $* > gpurun_out/rp_$TAG.log 2>&1 || exit 1
