#!/bin/bash
# A/B of library variants through the whole bench step on one box: tools/ab_bench.sh <name>...
mkdir -p gpurun_out
: > gpurun_out/ab_bench.log
for rep in 1 2; do
  for v in "$@"; do
    DDSP_HIP_LIB=$PWD/build/ab_$v.so timeout -k 10 120 python bench.py --no-train-leg --no-loss-leg --no-model-train-leg --no-decoder-leg --no-op-leg --no-cpu-baseline --no-uncached-leg > gpurun_out/ab_b.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_b.json').read().strip().split(chr(10))[-1]); print('$v', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['kernel_ms'])" >> gpurun_out/ab_bench.log
  done
done
