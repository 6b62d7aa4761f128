#!/bin/bash
# Frame table on / off in the bench step of configs 4 and 5 (run via gpurun from the repo root).
mkdir -p gpurun_out
: > gpurun_out/tc.log
for rep in 1 2; do
  for c in 4 5 2; do
    for v in 0 1; do
      DDSP_HIP_FRAME_TABLE=$v timeout -k 10 120 python bench.py --config $c --no-train-leg --no-loss-leg \
        --no-model-train-leg --no-decoder-leg --no-op-leg --no-cpu-baseline --no-uncached-leg > gpurun_out/tc.json 2>/dev/null || exit 1
      python3 -c "import json; d=json.loads(open('gpurun_out/tc.json').read().strip().split(chr(10))[-1]); print('config $c table=$v', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['kernel_ms'], d.get('pipelined', {}).get('ms_per_step'))" >> gpurun_out/tc.log
    done
  done
done
cat gpurun_out/tc.log
