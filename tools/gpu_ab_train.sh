#!/bin/bash
# Same-box A/B of the bench's train leg for library variants build/ab_<name>.so
mkdir -p gpurun_out
: > gpurun_out/ab_train.log
for rep in 1 2; do
  for v in "$@"; do
    DDSP_HIP_LIB=$PWD/build/ab_$v.so timeout -k 10 150 python bench.py --no-loss-leg --no-model-train-leg \
      --no-decoder-leg --no-op-leg --no-cpu-baseline --no-uncached-leg --no-pipelined-leg > gpurun_out/ab_tr.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_tr.json').read().strip().split(chr(10))[-1]); print('$v', d['ms_per_step'], d['train_step']['ms_per_step'], d['train_step']['event_ms'])" >> gpurun_out/ab_train.log
  done
done
cat gpurun_out/ab_train.log
