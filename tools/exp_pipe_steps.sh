#!/bin/bash
# The pipelined serving leg against the one-stream step at the driver's step count and at 200 / 400
# batches (run via gpurun from the repo root).
mkdir -p gpurun_out
ARGS="--no-train-leg --no-loss-leg --no-model-train-leg --no-decoder-leg --no-op-leg --no-cpu-baseline --no-uncached-leg"
for s in 20 200 400; do
  timeout -k 10 120 python3 bench.py --steps $s --warmup 5 $ARGS > gpurun_out/pipe_$s.json 2>gpurun_out/pipe_$s.err || { tail -5 gpurun_out/pipe_$s.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('steps', sys.argv[2], 'step', d['ms_per_step'], 'pipelined', d['pipelined'])" gpurun_out/pipe_$s.json $s
done
