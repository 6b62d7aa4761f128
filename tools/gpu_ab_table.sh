#!/bin/bash
# Frame-table A/B on one box (run via gpurun from the repo root): parity tests of the two-launch form,
# then the bench step with DDSP_HIP_FRAME_TABLE=0 / 1 alternated, then rocprofv3 kernel stats of each.
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_frame_table.py tests/test_gpu_persist.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/ab_table_pytest.log 2>&1 || { tail -30 gpurun_out/ab_table_pytest.log; exit 1; }
tail -1 gpurun_out/ab_table_pytest.log
: > gpurun_out/ab_table.log
for rep in 1 2; do
  for v in 0 1 1p6 1p5 1p4 0p6; do
    export DDSP_HIP_FRAME_TABLE=${v:0:1}
    if [ "${v:1:1}" = p ]; then export DDSP_HIP_PERSIST_WPC=${v:2:1}; else unset DDSP_HIP_PERSIST_WPC; fi
    timeout -k 10 120 python bench.py --no-train-leg --no-loss-leg --no-model-train-leg \
      --no-decoder-leg --no-op-leg --no-cpu-baseline --no-uncached-leg > gpurun_out/ab_t.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_t.json').read().strip().split(chr(10))[-1]); print('table=$v', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['kernel_ms'], d.get('pipelined', {}).get('ms_per_step'))" >> gpurun_out/ab_table.log
  done
done
unset DDSP_HIP_PERSIST_WPC
cat gpurun_out/ab_table.log
for v in 0 1 1p6; do
  export DDSP_HIP_FRAME_TABLE=${v:0:1}
  if [ "${v:1:1}" = p ]; then export DDSP_HIP_PERSIST_WPC=${v:2:1}; else unset DDSP_HIP_PERSIST_WPC; fi
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_table$v -o run -- \
    python3 bench.py --steps 100 --no-train-leg --no-loss-leg --no-model-train-leg --no-decoder-leg --no-op-leg \
    --no-cpu-baseline --no-uncached-leg --no-pipelined-leg > gpurun_out/prof_table$v.out 2>&1 || exit 1
done
for v in 0 1 1p6; do
  f=$(find gpurun_out/prof_table$v -name '*kernel_stats.csv' | head -1)
  echo "== table=$v"; cut -c1-160 "$f" | head -8
done
