#!/bin/bash
# Frame-table check on one box (via gpurun): its parity tests, then rocprofv3 kernel stats of the bench step
# with DDSP_HIP_FRAME_TABLE=0 and 1, and the bench's in-region synthesis time of each (alternated).
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_frame_table.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pt_pytest.log 2>&1 || { tail -30 gpurun_out/pt_pytest.log; exit 1; }
tail -1 gpurun_out/pt_pytest.log
for v in 0 1; do
  DDSP_HIP_FRAME_TABLE=$v timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pt$v -o run -- \
    python3 bench.py --steps 100 --no-train-leg --no-loss-leg --no-model-train-leg --no-decoder-leg --no-op-leg \
    --no-cpu-baseline --no-uncached-leg --no-pipelined-leg > gpurun_out/pt$v.out 2>&1 || exit 1
done
for v in 0 1; do
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/pt$v/run_kernel_stats.csv')):
    if any(k in r['Name'] for k in ('synth_', 'frame_table', 'upols')):
        print('table=$v', r['Name'][:60], r['Calls'], round(float(r['AverageNs']) / 1000, 2), round(float(r['MinNs']) / 1000, 2))
"
done
: > gpurun_out/pt_bench.log
for rep in 1 2; do
  for v in 0 1; do
    DDSP_HIP_FRAME_TABLE=$v timeout -k 10 120 python bench.py --no-train-leg --no-loss-leg --no-model-train-leg \
      --no-decoder-leg --no-op-leg --no-cpu-baseline --no-uncached-leg > gpurun_out/pt_b.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/pt_b.json').read().strip().split(chr(10))[-1]); print('table=$v', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['kernel_ms'], d.get('pipelined', {}).get('ms_per_step'))" >> gpurun_out/pt_bench.log
  done
done
cat gpurun_out/pt_bench.log
