#!/bin/bash
# Round validation on one GPU box (run via gpurun from the repo root):
#   bash tools/round_check.sh <tag>
# GPU tests, smoke, the default bench line, configs 4 and 5 bench lines, rocprofv3 kernel stats
# and PMC traffic (tools/profile.sh), PMC counters of the reverb kernels.  Every GPU step has its
# own time limit and the chain stops at the first failure.
TAG=${1:-check}
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
step() { echo "== $1"; }
step pytest
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1 || { tail -20 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
step smoke
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { cat gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
step bench-driver-command
# the driver's exact command (BENCH_rNN.json): 20 timed steps after 5 warmup steps
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_${TAG}_driver.json \
  2> gpurun_out/bench_${TAG}_driver.err || { tail -20 gpurun_out/bench_${TAG}_driver.err; exit 1; }
step bench
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
step bench-config4
timeout -k 10 300 python -u bench.py --config 4 --no-train-leg --no-loss-leg --no-model-train-leg --no-decoder-leg \
  > gpurun_out/bench_${TAG}_c4.json 2> gpurun_out/bench_${TAG}_c4.err || { tail -20 gpurun_out/bench_${TAG}_c4.err; exit 1; }
step bench-config5
timeout -k 10 300 python -u bench.py --config 5 --no-train-leg --no-loss-leg --no-model-train-leg --no-decoder-leg \
  > gpurun_out/bench_${TAG}_c5.json 2> gpurun_out/bench_${TAG}_c5.err || { tail -20 gpurun_out/bench_${TAG}_c5.err; exit 1; }
step profile
bash tools/profile.sh $TAG || exit 1
step pmc-reverb
bash tools/pmc_probe.sh reverb $TAG || exit 1
step pmc-fused
bash tools/pmc_probe.sh fused $TAG || exit 1
echo round check $TAG done
