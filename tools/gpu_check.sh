#!/bin/bash
# One GPU box call: the GPU test suite, then kernel timings of the reverb and the fused synthesis
# (rocprofv3 kernel stats).  Run via gpurun from the repo root:  bash tools/gpu_check.sh <tag>
TAG=${1:-check}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && exit $rc
DDSP_AB_WHAT=reverb timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rp_${TAG}_reverb -o t -- python3 tools/exp_synth_time.py > gpurun_out/rp_${TAG}_reverb.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rp_${TAG}_synth -o t -- python3 tools/exp_synth_time.py > gpurun_out/rp_${TAG}_synth.log 2>&1 || exit 1
grep median gpurun_out/rp_${TAG}_*.log
