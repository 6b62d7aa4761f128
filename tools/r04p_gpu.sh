#!/bin/bash
# Second half of tools/r04m_gpu.sh (uncached-IR step, decoder kernel profile, default / config 4 / config 5
# lines, rocprofv3 + PMC traffic, PMC VALU of the fused kernel): bash tools/r04p_gpu.sh <tag>
TAG=${1:-r04p}
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/exp_uncached.py > gpurun_out/unc_$TAG.log 2>&1 || { cat gpurun_out/unc_$TAG.log; exit 1; }
cat gpurun_out/unc_$TAG.log
echo "== decoder profile $(date +%T)"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dec_$TAG -o t -- python3 tools/exp_decoder2.py outmlp outmlp_gemm fwd > gpurun_out/prof_dec_$TAG.log 2>&1 || exit 1
echo "== bench default $(date +%T)"
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
echo "== bench config 4/5 $(date +%T)"
timeout -k 10 300 python -u bench.py --config 4 --no-train-leg --no-loss-leg --no-model-train-leg --no-decoder-leg \
  > gpurun_out/bench_${TAG}_c4.json 2> gpurun_out/bench_${TAG}_c4.err || { tail -20 gpurun_out/bench_${TAG}_c4.err; exit 1; }
timeout -k 10 300 python -u bench.py --config 5 --no-train-leg --no-loss-leg --no-model-train-leg --no-decoder-leg \
  > gpurun_out/bench_${TAG}_c5.json 2> gpurun_out/bench_${TAG}_c5.err || { tail -20 gpurun_out/bench_${TAG}_c5.err; exit 1; }
echo "== profile $(date +%T)"
bash tools/profile.sh $TAG || exit 1
echo "== pmc $(date +%T)"
bash tools/pmc_probe.sh fused $TAG || exit 1
bash tools/pmc_probe.sh reverb $TAG || exit 1
echo "r04m done $(date +%T)"
