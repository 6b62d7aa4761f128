#!/bin/bash
# Round validation on one GPU box (run via gpurun from the repo root):  bash tools/round_check.sh <tag>
# GPU tests, smoke, the driver's exact bench command (twice), decoder / GRU / uncached-IR timings, the
# decoder's kernel profile, default / config 4 / config 5 lines, rocprofv3 kernel stats + PMC traffic
# (tools/profile.sh), PMC VALU and wave counters of the fused synthesis and reverb kernels
# (tools/pmc_probe.sh; then tools/pmc_valu.py and tools/pmc_traffic.py re-key profiles/ to the build).
# Each GPU step has its own time limit; the chain stops at the first failure.
TAG=${1:-check}
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== pytest $(date +%T)"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
echo "== smoke $(date +%T)"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { cat gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
for i in 1 2; do
  echo "== driver $i $(date +%T)"
  timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/driver_${TAG}_$i.json \
    2> gpurun_out/driver_${TAG}_$i.err || { tail -20 gpurun_out/driver_${TAG}_$i.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('value', d['value'], 'ms', d['ms_per_step'], 'synth', d['roofline']['avg_launch_ms'], 'frac_alg', d['roofline']['frac_algorithmic'], 'kern', d['kernel_ms'], 'pipe', d.get('pipelined',{}).get('ms_per_step'), 'unc', d.get('uncached_ir',{}).get('ms_per_step'), 'train', d.get('train_step',{}).get('ms_per_step'), 'dec', d.get('decoder_forward',{}).get('ms_per_step'), 'dsyn', d.get('decoder_synthesis',{}).get('ms_per_step'))" gpurun_out/driver_${TAG}_$i.json
done
echo "== decoder $(date +%T)"
timeout -k 10 200 python3 tools/exp_decoder2.py net net_gemm outmlp outmlp_gemm mlps gru proj dsyn fwd > gpurun_out/dec_$TAG.log 2>&1 || { tail gpurun_out/dec_$TAG.log; exit 1; }
cat gpurun_out/dec_$TAG.log
timeout -k 10 100 python3 tools/exp_gru.py > gpurun_out/gru_$TAG.log 2>&1 || exit 1
cat gpurun_out/gru_$TAG.log
timeout -k 10 200 python3 tools/exp_uncached.py > gpurun_out/unc_$TAG.log 2>&1 || exit 1
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
echo "round check $TAG done $(date +%T)"
