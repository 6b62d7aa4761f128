#!/bin/bash
# One GPU box pass (run via gpurun from the repo root):  bash tools/gpu_run.sh <tag> [steps...]
# steps: pytest | driver (the driver's exact bench command, twice) | profile (tools/profile.sh) |
#        pmc (VALU + traffic PMC passes) | smoke.  Each GPU step has its own time limit; the chain
# stops at the first failure.
TAG=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
for s in "$@"; do
  echo "== $s $(date +%T)"
  case $s in
    pytest)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
        > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
      tail -1 gpurun_out/pytest_$TAG.log ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 \
        || { cat gpurun_out/smoke_$TAG.log; exit 1; }
      tail -1 gpurun_out/smoke_$TAG.log ;;
    driver)
      for i in 1 2; do
        timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/driver_${TAG}_$i.json \
          2> gpurun_out/driver_${TAG}_$i.err || { tail -20 gpurun_out/driver_${TAG}_$i.err; exit 1; }
        python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('value', d['value'], 'ms', d['ms_per_step'], 'synth', d['roofline']['avg_launch_ms'], 'frac_alg', d['roofline']['frac_algorithmic'], 'kern', d['kernel_ms'], 'pipe', d.get('pipelined',{}).get('ms_per_step'), 'unc', d.get('uncached_ir',{}).get('ms_per_step'), 'train', d.get('train_step',{}).get('ms_per_step'))" gpurun_out/driver_${TAG}_$i.json
      done ;;
    profile)
      bash tools/profile.sh $TAG || exit 1
      python3 tools/kstats.py gpurun_out/prof_$TAG/trace_kernel_stats.csv 2>/dev/null | head -20 ;;
    pmc)
      bash tools/pmc_probe.sh fused $TAG && bash tools/pmc_probe.sh reverb $TAG || exit 1 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "gpu_run $TAG done $(date +%T)"
