#!/bin/bash
# Same-box A/B of library variants in the bench step (run via gpurun from the repo root):
#   bash tools/ab_step.sh <name>...      (build/ab_<name>.so from tools/ab_build.sh; "base" = the in-tree lib)
# Per variant, twice, interleaved: bench.py at 200 steps (step ms, in-region synthesis ms), then a
# rocprofv3 kernel trace of a 60-step bench (average kernel times in the step's order).
mkdir -p gpurun_out
export TMPDIR=/tmp
LOG=gpurun_out/ab_step.log
: > $LOG
ARGS="--no-train-leg --no-loss-leg --no-model-train-leg --no-decoder-leg --no-op-leg --no-cpu-baseline --no-uncached-leg --no-pipelined-leg"
for rep in 1 2; do
  for v in "$@"; do
    if [ "$v" = base ]; then LIB=$PWD/ddsp_pytorch_amd/lib/libddsp_hip.so; else LIB=$PWD/build/ab_$v.so; fi
    DDSP_HIP_LIB=$LIB timeout -k 10 120 python3 bench.py --steps 200 --warmup 20 $ARGS > gpurun_out/ab_s.json 2>gpurun_out/ab_s.err || { tail -5 gpurun_out/ab_s.err; exit 1; }
    D=gpurun_out/abs_${v}_$rep
    DDSP_HIP_LIB=$LIB timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o t -- python3 bench.py --steps 60 --warmup 10 $ARGS > $D.log 2>&1 || { tail -5 $D.log; exit 1; }
    python3 - $v gpurun_out/ab_s.json $D >> $LOG <<'PY'
import csv, glob, json, sys
v, js, d = sys.argv[1:4]
b = json.loads(open(js).read().strip().split("\n")[-1])
ks = {}
for f in glob.glob(d + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        for short, key in (("synth", "synth_frame_kernel"), ("mac", "upols_mac_"), ("fwd", "upols_forward"), ("inv", "upols_inverse")):
            if key in n:
                ks[short] = float(r["AverageNs"]) / 1e3
print(f"{v:10s} step {b['ms_per_step']:.4f} ms  synth(in-region) {b['roofline']['avg_launch_ms']:.4f}  rocprof " +
      " ".join(f"{k} {ks.get(k, float('nan')):6.1f}" for k in ("synth", "mac", "fwd", "inv")), flush=True)
PY
    tail -1 $LOG
  done
done
