#!/bin/bash
# Does the f32 MFMA FIR take VALU issue from the sine loops?  One PMC pass per library variant
# (run via gpurun from the repo root):  bash tools/pmc_mfma.sh <name>...   ("base" = the in-tree library)
ROOT=$(pwd)
export TMPDIR=/tmp
mkdir -p $ROOT/gpurun_out
LOG=$ROOT/gpurun_out/pmc_mfma.log
: > $LOG
for v in "$@"; do
  if [ "$v" = base ]; then LIB=$ROOT/ddsp_pytorch_amd/lib/libddsp_hip.so; else LIB=$ROOT/build/ab_$v.so; fi
  D=$ROOT/gpurun_out/pmcm_$v
  (cd /tmp && DDSP_HIP_LIB=$LIB timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_TRANS_F32 SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_LDS \
    --output-format csv -d $D -o p -- python3 $ROOT/tools/kernel_probe.py fused 10 > $D.log 2>&1) || { tail -5 $D.log; exit 1; }
  python3 - $v $D >> $LOG <<'PY'
import csv, glob, sys
from collections import defaultdict
v, d = sys.argv[1:3]
vals = defaultdict(list); durs = []
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "synth_frame_kernel" in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "synth_frame_kernel" in r["Kernel_Name"]:
            durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
m = {k: sum(x) / len(x) for k, x in vals.items()}
durs.sort()
print(v, " ".join(f"{k} {m[k] / 1e6:.3f}M" for k in sorted(m)), f"median {durs[len(durs) // 2] if durs else 0:.1f} us", flush=True)
PY
  tail -1 $LOG
done
