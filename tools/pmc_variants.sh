#!/bin/bash
# One PMC pass (VALU / SALU / LDS instruction counts) of the fused synthesis kernel per library
# variant (run via gpurun from the repo root):  bash tools/pmc_variants.sh <name>...
# ("base" = the in-tree library, else build/ab_<name>.so, e.g. tools/probe_build.py's probes)
ROOT=$(pwd)
export TMPDIR=/tmp
mkdir -p $ROOT/gpurun_out
LOG=$ROOT/gpurun_out/pmc_variants.log
: > $LOG
for v in "$@"; do
  if [ "$v" = base ]; then LIB=$ROOT/ddsp_pytorch_amd/lib/libddsp_hip.so; else LIB=$ROOT/build/ab_$v.so; fi
  D=$ROOT/gpurun_out/pmcv_$v
  (cd /tmp && DDSP_HIP_LIB=$LIB timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES \
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
print(f"{v:10s} VALU {m.get('SQ_INSTS_VALU', 0) / 1e6:7.2f} M  SALU {m.get('SQ_INSTS_SALU', 0) / 1e6:6.2f} M  "
      f"LDS {m.get('SQ_INSTS_LDS', 0) / 1e6:5.2f} M  waves {m.get('SQ_WAVES', 0):.0f}  median {durs[len(durs) // 2] if durs else 0:7.1f} us", flush=True)
PY
  tail -1 $LOG
done
