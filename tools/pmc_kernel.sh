#!/bin/bash
# One rocprofv3 PMC pass per counter set for one kernel of a command (run via gpurun from the repo root):
#   bash tools/pmc_kernel.sh <kernel-substring> <tag> <python script> [args...]
# Prints the per-launch mean of each counter for launches whose name contains the substring.
K=$1; TAG=$2; shift 2
ROOT=$(pwd)
export TMPDIR=/tmp
mkdir -p $ROOT/gpurun_out
i=0
for SET in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
  i=$((i + 1))
  D=$ROOT/gpurun_out/pmck_${TAG}_$i
  (cd /tmp && timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $SET --output-format csv -d $D -o p -- python3 "$@" > $D.log 2>&1) || { tail -5 $D.log; exit 1; }
  python3 - "$K" $D <<'PY'
import csv, glob, sys
from collections import defaultdict
k, d = sys.argv[1:3]
vals = defaultdict(list)
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if k in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(" ".join(f"{c} {sum(v) / len(v) / 1e6:.3f}M" for c, v in sorted(vals.items())), flush=True)
PY
done
