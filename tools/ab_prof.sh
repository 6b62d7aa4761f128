#!/bin/bash
# Kernel-level A/B of C-ABI library variants (run via gpurun from the repo root):
#   tools/ab_prof.sh <probe> <kernel-substring> <name>...
# runs tools/kernel_probe.py <probe> under rocprofv3 --kernel-trace --stats with
# DDSP_HIP_LIB=build/ab_<name>.so, twice per variant, and prints the kernel's average duration.
PROBE=$1; KERN=$2; shift 2
ROOT=$(pwd)
export TMPDIR=/tmp
mkdir -p $ROOT/gpurun_out
: > $ROOT/gpurun_out/ab_prof.log
for rep in 1 2; do
  for v in "$@"; do
    D=$ROOT/gpurun_out/abp_${v}_$rep
    (cd /tmp && DDSP_HIP_LIB=$ROOT/build/ab_$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $D -o t -- python3 $ROOT/tools/kernel_probe.py $PROBE 30 > $D.log 2>&1) || exit 1
    python3 - "$D/t_kernel_stats.csv" "$KERN" "$v" >> $ROOT/gpurun_out/ab_prof.log <<'EOF'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if sys.argv[2] in r["Name"].replace(" ", ""):
        print(f"{sys.argv[3]:10s} {float(r['AverageNs']) / 1000:8.1f} us  (min {float(r['MinNs']) / 1000:.1f}, {r['Calls']} calls)")
EOF
  done
done
cat $ROOT/gpurun_out/ab_prof.log
