#!/bin/bash
# rocprofv3 kernel times of the reverb's three kernels against batch (tools/exp_mac_scaling.py)
ROOT=$(pwd)
export TMPDIR=/tmp
mkdir -p $ROOT/gpurun_out
: > $ROOT/gpurun_out/mac_scaling.log
for B in "$@"; do
  D=$ROOT/gpurun_out/macs_$B
  (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o t -- \
    python3 $ROOT/tools/exp_mac_scaling.py $B 30 > $D.log 2>&1) || exit 1
  python3 - "$D/t_kernel_stats.csv" "$B" >> $ROOT/gpurun_out/mac_scaling.log <<'PY'
import csv, sys
out = {"B": int(sys.argv[2])}
for r in csv.DictReader(open(sys.argv[1])):
    for k in ("upols_forward_ir", "upols_mac_stream", "upols_mac_ring", "upols_inverse"):
        if k in r["Name"]:
            out[k] = round(float(r["AverageNs"]) / 1000, 2)
print(out)
PY
done
cat $ROOT/gpurun_out/mac_scaling.log
