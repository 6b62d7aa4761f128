#!/bin/bash
# VALU / wave-cycle counters for one kernel of the path (run via gpurun from the repo root):
#   tools/pmc_probe.sh <kernel> <tag>
set -e
K=${1:-harmonic}; TAG=${2:-probe}
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmc_${TAG}_${K}
export TMPDIR=/tmp
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
  --output-format csv -d $OUT/a -o a -- python3 $ROOT/tools/kernel_probe.py $K 10 > $OUT.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT GRBM_COUNT \
  --output-format csv -d $OUT/b -o b -- python3 $ROOT/tools/kernel_probe.py $K 10 >> $OUT.log 2>&1
echo probe $K done
