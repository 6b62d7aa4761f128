#!/bin/bash
# Wave-cycle / MFMA counters of the decoder's MLP block kernels (tools/exp_mlp.py), run via gpurun from the
# repo root: tools/pmc_mlp.sh <tag>.  Two passes, counters per dispatch in gpurun_out/pmc_mlp_<tag>/.
set -e
TAG=${1:-probe}
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmc_mlp_${TAG}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE \
  --output-format csv -d $OUT/a -o a -- python3 $ROOT/tools/exp_mlp.py > $OUT/a.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM GRBM_COUNT \
  --output-format csv -d $OUT/b -o b -- python3 $ROOT/tools/exp_mlp.py > $OUT/b.log 2>&1
echo pmc mlp done
