set -e
export TMPDIR=/tmp
ROOT=$(pwd); mkdir -p gpurun_out
cd /tmp
for K in proj mlp; do
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $ROOT/gpurun_out/pmc_r05_$K -o a -- python3 $ROOT/tools/kernel_probe.py $K 10 > $ROOT/gpurun_out/pmc_r05_$K.log 2>&1
done
echo ok
