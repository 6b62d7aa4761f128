#!/bin/bash
# Parity of variant build/ab_<b>.so (frame-table bit-identity, device noise, parity suites), then the
# same-box A/B of ab_<a> vs ab_<b> (tools/gpu_ab2.sh).
mkdir -p gpurun_out
export TMPDIR=/tmp
DDSP_HIP_LIB=$PWD/build/ab_$2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_frame_table.py \
  tests/test_gpu_device_noise.py tests/test_gpu_parity.py tests/test_gpu_synth_reverb.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/ab3_pytest.log 2>&1 || { tail -30 gpurun_out/ab3_pytest.log; exit 1; }
tail -1 gpurun_out/ab3_pytest.log
bash tools/gpu_ab2.sh $1 $2
