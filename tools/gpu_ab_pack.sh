#!/bin/bash
# GPU tests on the built library, then same-box A/B of build/ab_old.so vs build/ab_new.so: the bench step
# (tools/ab_bench.sh) and rocprofv3 kernel averages of the fused synthesis kernel (tools/ab_prof.sh).
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pack_pytest.log 2>&1 || { tail -30 gpurun_out/pack_pytest.log; exit 1; }
tail -1 gpurun_out/pack_pytest.log
bash tools/ab_bench.sh old new old new || exit 1
cat gpurun_out/ab_bench.log
bash tools/ab_prof.sh fused "synth_frame_kernel<true, false, false>" old new || exit 1
