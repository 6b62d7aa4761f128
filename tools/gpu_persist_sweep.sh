# persistent synthesis kernel: tests, phase probe, and the timing sweep over workgroups per CU
timeout -k 10 300 python -u -m pytest tests/test_gpu_persist.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_persist.log 2>&1; tail -3 gpurun_out/pytest_persist.log
DDSP_HIP_LIB=$PWD/build/ab_pclk.so timeout -k 10 100 python tools/exp_persist.py > gpurun_out/exp_persist.log 2>&1 || exit 1
for w in 0 5 6; do echo "wpc=$w" >> gpurun_out/exp_timing_wpc.log; DDSP_HIP_PERSIST_WPC=$w timeout -k 10 100 python tools/exp_timing.py --short >> gpurun_out/exp_timing_wpc.log 2>&1 || exit 1; done
