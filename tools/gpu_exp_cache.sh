# fused synthesis + transform: new C-entry test, PMC HBM bytes of the fused route's kernels
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_synth_reverb.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sr_tests.log 2>&1 || { tail -30 gpurun_out/sr_tests.log; exit 1; }
tail -1 gpurun_out/sr_tests.log
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_sr_fetch -o fetch -- python tools/exp_synth_reverb.py --fused-only > gpurun_out/pmc_sr_fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_sr_write -o write -- python tools/exp_synth_reverb.py --fused-only > gpurun_out/pmc_sr_write.log 2>&1 || exit 1
echo pmc done
