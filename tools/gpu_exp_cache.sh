timeout -k 10 300 python -u -m pytest tests/test_gpu_synth_reverb.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sr_tests.log 2>&1; tail -1 gpurun_out/sr_tests.log
timeout -k 10 200 python tools/exp_synth_reverb.py > gpurun_out/exp_sr2.log 2>&1
