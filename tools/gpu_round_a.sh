# one GPU call: persistent-kernel tests + phase probe + workgroup sweep, the GPU test suite, the default bench
mkdir -p gpurun_out
bash tools/gpu_persist_sweep.sh || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r03b.log 2>&1; tail -2 gpurun_out/pytest_r03b.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_r03b.json 2> gpurun_out/bench_r03b.err || { tail -5 gpurun_out/bench_r03b.err; exit 1; }
