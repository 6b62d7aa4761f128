# one GPU call: per-frame prologue A/B, persistent-kernel tests + probe + sweep, GPU test suite, default bench
mkdir -p gpurun_out
for rep in 1 2; do for v in prev new; do echo "== $v" >> gpurun_out/ab_prologue.log; DDSP_HIP_LIB=$PWD/build/ab_$v.so timeout -k 10 100 python tools/exp_timing.py --short >> gpurun_out/ab_prologue.log 2>&1 || exit 1; done; done
bash tools/gpu_persist_sweep.sh || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r03b.log 2>&1; tail -2 gpurun_out/pytest_r03b.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_r03b.json 2> gpurun_out/bench_r03b.err || { tail -5 gpurun_out/bench_r03b.err; exit 1; }
