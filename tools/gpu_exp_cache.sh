# streaming policies elsewhere in the step (same-box bench A/B, config 2)
F="--no-train-leg --no-loss-leg --no-model-train-leg --no-decoder-leg --no-cpu-baseline --no-op-leg --no-uncached-leg --no-pipelined-leg"
for v in cur so fx iy cur so fx iy; do echo "== $v" >> gpurun_out/bench_ab_nt.log; DDSP_HIP_LIB=$PWD/build/ab_$v.so timeout -k 10 200 python bench.py $F >> gpurun_out/bench_ab_nt.log 2>/dev/null || exit 1; done
