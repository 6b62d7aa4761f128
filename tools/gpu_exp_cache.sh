# same-box bench A/B: the MAC's round-2 cache policy (old) vs the non-temporal loads (cur)
F="--no-train-leg --no-loss-leg --no-model-train-leg --no-decoder-leg --no-cpu-baseline --no-op-leg --no-uncached-leg"
for v in old cur old cur; do echo "== $v" >> gpurun_out/bench_ab.log; DDSP_HIP_LIB=$PWD/build/ab_$v.so timeout -k 10 200 python bench.py $F >> gpurun_out/bench_ab.log 2>/dev/null || exit 1; done
