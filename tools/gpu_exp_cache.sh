# streaming-policy variants (cur = z2g3 default; old = round-2 policy), then the train step with the adjoint MAC's loads nt
for v in old cur z2g3y z2g3i z2g3f z3g3 old cur; do echo "== $v" >> gpurun_out/exp_aux3.log; DDSP_HIP_LIB=$PWD/build/ab_$v.so timeout -k 10 200 python tools/exp_timing.py --short >> gpurun_out/exp_aux3.log 2>&1 || exit 1; done
for v in cur adjnt cur adjnt; do echo "== $v" >> gpurun_out/exp_train.log; DDSP_HIP_LIB=$PWD/build/ab_$v.so timeout -k 10 200 python tools/exp_train_time.py >> gpurun_out/exp_train.log 2>&1 || exit 1; done
