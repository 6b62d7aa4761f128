# A/B of the persistent kernel's probe variants (tools/exp_timing.py --short, wpc 8)
for v in base noprep noosc; do echo "== $v" >> gpurun_out/ab_persist.log; DDSP_HIP_LIB=$PWD/build/ab_$v.so timeout -k 10 100 python tools/exp_timing.py --short >> gpurun_out/ab_persist.log 2>&1 || exit 1; done
for v in base noosc; do echo "== $v per-frame (wpc 0)" >> gpurun_out/ab_persist.log; DDSP_HIP_PERSIST_WPC=0 DDSP_HIP_LIB=$PWD/build/ab_$v.so timeout -k 10 100 python tools/exp_timing.py --short >> gpurun_out/ab_persist.log 2>&1 || exit 1; done
