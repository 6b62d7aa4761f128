DDSP_HIP_LIB=$PWD/build/ab_clk.so timeout -k 10 300 python tools/exp_clock.py --in-kernel > gpurun_out/exp_clock_ik3.log 2>&1
