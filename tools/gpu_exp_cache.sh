# does a small kernel between the reverb and the next synthesis launch remove the slowdown? (tools/exp_gap.py --reset)
timeout -k 10 200 python tools/exp_gap.py --reset > gpurun_out/exp_gap2.log 2>&1
