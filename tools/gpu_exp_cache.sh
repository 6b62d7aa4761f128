# oscillator encodings A/B (tools/ab_build.sh variants of synth_frame.hip)
for v in cur rndnep vconst vconstp rndlit cur; do echo "== $v" >> gpurun_out/exp_enc.log; DDSP_HIP_LIB=$PWD/build/ab_$v.so timeout -k 10 200 python tools/exp_timing.py --short >> gpurun_out/exp_enc.log 2>&1 || exit 1; done
