mkdir -p gpurun_out; : > gpurun_out/cumask.log
for m in plain 64:block 64:spread 64:xcd 48:xcd 32:xcd 96:xcd 56:block; do
  timeout -k 10 60 python -u tools/exp_cumask.py $m >> gpurun_out/cumask.log 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/cumask.log
