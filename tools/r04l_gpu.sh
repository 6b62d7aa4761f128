set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_gru.py tests/test_gpu_mlp.py tests/test_gpu_decoder_route.py tests/test_autoencoder.py tests/test_gpu_grad.py tests/test_gpu_realtime.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r04l.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r04l.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python3 tools/exp_decoder2.py net net_gemm outmlp outmlp_gemm mlps gru proj dsyn fwd > gpurun_out/dec_r04l.log 2>&1 || exit 1
cat gpurun_out/dec_r04l.log
timeout -k 10 100 python3 tools/exp_gru.py > gpurun_out/gru_r04l.log 2>&1 || exit 1
cat gpurun_out/gru_r04l.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mlp2 -o t -- python3 tools/exp_decoder2.py outmlp outmlp_gemm fwd > gpurun_out/prof_mlp2.log 2>&1 || exit 1
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/prof_mlp2/t_kernel_stats.csv')))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:16]:
    print(f"{r['Name'][:90]:90s} {int(r['Calls']):6d} {float(r['AverageNs'])/1000:8.1f} us")
PY
bash tools/ab_prof.sh gru step_kernel grunew grumfma || exit 1
cat gpurun_out/ab_prof.log; cp gpurun_out/ab_prof.log gpurun_out/ab_prof_fwd.log
bash tools/ab_prof.sh gru_train bwd_step grunew grumfma || exit 1
cat gpurun_out/ab_prof.log
echo ALLDONE
