set -o pipefail
export TMPDIR=/tmp
timeout -k 10 100 python3 tools/exp_gru.py > gpurun_out/gru_r04n.log 2>&1 || { cat gpurun_out/gru_r04n.log; exit 1; }
cat gpurun_out/gru_r04n.log
AB_SCRIPT=tools/exp_gru.py bash tools/ab_time.sh grunew grumfma || exit 1
grep -v amdgpu.ids gpurun_out/ab.log
timeout -k 10 200 python3 tools/exp_uncached.py > gpurun_out/unc_r04n.log 2>&1 || { cat gpurun_out/unc_r04n.log; exit 1; }
cat gpurun_out/unc_r04n.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dec_r04n -o t -- python3 tools/exp_decoder2.py outmlp outmlp_gemm mlps net > gpurun_out/prof_dec_r04n.log 2>&1 || exit 1
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/prof_dec_r04n/t_kernel_stats.csv')))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:16]:
    print(f"{r['Name'][:90]:90s} {int(r['Calls']):6d} {float(r['AverageNs'])/1000:8.1f} us")
PY
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gru_r04n -o t -- python3 tools/exp_gru.py > gpurun_out/prof_gru_r04n.log 2>&1 || exit 1
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/prof_gru_r04n/t_kernel_stats.csv')))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:10]:
    print(f"{r['Name'][:90]:90s} {int(r['Calls']):6d} {float(r['AverageNs'])/1000:8.1f} us")
PY
bash tools/ab_prof.sh gru step_kernel grunew grumfma || exit 1
cp gpurun_out/ab_prof.log gpurun_out/ab_prof_fwd_r04n.log; cat gpurun_out/ab_prof.log
bash tools/ab_prof.sh gru_train bwd_step grunew grumfma || exit 1
cp gpurun_out/ab_prof.log gpurun_out/ab_prof_bwd_r04n.log; cat gpurun_out/ab_prof.log
echo ALLDONE
