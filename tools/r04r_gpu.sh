set -o pipefail
export TMPDIR=/tmp
for m in cached uncached; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_unc_$m -o t -- python3 tools/exp_uncached.py $m > gpurun_out/prof_unc_$m.log 2>&1 || exit 1
  grep -v amdgpu gpurun_out/prof_unc_$m.log
  python3 - $m <<'PY'
import csv, sys
rows=list(csv.DictReader(open(f'gpurun_out/prof_unc_{sys.argv[1]}/t_kernel_stats.csv')))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:7]:
    print(f"{r['Name'][:70]:70s} {int(r['Calls']):6d} {float(r['AverageNs'])/1000:8.1f} us")
PY
done
echo ALLDONE
