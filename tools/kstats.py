"""Print a rocprofv3 kernel-stats CSV compactly: short kernel name, calls, average us.
    python tools/kstats.py <dir-or-csv> [filter]"""
import csv
import glob
import os
import sys

p = sys.argv[1]
files = [p] if p.endswith(".csv") else glob.glob(os.path.join(p, "**", "*kernel_stats.csv"), recursive=True)
flt = sys.argv[2] if len(sys.argv) > 2 else ""
for f in files:
    for r in csv.DictReader(open(f)):
        name = r["Name"].replace("(anonymous namespace)::", "").replace("void ", "").replace("ddsp::", "")
        name = name.split("(")[0]
        if flt in name:
            print(f"{name[:60]:60s} calls {int(r['Calls']):6d}  avg {float(r['AverageNs'])/1e3:8.2f} us  "
                  f"total% {float(r['Percentage']):5.1f}")
