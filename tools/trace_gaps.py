"""Kernel sequence with start gaps from a rocprofv3 kernel trace (development aid):
    python tools/trace_gaps.py <kernel_trace.csv> <first-kernel-substring> [count]
prints the `count` kernels from the last occurrence of the first kernel, with the idle gap before each."""
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
key, n = sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 20
idx = [i for i, r in enumerate(rows) if key in r["Kernel_Name"]]
i0 = idx[-2] if len(idx) > 1 else idx[-1]
prev_end = None
for r in rows[i0:i0 + n]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev_end) / 1000 if prev_end else 0.0
    print(f"gap {gap:7.1f} us  dur {(e - s) / 1000:7.1f} us  {r['Kernel_Name'][:90]}")
    prev_end = e
