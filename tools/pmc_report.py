"""Summarise tools/pmc_probe.sh output: per-kernel mean counters and derived rates.

    python tools/pmc_report.py gpurun_out/pmc_<tag>_<kernel>
"""
import csv
import glob
import sys
from collections import defaultdict


def load(d):
    vals = defaultdict(lambda: defaultdict(list))
    durs = defaultdict(list)
    for f in glob.glob(d + "/*/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("(anonymous namespace)", "anon").split("(")[0].split("::")[-1]
            vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for f in glob.glob(d + "/*/*kernel_trace.csv"):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("(anonymous namespace)", "anon").split("(")[0].split("::")[-1]
            durs[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    return vals, durs


def main():
    vals, durs = load(sys.argv[1])
    for k, c in vals.items():
        if "ddsp" not in k and "kernel" not in k:
            continue
        m = {n: sum(v) / len(v) for n, v in c.items()}
        t = sorted(durs.get(k, [0]))[len(durs.get(k, [0])) // 2]
        print(f"== {k}  (median {t*1e6:.1f} us)")
        for n in sorted(m):
            print(f"   {n:24s} {m[n]:.4g}")
        if "GRBM_GUI_ACTIVE" in m and t > 0:
            clk = m["GRBM_GUI_ACTIVE"] / 8 / t
            print(f"   effective clock ~ {clk/1e9:.2f} GHz (GRBM_GUI_ACTIVE/8/t; reads high below 0.3 ms)")
            if "SQ_INSTS_VALU" in m:
                # SQ_INSTS_VALU counts wave-instructions; peak = 256 CU * 4 SIMD * clk / 2 cycles
                rate = m["SQ_INSTS_VALU"] / t
                peak = 256 * 4 * clk / 2
                print(f"   VALU wave-instr/s {rate:.3e} = {rate/peak*100:.1f}% of {peak:.3e} at that clock")
        if "SQ_ACTIVE_INST_VALU" in m and "SQ_WAVE_CYCLES" in m:
            print(f"   ACTIVE_INST_VALU / WAVE_CYCLES = {m['SQ_ACTIVE_INST_VALU']/m['SQ_WAVE_CYCLES']:.3f}")


if __name__ == "__main__":
    main()
