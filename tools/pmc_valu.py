"""PMC VALU instruction counts of the fused synthesis kernel (tools/pmc_probe.sh fused <tag>) ->
profiles/pmc_valu.json, which bench.py's roofline reads (issue slots per launch).

    python tools/pmc_valu.py gpurun_out/pmc_<tag>_fused [config]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    d = sys.argv[1]
    cfg = sys.argv[2] if len(sys.argv) > 2 else "2"
    vals = defaultdict(list)
    for f in glob.glob(d + "/*/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "synth_frame_kernel" in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    m = {k: sum(v) / len(v) for k, v in vals.items()}
    path = os.path.join(ROOT, "profiles", "pmc_valu.json")
    try:
        out = json.load(open(path))
    except (OSError, ValueError):
        out = {}
    sys.path.insert(0, ROOT)
    from bench import DOMINANT_KERNEL, kernel_source_sha
    out[f"config{cfg}"] = {"kernel": DOMINANT_KERNEL,
                           "source": os.path.relpath(d, ROOT).replace("gpurun_out/", "profiles/") + ".txt",
                           "kernel_sha": kernel_source_sha(),
                           **{k: m[k] for k in sorted(m) if k.startswith("SQ_")}}
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out[f"config{cfg}"], indent=1))


if __name__ == "__main__":
    main()
