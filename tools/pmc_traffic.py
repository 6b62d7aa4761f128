"""Summarise rocprofv3 runs (tools/profile.sh) into profiles/:

  * <tag>_kernel_stats.csv      — rocprofv3 --kernel-trace --stats summary (copied)
  * <tag>_pmc.json              — per-kernel mean FETCH_SIZE / WRITE_SIZE per launch
  * pmc_traffic.json            — HBM bytes per launch for the kernels bench.py reports

Counter conventions (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide (16 B/lane) coalesced streaming
read, so it is doubled for kernels whose dominant reads are 16-byte vector loads.  The
correction is applied only where that access shape holds (listed in WIDE_READS).

    python tools/pmc_traffic.py <tag> [gpurun_out]
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# kernels whose FETCH_SIZE is doubled: 16-B/lane streaming amplitude reads (the guide's rule), and
# the UPOLS kernels' 4- and 8-B/lane coalesced streaming reads, calibrated on known byte counts in
# their own access pattern (MI355X_MICROARCH.md: other widths "uncalibrated: calibrate"): the
# inverse reads the Y spectra exactly once (51.2 MB at config 2) and reports 25.7 MB; the forward
# reads the signal exactly once (26.2 MB) and reports 12.9 MB
WIDE_READS = ("harmonic_samples_tiled_kernel", "upols_forward_kernel", "upols_forward_ir_kernel", "upols_inverse_kernel",
              "upols_mac_kernel", "upols_mac_ring_kernel", "upols_mac_stream_kernel")
REPORT = {  # bench.py roofline key -> kernels whose bytes add up to one launch of it (a name with its template
    # arguments matches that instantiation only: bench.py's realtime leg launches the one-sample-per-thread
    # instantiation of the fused kernel at 4 frames per call, whose launches must not dilute config 2's mean)
    "synth_frame_kernel": ("synth_frame_kernel<true, false, false, false>",),
    "harmonic_frames_kernel": ("harmonic_frames_kernel",),
    "harmonic_samples_kernel": ("phase_chunk_sums_kernel", "harmonic_samples_tiled_kernel"),
    "filtered_noise_kernel": ("filtered_noise_kernel",),
    "reverb": ("upols_forward_kernel", "upols_forward_ir_kernel", "upols_mac_kernel", "upols_mac_ring_kernel",
               "upols_mac_stream_kernel", "upols_inverse_kernel"),
}


def short(name):
    """kernel name with its template arguments, without namespace, return type and parameters"""
    base = name.replace("(anonymous namespace)", "anon").split("(")[0]
    return base.replace("void ", "").split("::")[-1]


def base(name):
    return name.split("<")[0]


def matches(k, pattern):
    return k == pattern if "<" in pattern else base(k) == pattern


def per_kernel(path):
    acc = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            acc[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out")
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = os.path.join(out, f"prof_{tag}", "trace_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(prof, f"{tag}_kernel_stats.csv"))
    fetch = per_kernel(os.path.join(out, f"pmc_{tag}_fetch", "fetch_counter_collection.csv"))
    write = per_kernel(os.path.join(out, f"pmc_{tag}_write", "write_counter_collection.csv"))
    table = {}
    for k in sorted(set(fetch) | set(write)):
        f_kib, w_kib = fetch.get(k, 0.0), write.get(k, 0.0)
        corr = 2.0 if base(k) in WIDE_READS else 1.0
        table[k] = {"fetch_kib_raw": round(f_kib, 1), "fetch_correction": corr,
                    "write_kib": round(w_kib, 1),
                    "hbm_bytes": int((f_kib * corr + w_kib) * 1024)}
    with open(os.path.join(prof, f"{tag}_pmc.json"), "w") as f:
        json.dump(table, f, indent=1)
    traffic = {key: sum(v["hbm_bytes"] for k, v in table.items() if any(matches(k, p) for p in ks))
               for key, ks in REPORT.items() if any(matches(k, p) for k in table for p in ks)}
    traffic["_source"] = f"profiles/{tag}_pmc.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes)"
    with open(os.path.join(prof, "pmc_traffic.json"), "w") as f:
        json.dump(traffic, f, indent=1)
    print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    main()
