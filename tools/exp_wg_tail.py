"""How full is the chip over one fused synthesis launch?  (measurement only.)
Runs config 2's synthesis step (fused kernel + reverb, as bench.py) through the wgclk probe build
(tools/probe_build.py wgclk -> build/ab_wgclk.so, loaded through DDSP_HIP_LIB), then reads the last
launch's per-workgroup start / end stamps (s_memrealtime, 100 MHz) and prints the resident-workgroup
count over time, the workgroup durations by dispatch round and the fill efficiency
(sum of workgroup time / (span x peak residency)).

    DDSP_HIP_LIB=build/ab_wgclk.so python tools/exp_wg_tail.py
"""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddsp_pytorch_amd import _lib  # noqa: E402
from ddsp_pytorch_amd.synth import SynthPath, make_inputs  # noqa: E402


def main():
    B, F, H, NB, bs, sr = 64, 200, 100, 65, 512, 48000
    inp = make_inputs(B, F, H, NB, bs, device="cuda")
    path = SynthPath(bs, sr, reverb_length=48000).to("cuda")
    with torch.no_grad():
        t = time.perf_counter()
        while time.perf_counter() - t < 0.5:
            path(inp["f0"], inp["param"], inp["mags"])
        torch.cuda.synchronize()
    n = B * F
    st = np.zeros(3 * n, dtype=np.uint64)
    rc = _lib.load().ddsp_probe_wg_stamps(st.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(n))
    assert rc == 0, rc
    st = st.reshape(n, 3)
    t0 = st[:, 0].astype(np.int64)
    t1 = st[:, 1].astype(np.int64)
    base = t0.min()
    s, e = (t0 - base) * 0.01, (t1 - base) * 0.01  # us
    span = e.max()
    dur = e - s
    grid = np.arange(0.0, span + 0.5, 0.5)
    active = np.array([np.count_nonzero((s <= g) & (e > g)) for g in grid])
    peak = active.max()
    order = np.argsort(s)
    rounds = {}
    per = 4096
    for r in range(int(np.ceil(n / per))):
        idx = order[r * per:(r + 1) * per]
        rounds[r] = {"n": int(idx.size), "start_us": round(float(s[idx].min()), 2),
                     "last_start_us": round(float(s[idx].max()), 2),
                     "dur_median_us": round(float(np.median(dur[idx])), 2),
                     "dur_p90_us": round(float(np.percentile(dur[idx], 90)), 2)}
    below = grid[active < 0.9 * peak]
    tail_start = float(below[below > span * 0.3].min()) if (below > span * 0.3).any() else span
    xcc = (st[:, 2] >> np.uint64(32)).astype(np.int64)
    hw = (st[:, 2] & np.uint64(0xFFFFFFFF)).astype(np.int64)
    cu = xcc * 256 + ((hw >> 8) & 0xFF)  # HW_ID [15:8]: cu_id, sh_id, se_id
    per_cu_peak = []
    for c in np.unique(cu):
        m = cu == c
        ev = sorted([(t, 1) for t in s[m]] + [(t, -1) for t in e[m]], key=lambda x: (x[0], x[1]))
        cur = top = 0
        for _, d in ev:
            cur += d
            top = max(top, cur)
        per_cu_peak.append(top)
    occ = {str(t): _lib.load().ddsp_probe_occupancy(ctypes.c_int(t), ctypes.c_int64(6480)) for t in (64, 128, 256)}
    out = {"span_us": round(float(span), 2), "peak_resident_wg": int(peak), "runtime_occupancy_blocks_per_cu": occ,
           "fill_efficiency": round(float(dur.sum() / (span * peak)), 4),
           "tail_from_us": round(tail_start, 2),
           "wg_time_in_tail_frac": round(float(np.clip(np.minimum(e, span) - np.maximum(s, tail_start), 0,
                                                        None).sum() / dur.sum()), 4),
           "rounds": rounds,
           "wg_per_xcc": np.bincount(xcc, minlength=8).tolist(),
           "distinct_cus": int(np.unique(cu).size),
           "per_cu_peak_resident": {str(k): int(v) for k, v in zip(*np.unique(per_cu_peak, return_counts=True))},
           "xcc_span_us": [round(float(e[xcc == x].max() - s[xcc == x].min()), 2) for x in range(8)],
           "active_every_5us": active[::10].tolist()}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
