"""Launch time of the fused synthesis kernel (and the synthesis VJP) against grid size: is a workgroup's
lifetime set by its own latency chain (flat time while the grid fits the chip) or by sharing the SIMDs
(time growing with the resident workgroups)?  Config-2 frames (F=200, bs=512, H=100, NB=65), batch B.

    python tools/exp_occupancy_curve.py [reps]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddsp_pytorch_amd import core  # noqa: E402
from ddsp_pytorch_amd.synth import make_inputs  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = None
    for _ in range(3):
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        b.synchronize()
        t = a.elapsed_time(b) * 1000.0 / reps
        best = t if best is None else min(best, t)
    return best


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda", 0)
    F, H, NB, bs, sr = 200, 100, 65, 512, 48000
    rows = []
    for B in (1, 2, 4, 8, 12, 18, 27, 36, 48, 64):
        inp = make_inputs(B, F, H, NB, bs, seed=0, device=dev, with_noise=False)
        with torch.no_grad():
            fwd = timed(lambda: core.synth_frames(inp["f0"], inp["param"], inp["mags"], bs, sr), reps)
        param = inp["param"].clone().requires_grad_(True)
        mags = inp["mags"].clone().requires_grad_(True)
        out = core.synth_frames(inp["f0"], param, mags, bs, sr)
        g = torch.randn_like(out)
        bwd = timed(lambda: out.backward(g, retain_graph=True), reps)
        rows.append({"B": B, "workgroups": B * F, "fused_us": round(fwd, 2), "backward_us": round(bwd, 2)})
        print(json.dumps(rows[-1]), flush=True)


if __name__ == "__main__":
    main()
