"""The fused synthesis + forward-transform route against the two launch groups (development
experiment): event-timed back-to-back steps at config 2, and the parity between them.

    python tools/exp_synth_reverb.py
"""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddsp_pytorch_amd import core  # noqa: E402
from ddsp_pytorch_amd.synth import SynthPath, make_inputs  # noqa: E402


def main():
    B, F, H, NB, bs, sr = 64, 200, 100, 65, 512, 48000
    inp = make_inputs(B, F, H, NB, bs, device="cuda", with_noise=False)
    syn = SynthPath(bs, sr, reverb_length=48000).to("cuda")
    spec = syn.reverb._spectrum(F * bs)
    two = lambda: core.reverb_apply(core.synth_frames(inp["f0"], inp["param"], inp["mags"], bs, sr), spec, 48000)
    fused = lambda: core.synth_reverb(inp["f0"], inp["param"], inp["mags"], bs, sr, spec, 48000)
    E = lambda: torch.cuda.Event(enable_timing=True)
    if "--fused-only" in sys.argv:  # a short run for rocprofv3 --pmc passes
        for _ in range(20):
            fused()
        torch.cuda.synchronize()
        return

    def group(fn, n=50, reps=7):
        t = time.perf_counter()
        while time.perf_counter() - t < 0.3:
            fn()
        out = []
        for _ in range(reps):
            e0, e1 = E(), E()
            e0.record()
            for _ in range(n):
                fn()
            e1.record()
            torch.cuda.synchronize()
            out.append(e0.elapsed_time(e1) / n * 1e3)
        return statistics.median(out), min(out)

    for rep in range(2):
        for name, fn in (("two launch groups", two), ("fused synthesis + transform", fused)):
            med, lo = group(fn)
            print(f"{name:30s}: step {med:7.1f} us (min {lo:7.1f})", flush=True)
    core.set_noise_seed(5)
    a = two()
    core.set_noise_seed(5)
    b = fused()
    torch.cuda.synchronize()
    print(f"max |fused - two| = {float((a - b).abs().max()):.3e}, rms(out) = {float(a.pow(2).mean().sqrt()):.3f}")


if __name__ == "__main__":
    main()
