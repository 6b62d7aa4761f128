"""Reverb (UPOLS) time vs batch at T = 102400, L = 48000: is each kernel bandwidth-bound
(time ~ batch) or latency/occupancy-bound (flat until the grid fills another round)?
Run under rocprofv3 --kernel-trace --stats for the per-kernel split.

    python tools/exp_reverb_scaling.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddsp_pytorch_amd import core  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    T, L = 102400, 48000
    h = torch.randn(L, device=dev) * 0.01
    h[0] = 1
    spec = core.reverb_spectrum(h, T)
    for B in (int(a) for a in (sys.argv[1:] or [8, 16, 32, 40, 48, 64, 82, 96, 128])):
        x = torch.randn(B, T, 1, device=dev)
        with torch.no_grad():
            for _ in range(3):
                core.reverb_apply(x, spec, L)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                core.reverb_apply(x, spec, L)
            e1.record()
            torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        print(f"B={B:4d} pairs={(B + 1) // 2:3d} reverb {ms * 1e3:7.1f} us  {B * T / ms / 1e6:6.2f} G samples/s",
              flush=True)


if __name__ == "__main__":
    main()
