"""Does the synthesis backward run faster as its two halves on two streams than fused in one
launch?  Times, at config 2 with device noise: the fused kernel (ddsp_hip_synth_frames_backward),
the harmonic half (ddsp_hip_harmonic_synth_params_backward) and the noise half
(ddsp_hip_filtered_noise_backward) alone, both halves back to back on one stream, and both halves
on two streams (development experiment).

    python tools/exp_bwd_split.py
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddsp_pytorch_amd import _lib, core  # noqa: E402
from ddsp_pytorch_amd.synth import make_inputs  # noqa: E402

B, F, H, NB, bs, sr = 64, 200, 100, 65, 512, 48000
N = 50


def main():
    inp = make_inputs(B, F, H, NB, bs, device="cuda", with_noise=False)
    f0, param, mags = (core._c(inp[k]) for k in ("f0", "param", "mags"))
    g = torch.randn(B, F * bs, 1, device="cuda")
    dp = torch.empty(B, F, H + 1, device="cuda")
    dm = torch.empty(B, F, NB, device="cuda")
    seed, off, bias = 1234, 0, -5.0
    P = _lib.ptr
    s2 = torch.cuda.Stream()

    def fused(stream=None):
        _lib.call("synth_frames_backward", P(f0), P(param), P(mags), bias, None, seed, off, P(g), P(g), P(dp),
                  P(dm), B, F, H, NB, bs, float(sr), stream or _lib.stream_of(dp))

    def harm(stream=None):
        _lib.call("harmonic_synth_params_backward", P(f0), P(param), P(g), P(dp), B, F, H, bs, float(sr),
                  stream or _lib.stream_of(dp))

    def noise(stream=None):
        _lib.call("filtered_noise_backward", P(mags), None, seed, off, 1, bias, P(g), P(dm), B, F, NB, bs,
                  stream or _lib.stream_of(dm))

    def two_streams():
        e = torch.cuda.Event()
        e.record()
        s2.wait_event(e)
        harm()
        noise(s2.cuda_stream)
        e2 = torch.cuda.Event()
        e2.record(s2)
        torch.cuda.current_stream().wait_event(e2)

    def timed(fn):
        t = time.perf_counter()
        while time.perf_counter() - t < 0.3:
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(N):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / N * 1e6

    for name, fn in (("fused", fused), ("harmonic half", harm), ("noise half", noise),
                     ("halves, one stream", lambda: (harm(), noise())), ("halves, two streams", two_streams),
                     ("fused again", fused)):
        print(f"{name:22s} {timed(fn):7.1f} us", flush=True)


if __name__ == "__main__":
    main()
