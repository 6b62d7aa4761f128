"""Within one config-2 step: does splitting the batch in two and running reverb(first half) on a
second stream beside synth(second half) shorten the step?  (development experiment)

    python tools/exp_split_overlap.py
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
    dev = torch.device("cuda", 0)
    B, F, H, NB, bs, sr = 64, 200, 100, 65, 512, 48000
    inp = make_inputs(B, F, H, NB, bs, seed=0, device=dev, with_noise=False)
    syn = SynthPath(bs, sr, reverb_length=48000).to(dev)
    spec = syn.reverb._spectrum(F * bs)
    L = syn.reverb.length
    sA = torch.cuda.current_stream(dev)
    sB = torch.cuda.Stream(dev)
    h = B // 2
    halves = [{k: v[i * h:(i + 1) * h] for k, v in inp.items()} for i in range(2)]

    def plain():
        return syn(inp["f0"], inp["param"], inp["mags"])

    def split():
        s0 = core.synth_frames(halves[0]["f0"], halves[0]["param"], halves[0]["mags"], bs, sr)
        ev = torch.cuda.Event()
        ev.record(sA)
        s1 = core.synth_frames(halves[1]["f0"], halves[1]["param"], halves[1]["mags"], bs, sr)
        with torch.cuda.stream(sB):
            sB.wait_event(ev)
            y0 = core.reverb_apply(s0, spec, L)
            s0.record_stream(sB)
            y0.record_stream(sA)
        y1 = core.reverb_apply(s1, spec, L)
        sA.wait_stream(sB)
        return y0, y1

    def timed(fn, n=100):
        t = time.perf_counter()
        while time.perf_counter() - t < 0.3:
            fn()
        torch.cuda.synchronize()
        res = []
        for _ in range(5):
            t0 = time.perf_counter()
            for _ in range(n):
                fn()
            torch.cuda.synchronize()
            res.append((time.perf_counter() - t0) / n * 1e6)
        return statistics.median(res)

    with torch.no_grad():
        y0, y1 = split()
        ref = plain()
        torch.cuda.synchronize()
        err = float((torch.cat([y0, y1]) - ref).abs().max())
        for _ in range(2):
            print(f"plain step {timed(plain):6.1f} us | split + overlap {timed(split):6.1f} us | max |diff| {err:.2e}",
                  flush=True)


if __name__ == "__main__":
    main()
