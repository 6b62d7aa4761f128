"""How does the fused synthesis kernel's measured time depend on what runs around it?  (development
experiment: back-to-back groups vs per-launch events vs the bench step's synth -> reverb order)

    python tools/exp_timing.py
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
    synth = lambda: core.synth_frames(inp["f0"], inp["param"], inp["mags"], bs, sr)
    sig = synth()
    spec = syn.reverb._spectrum(F * bs)
    reverb = lambda: core.reverb_apply(sig, spec, 48000)
    E = lambda: torch.cuda.Event(enable_timing=True)

    def settle(fn, s=0.5):
        t = time.perf_counter()
        while time.perf_counter() - t < s:
            fn()
        torch.cuda.synchronize()

    def group(fn, n=20, reps=7):
        out = []
        for _ in range(reps):
            e0, e1 = E(), E()
            e0.record()
            for _ in range(n):
                fn()
            e1.record()
            torch.cuda.synchronize()
            out.append(e0.elapsed_time(e1) / n * 1e3)
        return statistics.median(out)

    def per_launch(fn, between=None, n=140):
        ps = []
        for _ in range(n):
            e0, e1 = E(), E()
            e0.record()
            fn()
            e1.record()
            ps.append((e0, e1))
            if between:
                between()
        torch.cuda.synchronize()
        return statistics.median(a.elapsed_time(b) * 1e3 for a, b in ps)

    settle(synth)
    print(f"A synth back-to-back, group events      : {group(synth):7.1f} us", flush=True)
    print(f"B synth, events around each launch      : {per_launch(synth):7.1f} us", flush=True)
    settle(lambda: (synth(), reverb()))
    print(f"C synth then reverb, events around synth: {per_launch(synth, reverb):7.1f} us", flush=True)
    if "--short" in sys.argv:
        print(f"E synth+reverb step group               : {group(lambda: (synth(), reverb())):7.1f} us", flush=True)
        return
    print(f"D reverb group                          : {group(reverb):7.1f} us", flush=True)
    print(f"E synth+reverb step group               : {group(lambda: (synth(), reverb())):7.1f} us", flush=True)
    def synced():
        torch.cuda.synchronize()
    print(f"F synth, host sync between launches     : {per_launch(synth, synced):7.1f} us", flush=True)
    settle(synth)
    print(f"G synth back-to-back again (settled)    : {group(synth):7.1f} us", flush=True)
    tiny = torch.zeros(16, device="cuda")
    print(f"H synth, a tiny fill kernel between     : {per_launch(synth, lambda: tiny.fill_(1.0)):7.1f} us", flush=True)
    harm = lambda: core.harmonic_synth_params(inp["f0"], inp["param"], bs, sr)
    print(f"I synth, harmonic_synth_params between  : {per_launch(synth, harm):7.1f} us", flush=True)
    print(f"J harmonic_synth_params back-to-back    : {group(harm):7.1f} us", flush=True)
    print(f"K harmonic_synth_params after synth     : {per_launch(harm, synth):7.1f} us", flush=True)
    half = {k: v[:, :100].contiguous() for k, v in inp.items()}
    synth_h = lambda: core.synth_frames(half["f0"], half["param"], half["mags"], bs, sr)
    settle(synth_h)
    print(f"L synth F=100 back-to-back              : {group(synth_h):7.1f} us", flush=True)
    print(f"M synth F=100, reverb between           : {per_launch(synth_h, reverb):7.1f} us", flush=True)
    quarter = {k: v[:16].contiguous() for k, v in inp.items()}
    synth_q = lambda: core.synth_frames(quarter["f0"], quarter["param"], quarter["mags"], bs, sr)
    settle(synth_q)
    print(f"N synth B=16 back-to-back               : {group(synth_q):7.1f} us", flush=True)
    print(f"O synth B=16, reverb between            : {per_launch(synth_q, reverb):7.1f} us", flush=True)


if __name__ == "__main__":
    main()
