"""Why does the fused synthesis kernel run ~13 % slower after the reverb than back to back?  Cache-state
experiments (development): the kernel after kernels that leave L2 / the MALL in different states.

    python tools/exp_cache.py
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
    synth = lambda **kw: core.synth_frames(inp["f0"], inp["param"], inp["mags"], bs, sr, **kw)
    sig = synth()
    spec = syn.reverb._spectrum(F * bs)
    reverb = lambda: core.reverb_apply(sig, spec, 48000)
    big = torch.empty(300 * 2 ** 20 // 4, device="cuda")
    big.fill_(1.0)
    E = lambda: torch.cuda.Event(enable_timing=True)
    keep = []

    def per_launch(fn, between=None, n=60):
        t = time.perf_counter()
        while time.perf_counter() - t < 0.3:
            fn()
            if between:
                between()
        torch.cuda.synchronize()
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
        keep.clear()
        return statistics.median(a.elapsed_time(b) * 1e3 for a, b in ps)

    cases = [
        ("back to back (output block reused)", synth, None),
        ("back to back, a fresh output block each launch", lambda: keep.append(synth()), None),
        ("back to back, parts (3 outputs)", lambda: synth(parts=True), None),
        ("after the reverb", synth, reverb),
        ("after reading 300 MB (clean lines)", synth, lambda: big.sum()),
        ("after writing 300 MB (dirty lines)", synth, lambda: big.fill_(2.0)),
        ("after writing 16 MB (dirty lines)", synth, lambda: big[: 4 * 2 ** 20].fill_(3.0)),
        ("after reading the 8.5 MB of controls", synth, lambda: (inp["param"].sum(), inp["mags"].sum())),
        ("after the reverb, then reading the controls", synth,
         lambda: (reverb(), inp["param"].sum(), inp["mags"].sum())),
    ]
    if "--short" in sys.argv:
        cases = [cases[0], cases[3]]
    for name, fn, between in cases:
        print(f"{name:48s}: {per_launch(fn, between):7.1f} us", flush=True)


if __name__ == "__main__":
    main()
