"""Does the fused synthesis kernel's slowdown after the reverb depend on how long the rest of the GPU
was quiet or memory-bound before it, rather than on which kernel ran?  (development experiment)

    DDSP_HIP_LIB=build/ab_rvfwd.so python tools/exp_gap.py
"""
import os
import statistics
import sys

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

    def per_launch(fn, between, n=120):
        ps, gs = [], []
        for _ in range(n):
            e0, e1, e2 = E(), E(), E()
            e0.record()
            fn()
            e1.record()
            between()
            e2.record()
            ps.append((e0, e1))
            gs.append((e1, e2))
        torch.cuda.synchronize()
        return (statistics.median(a.elapsed_time(b) * 1e3 for a, b in ps),
                statistics.median(a.elapsed_time(b) * 1e3 for a, b in gs))

    cases = [("nothing", lambda: None)]
    if "--reset" in sys.argv:
        tiny = torch.zeros(16, device="cuda")
        mid = torch.empty(64 << 20, dtype=torch.uint8, device="cuda")
        wide = torch.empty(256 * 512, device="cuda")
        cases += [("reverb", reverb),
                  ("reverb + tiny fill", lambda: (reverb(), tiny.fill_(1.0))),
                  ("reverb + 512-WG fill", lambda: (reverb(), wide.fill_(1.0))),
                  ("reverb + spin 20000", lambda: (reverb(), torch.cuda._sleep(20000))),
                  ("reverb + 64 MB fill", lambda: (reverb(), mid.fill_(1))),
                  ("reverb + harmonic_synth_params", lambda: (reverb(), core.harmonic_synth_params(inp["f0"], inp["param"], bs, sr)))]
        for name, between in cases:
            for _ in range(20):
                synth(); between()
            t, g = per_launch(synth, between)
            print(f"{name:32s}: synth {t:7.1f} us   gap {g:7.1f} us", flush=True)
        return
    for k in (1, 2, 3, 4):
        cases.append((f"reverb-variant x{k}", lambda k=k: [reverb() for _ in range(k)]))
    for cyc in (20000, 50000, 100000, 150000, 250000):
        cases.append((f"one-wave spin {cyc} cycles", lambda c=cyc: torch.cuda._sleep(c)))
    for name, between in cases:
        for _ in range(20):
            synth(); between()
        t, g = per_launch(synth, between)
        print(f"{name:32s}: synth {t:7.1f} us   gap {g:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
