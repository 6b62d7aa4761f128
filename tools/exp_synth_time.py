"""Time the fused synthesis kernel (core.synth_frames) at config 2 after the device has
settled: median of several event-timed groups (development experiment for launch-shape
variants selected through environment variables read by the library).

    python tools/exp_synth_time.py [batch frames harmonics]     (DDSP_AB_INJECT=1: injected noise;
                                                                 DDSP_AB_WHAT=reverb: the 1 s reverb)
"""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddsp_pytorch_amd import core  # noqa: E402
from ddsp_pytorch_amd.synth import make_inputs  # noqa: E402


def main():
    B, F, H = (int(a) for a in (sys.argv[1:4] if len(sys.argv) > 3 else (64, 200, 100)))
    NB, bs, sr = 65, 512, 48000
    inject = os.environ.get("DDSP_AB_INJECT") == "1"
    inp = make_inputs(B, F, H, NB, bs, device="cuda", with_noise=inject)
    run = lambda: core.synth_frames(inp["f0"], inp["param"], inp["mags"], bs, sr, noise=inp.get("noise"))
    if os.environ.get("DDSP_AB_WHAT") == "reverb":
        from ddsp_pytorch_amd.synth import SynthPath
        rv = SynthPath(bs, sr, reverb_length=48000).to("cuda").reverb
        sig = run()
        spec = rv._spectrum(F * bs)
        run = lambda: core.reverb_apply(sig, spec, rv.length)
    t = time.perf_counter()
    while time.perf_counter() - t < 0.5:
        run()
    torch.cuda.synchronize()
    groups = []
    for _ in range(7):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            run()
        e1.record()
        torch.cuda.synchronize()
        groups.append(e0.elapsed_time(e1) / 20)
    env = {k: v for k, v in os.environ.items() if k.startswith("DDSP_HIP_")}
    print(f"{env} B={B} F={F} H={H}: median {statistics.median(groups) * 1e3:.1f} us "
          f"(min {min(groups) * 1e3:.1f}, max {max(groups) * 1e3:.1f})", flush=True)


if __name__ == "__main__":
    main()
