"""Does running the reverb of batch chunk i beside the synthesis of chunk i+1 (two HIP streams)
shorten the config-2 step?  The synthesis kernel is VALU-bound, the reverb kernels are
HBM/LDS-latency-bound, so their workgroups can share CUs.

    python tools/exp_overlap.py [chunks ...]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddsp_pytorch_amd import core  # noqa: E402
from ddsp_pytorch_amd.synth import SynthPath, make_inputs  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    B, F, H, NB, bs = 64, 200, 100, 65, 512
    inp = make_inputs(B, F, H, NB, bs, seed=0, device=dev, with_noise=False)
    f0, param, mags = inp["f0"], inp["param"], inp["mags"]
    syn = SynthPath(bs, 48000, reverb_length=48000).to(dev)
    L = syn.reverb.length
    spec = syn.reverb._spectrum(F * bs)
    sA = torch.cuda.current_stream(dev)
    sB = torch.cuda.Stream(dev)

    def step(chunks):
        if chunks == 1:
            return syn(f0, param, mags)
        if chunks == 0:  # inter-step pipeline: reverb(i) on sB beside synth(i+1) on sA
            sig = core.synth_frames(f0, param, mags, bs, 48000)
            ev = torch.cuda.Event()
            ev.record(sA)
            with torch.cuda.stream(sB):
                sB.wait_event(ev)
                y = core.reverb_apply(sig, spec, L)
                sig.record_stream(sB)
            return y
        out = torch.empty(B, F * bs, 1, device=dev)
        cb = (B + chunks - 1) // chunks
        for c0 in range(0, B, cb):
            c1 = min(B, c0 + cb)
            sig = core.synth_frames(f0[c0:c1], param[c0:c1], mags[c0:c1], bs, 48000)
            ev = torch.cuda.Event()
            ev.record(sA)
            with torch.cuda.stream(sB):
                sB.wait_event(ev)
                y = core.reverb_apply(sig, spec, L)
                sig.record_stream(sB)
                y.record_stream(sB)
        ev = torch.cuda.Event()
        ev.record(sB)
        sA.wait_event(ev)
        return out

    with torch.no_grad():
        for chunks in (int(a) for a in (sys.argv[1:] or [1, 2, 4, 8])):
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < 0.3:
                step(chunks)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            t0 = time.perf_counter()
            for _ in range(50):
                step(chunks)
            cpu_us = (time.perf_counter() - t0) / 50 * 1e6
            if chunks == 0:
                ev = torch.cuda.Event()
                ev.record(sB)
                sA.wait_event(ev)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 50
            print(f"chunks={chunks} step {ms * 1e3:7.1f} us  {B * F * bs / ms / 1e6:6.2f} G samples/s"
                  f"  (host enqueue {cpu_us:6.1f} us/step)", flush=True)


if __name__ == "__main__":
    main()
