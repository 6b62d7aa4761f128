"""Do the VALU-bound synthesis kernel and the HBM/LDS-bound reverb kernels overlap when they run
on two HIP streams at once?  Independent inputs (no dependency between the streams), N launches
enqueued per stream, device time of each alone and both together (development experiment).

    python tools/exp_concurrency.py [batch]
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
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    F, H, NB, bs, N = 200, 100, 65, 512, 50
    inp = make_inputs(B, F, H, NB, bs, seed=0, device=dev, with_noise=False)
    syn = SynthPath(bs, 48000, reverb_length=48000).to(dev)
    L = syn.reverb.length
    spec = syn.reverb._spectrum(F * bs)
    sig = core.synth_frames(inp["f0"], inp["param"], inp["mags"], bs, 48000)
    sA, sB = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def synth():
        core.synth_frames(inp["f0"], inp["param"], inp["mags"], bs, 48000)

    def reverb():
        core.reverb_apply(sig, spec, L)

    def timed(fn_a, fn_b):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if fn_a:
            with torch.cuda.stream(sA):
                for _ in range(N):
                    fn_a()
        if fn_b:
            with torch.cuda.stream(sB):
                for _ in range(N):
                    fn_b()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / N * 1e6

    t = time.perf_counter()
    while time.perf_counter() - t < 0.5:
        synth()
        reverb()
    for rep in range(2):
        ts, tr, tb = timed(synth, None), timed(None, reverb), timed(synth, reverb)
        print(f"batch {B}: synth alone {ts:6.1f} us, reverb alone {tr:6.1f} us, sum {ts + tr:6.1f}, "
              f"both on two streams {tb:6.1f} us per pair", flush=True)


if __name__ == "__main__":
    main()
