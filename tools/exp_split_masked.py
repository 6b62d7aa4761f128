"""Within one step: does splitting the batch into chunks and overlapping reverb(chunk i) on a 64-CU
partition with synthesis(chunk i+1) on the other 192 CUs beat the one-stream step?  (The unmasked
form of this split measured slower in round 1, tools/exp_split_overlap.py.)  Schedule for C chunks:
synth(0) on all CUs; then for i = 1..C-1: synth(i) on 192 CUs beside reverb(i-1) on 64; then
reverb(C-1) on all CUs.  Development experiment.

    python tools/exp_split_masked.py [chunks ...]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddsp_pytorch_amd import core  # noqa: E402
from ddsp_pytorch_amd.synth import SynthPath, make_inputs  # noqa: E402

N = 60


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


def main():
    B, F, H, NB, bs = 64, 200, 100, 65, 512
    inp = make_inputs(B, F, H, NB, bs, seed=0, device="cuda", with_noise=False)
    syn = SynthPath(bs, 48000, reverb_length=48000).cuda()
    spec = syn.reverb._spectrum(F * bs)
    L = syn.reverb.length
    # the split runs on a non-default stream: the masked streams are blocking streams, so anything
    # recorded on the legacy default stream would serialise them
    main_s = torch.cuda.Stream()
    sa = core.cu_masked_stream(range(64, 256))
    sb = core.cu_masked_stream(range(64))
    print(f"one-stream step: {timed(lambda: syn(inp['f0'], inp['param'], inp['mags'])):6.1f} us", flush=True)

    def split(C):
        step = B // C
        sl = [slice(i * step, (i + 1) * step) for i in range(C)]
        sig = [None] * C
        ev = [None] * C
        out = []
        sig[0] = core.synth_frames(inp["f0"][sl[0]], inp["param"][sl[0]], inp["mags"][sl[0]], bs, 48000)
        for i in range(1, C):
            e0 = torch.cuda.Event()
            e0.record(main_s)
            sa.wait_event(e0)
            sb.wait_event(e0)
            with torch.cuda.stream(sa):
                sig[i] = core.synth_frames(inp["f0"][sl[i]], inp["param"][sl[i]], inp["mags"][sl[i]], bs, 48000)
                ev[i] = torch.cuda.Event()
                ev[i].record(sa)
            with torch.cuda.stream(sb):
                sig[i - 1].record_stream(sb)
                out.append(core.reverb_apply(sig[i - 1], spec, L))
                eb = torch.cuda.Event()
                eb.record(sb)
            main_s.wait_event(ev[i])
            main_s.wait_event(eb)
        out.append(core.reverb_apply(sig[C - 1], spec, L))
        return out

    with torch.cuda.stream(main_s):
        print(f"one-stream step on a side stream: {timed(lambda: syn(inp['f0'], inp['param'], inp['mags'])):6.1f} us",
              flush=True)
        for C in [int(a) for a in sys.argv[1:]] or [2, 4]:
            print(f"split into {C} chunks, masked overlap: {timed(lambda: split(C)):6.1f} us", flush=True)


if __name__ == "__main__":
    main()
