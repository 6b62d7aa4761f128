"""Is the eager bench step host-bound?  Host enqueue time vs GPU time per step, the fused kernel's
event time with the queue kept ahead of the GPU, and the captured-graph step.  (development experiment)

    python tools/exp_host.py
"""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddsp_pytorch_amd import core  # noqa: E402
from ddsp_pytorch_amd.synth import SynthGraph, SynthPath, make_inputs  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import EventTimer  # noqa: E402


def main():
    B, F, H, NB, bs, sr = 64, 200, 100, 65, 512, 48000
    inp = make_inputs(B, F, H, NB, bs, device="cuda", with_noise=False)
    syn = SynthPath(bs, sr, reverb_length=48000).to("cuda")
    step = lambda: syn(inp["f0"], inp["param"], inp["mags"])
    n = 200

    def loop(fn, head_start_cycles=0):
        torch.cuda.synchronize()
        if head_start_cycles:
            torch.cuda._sleep(head_start_cycles)  # one wave spins: the host gets ahead of the GPU
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        t1 = time.perf_counter()
        e1.record()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        return (t1 - t0) / n * 1e6, (t2 - t0) / n * 1e6, e0.elapsed_time(e1) / n * 1e3

    for _ in range(300):
        step()
    for name, head in (("eager step", 0), ("eager step, host 100 ms ahead", 250_000_000)):
        for timed in (False, True):
            timer = EventTimer(["synth_frames"])
            timer.enabled = timed
            syn.timer = timer
            enq, wall, gpu = loop(step, head)
            extra = f"   synth event mean {timer.mean_ms('synth_frames') * 1e3:6.1f} us" if timed else ""
            print(f"{name:32s} events={timed!s:5s}: host enqueue {enq:6.1f} us/step, wall {wall:6.1f}, "
                  f"GPU span {gpu:6.1f}{extra}", flush=True)
    syn.timer = None
    for name, fn in (("core.synth_frames alone", lambda: core.synth_frames(inp["f0"], inp["param"], inp["mags"], bs, sr)),
                     ("reverb alone", lambda: syn.reverb(inp["f0"].new_zeros(B, F * bs, 1)))):
        enq, wall, gpu = loop(fn)
        print(f"{name:32s}: host enqueue {enq:6.1f} us/call, wall {wall:6.1f}, GPU span {gpu:6.1f}", flush=True)
    g = SynthGraph(syn, inp["f0"], inp["param"], inp["mags"])
    for _ in range(50):
        g.replay()
    enq, wall, gpu = loop(g.replay)
    print(f"{'graph replay':32s}: host enqueue {enq:6.1f} us/step, wall {wall:6.1f}, GPU span {gpu:6.1f}", flush=True)


if __name__ == "__main__":
    main()
