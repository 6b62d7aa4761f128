"""Why is synth.PipelinedSynthPath slower than the inline two-stream loop of tools/exp_cumask.py?
Times, at config 2: the one-stream step, the inline pipelined loop, and PipelinedSynthPath with
its per-call extras switched off one at a time (development experiment).

    python tools/exp_pipeline_leg.py
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddsp_pytorch_amd import core  # noqa: E402
from ddsp_pytorch_amd.synth import PipelinedSynthPath, SynthGraph, SynthPath, make_inputs  # noqa: E402

N = 100


def timed(fn, join=None):
    for _ in range(10):
        fn()
    if join:
        join()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(N):
        fn()
    if join:
        join()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / N * 1e6


def main():
    B, F, H, NB, bs = 64, 200, 100, 65, 512
    inp = make_inputs(B, F, H, NB, bs, seed=0, device="cuda", with_noise=False)
    syn = SynthPath(bs, 48000, reverb_length=48000).cuda()
    args = (inp["f0"], inp["param"], inp["mags"], None)
    print(f"one stream: {timed(lambda: syn(*args)):6.1f} us", flush=True)
    pipe = PipelinedSynthPath(syn)
    cur = torch.cuda.current_stream()
    print("current is default:", cur == torch.cuda.default_stream(cur.device), cur, flush=True)
    print(f"PipelinedSynthPath: {timed(lambda: pipe(*args), pipe.join):6.1f} us", flush=True)
    sa, sb = pipe.s_synth, pipe.s_reverb
    spec = syn.reverb._spectrum(F * bs)

    def inline(use_module):
        with torch.cuda.stream(sa):
            x = syn.synthesize(*args)
            e = torch.cuda.Event()
            e.record(sa)
        with torch.cuda.stream(sb):
            sb.wait_event(e)
            x.record_stream(sb)
            if use_module:
                syn.reverb(x)
            else:
                core.reverb_apply(x, spec, syn.reverb.length)

    print(f"inline, reverb_apply: {timed(lambda: inline(False)):6.1f} us", flush=True)
    print(f"inline, Reverb module: {timed(lambda: inline(True)):6.1f} us", flush=True)
    print(f"PipelinedSynthPath again: {timed(lambda: pipe(*args), pipe.join):6.1f} us", flush=True)
    g = SynthGraph(syn, inp["f0"], inp["param"], inp["mags"])
    print(f"one stream, HIP graph replay: {timed(g.replay):6.1f} us", flush=True)
    cur = torch.cuda.current_stream()
    print("current is default:", cur == torch.cuda.default_stream(cur.device), cur, flush=True)
    print(f"PipelinedSynthPath after the graph: {timed(lambda: pipe(*args), pipe.join):6.1f} us", flush=True)
    print(f"one stream again: {timed(lambda: syn(*args)):6.1f} us", flush=True)


if __name__ == "__main__":
    main()
