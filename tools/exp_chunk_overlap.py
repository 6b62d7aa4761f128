"""Within one config-2 step, overlap the reverb of batch chunk i with the synthesis of chunk i+1 on two
unmasked HIP streams (the synthesis launches queue on the first, each chunk's reverb on the second after
an event), against the one-stream step — eager and as captured HIP graphs.  (Measurement only: the chunks
draw device noise from their own frame indices, so their audio differs from the one-launch step's.)

    python tools/exp_chunk_overlap.py
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
    dev = torch.device("cuda", 0)
    inp = make_inputs(B, F, H, NB, bs, device=dev, with_noise=False)
    path = SynthPath(bs, sr, reverb_length=48000).to(dev)
    rv = path.reverb
    s2 = torch.cuda.Stream(dev)

    def one_stream():
        return path(inp["f0"], inp["param"], inp["mags"])

    def chunked(n):
        step = B // n
        main = torch.cuda.current_stream(dev)
        outs = []
        for c in range(n):
            sl = slice(c * step, (c + 1) * step)
            sig = core.synth_frames(inp["f0"][sl], inp["param"][sl], inp["mags"][sl], bs, sr, bias=-5.0)
            s2.wait_stream(main)
            with torch.cuda.stream(s2):
                outs.append(rv(sig))
        main.wait_stream(s2)
        return outs

    runs = {"one_stream": one_stream, "chunks2": lambda: chunked(2), "chunks4": lambda: chunked(4)}
    res = {}
    with torch.no_grad():
        for name, fn in runs.items():
            t = time.perf_counter()
            while time.perf_counter() - t < 0.3:
                fn()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            side = torch.cuda.Stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                fn()
            torch.cuda.current_stream(dev).wait_stream(side)
            with torch.cuda.graph(g):
                fn()
            for mode, call in (("eager", fn), ("graph", g.replay)):
                ms = []
                for _ in range(5):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(50):
                        call()
                    e1.record()
                    torch.cuda.synchronize()
                    ms.append(e0.elapsed_time(e1) / 50)
                res[f"{name}_{mode}"] = round(statistics.median(ms) * 1e3, 1)
                print(f"{name:10s} {mode:5s} {res[f'{name}_{mode}']:7.1f} us per step (min {min(ms) * 1e3:.1f})",
                      flush=True)


if __name__ == "__main__":
    main()
