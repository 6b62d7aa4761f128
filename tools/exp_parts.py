"""Fused synthesis at config 2 in the decoder's form (parts + control dicts) and the step's (signal only):
ms per launch over 100 back-to-back launches, event-timed.  For library A/Bs (DDSP_HIP_LIB, tools/ab_time.sh)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddsp_pytorch_amd import core  # noqa: E402
from ddsp_pytorch_amd.synth import make_inputs  # noqa: E402

dev = torch.device("cuda", 0)
inp = make_inputs(64, 200, 100, 65, 512, seed=0, device=dev, with_noise=False)


def timed(fn, reps=100):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


with torch.no_grad():
    for _ in range(400):  # ~50 ms of launches: a cold MI355X runs the first launches ~10 % slower
        core.synth_frames(inp["f0"], inp["param"], inp["mags"], 512, 48000)
    torch.cuda.synchronize()
    res = {}
    for parts in (False, True):
        for controls in (False, True):
            res[f"parts={parts} controls={controls}"] = round(timed(
                lambda: core.synth_frames(inp["f0"], inp["param"], inp["mags"], 512, 48000, parts=parts,
                                          controls=controls)), 4)
print(res)
