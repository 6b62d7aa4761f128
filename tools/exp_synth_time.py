"""Steady-state time of the fused synthesis kernel at config 2 (library chosen by DDSP_HIP_LIB):
A/B experiments on kernel variants.   python tools/exp_synth_time.py [H ...]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddsp_pytorch_amd import core  # noqa: E402
from ddsp_pytorch_amd.synth import make_inputs  # noqa: E402

B, F, bs, sr = 64, 200, 512, 48000
for H in [int(a) for a in sys.argv[1:]] or [100]:
    inp = make_inputs(B, F, H, 65, bs, device="cuda", with_noise=False)
    fn = lambda: core.synth_frames(inp["f0"], inp["param"], inp["mags"], bs, sr)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        fn()
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(200):
        fn()
    e1.record()
    torch.cuda.synchronize()
    print(f"{os.environ.get('DDSP_HIP_LIB', 'default')} H={H} synth_frames {e0.elapsed_time(e1) / 200 * 1e3:.1f} us", flush=True)
