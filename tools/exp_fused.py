"""Cost breakdown of the fused synthesis-frame kernel (development experiment):
time synth_frames over harmonic counts / band counts at config-2 batch shape."""
import sys, os, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddsp_pytorch_amd import core
from ddsp_pytorch_amd.synth import make_inputs


def t_ms(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


B, F, bs, sr = 64, 200, 512, 48000
res = {}
import time
_w = make_inputs(B, F, 100, 65, bs, device="cuda", with_noise=False)
_t = time.perf_counter()
while time.perf_counter() - _t < 0.5:  # clocks / power state settle
    core.synth_frames(_w["f0"], _w["param"], _w["mags"], bs, sr)
torch.cuda.synchronize()
for H in (1, 2, 25, 50, 100, 128):
    for NB in (2, 65):
        inp = make_inputs(B, F, H, NB, bs, device="cuda", with_noise=False)
        res[f"H{H}_NB{NB}"] = round(t_ms(lambda: core.synth_frames(inp["f0"], inp["param"], inp["mags"], bs, sr)), 4)
inp = make_inputs(B, F, 100, 65, bs, device="cuda", with_noise=False)
res["separate_harm"] = round(t_ms(lambda: core.harmonic_synth_params(inp["f0"], inp["param"], bs, sr)), 4)
res["separate_noise"] = round(t_ms(lambda: core.filtered_noise(inp["mags"], bs, raw_bias=-5.0)), 4)
print(json.dumps(res))
