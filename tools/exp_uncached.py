"""Development experiment: bench.py's step at config 2 with the reverb IR cached and rebuilt every call
(Reverb.cache_spectrum = False), host-timed over 200 steps after warmup.  (Round 4's r04n run also timed
a side-stream prefetch of the rebuild, since removed: profiles/r04n_uncached.log.)"""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddsp_pytorch_amd.synth import SynthPath, make_inputs

dev = "cuda"
syn = SynthPath(512, 48000, reverb_length=48000, noise_mode="device").to(dev)
inp = make_inputs(64, 200, 100, 65, 512, seed=0, device=dev, with_noise=False)


def step():
    with torch.no_grad():
        return syn(inp["f0"], inp["param"], inp["mags"], inp.get("noise"))


def t(reps=200):
    for _ in range(20):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        step()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t0) / reps * 1e3, 4)


res = {"cached_ms": t()}
syn.reverb.cache_spectrum = False
res["uncached_ms"] = t()
syn.reverb.cache_spectrum = True
res["cached_again_ms"] = t()
print(json.dumps(res), flush=True)
