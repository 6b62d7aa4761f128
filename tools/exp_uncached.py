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


def t_fn(fn, reps=200):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t0) / reps * 1e3, 4)


mode = sys.argv[1] if len(sys.argv) > 1 else "both"  # cached | uncached | both | order
if mode == "order":  # where the rebuild goes in the step: after the synthesis (as Reverb.forward does) or before
    from ddsp_pytorch_amd.modules import Reverb
    T = 200 * 512

    def after():
        with torch.no_grad():
            syn.reverb.decay.add_(0.0)  # a version bump: the forward rebuilds
        return step()

    def before():
        with torch.no_grad():
            syn.reverb.decay.add_(0.0)
            Reverb._spectrum(syn.reverb, T)  # rebuilt ahead of the synthesis launch
        return step()

    print(json.dumps({"rebuild_after_synth_ms": t_fn(after), "rebuild_before_synth_ms": t_fn(before),
                      "rebuild_after_synth_ms_2": t_fn(after), "rebuild_before_synth_ms_2": t_fn(before),
                      "cached_ms": t()}), flush=True)
    sys.exit(0)
res = {}
if mode in ("cached", "both"):
    res["cached_ms"] = t()
if mode in ("uncached", "both"):
    syn.reverb.cache_spectrum = False
    res["uncached_ms"] = t()
    syn.reverb.cache_spectrum = True
if mode == "both":
    res["cached_again_ms"] = t()
print(json.dumps(res), flush=True)
