"""Development experiment: host (CPU) cost of bench.py's train_step pieces at config 2 — each piece
called after a device synchronize — against their device time (HIP events)."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddsp_pytorch_amd import core
from ddsp_pytorch_amd.modules import Reverb
from ddsp_pytorch_amd.synth import make_inputs

dev = "cuda"
B, F, H, NB, bs, sr = 64, 200, 100, 65, 512, 48000
inp = make_inputs(B, F, H, NB, bs, seed=0, device=dev, with_noise=False)
torch.manual_seed(1)
rv = Reverb(48000, sr).to(dev)
param = inp["param"].clone().requires_grad_(True)
mags = inp["mags"].clone().requires_grad_(True)
w = torch.randn(B, F * bs, 1, device=dev)
res = {}


def measure(name, fn, reps=50, setup=None):
    host = 0.0
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    devt = 0.0
    for i in range(reps + 5):
        if setup is not None:
            setup()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        a.record()
        fn()
        b.record()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        if i >= 5:
            host += t1 - t0
            devt += a.elapsed_time(b) * 1e-3
    res[name] = {"host_us": round(host / reps * 1e6, 1), "device_us": round(devt / reps * 1e6, 1)}


state = {}


def fwd_synth():
    state["sig"] = core.synth_frames(inp["f0"], param, mags, bs, sr)


def fwd_rev():
    state["out"] = rv(state["sig"])


def bwd():
    state["out"].backward(w)


def zero():
    param.grad = mags.grad = None
    for p_ in rv.parameters():
        p_.grad = None


for _ in range(3):
    zero(); fwd_synth(); fwd_rev(); bwd()
measure("zero_grads", zero)
measure("synth_frames_fwd", fwd_synth)
measure("reverb_fwd", fwd_rev, setup=fwd_synth)
measure("backward", bwd, setup=lambda: (zero(), fwd_synth(), fwd_rev()))
print(json.dumps(res), flush=True)
