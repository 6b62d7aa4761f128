"""Bit-identity of two C-ABI library builds on the fused synthesis kernel (development check for
changes that must not move a bit, e.g. a different FIR schedule):

    DDSP_HIP_LIB=build/ab_<a>.so python tools/exp_bits.py save <a>
    DDSP_HIP_LIB=build/ab_<b>.so python tools/exp_bits.py save <b>
    python tools/exp_bits.py compare <a> <b>

`save` renders config 2 with device noise and with injected noise (signal, harmonic and noise parts),
plus the controls form, to gpurun_out/bits_<name>.pt; `compare` prints the number of differing
elements and the largest difference per tensor.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def save(name):
    from ddsp_pytorch_amd import core
    from ddsp_pytorch_amd.synth import make_inputs
    out = {}
    for B, F, H, bs in ((64, 200, 100, 512), (4, 40, 128, 512), (8, 80, 64, 256), (2, 24, 64, 256)):
        inp = make_inputs(B, F, H, 65, bs, device="cuda", with_noise=True)
        key = f"{B}x{F}x{H}x{bs}"
        out[key + "_device"] = core.synth_frames(inp["f0"], inp["param"], inp["mags"], bs, 48000).cpu()
        parts = core.synth_frames(inp["f0"], inp["param"], inp["mags"], bs, 48000, noise=inp["noise"],
                                  parts=True, controls=True)
        for i, p in enumerate(parts):
            for j, t in enumerate(p.values() if isinstance(p, dict) else (p,)):
                out[f"{key}_inject{i}_{j}"] = t.cpu()
    # the reverb (forward transform + IR cache, MAC, inverse) and its backward (modules.Reverb under autograd)
    from ddsp_pytorch_amd.synth import SynthPath
    from ddsp_pytorch_amd.modules import Reverb
    inp = make_inputs(64, 200, 100, 65, 512, device="cuda", with_noise=True)
    path = SynthPath(512, 48000, reverb_length=48000).to("cuda")
    out["reverb_path"] = path(inp["f0"], inp["param"], inp["mags"]).cpu()
    torch.manual_seed(1)
    rv = Reverb(48000, 48000).to("cuda")
    x = (torch.randn(6, 40000, 1, device="cuda") * 0.3).requires_grad_(True)
    y = rv(x)
    y.backward(torch.randn_like(y))
    out["reverb_y"], out["reverb_dx"] = y.detach().cpu(), x.grad.cpu()
    out["reverb_dnoise"] = rv.noise.grad.cpu()
    os.makedirs("gpurun_out", exist_ok=True)
    torch.save(out, f"gpurun_out/bits_{name}.pt")
    print("saved", name, len(out), "tensors")


def compare(a, b):
    A = torch.load(f"gpurun_out/bits_{a}.pt", weights_only=True)
    B = torch.load(f"gpurun_out/bits_{b}.pt", weights_only=True)
    bad = 0
    for k in A:
        d = (A[k] - B[k]).abs()
        n = int((A[k] != B[k]).sum())
        bad += n
        print(f"{k:28s} differing {n:9d}  max |diff| {float(d.max()):.3e}")
    print("BIT-IDENTICAL" if bad == 0 else f"DIFFERENT ({bad} elements)")


if __name__ == "__main__":
    if sys.argv[1] == "save":
        save(sys.argv[2])
    else:
        compare(sys.argv[2], sys.argv[3])
