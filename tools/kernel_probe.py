"""Run one kernel of the synthesis path repeatedly at configuration 2 (for rocprofv3 PMC passes).

    python tools/kernel_probe.py {fused,bwd,reverb_bwd,gru,gru_train,harmonic,harmonic_frames,noise,reverb,op} [reps]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddsp_pytorch_amd import core  # noqa: E402
from ddsp_pytorch_amd.synth import SynthPath, make_inputs  # noqa: E402


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "harmonic"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda", 0)
    B, F, H, NB, bs, sr = 64, 200, 100, 65, 512, 48000
    inp = make_inputs(B, F, H, NB, bs, seed=0, device=dev, with_noise=False)
    syn = SynthPath(bs, sr, reverb_length=48000).to(dev)
    if which == "bwd":  # the fused synthesis backward (frame_backward_kernel<2, 2, true>)
        param = inp["param"].clone().requires_grad_(True)
        mags = inp["mags"].clone().requires_grad_(True)
        out = core.synth_frames(inp["f0"], param, mags, bs, sr)
        g = torch.randn_like(out)
        for _ in range(reps):
            out.backward(g, retain_graph=True)
        torch.cuda.synchronize()
        return
    if which in ("proj", "mlp"):  # the decoder's projections (one launch) / one 512-wide MLP block
        torch.manual_seed(0)
        h = torch.randn(B * F, 512, device=dev)
        l1, l2 = torch.nn.Linear(512, H + 1).to(dev), torch.nn.Linear(512, NB).to(dev)
        lin, ln, act = torch.nn.Linear(512, 512).to(dev), torch.nn.LayerNorm(512).to(dev), torch.nn.LeakyReLU()
        with torch.no_grad():
            for _ in range(reps):
                if which == "proj":
                    core.projections(h, l1, l2)
                else:
                    core.mlp_block(h, lin, ln, act)
        torch.cuda.synchronize()
        return
    if which == "gru":  # the decoder's GRU recurrence (B=64, T=200, hidden 512): step kernels
        torch.manual_seed(0)
        g = torch.nn.GRU(1024, 512, batch_first=True).to(dev)
        xg = torch.randn(B, F, 1024, device=dev)
        with torch.no_grad():
            for _ in range(reps):
                core.gru(xg, g)
        torch.cuda.synchronize()
        return
    if which == "gru_train":  # the same recurrence under autograd: forward step kernels + BPTT step kernels
        torch.manual_seed(0)
        g = torch.nn.GRU(1024, 512, batch_first=True).to(dev)
        xg = torch.randn(B, F, 1024, device=dev, requires_grad=True)
        for _ in range(reps):
            out, _h = core.gru(xg, g)
            out.sum().backward()
        torch.cuda.synchronize()
        return
    if which == "reverb_bwd":  # the UPOLS backward (input and IR gradients)
        x = torch.randn(B, F * bs, 1, device=dev, requires_grad=True)
        g = torch.randn(B, F * bs, 1, device=dev)
        for _ in range(reps):  # forward each time: the backward releases the kept input spectra
            syn.reverb(x).backward(g)
        torch.cuda.synchronize()
        return
    with torch.no_grad():
        amps, dist = core.harmonic_controls(inp["param"][..., :1], inp["param"][..., 1:], inp["f0"], sr)
        x = torch.randn(B, F * bs, 1, device=dev)
        if which == "op":
            f0s = core.upsample(inp["f0"], bs)
            a = core.upsample(dist, bs)
        for _ in range(reps):
            if which == "fused":
                core.synth_frames(inp["f0"], inp["param"], inp["mags"], bs, sr)
            elif which == "harmonic":
                core.harmonic_synth_params(inp["f0"], inp["param"], bs, sr)
            elif which == "harmonic_frames":
                core.harmonic_synth_frames(inp["f0"], amps, dist, bs, sr, write_back=False)
            elif which == "noise":
                core.filtered_noise(inp["mags"], bs, add=x, raw_bias=-5.0)
            elif which == "reverb":
                syn.reverb(x)
            elif which == "op":
                core.harmonic_synth(f0s, a, sr)
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
