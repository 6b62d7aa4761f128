"""Pin the oracle's gradients to the reference's own autograd (tests/golden/g6_*.npz, written by
make_goldens.py running hugofloresgarcia/ddsp_pytorch with loss = sum(signal * w)).

oracle/torch_ref.py re-issues the reference's ATen op sequence, so its autograd must give the
reference's gradients; it is then the checker for the gfx950 backward kernels
(tests/test_gpu_grad.py)."""
import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import torch_ref as tr

T = torch.from_numpy


def relerr(a, b):
    a = torch.as_tensor(a, dtype=torch.float64)
    b = torch.as_tensor(b, dtype=torch.float64)
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.mark.parametrize("tag", ["small", "crop"])
def test_reverb_grad(tag):
    g = load_golden(f"g6_grad_reverb_{tag}")
    noise, decay, wet = (T(g[k]).clone().requires_grad_(True) for k in ("noise", "decay", "wet"))
    rv = tr.Reverb(noise, decay, wet, int(g["length"]), int(g["sample_rate"]))
    x = T(g["x"]).clone().requires_grad_(True)
    out = rv(x)
    assert torch.equal(out.detach(), T(g["out"]))
    (out * T(g["weight"])).sum().backward()
    for name, t in (("grad_x", x), ("grad_noise", noise), ("grad_decay", decay), ("grad_wet", wet)):
        assert relerr(t.grad, g[name]) < 1e-6, (name, relerr(t.grad, g[name]))


def test_decoder_synth_grad():
    """Gradients of the synthesis section w.r.t. its inputs (the harmonic and noise projections)
    and the reverb parameters, from the reference's full DDSPDecoder backward."""
    g = load_golden("g6_grad_decoder")
    bs, sr = int(g["block_size"]), int(g["sample_rate"])
    f0 = T(g["pitch"])
    param = T(g["param"]).clone().requires_grad_(True)
    mags = T(g["mags"]).clone().requires_grad_(True)
    B, F = param.shape[0], param.shape[1]
    noise, decay, wet = (T(g["sd.reverb." + k]).clone().requires_grad_(True) for k in ("noise", "decay", "wet"))
    rv = tr.Reverb(noise, decay, wet, noise.shape[0], sr)
    torch.manual_seed(123)
    nz = torch.rand(B, F, bs) * 2 - 1
    sig = tr.synth_path_autograd(f0, param, mags, nz, rv, bs, sr)
    assert torch.equal(sig.detach(), T(g["signal"]))
    (sig * T(g["weight"])).sum().backward()
    assert relerr(param.grad, g["grad_param"]) < 1e-6, relerr(param.grad, g["grad_param"])
    assert relerr(mags.grad, g["grad_mags"]) < 1e-6, relerr(mags.grad, g["grad_mags"])
    for k, t in (("noise", noise), ("decay", decay), ("wet", wet)):
        assert relerr(t.grad, g["grad.reverb." + k]) < 1e-6, (k, relerr(t.grad, g["grad.reverb." + k]))


def test_stft_loss_oracle():
    """The oracle's multiscale STFT loss and its gradient reproduce the reference's (g7)."""
    g = load_golden("g7_stft_loss")
    scales, overlap = [int(s) for s in g["scales"]], float(g["overlap"])
    rec = T(g["rec"]).clone().requires_grad_(True)
    ori = tr.multiscale_fft(T(g["sig"]), scales, overlap)
    rs = tr.multiscale_fft(rec, scales, overlap)
    for s, m in zip(scales, rs):
        assert torch.equal(m.detach(), T(g[f"stft_{s}"]))
    loss = tr.multiscale_spec_loss(ori, rs)
    assert torch.equal(loss.detach(), T(g["loss"]))
    loss.backward()
    assert relerr(rec.grad, g["grad_rec"]) < 1e-6


def test_masked_stft_loss_oracle():
    """The oracle reproduces the reference's masked-loss gradient (g7b: train.py's loss on the
    well-conditioned bins, tests/golden/make_goldens.py masked_loss_golden) bit for bit."""
    g = load_golden("g7_stft_loss")
    gb = load_golden("g7b_stft_loss_masked")
    scales, overlap = [int(s) for s in g["scales"]], float(g["overlap"])
    rec = T(g["rec"]).clone().requires_grad_(True)
    ori = tr.multiscale_fft(T(g["sig"]), scales, overlap)
    rs = tr.multiscale_fft(rec, scales, overlap)
    loss = 0
    for s, mx, my in zip(scales, ori, rs):
        m = T(gb[f"mask_{s}"]).float()
        loss = loss + (m * (mx - my).abs()).mean() + (m * (tr.safe_log(mx) - tr.safe_log(my)).abs()).mean()
    assert torch.equal(loss.detach(), T(gb["loss"]))
    loss.backward()
    assert torch.equal(rec.grad, T(gb["grad_rec"]))
