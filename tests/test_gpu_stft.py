"""Multiscale STFT magnitudes and the training loss on gfx950 kernels,
against torch.stft on the CPU (the reference's own call, ddsp/core.py:27-41) and the reference's
golden loss and gradient (g7, tests/golden/make_goldens.py).

Tolerances: spectrogram relative L2 error <= 1e-5 (fp32 FFTs of different structure);
gradient of sum(M * W) <= 2e-5; the loss value <= 1e-5; the loss gradient <= 1e-3 on the golden's
small case and <= 1e-4 for the squared linear-magnitude form at config 2's length (see the last test
for why the L1 / log form's gradient is not a well-conditioned comparison there).
"""
import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import torch_ref as tr

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dd():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import ddsp_pytorch_amd
    ddsp_pytorch_amd._lib.load()
    return ddsp_pytorch_amd


def relerr(a, b):
    a = torch.as_tensor(a).detach().double().cpu()
    b = torch.as_tensor(b).detach().double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def ref_stft(x, n, hop):
    return torch.stft(x, n, hop, n, torch.hann_window(n), True, normalized=True, return_complex=True).abs()


@pytest.mark.parametrize("n", [16, 32, 64, 128, 256, 512, 1024, 2048, 4096])
@pytest.mark.parametrize("T,hop_div", [(10000, 4), (9001, 4), (5000, 2), (4097, 8)])
def test_stft_magnitude(dd, n, T, hop_div):
    if n // 2 >= T:
        pytest.skip("reflect padding needs T > n/2")
    hop = max(1, n // hop_div)
    x = torch.randn(3, T, generator=torch.Generator().manual_seed(n + T)) * 0.3
    ref = ref_stft(x, n, hop)
    got = dd.core.stft_magnitude(x.cuda(), n, hop)
    assert got.shape == ref.shape
    assert relerr(got, ref) < 1e-5, relerr(got, ref)


@pytest.mark.parametrize("n,T", [(16, 12000), (128, 12000), (512, 12000), (1024, 12000), (4096, 12000),
                                 (128, 102400), (4096, 102400)])
def test_stft_magnitude_grad(dd, n, T):
    hop = n // 4
    g = torch.Generator().manual_seed(n)
    x = torch.randn(2, T, generator=g) * 0.3
    ref_m = ref_stft(x, n, hop)
    W = torch.randn(ref_m.shape, generator=g)
    xc = x.clone().requires_grad_(True)
    (ref_stft(xc, n, hop) * W).sum().backward()
    xg = x.cuda().requires_grad_(True)
    (dd.core.stft_magnitude(xg, n, hop) * W.cuda()).sum().backward()
    assert relerr(xg.grad, xc.grad) < 2e-5, relerr(xg.grad, xc.grad)


def test_spectral_loss_golden(dd):
    g = load_golden("g7_stft_loss")
    scales, overlap = [int(s) for s in g["scales"]], float(g["overlap"])
    from ddsp_pytorch_amd import loss as L
    rec = torch.as_tensor(g["rec"]).cuda().requires_grad_(True)
    sig = torch.as_tensor(g["sig"]).cuda()
    rs = dd.core.multiscale_fft(rec, scales, overlap)
    for s, m in zip(scales, rs):
        assert relerr(m, g[f"stft_{s}"]) < 1e-5, (s, relerr(m, g[f"stft_{s}"]))
    val = L.multiscale_spec_loss(dd.core.multiscale_fft(sig, scales, overlap), rs)
    assert relerr(val, g["loss"]) < 1e-5, (float(val), float(g["loss"]))
    val.backward()
    assert relerr(rec.grad, g["grad_rec"]) < 1e-3, relerr(rec.grad, g["grad_rec"])


def test_spectral_loss_config2_size(dd):
    """config 2's signal length (T = 102400) and batch 4, against the oracle on the CPU.

    The loss value is compared directly.  Its gradient is compared on the linear-magnitude part
    in squared form: train.py's L1 terms take sign(|X| - |Y|), decided by transform round-off for
    bins whose magnitudes agree to fp32 precision, and its log terms weight each bin by
    1/(|X| + 1e-7), so the few smallest of ~10^6 bins per scale dominate that gradient and carry
    the fp32 transform's relative error of those tiny magnitudes (two correct fp32 transforms
    differ there by several percent of the gradient norm).  Both are conditioning of the loss,
    not of the kernels, whose vector-Jacobian product is checked directly in
    test_stft_magnitude_grad (including at this length)."""
    g = torch.Generator().manual_seed(3)
    sig = torch.randn(4, 102400, generator=g) * 0.3
    rec = sig + 0.05 * torch.randn(4, 102400, generator=g)
    scales = [4096, 2048, 1024, 512, 256, 128]
    from ddsp_pytorch_amd import loss as L
    lc = tr.multiscale_spec_loss(tr.multiscale_fft(sig, scales, 0.75), tr.multiscale_fft(rec, scales, 0.75))
    lg = L.spectral_loss(sig.cuda(), rec.cuda())
    assert relerr(lg, lc) < 1e-5

    def lin_sq(ori, rs):
        out = 0
        for s_x, s_y in zip(ori, rs):
            out = out + ((s_x - s_y) ** 2).mean()
        return out

    rc = rec.clone().requires_grad_(True)
    lin_sq(tr.multiscale_fft(sig, scales, 0.75), tr.multiscale_fft(rc, scales, 0.75)).backward()
    rg = rec.cuda().requires_grad_(True)
    lin_sq(dd.core.multiscale_fft(sig.cuda(), scales, 0.75), dd.core.multiscale_fft(rg, scales, 0.75)).backward()
    assert relerr(rg.grad, rc.grad) < 1e-4, relerr(rg.grad, rc.grad)


def test_fused_spectral_loss_matches_unfused(dd):
    """ddsp_hip_spectral_loss (one fused pass per scale) against the spectrogram route on the same
    kernels: same loss, and the same gradient up to the sign-flip ambiguity of the L1 terms
    (checked on the golden's small case, where no bin pair is within rounding)."""
    from ddsp_pytorch_amd import loss as L
    g = load_golden("g7_stft_loss")
    scales, overlap = [int(s) for s in g["scales"]], float(g["overlap"])
    sig = torch.as_tensor(g["sig"]).cuda()
    rec = torch.as_tensor(g["rec"]).cuda().requires_grad_(True)
    lf = L.spectral_loss(sig, rec, scales, overlap)
    lf.backward()
    assert relerr(lf, g["loss"]) < 1e-5, (float(lf), float(g["loss"]))
    assert relerr(rec.grad, g["grad_rec"]) < 1e-3, relerr(rec.grad, g["grad_rec"])
    with torch.no_grad():
        l0 = L.spectral_loss(sig, rec.detach(), scales, overlap)
    assert torch.equal(l0, lf.detach())
    # config 2's length: the loss value against the oracle
    gg = torch.Generator().manual_seed(3)
    s2 = torch.randn(4, 102400, generator=gg) * 0.3
    r2 = s2 + 0.05 * torch.randn(4, 102400, generator=gg)
    lc = tr.multiscale_spec_loss(tr.multiscale_fft(s2, scales, 0.75), tr.multiscale_fft(r2, scales, 0.75))
    assert relerr(L.spectral_loss(s2.cuda(), r2.cuda()), lc) < 1e-5
