"""Backward kernels: gradients of the gfx950 path, through the C-ABI,
against the reference's own autograd — its golden gradients (g6_*, written by
tests/golden/make_goldens.py) and the torch-CPU oracle's autograd, which tests/test_oracle_grad.py
pins to those goldens.

Tolerance: relative L2 error of each gradient ||got - ref|| / ||ref|| <= GRAD_REL (1e-5) for
the synthesis path (fp32 sums in a different order; the sine and scale_function
approximations of the forward kernels are ~2e-7 / 1e-6 relative), 1e-4 for the full
decoder's network parameters (their gradients also pass through the GRU on MIOpen).
"""
import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import torch_ref as tr

pytestmark = pytest.mark.gpu

GRAD_REL = 1e-5
NET_REL = 1e-4


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


def leaf(x, dev="cpu"):
    return torch.as_tensor(np.asarray(x)).float().to(dev).clone().requires_grad_(True)


def both(x):
    """the same values as a CPU leaf and a cuda leaf"""
    x = torch.as_tensor(np.asarray(x)).float()
    return x.clone().requires_grad_(True), x.cuda().requires_grad_(True)


def f0_frames(B, F, seed=0):
    g = torch.Generator().manual_seed(seed)
    return 50.0 * 20.0 ** torch.rand(B, F, 1, generator=g)


# ------------------------------------------------------------------ function level
def test_scale_function_grad(dd):
    x = torch.randn(5000, generator=torch.Generator().manual_seed(0)) * 4
    w = torch.randn(5000)
    xc, xg = both(x)
    (tr.scale_function(xc) * w).sum().backward()
    (dd.core.scale_function(xg) * w.cuda()).sum().backward()
    assert relerr(xg.grad, xc.grad) < GRAD_REL
    xc, xg = both(x)
    (tr.scale_function(xc + (-5.0)) * w).sum().backward()
    (dd.core.scale_with_bias(xg, -5.0) * w.cuda()).sum().backward()
    assert relerr(xg.grad, xc.grad) < GRAD_REL


def test_nyquist_and_upsample_grad(dd):
    g = torch.Generator().manual_seed(1)
    amps = torch.rand(2, 7, 33, generator=g)
    f0 = f0_frames(2, 7, 1)
    ac, ag = both(amps)
    w = torch.randn(2, 7 * 64, 33, generator=g)
    (tr.upsample(tr.remove_above_nyquist(ac, f0, 48000), 64) * w).sum().backward()
    (dd.core.upsample(dd.core.remove_above_nyquist(ag, f0.cuda(), 48000), 64) * w.cuda()).sum().backward()
    assert relerr(ag.grad, ac.grad) < GRAD_REL


def test_harmonic_synth_grad(dd):
    g = torch.Generator().manual_seed(2)
    f0 = tr.upsample(f0_frames(2, 8, 2), 512)
    amps = torch.rand(2, 8 * 512, 16, generator=g) / 16
    w = torch.randn(2, 8 * 512, 1, generator=g)
    ac, ag = both(amps)
    (tr.harmonic_synth(f0, ac, 48000) * w).sum().backward()
    (dd.core.harmonic_synth(f0.cuda(), ag, 48000) * w.cuda()).sum().backward()
    assert relerr(ag.grad, ac.grad) < GRAD_REL


def test_f0_grad_refused(dd):
    f0 = torch.full((1, 64, 1), 220.0, device="cuda", requires_grad=True)
    a = torch.rand(1, 64, 4, device="cuda", requires_grad=True)
    with pytest.raises(NotImplementedError):
        dd.core.harmonic_synth(f0, a, 48000)


@pytest.mark.parametrize("NB,target", [(65, 512), (17, 40), (17, 20), (5, 16), (65, 64)])
def test_impulse_response_grad(dd, NB, target):
    g = torch.Generator().manual_seed(NB + target)
    amp = torch.rand(3, 5, NB, generator=g)
    w = torch.randn(3, 5, target, generator=g)
    ac, ag = both(amp)
    (tr.amp_to_impulse_response(ac, target) * w).sum().backward()
    (dd.core.amp_to_impulse_response(ag, target) * w.cuda()).sum().backward()
    assert relerr(ag.grad, ac.grad) < GRAD_REL, relerr(ag.grad, ac.grad)


@pytest.mark.parametrize("rows,krows,N", [(4, 4, 100), (3, 1, 10000), (2, 2, 5000)])
def test_fft_convolve_grad(dd, rows, krows, N):
    g = torch.Generator().manual_seed(rows * N)
    s = torch.randn(rows, N, generator=g)
    k = torch.randn(krows, N, generator=g) * 0.1
    w = torch.randn(rows, N, generator=g)
    sc, sg = both(s)
    kc, kg = both(k)
    (tr.fft_convolve(sc, kc) * w).sum().backward()
    (dd.core.fft_convolve(sg, kg) * w.cuda()).sum().backward()
    assert relerr(sg.grad, sc.grad) < GRAD_REL, relerr(sg.grad, sc.grad)
    assert relerr(kg.grad, kc.grad) < GRAD_REL, relerr(kg.grad, kc.grad)


# ------------------------------------------------------------------ module level
@pytest.mark.parametrize("B,F,bs,H", [(2, 16, 64, 16), (1, 200, 512, 100), (2, 20, 256, 64)])
def test_harmonic_module_grad(dd, B, F, bs, H):
    g = torch.Generator().manual_seed(3)
    f0 = f0_frames(B, F, 3)
    param = torch.randn(B, F, H + 1, generator=g)
    w = torch.randn(B, F * bs, 1, generator=g)
    pc, pg = both(param)
    a, d = tr.harmonic_controls(pc[..., :1], pc[..., 1:], f0, 48000)
    (tr.harmonic_forward(a, d, f0, bs, 48000) * w).sum().backward()
    hs = dd.modules.HarmonicSynth(bs, 48000)
    ctrls = hs.get_controls(pg[..., :1], pg[..., 1:], f0.cuda())
    out = hs(**ctrls)
    # the in-place side effect of modules.py:73 is reproduced under autograd too
    assert relerr(ctrls["harmonic_distribution"], d) < 1e-6
    (out * w.cuda()).sum().backward()
    assert relerr(pg.grad, pc.grad) < GRAD_REL, relerr(pg.grad, pc.grad)
    # the fused params op
    pg2 = param.cuda().requires_grad_(True)
    (dd.core.harmonic_synth_params(f0.cuda(), pg2, bs, 48000) * w.cuda()).sum().backward()
    assert relerr(pg2.grad, pc.grad) < GRAD_REL, relerr(pg2.grad, pc.grad)


@pytest.mark.parametrize("B,F,bs,NB", [(2, 16, 512, 65), (1, 8, 256, 65), (2, 4, 64, 17),
                                       # the wave-per-frame noise VJP's lag-segment tails (bs/8 = 80, 96, 112, 128
                                       # lags: 64 + 16, 64 + 32, 64 + 32 + 16, 2 x 64) and a frame count that
                                       # leaves its last workgroup partly empty
                                       (1, 5, 640, 65), (1, 6, 768, 65), (1, 3, 896, 65), (2, 3, 1024, 65)])
def test_noise_module_grad(dd, B, F, bs, NB):
    g = torch.Generator().manual_seed(4)
    mags = torch.randn(B, F, NB, generator=g)
    w = torch.randn(B, F * bs, 1, generator=g)
    mc, mg = both(mags)
    torch.manual_seed(123)
    nz = torch.rand(B, F, bs) * 2 - 1
    (tr.noise_forward(tr.scale_function(mc + (-5.0)), nz, bs) * w).sum().backward()
    fn = dd.modules.FilteredNoise(bs, NB)
    torch.manual_seed(123)  # noise_mode "torch" draws the same tensor
    (fn(**fn.get_controls(mg)) * w.cuda()).sum().backward()
    assert relerr(mg.grad, mc.grad) < GRAD_REL, relerr(mg.grad, mc.grad)
    # fused get_controls + forward (raw magnitudes)
    mg2 = mags.cuda().requires_grad_(True)
    (dd.core.filtered_noise(mg2, bs, noise=nz.cuda(), raw_bias=-5.0) * w.cuda()).sum().backward()
    assert relerr(mg2.grad, mc.grad) < GRAD_REL, relerr(mg2.grad, mc.grad)


def test_noise_device_rng_grad_linear(dd):
    """On-device noise: the backward regenerates the forward's Philox stream.  The output is
    linear in the (scaled) magnitudes, so <dA, delta> = <w, y(A + delta) - y(A)> up to rounding."""
    B, F, bs, NB = 2, 12, 512, 65
    g = torch.Generator().manual_seed(5)
    A = (torch.rand(B, F, NB, generator=g) + 0.1).cuda().requires_grad_(True)
    delta = (torch.randn(B, F, NB, generator=g) * 0.1).cuda()
    w = torch.randn(B, F * bs, 1, generator=g).cuda()
    dd.core.set_noise_seed(77)
    y = dd.core.filtered_noise(A, bs)
    (y * w).sum().backward()
    with torch.no_grad():
        dd.core.set_noise_seed(77)
        y1 = dd.core.filtered_noise(A + delta, bs)
        lhs = float((A.grad.double() * delta.double()).sum())
        rhs = float(((y1 - y).double() * w.double()).sum())
    assert abs(lhs - rhs) <= 1e-4 * abs(rhs), (lhs, rhs)


@pytest.mark.parametrize("parts", [False, True])
def test_synth_frames_grad(dd, parts):
    B, F, bs, H, NB = 2, 40, 512, 100, 65
    g = torch.Generator().manual_seed(6)
    f0 = f0_frames(B, F, 6)
    param = torch.randn(B, F, H + 1, generator=g)
    mags = torch.randn(B, F, NB, generator=g)
    nz = torch.rand(B, F, bs, generator=g) * 2 - 1
    w = torch.randn(B, F * bs, 1, generator=g)
    w2 = torch.randn(B, F * bs, 1, generator=g)
    pc, pg = both(param)
    mc, mg = both(mags)
    a, d = tr.harmonic_controls(pc[..., :1], pc[..., 1:], f0, 48000)
    h = tr.harmonic_forward(a, d, f0, bs, 48000)
    n = tr.noise_forward(tr.scale_function(mc + (-5.0)), nz, bs)
    loss = ((h + n) * w).sum() + ((h * w2).sum() if parts else 0.0)
    loss.backward()
    res = dd.core.synth_frames(f0.cuda(), pg, mg, bs, 48000, noise=nz.cuda(), parts=parts)
    if parts:
        out, harm, _ = res
        loss_g = (out * w.cuda()).sum() + (harm * w2.cuda()).sum()
    else:
        loss_g = (res * w.cuda()).sum()
    loss_g.backward()
    assert relerr(pg.grad, pc.grad) < GRAD_REL, relerr(pg.grad, pc.grad)
    assert relerr(mg.grad, mc.grad) < GRAD_REL, relerr(mg.grad, mc.grad)


# ------------------------------------------------------------------ reverb
@pytest.mark.parametrize("tag", ["small", "crop"])
def test_reverb_grad_golden(dd, tag):
    g = load_golden(f"g6_grad_reverb_{tag}")
    L, sr = int(g["length"]), int(g["sample_rate"])
    rv = dd.modules.Reverb(L, sr)
    with torch.no_grad():
        rv.noise.copy_(torch.as_tensor(g["noise"]))
        rv.decay.copy_(torch.as_tensor(g["decay"]))
        rv.wet.copy_(torch.as_tensor(g["wet"]))
    rv = rv.cuda()
    x = leaf(g["x"], "cuda")
    out = rv(x)
    (out * torch.as_tensor(g["weight"]).cuda()).sum().backward()
    assert relerr(out, g["out"]) < 2e-6
    for name, t in (("grad_x", x), ("grad_noise", rv.noise), ("grad_decay", rv.decay), ("grad_wet", rv.wet)):
        assert relerr(t.grad, g[name]) < GRAD_REL, (name, relerr(t.grad, g[name]))


# (2, 102400, 96000): config 4's 48 kernel windows, more than one round of the adjoint MAC's
# 27-slot register ring; (1, 131072, 120000): 60 windows, three rounds, and the IR correlation's
# 25-lag kernel over three lag blocks
# (3, 102400, 48000) and (2, 102400, 30000): 50 blocks, the streaming adjoint MAC (all 25 / 16 windows)
@pytest.mark.parametrize("B,T,L", [(3, 102400, 48000), (2, 102400, 30000), (2, 30000, 96000), (1, 2048, 2048),
                                   (2, 102400, 96000), (1, 131072, 120000)])
def test_reverb_grad_oracle(dd, B, T, L):
    g = torch.Generator().manual_seed(B * T + L)
    torch.manual_seed(1)
    rv = dd.modules.Reverb(L, 48000, initial_wet=0.3, initial_decay=4.0)
    noise, decay, wet = (p.detach().clone().requires_grad_(True) for p in (rv.noise, rv.decay, rv.wet))
    ref = tr.Reverb(noise, decay, wet, L, 48000)
    x = torch.randn(B, T, 1, generator=g) * 0.3
    w = torch.randn(B, T, 1, generator=g)
    xc, xg = both(x)
    (ref(xc) * w).sum().backward()
    rv = rv.cuda()
    (rv(xg) * w.cuda()).sum().backward()
    assert relerr(xg.grad, xc.grad) < GRAD_REL, relerr(xg.grad, xc.grad)
    for name, a, b in (("noise", rv.noise, noise), ("decay", rv.decay, decay), ("wet", rv.wet, wet)):
        assert relerr(a.grad, b.grad) < GRAD_REL, (name, relerr(a.grad, b.grad))


# ------------------------------------------------------------------ the full model
def test_decoder_grad_golden(dd):
    """One training step's backward of DDSPDecoder (decoder.py:101 -> loss) against the
    reference's own gradients for every parameter."""
    g = load_golden("g6_grad_decoder")
    m = dd.DDSPDecoder(int(g["hidden_size"]), int(g["n_harmonic"]), int(g["n_bands"]), int(g["sample_rate"]),
                       int(g["block_size"]), True)
    m.load_state_dict({k[3:]: torch.as_tensor(v) for k, v in g.items() if k.startswith("sd.")})
    m = m.cuda()
    acts = {}

    def keep(name):
        def hook(mod, inp, out):
            out.retain_grad()
            acts[name] = out
        return hook

    m.harmonic_proj.register_forward_hook(keep("param"))
    m.noise_proj.register_forward_hook(keep("mags"))
    torch.manual_seed(123)
    o = m({"pitch": torch.as_tensor(g["pitch"]).cuda(), "loudness": torch.as_tensor(g["loudness"]).cuda()})
    (o["signal"] * torch.as_tensor(g["weight"]).cuda()).sum().backward()
    assert relerr(acts["param"].grad, g["grad_param"]) < GRAD_REL, relerr(acts["param"].grad, g["grad_param"])
    assert relerr(acts["mags"].grad, g["grad_mags"]) < GRAD_REL, relerr(acts["mags"].grad, g["grad_mags"])
    checked = 0
    for name, p in m.named_parameters():
        key = "grad." + name
        if key in g:
            tol = GRAD_REL if name.startswith("reverb.") else NET_REL
            assert p.grad is not None, name
            assert relerr(p.grad, g[key]) < tol, (name, relerr(p.grad, g[key]))
            checked += 1
    assert checked >= 20


def test_reverb_backward_entry_points(dd):
    """The C-ABI's three ways to the reverb gradients agree: ddsp_hip_reverb_backward with the
    forward's kept input spectra (the autograd path), the same entry recomputing them from x, and
    ddsp_hip_reverb_apply_transposed for the input gradient."""
    from ddsp_pytorch_amd import _lib, core, grad
    g_ = torch.Generator().manual_seed(21)
    B, T, L = 5, 20000, 9000
    x = (torch.randn(B, T, 1, generator=g_) * 0.3).cuda()
    w = torch.randn(B, T, 1, generator=g_).cuda()
    torch.manual_seed(1)
    rv = dd.modules.Reverb(L, 48000).cuda()
    with torch.no_grad():
        spec = core.reverb_spectrum(rv.build_impulse(), T)
        _, ws = core._reverb_apply_launch(x, spec, L)
    dx1, di1 = grad.reverb_backward(None, ws, spec, w, L, True, True)
    dx2, di2 = grad.reverb_backward(x, None, spec, w, L, True, True)
    assert torch.equal(dx1, dx2) and torch.equal(di1, di2)
    dx3 = torch.empty_like(dx1)
    ws3 = core._workspace(_lib.query("reverb_workspace_size", B, T, L), x.device)
    _lib.call("reverb_apply_transposed", _lib.ptr(w), _lib.ptr(spec), _lib.ptr(dx3), B, T, L, _lib.ptr(ws3),
              ws3.numel(), _lib.stream_of(w))
    assert relerr(dx3, dx1) < 1e-6
    # against the oracle
    noise, decay, wet = (p.detach().cpu().clone() for p in (rv.noise, rv.decay, rv.wet))
    imp = tr.Reverb(noise, decay, wet, L, 48000).build_impulse().reshape(-1)
    xc = x.cpu().requires_grad_(True)
    ic = imp.clone().requires_grad_(True)
    y = tr.fft_convolve(xc.squeeze(-1), torch.nn.functional.pad(ic, (0, T - L)))
    (y * w.cpu().squeeze(-1)).sum().backward()
    assert relerr(dx1, xc.grad) < GRAD_REL
    assert relerr(di1, ic.grad) < GRAD_REL
