"""Long renders: past core.FRAME_PREFIX_MIN_FRAMES frames per item the fused synthesis
kernel reads every frame's phase prefix from one ddsp_hip_frame_phase_prefix launch instead of summing its
earlier frames itself (O(F) per frame, O(F^2) per item).  The prefix is the reference's cumsum
(core.py:138) at each frame's start, exact in fp64, so both routes give the same bits; the harmonic output
at F = 4096 matches the numpy oracle (oracle/numpy_oracle.py).  (Bit identity holds while every partial sum is
exact in fp64 — audio pitch; near-zero f0 mixed in rounds the sums, and the routes are then held to a
tolerance: test_prefix_route_near_zero_f0.)"""
import numpy as np
import pytest
import torch

from conftest import rms

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dd():
    import ddsp_pytorch_amd
    return ddsp_pytorch_amd


def _inputs(B, F, H, NB, bs, seed):
    rng = np.random.default_rng(seed)
    f0 = (50.0 * 20.0 ** rng.random((B, F, 1))).astype(np.float32)
    param = rng.standard_normal((B, F, H + 1)).astype(np.float32)
    mags = rng.standard_normal((B, F, NB)).astype(np.float32)
    noise = (rng.random((B, F, bs)) * 2 - 1).astype(np.float32)
    return f0, param, mags, noise


def test_frame_phase_prefix_exact(dd):
    """ddsp_hip_frame_phase_prefix equals the exact fp64 running sum of bs * fl32 increment, bit for bit."""
    from oracle import numpy_oracle as no
    from ddsp_pytorch_amd import _lib
    B, F, bs = 3, 5000, 512
    f0 = _inputs(B, F, 1, 2, 4, 1)[0]
    inc = no.phase_increment(f0[..., 0], 48000).astype(np.float64) * bs
    ref = np.concatenate([np.zeros((B, 1)), np.cumsum(inc, 1)[:, :-1]], 1)
    f0d = torch.as_tensor(f0).cuda()
    out = torch.empty(B * F, dtype=torch.float64, device="cuda")
    _lib.call("frame_phase_prefix", _lib.ptr(f0d), B, F, bs, 48000.0, _lib.ptr(out), _lib.stream_of(out))
    np.testing.assert_array_equal(out.view(B, F).cpu().numpy(), ref)


def test_prefix_route_is_bit_identical(dd, monkeypatch):
    """The same launch with and without the precomputed prefix: identical signal, parts and controls."""
    B, F, H, NB, bs = 2, 700, 24, 65, 512
    f0, param, mags, noise = (torch.as_tensor(a).cuda() for a in _inputs(B, F, H, NB, bs, 2))
    with torch.no_grad():
        a = dd.core.synth_frames(f0, param, mags, bs, 48000, noise=noise, parts=True, controls=True)
        monkeypatch.setattr(dd.core, "FRAME_PREFIX_MIN_FRAMES", 1 << 30)
        b = dd.core.synth_frames(f0, param, mags, bs, 48000, noise=noise, parts=True, controls=True)
    for x, y in zip(a[:3], b[:3]):
        assert torch.equal(x, y)
    for k in a[3]:
        assert torch.equal(a[3][k], b[3][k])


def test_long_render_vs_oracle(dd):
    """F = 4096 frames (block 64: 262,144 samples per item, |phase| to ~2e5 rad) against the oracle's
    harmonic synth and filtered noise (north_star: 1e-5 RMS; the harmonic part is held to 1e-6)."""
    from oracle import numpy_oracle as no
    B, F, H, NB, bs = 2, 4096, 8, 17, 64
    f0, param, mags, noise = _inputs(B, F, H, NB, bs, 3)
    f0 = np.minimum(f0, 600.0).astype(np.float32)
    c = no.harmonic_get_controls(param[..., :1], param[..., 1:], f0, 48000)
    harm_ref, _ = no.harmonic_forward(c["amplitudes"], c["harmonic_distribution"], f0, bs, 48000)
    noise_ref = no.noise_forward(no.noise_get_controls(mags)["magnitudes"], noise, bs)
    with torch.no_grad():
        out, harm, nz = dd.core.synth_frames(*(torch.as_tensor(a).cuda() for a in (f0, param, mags)), bs, 48000,
                                             noise=torch.as_tensor(noise).cuda(), parts=True)
    assert rms(harm.cpu().numpy(), harm_ref) < 1e-6
    assert rms(nz.cpu().numpy(), noise_ref) < 1e-7
    assert rms(out.cpu().numpy(), harm_ref + noise_ref) < 1e-5


def test_prefix_route_near_zero_f0(dd, monkeypatch):
    """unvoiced frames (f0 near 0, down to 1e-30 Hz, and exact zeros) among audio-pitch frames: the
    fp64 partial sums are no longer all exact, so the precomputed prefix and the per-frame sums may round
    differently.  Both routes stay within 1e-6 RMS of each other and of the oracle on the harmonic part."""
    from oracle import numpy_oracle as no
    B, F, H, NB, bs = 2, 700, 16, 65, 512
    f0, param, mags, noise = _inputs(B, F, H, NB, bs, 4)
    rng = np.random.default_rng(9)
    tiny = (10.0 ** rng.uniform(-30, -3, size=f0.shape)).astype(np.float32)
    f0 = np.where(rng.random(f0.shape) < 0.4, tiny, f0).astype(np.float32)
    f0[:, ::50] = 0.0
    c = no.harmonic_get_controls(param[..., :1], param[..., 1:], f0, 48000)
    harm_ref, _ = no.harmonic_forward(c["amplitudes"], c["harmonic_distribution"], f0, bs, 48000)
    args = [torch.as_tensor(a).cuda() for a in (f0, param, mags)]
    with torch.no_grad():
        a = dd.core.synth_frames(*args, bs, 48000, noise=torch.as_tensor(noise).cuda(), parts=True)
        monkeypatch.setattr(dd.core, "FRAME_PREFIX_MIN_FRAMES", 1 << 30)
        b = dd.core.synth_frames(*args, bs, 48000, noise=torch.as_tensor(noise).cuda(), parts=True)
    monkeypatch.undo()
    assert F >= dd.core.FRAME_PREFIX_MIN_FRAMES  # a is the prefix route
    assert rms(a[1].cpu().numpy(), b[1].cpu().numpy()) < 1e-6
    assert rms(a[1].cpu().numpy(), harm_ref) < 1e-6 and rms(b[1].cpu().numpy(), harm_ref) < 1e-6
