"""The fused IR rebuild (ddsp_hip_reverb_impulse_spectrum: modules.py:21-26's build_impulse and the
partition spectra of modules.py:30-35 in one launch) equals the two-launch form bit for bit, for crop
and pad cases and non-default wet/decay; the module's uncached forward matches golden g4."""
import numpy as np
import pytest
import torch

from conftest import load_golden, rms

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dd():
    import ddsp_pytorch_amd
    return ddsp_pytorch_amd


@pytest.mark.parametrize("L,T,wet,decay", [(48000, 102400, 0.0, 5.0), (48000, 24000, 0.0, 5.0),
                                           (4800, 9600, 1.5, 2.0), (96000, 102400, -0.7, 25.0),
                                           (2049, 4097, 0.3, 1.0)])
def test_impulse_spectrum_bitexact(dd, L, T, wet, decay):
    torch.manual_seed(1)
    rv = dd.Reverb(L, 48000, initial_wet=wet, initial_decay=decay).cuda()
    with torch.no_grad():
        two = dd.core.reverb_spectrum(rv.build_impulse(), T)
        one = dd.core.reverb_impulse_spectrum(rv.noise, rv.decay, rv.wet, 48000, T)
    assert torch.equal(one, two)


@pytest.mark.parametrize("tag", ["small", "1s", "crop", "wet"])
def test_uncached_reverb_golden(dd, tag):
    g = load_golden(f"g4_reverb_{tag}")
    rv = dd.Reverb(int(g["length"]), int(g["sample_rate"])).cuda()
    with torch.no_grad():
        rv.noise.copy_(torch.as_tensor(g["noise"]))
        rv.decay.copy_(torch.as_tensor(g["decay"]))
        rv.wet.copy_(torch.as_tensor(g["wet"]))
    rv.cache_spectrum = False
    with torch.no_grad():
        out = rv(torch.as_tensor(g["x"]).cuda())
    ref = g["out"]
    assert rms(out.cpu().numpy(), ref) < 2e-6 * max(1.0, float(np.sqrt(np.mean(ref ** 2))))


def test_ir_rebuild_every_call_and_after_updates(dd):
    """With the cache off (the reference's rebuild-every-forward) and after in-place parameter updates
    (an optimizer step), every SynthPath call equals the same step with the IR built by the separate
    build_impulse + reverb_spectrum calls."""
    from ddsp_pytorch_amd.synth import SynthPath, make_inputs
    B, F, H, NB, bs, sr = 4, 20, 30, 65, 512, 48000
    inp = make_inputs(B, F, H, NB, bs, seed=2, device="cuda", with_noise=True)
    syn = SynthPath(bs, sr, reverb_length=4800, noise_mode="inject").cuda()
    args = (inp["f0"], inp["param"], inp["mags"], inp["noise"])
    T = F * bs

    def inline():
        with torch.no_grad():
            sig = syn.synthesize(*args)
            spec = dd.core.reverb_spectrum(syn.reverb.build_impulse(), T)
            return dd.core.reverb_apply(sig, spec, syn.reverb.length)

    syn.reverb.cache_spectrum = False
    for _ in range(3):
        assert torch.equal(syn(*args), inline())
    syn.reverb.cache_spectrum = True
    for k in range(3):
        with torch.no_grad():
            syn.reverb.decay.add_(0.5)    # version bump: the next forward rebuilds
            syn.reverb.wet.sub_(0.1)
        out = syn(*args)
        assert torch.equal(out, inline())


@pytest.mark.parametrize("L,T", [(48000, 102400), (48000, 24000), (4800, 9600)])
def test_device_cache_is_the_impulse_spectrum(dd, L, T):
    """The module's device cache (ddsp_hip_reverb_forward) holds ddsp_hip_reverb_impulse_spectrum's
    spectrum bit for bit, after the first call, after a rebuild, and in the every-call (force) mode."""
    torch.manual_seed(1)
    rv = dd.Reverb(L, 48000, initial_wet=0.3, initial_decay=3.0).cuda()
    x = torch.randn(3, T, 1, device="cuda")
    with torch.no_grad():
        a = rv(x)
        ref = dd.core.reverb_impulse_spectrum(rv.noise, rv.decay, rv.wet, 48000, T)
        assert torch.equal(rv._spectrum(T), ref)
        rv.cache_spectrum = False
        b = rv(x)
        assert torch.equal(a, b) and torch.equal(rv._spectrum(T), ref)
        assert torch.equal(a, dd.core.reverb_apply(x, ref, L))


def test_device_cache_sees_writes_through_data(dd):
    """an EMA-style update through ``p.data`` (no autograd version bump) between two
    forwards is seen by the second — the launch compares the parameters with the cached spectrum's inputs
    bit for bit — and one changed tap rebuilds only what it touches yet equals a fresh module."""
    torch.manual_seed(1)
    rv = dd.Reverb(48000, 48000).cuda()
    x = torch.randn(4, 102400, 1, device="cuda")
    with torch.no_grad():
        a = rv(x)
        for p in (rv.noise, rv.decay, rv.wet):  # EMA toward a shadow copy, through .data
            p.data.mul_(0.999).add_(0.001 * torch.randn_like(p))
        b = rv(x)
        rv.noise.data[30000, 0] += 0.25  # one tap, in one window pair
        c = rv(x)
    assert not torch.equal(a, b) and not torch.equal(b, c)
    for out in (c,):
        fresh = dd.Reverb(48000, 48000).cuda()
        fresh.load_state_dict(rv.state_dict())
        with torch.no_grad():
            ref = fresh(x)
        assert torch.equal(out, ref)
    with torch.no_grad():  # the cached spectrum is rebuilt bit-identically to the one-launch rebuild
        assert torch.equal(rv._spectrum(102400), dd.core.reverb_impulse_spectrum(rv.noise, rv.decay, rv.wet, 48000,
                                                                                  102400))


def test_device_cache_training_step(dd):
    """Under autograd (ReverbFn) with an optimizer step between forwards, the cache follows the updated
    parameters, and the gradients equal those of a module rebuilding every call."""
    torch.manual_seed(1)
    a = dd.Reverb(4800, 48000, initial_wet=0.5, initial_decay=3.0).cuda()
    b = dd.Reverb(4800, 48000, initial_wet=0.5, initial_decay=3.0).cuda()
    b.load_state_dict(a.state_dict())
    b.cache_spectrum = False
    oa, ob = torch.optim.SGD(a.parameters(), lr=0.05), torch.optim.SGD(b.parameters(), lr=0.05)
    x = torch.randn(3, 9600, 1, device="cuda")
    w = torch.randn(3, 9600, 1, device="cuda")
    for _ in range(3):
        for m, o in ((a, oa), (b, ob)):
            o.zero_grad()
            (m(x) * w).sum().backward()
            o.step()
        for pa, pb in zip(a.parameters(), b.parameters()):
            assert torch.equal(pa, pb)
