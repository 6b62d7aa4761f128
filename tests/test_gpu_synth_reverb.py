"""The synthesis kernel fused with the reverb's forward transform (ddsp_hip_synth_reverb,
core.synth_reverb): decoder.py:106-125's synthesis section + Reverb.forward (modules.py:28-35) with
the dry signal never written.  Checked against the two-launch-group route (synth_frames +
reverb_apply, the same Philox draw) and against the reference's ATen op sequence
(oracle/torch_ref.py) at the north_star tolerance (1e-5 RMS)."""
import pytest
import torch

from conftest import rms

pytestmark = pytest.mark.gpu


def _setup(B, F, bs, H=100, NB=65, L=48000, seed=0, with_noise=True):
    from ddsp_pytorch_amd.synth import SynthPath, make_inputs
    inp = make_inputs(B, F, H, NB, bs, seed=seed, device="cuda", with_noise=with_noise)
    syn = SynthPath(bs, 48000, reverb_length=L, noise_mode="inject" if with_noise else "device").cuda()
    return inp, syn


def _two_launch(inp, syn, noise=None):
    from ddsp_pytorch_amd import core
    sig = core.synth_frames(inp["f0"], inp["param"], inp["mags"], syn.block_size, syn.sample_rate, noise=noise)
    return core.reverb_apply(sig, syn.reverb._spectrum(sig.shape[1]), syn.reverb.length)


def _fused(inp, syn, noise=None):
    from ddsp_pytorch_amd import core
    T = inp["f0"].shape[1] * syn.block_size
    return core.synth_reverb(inp["f0"], inp["param"], inp["mags"], syn.block_size, syn.sample_rate,
                             syn.reverb._spectrum(T), syn.reverb.length, noise=noise)


@pytest.mark.parametrize("B,F,bs,L", [(64, 200, 512, 48000),  # config 2
                                      (3, 7, 512, 48000),     # odd batch (a pair with one row), T < L, partial block
                                      (4, 33, 256, 4800),     # 8 frames per block
                                      (2, 9, 1024, 9000)])    # 2 frames per block, T not a block multiple
def test_fused_vs_two_launch_groups(B, F, bs, L):
    with torch.no_grad():
        inp, syn = _setup(B, F, bs, L=L)
        ref = _two_launch(inp, syn, inp["noise"])
        out = _fused(inp, syn, inp["noise"])
    torch.cuda.synchronize()
    assert out.shape == ref.shape
    scale = max(1.0, float(ref.pow(2).mean().sqrt()))
    # the same samples through a radix-8 instead of the radix-16 forward transform: fp32 rounding only
    assert float((out - ref).abs().max()) < 2e-6 * scale * 10
    assert rms(out.cpu().numpy(), ref.cpu().numpy()) < 1e-6 * scale


def test_fused_device_noise_matches_two_launch_groups():
    """Device Philox noise: one offset per call, the same draw as synth_frames at that offset."""
    from ddsp_pytorch_amd import core
    with torch.no_grad():
        inp, syn = _setup(8, 40, 512, with_noise=False)
        core.set_noise_seed(77)
        a1, a2 = _fused(inp, syn), _fused(inp, syn)
        core.set_noise_seed(77)
        b1, b2 = _two_launch(inp, syn), _two_launch(inp, syn)
    torch.cuda.synchronize()
    assert float((a1 - b1).abs().max()) < 2e-5 and float((a2 - b2).abs().max()) < 2e-5
    assert float((a1 - a2).abs().max()) > 1e-3  # consecutive calls draw fresh noise


def test_fused_vs_oracle_config2_items():
    """Config-2 batch, two items (incl. the last pair's second row) against the reference's ATen op
    sequence at the north_star tolerance."""
    from oracle import torch_ref as tr
    with torch.no_grad():
        inp, syn = _setup(64, 200, 512, seed=5)
        out = _fused(inp, syn, inp["noise"]).cpu().numpy()
    rv = tr.Reverb(syn.reverb.noise.detach().cpu(), syn.reverb.decay.detach().cpu(),
                   syn.reverb.wet.detach().cpu(), 48000, 48000)
    for b in (0, 63):
        sl = slice(b, b + 1)
        ref = tr.synth_path(inp["f0"][sl].cpu(), inp["param"][sl].cpu(), inp["mags"][sl].cpu(),
                            inp["noise"][sl].cpu(), rv, 512, 48000).numpy()
        assert rms(out[sl], ref) < 1e-5, b


def test_fused_outside_envelope_falls_back():
    """block_size 128 (16 frames per block would need 2048 threads): ERANGE inside, the two-group
    route outside, same result."""
    with torch.no_grad():
        inp, syn = _setup(2, 40, 128, L=4800)
        ref = _two_launch(inp, syn, inp["noise"])
        out = _fused(inp, syn, inp["noise"])
    torch.cuda.synchronize()
    assert torch.equal(out, ref)


def test_synth_path_fused_route():
    """SynthPath.forward with fused_reverb equals the two-group route (its default)."""
    with torch.no_grad():
        inp, syn = _setup(6, 50, 512, L=48000, seed=2)
        ref = syn(inp["f0"], inp["param"], inp["mags"], inp["noise"])
        syn.fused_reverb = True
        fused = syn(inp["f0"], inp["param"], inp["mags"], inp["noise"])
    torch.cuda.synchronize()
    assert float((fused - ref).abs().max()) < 2e-5


def test_one_call_c_entry_matches_halves():
    """ddsp_hip_synth_reverb (one C call: spectra + reverb in the caller's workspace) equals
    synth_reverb_spectra + reverb_apply_spectra; bad workspace sizes are refused."""
    from ddsp_pytorch_amd import _lib, core
    with torch.no_grad():
        inp, syn = _setup(4, 24, 512, L=4800, seed=4)
        B, F, bs = 4, 24, 512
        T = F * bs
        spec = syn.reverb._spectrum(T)
        ref = _fused(inp, syn, inp["noise"])
        out = torch.empty(B, T, 1, device="cuda")
        need = int(_lib.query("synth_reverb_workspace_size", B, F, bs))
        ws = torch.empty(need, dtype=torch.uint8, device="cuda")
        p, m = inp["param"].contiguous(), inp["mags"].contiguous()
        args = lambda nbytes: (_lib.ptr(inp["f0"].contiguous()), _lib.ptr(p), p.shape[-1], _lib.ptr(m), m.shape[-1],
                               -5.0, _lib.ptr(inp["noise"].contiguous()), 0, 0, _lib.ptr(spec), syn.reverb.length,
                               _lib.ptr(out), _lib.ptr(ws), nbytes, B, F, p.shape[-1] - 1, m.shape[-1], bs, 48000.0,
                               _lib.stream_of(out))
        assert _lib.call("synth_reverb", *args(need - 1), allow=(core.EWORKSPACE,)) == core.EWORKSPACE
        _lib.call("synth_reverb", *args(need))
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
