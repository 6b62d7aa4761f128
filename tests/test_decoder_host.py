"""Host logic of the decoder's fused route (no GPU needed): the projections are never rebound, copied or
cached by the module (the round-4 shared padded buffer re-pointed the parameters' storage), the
fp32-only network kernels step aside for other dtypes and autocast, and hooked / overridden synth modules
keep their module calls."""
import copy
import io

import torch

import ddsp_pytorch_amd as dd
from ddsp_pytorch_amd.decoder import _fp32_inference_ok, _synth_overridden


def test_projections_leave_parameters_alone():
    """decoder_projections keeps no state on the module: parameters keep their own storage, the module's
    __dict__ gains nothing, deepcopy / state_dict / torch.save see exactly the reference's tensors."""
    torch.manual_seed(0)
    m = dd.DDSPDecoder(32, 10, 9, 48000, 64, False)
    ptrs = {k: p.data_ptr() for k, p in m.named_parameters()}
    keys = set(m.__dict__)
    with torch.no_grad():
        hp, npj = dd.decoder.decoder_projections(m, torch.randn(2, 3, 32))
    assert hp.shape == (2, 3, 11) and npj.shape == (2, 3, 9)
    assert {k: p.data_ptr() for k, p in m.named_parameters()} == ptrs and set(m.__dict__) == keys
    sd = m.state_dict()
    assert sd["harmonic_proj.weight"].shape == (11, 32) and sd["noise_proj.bias"].shape == (9,)
    assert sd["harmonic_proj.weight"].untyped_storage().data_ptr() != sd["noise_proj.weight"].untyped_storage().data_ptr()
    buf = io.BytesIO()
    torch.save(sd, buf)
    n_floats = sum(v.numel() for v in sd.values())
    assert len(buf.getvalue()) < 4 * n_floats + 64 * 1024  # no padded shared buffer serialised
    c = copy.deepcopy(m)
    for (k, a), b in zip(m.state_dict().items(), c.state_dict().values()):
        assert torch.equal(a, b), k


def test_fp32_inference_guard():
    lin = torch.nn.Linear(4, 3)
    x = torch.randn(2, 4)
    assert _fp32_inference_ok(x, (lin,))
    assert not _fp32_inference_ok(x.double(), (lin,))
    assert not _fp32_inference_ok(x, (torch.nn.Linear(4, 3).half(),))
    with torch.autocast("cpu", dtype=torch.bfloat16):
        assert not _fp32_inference_ok(x, (lin,))


def test_synth_overridden():
    m = dd.DDSPDecoder(32, 10, 9, 48000, 64, False)
    hs, ns = m.harmonic_synth, m.noise_synth
    assert not _synth_overridden(hs, dd.HarmonicSynth) and not _synth_overridden(ns, dd.FilteredNoise)
    h = hs.register_forward_hook(lambda *a: None)
    assert _synth_overridden(hs, dd.HarmonicSynth)
    h.remove()
    h = ns.register_forward_pre_hook(lambda *a: None)
    assert _synth_overridden(ns, dd.FilteredNoise)
    h.remove()

    class Louder(dd.HarmonicSynth):
        def forward(self, amplitudes, harmonic_distribution, f0):
            return 2 * super().forward(amplitudes, harmonic_distribution, f0)

    class OtherControls(dd.FilteredNoise):
        def get_controls(self, magnitudes):
            return super().get_controls(magnitudes * 0.5)

    assert _synth_overridden(Louder(64, 48000), dd.HarmonicSynth)
    assert _synth_overridden(OtherControls(64, 9), dd.FilteredNoise)
