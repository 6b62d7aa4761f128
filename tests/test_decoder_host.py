"""Host logic of the decoder's fused route (no GPU needed): the shared projection buffer stays live
under every way a parameter can change, and hooked / overridden synth modules keep their module calls
(ADVICE r03)."""
import torch

import ddsp_pytorch_amd as dd
from ddsp_pytorch_amd.decoder import _shared_projection, _synth_overridden


def _cat(m):
    return (torch.cat([m.harmonic_proj.weight, m.noise_proj.weight]).detach(),
            torch.cat([m.harmonic_proj.bias, m.noise_proj.bias]).detach())


def _sp(m):
    """The shared buffer's live rows (it is zero-padded to a multiple of 64 outputs for the GEMM)."""
    w, b = _shared_projection(m)
    n = m.harmonic_proj.out_features + m.noise_proj.out_features
    assert w.shape[0] % 64 == 0 and not w[n:].any() and not b[n:].any()
    return w[:n], b[:n]


def test_shared_projection_is_live():
    torch.manual_seed(0)
    m = dd.DDSPDecoder(32, 10, 9, 48000, 64, False)
    w, b = _sp(m)
    assert torch.equal(w, _cat(m)[0]) and torch.equal(b, _cat(m)[1])
    # the parameters are views of the shared buffer: in-place writes through .data are seen
    m.harmonic_proj.weight.data.mul_(2.0)
    w2, b2 = _sp(m)
    assert w2.data_ptr() == w.data_ptr() and torch.equal(w2, _cat(m)[0])
    m.noise_proj.bias.data.copy_(torch.arange(9.0))
    assert torch.equal(_sp(m)[1], _cat(m)[1])
    # load_state_dict copies into the parameters in place
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    sd["harmonic_proj.weight"].fill_(0.5)
    m.load_state_dict(sd)
    assert torch.equal(_sp(m)[0], _cat(m)[0])
    # a replaced .data (or a fresh module) is re-shared with its current values
    m.noise_proj.weight.data = torch.randn(9, 32)
    w3, _ = _sp(m)
    assert w3.data_ptr() != w.data_ptr() and torch.equal(w3, _cat(m)[0])
    m.harmonic_proj = torch.nn.Linear(32, 11)
    assert torch.equal(_sp(m)[0], _cat(m)[0])
    # an optimizer step updates the shared storage too
    opt = torch.optim.SGD(m.parameters(), lr=0.1)
    for p in m.parameters():
        p.grad = torch.ones_like(p)
    opt.step()
    assert torch.equal(_sp(m)[0], _cat(m)[0])


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
