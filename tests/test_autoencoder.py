"""DDSPAutoencoder (ddsp/models/encoder.py:29-103), the reference's second caller of the synthesis
path, against golden g9 (tests/golden/make_goldens.py: the reference's own DDSPAutoencoder at hidden
size 32, seeded, with its state_dict and an MFCC input tensor).

CPU: the state_dict layout is the reference's (every g9 key loads, nothing extra) and the encoder and
z-conditioned decoder network reproduce the reference's z and hidden state on the host (plain torch:
LayerNorm / GRU / Linear are not on the accelerated path).  GPU: the whole forward — the projections as one
GEMM, the synthesis section as the fused launch — matches signal, harmonic, noise, z and the control dicts
(north_star: 1e-5 RMS).  At g9's hidden size 32 the network itself stays on torch's modules (the GRU step
kernels need hidden % 64 == 0, the MLP block kernel 512 outputs); the shipped size (hidden 512), where the
encoder and decoder GRUs run the step kernels and the MLPs the block kernel, is pinned by g9b in
tests/test_decoder512.py."""
import numpy as np
import pytest
import torch

from conftest import load_golden, rms

PARITY_RMS = 1e-5


def _model(g):
    import ddsp_pytorch_amd as dd
    m = dd.DDSPAutoencoder(int(g["hidden_size"]), int(g["n_harmonic"]), int(g["n_bands"]),
                           int(g["sample_rate"]), int(g["block_size"]), True)
    sd = {k[3:]: torch.as_tensor(v) for k, v in g.items() if k.startswith("sd.")}
    res = m.load_state_dict(sd, strict=True)
    assert not res.missing_keys and not res.unexpected_keys
    return m.eval()


def test_autoencoder_state_dict_layout():
    g = load_golden("g9_autoencoder")
    m = _model(g)
    ref_keys = {k[3:] for k in g.keys() if k.startswith("sd.")}
    assert set(m.state_dict()) == ref_keys
    assert m.decoder.add_z and m.decoder.gru.input_size == 3 * int(g["hidden_size"])
    assert m.encoder.gru.input_size == 30 and m.encoder.proj.out_features == 16


def test_autoencoder_latent_on_host():
    """z = encoder(mfcc) (encoder.py:22-26) on the host equals the reference's z from g9."""
    g = load_golden("g9_autoencoder")
    m = _model(g)
    with torch.no_grad():
        z = m.encoder(torch.as_tensor(g["mfcc"]))
    np.testing.assert_allclose(z.numpy(), g["z"], rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_autoencoder_golden_gpu():
    g = load_golden("g9_autoencoder")
    m = _model(g).cuda()
    batch = {k: torch.as_tensor(g[v]).cuda() for k, v in (("pitch", "pitch"), ("loudness", "loudness"),
                                                          ("mfcc", "mfcc"))}
    with torch.no_grad():
        torch.manual_seed(123)  # the reference's FilteredNoise draw (noise_mode "torch")
        o = m(batch)
    for key in ("harmonic_audio", "noise", "signal"):
        e = rms(o[key].cpu().numpy(), g[key])
        assert e < PARITY_RMS, (key, e)
    assert rms(o["z"].cpu().numpy(), g["z"]) < PARITY_RMS
    np.testing.assert_allclose(o["harmonic_ctrls"]["amplitudes"].cpu().numpy(), g["amplitudes"], rtol=5e-5)
    np.testing.assert_allclose(o["harmonic_ctrls"]["harmonic_distribution"].cpu().numpy(), g["distribution"],
                               rtol=5e-5, atol=1e-10)
    np.testing.assert_allclose(o["noise_ctrls"]["magnitudes"].cpu().numpy(), g["magnitudes"], rtol=5e-5)
    assert o["harmonic_ctrls"]["f0"] is batch["pitch"]
