"""Pin the CPU oracles against the golden vectors produced by the reference itself.

tests/golden/*.npz were written by tests/golden/make_goldens.py running
hugofloresgarcia/ddsp_pytorch (torch 2.10 CPU).  numpy_oracle is an independent
restatement (explicit fp32/fp64 semantics); torch_ref re-issues the reference's
ATen op sequence and must be bit-exact.
"""
import numpy as np
import pytest
import torch

from conftest import load_golden, rms
from oracle import numpy_oracle as no
from oracle import torch_ref as tr

T = torch.from_numpy


def test_elementwise():
    g = load_golden("g0_elementwise")
    np.testing.assert_allclose(no.scale_function(g["scale_in"]), g["scale_out"], rtol=2e-6, atol=0)
    assert np.array_equal(no.remove_above_nyquist(g["nyq_amps"], g["nyq_f0"], 48000), g["nyq_out"])
    assert np.array_equal(no.remove_above_nyquist(g["nyq_amps"], g["nyq_f0"], 44100), g["nyq_out_44k"])
    assert np.array_equal(no.upsample(g["up_in"], 3), g["up_out_3"])
    assert np.array_equal(no.upsample(g["up_in"], 441), g["up_out_441"])
    assert torch.equal(tr.scale_function(T(g["scale_in"])), T(g["scale_out"]))
    assert torch.equal(tr.upsample(T(g["up_in"]), 441), T(g["up_out_441"]))


def test_phase_increment_bitexact():
    # the fp32 phase is the crux of 1e-5 parity: the closed form must match torch.cumsum bit for bit
    g = load_golden("g1_harmonic_persample")
    f0 = g["f0"]
    ref = torch.cumsum(2 * np.pi * T(f0) / 48000, 1).numpy()
    assert np.array_equal(no.phase(f0, 48000), ref)


@pytest.mark.parametrize("name", ["g1_harmonic_small", "g1_harmonic_full", "g1_harmonic_h128"])
def test_harmonic_frames(name):
    g = load_golden(name)
    out = no.harmonic_synth_frames(g["f0_frames"], g["amp_frames"], int(g["block_size"]), 48000)
    assert rms(out, g["out"]) < 2e-7, rms(out, g["out"])
    bs = int(g["block_size"])
    if name != "g1_harmonic_h128":
        o2 = tr.harmonic_synth(tr.upsample(T(g["f0_frames"]), bs), tr.upsample(T(g["amp_frames"]), bs), 48000)
        assert torch.equal(o2, T(g["out"]))


def test_harmonic_persample():
    g = load_golden("g1_harmonic_persample")
    assert rms(no.harmonic_synth(g["f0"], g["amps"], 48000), g["out"]) < 1e-7
    assert rms(no.harmonic_synth(g["f0"], g["amps"], 44100), g["out_44k"]) < 1e-7


@pytest.mark.parametrize("name", ["g2_controls", "g2_controls_rt"])
def test_harmonic_module(name):
    g = load_golden(name)
    p, f0, bs = g["param"], g["f0"], int(g["block_size"])
    c = no.harmonic_get_controls(p[..., :1], p[..., 1:], f0, 48000)
    if "amplitudes" in g:
        np.testing.assert_allclose(c["amplitudes"], g["amplitudes"], rtol=2e-6)
        np.testing.assert_allclose(c["harmonic_distribution"], g["distribution"], rtol=2e-6, atol=1e-12)
    out, dist = no.harmonic_forward(c["amplitudes"], c["harmonic_distribution"], f0, bs, 48000)
    if "distribution_after_forward" in g:
        np.testing.assert_allclose(dist, g["distribution_after_forward"], rtol=4e-6, atol=1e-12)
    assert rms(out, g["out"]) < 1e-6


def test_noise():
    g = load_golden("g3_noise")
    mags = no.noise_get_controls(g["mags"])["magnitudes"]
    np.testing.assert_allclose(mags, g["magnitudes"], rtol=2e-6)
    ir = no.amp_to_impulse_response(g["magnitudes"], 512)
    np.testing.assert_allclose(ir, g["impulse"], atol=2e-7)
    out = no.noise_forward(g["magnitudes"], g["noise_in"], 512)
    assert rms(out, g["out"]) < 1e-7
    np.testing.assert_allclose(no.amp_to_impulse_response(g["amp_odd"], 40), g["ir_odd_40"], atol=1e-6)
    np.testing.assert_allclose(no.amp_to_impulse_response(g["amp_odd"], 20), g["ir_odd_20"], atol=1e-6)
    np.testing.assert_allclose(no.fft_convolve(g["sig_odd"], g["ker_odd"]), g["conv_odd"], atol=2e-5)
    # torch restatement is bit-exact
    assert torch.equal(tr.amp_to_impulse_response(T(g["magnitudes"]), 512), T(g["impulse"]))
    assert torch.equal(tr.noise_forward(T(g["magnitudes"]), T(g["noise_in"]), 512), T(g["out"]))


@pytest.mark.parametrize("tag", ["small", "1s", "crop", "wet"])
def test_reverb(tag):
    g = load_golden(f"g4_reverb_{tag}")
    L = int(g["length"])
    imp = no.reverb_build_impulse(g["noise"], g["decay"], g["wet"], L, 48000)
    np.testing.assert_allclose(imp, g["impulse"], rtol=2e-6, atol=1e-9)
    out = no.reverb(g["x"], g["impulse"])
    scale = float(np.sqrt(np.mean(g["out"].astype(np.float64) ** 2)))
    assert rms(out, g["out"]) < 1e-6 * max(1.0, scale), (rms(out, g["out"]), scale)
    rv = tr.Reverb(T(g["noise"]), T(g["decay"]), T(g["wet"]), L, 48000)
    assert torch.equal(rv.build_impulse(), T(g["impulse"]))
    assert torch.equal(rv(T(g["x"])), T(g["out"]))


def test_synth_path_decoder_golden():
    """The synthesis section of DDSPDecoder.forward, fed the golden's own controls."""
    g = load_golden("g5_decoder")
    f0 = g["pitch"]
    out, _ = no.harmonic_forward(g["amplitudes"], g["distribution"] / g["amplitudes"], f0, 512, 48000)
    assert rms(out, g["harmonic_audio"]) < 1e-6


def _sd(g):
    return {k[3:]: torch.as_tensor(v) for k, v in g.items() if k.startswith("sd.")}


def test_decoder_oracle_vs_golden():
    """torch_ref's control network + synthesis restatement vs the reference's DDSPDecoder.forward."""
    g = load_golden("g5_decoder")
    sd = _sd(g)
    f0, lo = T(g["pitch"]), T(g["loudness"])
    with torch.no_grad():
        hidden = tr.gru_decoder_forward(sd, f0, lo)
        torch.manual_seed(123)
        noise = torch.rand(1, 16, 512) * 2 - 1
        rv = tr.Reverb(sd["reverb.noise"], sd["reverb.decay"], sd["reverb.wet"], 48000, 48000)
        sig, harm, nz = tr.decoder_synthesis(sd, f0, hidden, noise, 512, 48000, rv)
    assert torch.equal(harm, T(g["harmonic_audio"]))
    assert torch.equal(nz, T(g["noise"]))
    assert torch.equal(sig, T(g["signal"]))


def test_realtime_oracle_vs_golden():
    """export.py:33-40 realtime calls (decimation, loudness normalisation, cache_gru carried across
    calls, decoder.py:56-60) restated in torch_ref vs the reference's modules (g8)."""
    g = load_golden("g8_realtime")
    sd = _sd(g)
    cache = sd["decoder.cache_gru"].clone()
    for k in range(3):
        out = tr.realtime_forward(sd, T(g[f"pitch_{k}"]), T(g[f"loudness_{k}"]), float(g["mean_loudness"]),
                                  float(g["std_loudness"]), cache, T(g[f"noise_in_{k}"]), 256, 48000)
        assert torch.equal(out, T(g[f"signal_{k}"])), k
        assert torch.equal(cache, T(g[f"cache_{k}"])), k
