"""The decoder network at the reference's SHIPPED size against the reference itself (config.yaml:16-21:
hidden 512, n_harmonic 64, n_bands 65, block 512, reverb on).

Goldens (tests/golden/make_goldens.py, run against /root/reference):
* g10  — ``DDSPDecoder(512, 64, 65, 48000, 512, True)`` built after ``torch.manual_seed(0)``, forward on
  B=2, F=24 (decoder.py:101-136), noise drawn after ``manual_seed(123)``;
* g9b  — ``DDSPAutoencoder(512, 100, 65, ...)`` (encoder.py:29-103), B=2, F=16;
* g6b  — the reference's autograd through g10's model at F=8 (train.py:84-130's backward).
Each stores the state_dict as per-tensor CRC32s: the tests rebuild this package's modules under the same
seed (their constructors draw in the reference's order) and check every CRC before using them.

At hidden 512 the GPU forward takes the shipped network kernels — the H=512 persistent GRU recurrence, the 512-wide
MLP blocks (LayerNorm + LeakyReLU epilogue, out_mlp's extras), the one-feature LayerNorm blocks, the
projection GEMM over the stacked parameters — and the fused synthesis launch; the tests assert each route was taken (a spy on the
C-ABI entry points called).  g5 / g9 (hidden 32) never reach those kernels.
"""
import json
import os
import zlib

import numpy as np
import pytest
import torch

from conftest import ROOT, load_golden, rms

PARITY_RMS = 1e-5  # north_star: outputs within 1e-5 RMS of the reference
GRAD_REL = 2e-5    # relative L2 of each parameter gradient's sampled entries (measured max 3.3e-6, r05b)


def _rebuild(cls, g, **kw):
    """This package's module under the golden's seed, every state_dict tensor checked by CRC32."""
    torch.manual_seed(int(g["model_seed"]))
    m = cls(int(g["hidden_size"]), int(g["n_harmonic"]), int(g["n_bands"]), int(g["sample_rate"]),
            int(g["block_size"]), True, **kw)
    keys = {k[4:] for k in g if k.startswith("crc.")}
    sd = m.state_dict()
    assert set(sd) == keys, (set(sd) ^ keys)
    for k, v in sd.items():
        a = np.ascontiguousarray(v.detach().cpu().numpy())
        assert tuple(a.shape) == tuple(g["shape." + k]), k
        assert np.uint32(zlib.crc32(a.tobytes())) == g["crc." + k], f"state_dict tensor {k} differs from the reference's"
    return m


def _decoder(g):
    import ddsp_pytorch_amd as dd
    return _rebuild(dd.DDSPDecoder, g)


def _autoencoder(g):
    import ddsp_pytorch_amd as dd
    return _rebuild(dd.DDSPAutoencoder, g)


def test_g10_state_dict_rebuilt_from_seed():
    _decoder(load_golden("g10_decoder512"))


def test_g6b_state_dict_rebuilt_from_seed():
    _decoder(load_golden("g6b_grad_decoder512"))


def test_g9b_state_dict_rebuilt_from_seed():
    _autoencoder(load_golden("g9b_autoencoder512"))


def test_g10_oracle_on_host():
    """The CPU oracle (oracle/torch_ref.py: the reference's ATen sequence over a state_dict) reproduces
    g10 at the shipped size — the checker the GPU tests' larger cases rely on.  Bit-close in this container
    (the reference's own host); another host's MKL kernels (the GPU box) give a 512-wide network's
    rounding a different order: 5.5e-7 RMS measured there, so the bound is 2e-6."""
    from oracle import torch_ref as R
    g = load_golden("g10_decoder512")
    m = _decoder(g)
    sd = {k: v.detach() for k, v in m.state_dict().items()}
    f0, lo = torch.as_tensor(g["pitch"]), torch.as_tensor(g["loudness"])
    with torch.no_grad():
        hidden = R.gru_decoder_forward(sd, f0, lo)
        rv = R.Reverb(sd["reverb.noise"], sd["reverb.decay"], sd["reverb.wet"], 48000, 48000)
        sig, harm, nz = R.decoder_synthesis(sd, f0, hidden, torch.as_tensor(g["noise_in"]), 512, 48000, rv)
    assert rms(sig.numpy(), g["signal"]) < 2e-6
    assert rms(harm.numpy(), g["harmonic_audio"]) < 1e-6
    assert rms(nz.numpy(), g["noise"]) < 1e-6


class _Spy:
    """Records the C-ABI entry points called (name, args) while active."""

    def __init__(self, monkeypatch):
        from ddsp_pytorch_amd import _lib
        self.calls = []
        real = _lib.call

        def call(name, *args, **kw):
            self.calls.append((name, args))
            return real(name, *args, **kw)
        monkeypatch.setattr(_lib, "call", call)

    def names(self):
        return [n for n, _ in self.calls]

    def count(self, name):
        return sum(n == name for n, _ in self.calls)


def _report(name, errs):
    """Keep the measured errors (read back from the GPU box under gpurun_out/)."""
    d = os.path.join(ROOT, "gpurun_out")
    if os.path.isdir(d):
        with open(os.path.join(d, f"parity_{name}.json"), "w") as f:
            json.dump(errs, f, indent=1)


def _check_outputs(o, g, batch):
    errs = {k: rms(o[k].cpu().numpy(), g[k]) for k in ("harmonic_audio", "noise", "signal")}
    errs["amplitudes_max_rel"] = float(np.max(np.abs(o["harmonic_ctrls"]["amplitudes"].cpu().numpy() / g["amplitudes"] - 1)))
    for key in ("harmonic_audio", "noise", "signal"):
        assert errs[key] < PARITY_RMS, (key, errs)
    np.testing.assert_allclose(o["harmonic_ctrls"]["amplitudes"].cpu().numpy(), g["amplitudes"], rtol=5e-5)
    np.testing.assert_allclose(o["harmonic_ctrls"]["harmonic_distribution"].cpu().numpy(), g["distribution"],
                               rtol=5e-5, atol=1e-10)
    np.testing.assert_allclose(o["noise_ctrls"]["magnitudes"].cpu().numpy(), g["magnitudes"], rtol=5e-5)
    assert o["harmonic_ctrls"]["f0"] is batch["pitch"]
    return errs


def _assert_network_routes(spy, n_gru_inputs):
    names = spy.names()
    gru = [a for n, a in spy.calls if n == "gru_forward_persistent"]  # hidden 512: the persistent recurrence
    assert gru and all(int(a[9]) == 512 for a in gru), "the H=512 GRU kernel did not run"
    assert len(gru) == n_gru_inputs and "gru_forward" not in names
    # f0_mlp / loudness_mlp blocks 2-3 and out_mlp's three blocks (+ z_mlp's) on the matrix-core block kernel
    assert spy.count("mlp_block") >= 7, names
    assert spy.count("layer_norm_leaky_relu") >= 2, names  # the one-feature first blocks
    assert any(int(a[1]) == 512 and a[6].value is not None for n, a in spy.calls if n == "mlp_block"), \
        "out_mlp's extras (f0, loudness) path did not run"
    assert spy.count("projections") == 1 and "stack_rows" not in names, names  # both projections: one launch
    assert spy.count("synth_frames_controls_prefix") == 1, names
    assert spy.count("reverb_forward") == 1, names  # the device-validated IR cache + UPOLS


@pytest.mark.gpu
def test_g10_decoder512_gpu(monkeypatch):
    """DDSPDecoder.forward at the shipped size on the GPU vs the reference (g10): signal, harmonic,
    noise <= 1e-5 RMS, the control dicts to 5e-5 relative, through the shipped network kernels."""
    from ddsp_pytorch_amd import decoder as dec
    g = load_golden("g10_decoder512")
    m = _decoder(g).cuda().eval()
    batch = {"pitch": torch.as_tensor(g["pitch"]).cuda(), "loudness": torch.as_tensor(g["loudness"]).cuda()}
    spy = _Spy(monkeypatch)
    proj = []
    real_proj = dec.decoder_projections
    monkeypatch.setattr(dec, "decoder_projections", lambda self, h: proj.append(h.shape) or real_proj(self, h))
    with torch.no_grad():
        torch.manual_seed(int(g["noise_seed"]))  # the reference's FilteredNoise draw (noise_mode "torch")
        o = m(batch)
    torch.cuda.synchronize()
    _assert_network_routes(spy, 1)
    assert proj == [torch.Size([2, 24, 512])]
    errs = _check_outputs(o, g, batch)
    _report("g10", errs)


@pytest.mark.gpu
def test_g10_decoder512_repeat_is_deterministic(monkeypatch):
    """Two forwards of the same module with the same noise seed give bit-identical audio (no stale
    cache state between calls at this size: the projection buffer, the reverb IR spectrum)."""
    g = load_golden("g10_decoder512")
    m = _decoder(g).cuda().eval()
    batch = {"pitch": torch.as_tensor(g["pitch"]).cuda(), "loudness": torch.as_tensor(g["loudness"]).cuda()}
    outs = []
    with torch.no_grad():
        for _ in range(2):
            torch.manual_seed(int(g["noise_seed"]))
            outs.append(m(batch)["signal"].cpu())
    assert torch.equal(outs[0], outs[1])


@pytest.mark.gpu
def test_g9b_autoencoder512_gpu(monkeypatch):
    """DDSPAutoencoder.forward at hidden 512 (g9b): the encoder GRU (30 inputs) and the z-conditioned
    decoder GRU (3H inputs) on the H=512 step kernel, z_mlp's K=16 block, out_mlp's extras, the fused
    synthesis — signal, parts and z <= 1e-5 RMS."""
    g = load_golden("g9b_autoencoder512")
    m = _autoencoder(g).cuda().eval()
    batch = {k: torch.as_tensor(g[k]).cuda() for k in ("pitch", "loudness", "mfcc")}
    spy = _Spy(monkeypatch)
    with torch.no_grad():
        torch.manual_seed(int(g["noise_seed"]))
        o = m(batch)
    torch.cuda.synchronize()
    _assert_network_routes(spy, 2)
    assert spy.count("mlp_block") >= 10  # + z_mlp's three blocks (K = 16, 512, 512)
    errs = _check_outputs(o, g, batch)
    errs["z"] = rms(o["z"].cpu().numpy(), g["z"])
    assert errs["z"] < PARITY_RMS, errs
    _report("g9b", errs)


@pytest.mark.gpu
def test_g6b_decoder512_gradients_gpu(monkeypatch):
    """The reference's autograd at the shipped size (g6b): loss = sum(signal * w) backward through the
    synthesis backward kernels, the reverb's adjoint and the GRU's BPTT (H=512: one persistent launch on the
    bf16 matrix cores) — the gradients at both projections' outputs and every parameter's
    gradient (2048 seeded entries + its norm) within GRAD_REL relative L2."""
    g = load_golden("g6b_grad_decoder512")
    m = _decoder(g).cuda().train()
    acts = {}

    def keep(name):
        def hook(mod, inp, out):
            out.retain_grad()
            acts[name] = out
        return hook

    m.harmonic_proj.register_forward_hook(keep("param"))
    m.noise_proj.register_forward_hook(keep("mags"))
    spy = _Spy(monkeypatch)
    batch = {"pitch": torch.as_tensor(g["pitch"]).cuda(), "loudness": torch.as_tensor(g["loudness"]).cuda()}
    torch.manual_seed(int(g["noise_seed"]))
    o = m(batch)
    w = torch.as_tensor(g["weight"]).cuda()
    (o["signal"] * w).sum().backward()
    torch.cuda.synchronize()
    assert spy.count("gru_backward_persistent") == 1 and spy.count("gru_forward_persistent") == 1, spy.names()
    assert spy.count("gru_backward") == 0, spy.names()
    errs = {"signal": rms(o["signal"].detach().cpu().numpy(), g["signal"])}
    assert errs["signal"] < PARITY_RMS, errs

    def rel(a, b):
        a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
        return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))

    errs["grad_param"] = rel(acts["param"].grad.cpu().numpy(), g["grad_param"])
    errs["grad_mags"] = rel(acts["mags"].grad.cpu().numpy(), g["grad_mags"])
    worst = 0.0
    for k, p in m.named_parameters():
        if "gidx." + k not in g:
            assert p.grad is None or not p.grad.abs().sum(), k
            continue
        gv = p.grad.reshape(-1).cpu()
        e = rel(gv[torch.as_tensor(g["gidx." + k]).long()].numpy(), g["gval." + k])
        en = abs(float(gv.double().norm()) / float(g["gnorm." + k]) - 1)
        errs["grad." + k] = (e, en)
        worst = max(worst, e, en)
    _report("g6b", errs)
    assert errs["grad_param"] < GRAD_REL and errs["grad_mags"] < GRAD_REL, errs
    assert worst < GRAD_REL, {k: v for k, v in errs.items() if isinstance(v, tuple) and max(v) >= GRAD_REL}
