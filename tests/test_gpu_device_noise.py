"""Parity of the device-noise mode (the mode bench.py times) and of the config-3 realtime outputs
against the CPU oracle.

The kernels draw U[-1,1) with Philox4x32-10 on the device (noise_mode="device"); oracle/philox.py
regenerates the same samples on the host from (seed, offset) and the counter layout, and the
torch-CPU restatement of the reference (oracle/torch_ref.py, bit-exact on the goldens) is fed
that noise.  A counter-layout bug (two items or frames drawing the same block, a wrong offset
advance across calls, a ragged block stride) fails these tests.

Tolerances: north_star's 1e-5 RMS on the full signal; 1e-6 on the harmonic part and 1e-7 on the
filtered noise (as the injected-noise parity tests).
"""
import numpy as np
import pytest
import torch

from conftest import load_golden, rms
from oracle import philox
from oracle import torch_ref as tr

pytestmark = pytest.mark.gpu

PARITY_RMS = 1e-5


@pytest.fixture(scope="module")
def dd():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import ddsp_pytorch_amd
    ddsp_pytorch_amd._lib.load()
    return ddsp_pytorch_amd


def C(x):
    return x.detach().cpu().numpy()


def host_noise(B, F, bs, seed, offset):
    return torch.from_numpy(philox.device_noise(B, F, bs, seed, offset))


def controls(B, F, H, NB, seed):
    g = torch.Generator().manual_seed(seed)
    f0 = 50.0 * 20.0 ** torch.rand(B, F, 1, generator=g)
    return f0, torch.randn(B, F, H + 1, generator=g), torch.randn(B, F, NB, generator=g)


def oracle_parts(f0, param, mags, noise, bs):
    amp, dist = tr.harmonic_controls(param[..., :1], param[..., 1:], f0, 48000)
    harm = tr.harmonic_forward(amp, dist, f0, bs, 48000)
    nz = tr.noise_forward(tr.scale_function(mags + (-5.0)), noise, bs)
    return harm, nz


# ------------------------------------------------------------------ fused synthesis kernel
@pytest.mark.parametrize("B,F,H,NB,bs", [(3, 7, 100, 65, 512), (2, 5, 17, 9, 64), (1, 3, 128, 129, 1024),
                                         (4, 2, 64, 65, 256)])
def test_synth_frames_device_noise_calls(dd, B, F, H, NB, bs):
    """Three successive calls of synth_frames (noise=None) after set_noise_seed: call k draws the
    noise of (seed, offset k); harmonic, filtered noise and their sum vs the oracle."""
    f0, param, mags = controls(B, F, H, NB, B * 1000 + H)
    seed = 0xABCDEF0123 + bs
    dd.core.set_noise_seed(seed)
    with torch.no_grad():
        for k in range(3):
            out, harm, nz = (C(t) for t in dd.core.synth_frames(f0.cuda(), param.cuda(), mags.cuda(), bs, 48000,
                                                                parts=True))
            h_ref, n_ref = oracle_parts(f0, param, mags, host_noise(B, F, bs, seed, k), bs)
            assert rms(harm, h_ref.numpy()) < 1e-6, k
            assert rms(nz, n_ref.numpy()) < 1e-7, (k, rms(nz, n_ref.numpy()))
            assert rms(out, (h_ref + n_ref).numpy()) < 1e-6, k


def test_synth_frames_device_noise_large_offset(dd):
    """64-bit offsets and seeds: the high words reach the counter and key."""
    f0, param, mags = controls(2, 4, 32, 65, 3)
    seed, off = 0xFEDCBA9876543210, (3 << 32) + 11
    with torch.no_grad():
        out = C(dd.core._synth_frames_launch(f0.cuda(), param.cuda(), mags.cuda(), 512, 48000, -5.0, None,
                                             False, seed, off))
    h_ref, n_ref = oracle_parts(f0, param, mags, host_noise(2, 4, 512, seed, off), 512)
    assert rms(out, (h_ref + n_ref).numpy()) < 1e-6


def test_synth_frames_counter_matches_host_noise(dd):
    """ddsp_hip_synth_frames_counter (the HIP-graph entry point): the offset is read from device
    memory and advanced by one per launch."""
    f0, param, mags = controls(1, 4, 64, 65, 4)
    counter = torch.zeros(1, dtype=torch.int64, device="cuda")
    seed = 77
    with torch.no_grad():
        for k in range(3):
            out = C(dd.core.synth_frames_counter(f0.cuda(), param.cuda(), mags.cuda(), 256, 48000, counter, seed))
            h_ref, n_ref = oracle_parts(f0, param, mags, host_noise(1, 4, 256, seed, k), 256)
            assert rms(out, (h_ref + n_ref).numpy()) < 1e-6, k
    assert int(counter.item()) == 3


# ------------------------------------------------------------------ filtered-noise kernels
@pytest.mark.parametrize("B,F,NB,bs", [(3, 9, 65, 512), (2, 4, 65, 441), (1, 6, 33, 30), (2, 3, 129, 1024)])
def test_filtered_noise_device_noise(dd, B, F, NB, bs):
    """noise.hip's Philox (also ragged blocks, bs % 4 != 0: per-frame stride ceil(bs/4)), scaled
    controls and raw projection with the bias, the module with noise_mode='device'."""
    g = torch.Generator().manual_seed(B * F + bs)
    raw = torch.randn(B, F, NB, generator=g)
    mags = tr.scale_function(raw + (-5.0))
    seed = 4242
    dd.core.set_noise_seed(seed)
    with torch.no_grad():
        a = C(dd.core.filtered_noise(mags.cuda(), bs))                    # offset 0
        b = C(dd.core.filtered_noise(raw.cuda(), bs, raw_bias=-5.0))      # offset 1
        mod = dd.FilteredNoise(bs, NB)
        mod.noise_mode = "device"
        c = C(mod(mags.cuda()))                                           # offset 2
    for k, out in enumerate((a, b, c)):
        ref = tr.noise_forward(mags, host_noise(B, F, bs, seed, k), bs)
        assert rms(out, ref.numpy()) < 1e-7, (k, rms(out, ref.numpy()))


# ------------------------------------------------------------------ full size, device noise
def test_config2_device_noise_all_items(dd):
    """Config 2 exactly as bench.py runs it (SynthPath, noise_mode='device', 1 s reverb), every one
    of the 64 items against the torch-CPU restatement of the reference fed the host-regenerated
    noise of the same call; two consecutive calls (offsets 0 and 1)."""
    from ddsp_pytorch_amd.synth import SynthPath, make_inputs
    inp = make_inputs(64, 200, 100, 65, 512, seed=0, device="cuda", with_noise=False)
    syn = SynthPath(512, 48000, reverb_length=48000, noise_mode="device").cuda()
    seed = 1234
    dd.core.set_noise_seed(seed)
    with torch.no_grad():
        outs = [C(syn(inp["f0"], inp["param"], inp["mags"])) for _ in range(2)]
    rv = tr.Reverb(syn.reverb.noise.detach().cpu(), syn.reverb.decay.detach().cpu(),
                   syn.reverb.wet.detach().cpu(), 48000, 48000)
    f0, param, mags = (inp[k].cpu() for k in ("f0", "param", "mags"))
    # call 0: every item (chunks of 16 bound the oracle's [B, T, H] temporaries); call 1: every 16th
    for k, (out, chunks) in enumerate(zip(outs, ([slice(i, i + 16) for i in range(0, 64, 16)],
                                                 [slice(i, i + 1) for i in range(0, 64, 16)]))):
        noise = host_noise(64, 200, 512, seed, k)
        worst = 0.0
        for sl in chunks:
            ref = tr.synth_path(f0[sl], param[sl], mags[sl], noise[sl], rv, 512, 48000).numpy()
            for i in range(ref.shape[0]):
                worst = max(worst, rms(out[sl][i], ref[i]))
        assert worst < PARITY_RMS, (k, worst)


def test_config5_device_noise_items(dd):
    """Config 5 shard shape (F=400, H=128, |arg| up to ~3.4e6 rad), device noise: 8 items."""
    from ddsp_pytorch_amd.synth import SynthPath, make_inputs
    inp = make_inputs(64, 400, 128, 65, 512, seed=5, device="cuda", with_noise=False)
    syn = SynthPath(512, 48000, reverb_length=48000, noise_mode="device").cuda()
    dd.core.set_noise_seed(99)
    with torch.no_grad():
        out = C(syn(inp["f0"], inp["param"], inp["mags"]))
    rv = tr.Reverb(syn.reverb.noise.detach().cpu(), syn.reverb.decay.detach().cpu(),
                   syn.reverb.wet.detach().cpu(), 48000, 48000)
    noise = host_noise(64, 400, 512, 99, 0)
    sl = slice(0, 64, 8)
    ref = tr.synth_path(inp["f0"].cpu()[sl], inp["param"].cpu()[sl], inp["mags"].cpu()[sl], noise[sl], rv, 512,
                        48000).numpy()
    for i in range(ref.shape[0]):
        assert rms(out[sl][i], ref[i]) < PARITY_RMS, i


# ------------------------------------------------------------------ backward with device noise
def test_synth_frames_grad_device_noise(dd):
    """The backward regenerates the forward's Philox noise (backward.hip): gradients w.r.t. the
    raw projections vs the oracle's autograd fed the host-regenerated noise."""
    B, F, H, NB, bs = 2, 6, 40, 65, 512
    f0, param, mags = controls(B, F, H, NB, 8)
    w = torch.randn(B, F * bs, 1, generator=torch.Generator().manual_seed(9))
    seed = 5150
    dd.core.set_noise_seed(seed)
    dd.core.synth_frames(f0.cuda(), param.cuda(), mags.cuda(), bs, 48000)  # consumes offset 0
    pg, mg = param.cuda().requires_grad_(True), mags.cuda().requires_grad_(True)
    out = dd.core.synth_frames(f0.cuda(), pg, mg, bs, 48000)              # offset 1
    (out * w.cuda()).sum().backward()
    pc, mc = param.clone().requires_grad_(True), mags.clone().requires_grad_(True)
    ref = tr.synth_path_autograd(f0, pc, mc, host_noise(B, F, bs, seed, 1), None, bs, 48000)
    (ref * w).sum().backward()
    assert rms(C(out), ref.detach().numpy()) < 1e-6
    for got, want in ((pg.grad, pc.grad), (mg.grad, mc.grad)):
        e = float((got.cpu().double() - want.double()).norm() / want.double().norm())
        assert e < 1e-5, e


# ------------------------------------------------------------------ config 3: realtime stream
BS, H, NB, N = 256, 64, 65, 1024


def _g8_model(dd, dev):
    g = load_golden("g8_realtime")
    m = dd.DDSPDecoder(int(g["hidden_size"]), int(g["n_harmonic"]), int(g["n_bands"]), 48000,
                       int(g["block_size"]), False)
    m.load_state_dict({k[3:]: torch.as_tensor(v) for k, v in g.items() if k.startswith("sd.")})
    return m.to(dev).eval(), g


def test_scripted_realtime_matches_reference_golden(dd, tmp_path):
    """export.py:33-40 realtime model scripted over torch.ops.ddsp_hip (noise_mode='torch': the
    reference's torch.rand draw): three successive calls vs the reference's own realtime outputs
    (g8: decimation, loudness normalisation, cache_gru carried, decoder.py:56-60), and the GRU
    state after each call."""
    from ddsp_pytorch_amd import script
    m, g = _g8_model(dd, "cuda")
    s = script.export(m, str(tmp_path / "rt.ts"), float(g["mean_loudness"]), float(g["std_loudness"]),
                      realtime=True)
    with torch.no_grad():
        for k in range(3):
            torch.manual_seed(int(g["noise_seeds"][k]))
            y = s(torch.as_tensor(g[f"pitch_{k}"]).cuda(), torch.as_tensor(g[f"loudness_{k}"]).cuda())
            assert y.shape == (1, N, 1)
            assert rms(C(y), g[f"signal_{k}"]) < PARITY_RMS, (k, rms(C(y), g[f"signal_{k}"]))
            np.testing.assert_allclose(C(s.ddsp.decoder.cache_gru), g[f"cache_{k}"], atol=2e-6)


def test_scripted_realtime_device_noise_vs_oracle(dd, tmp_path):
    """The scripted realtime model in device-noise mode: call k draws Philox (0x5EEDDD5B,
    offset k+1); full signal vs torch_ref.realtime_forward with that noise."""
    from ddsp_pytorch_amd import script
    m, g = _g8_model(dd, "cuda")
    sd = {k[3:]: torch.as_tensor(v).clone() for k, v in g.items() if k.startswith("sd.")}
    cache = sd["decoder.cache_gru"].clone()
    s = torch.jit.script(script.ScriptDDSP(m, float(g["mean_loudness"]), float(g["std_loudness"]), realtime=True,
                                           noise_mode="device").eval())
    mean, std = float(g["mean_loudness"]), float(g["std_loudness"])
    with torch.no_grad():
        for k in range(3):
            p, lo = torch.as_tensor(g[f"pitch_{k}"]), torch.as_tensor(g[f"loudness_{k}"])
            y = C(s(p.cuda(), lo.cuda()))
            ref = tr.realtime_forward(sd, p, lo, mean, std, cache, host_noise(1, N // BS, BS, 0x5EEDDD5B, k + 1),
                                      BS, 48000)
            assert rms(y, ref.numpy()) < PARITY_RMS, (k, rms(y, ref.numpy()))


@pytest.mark.parametrize("fused", [False, True])
def test_realtime_graph_full_signal_vs_oracle(dd, fused):
    """RealtimeGraph (HIP-graph replay, device-counter noise: call k = offset k) — the full audio
    of five successive calls vs torch_ref.realtime_forward (export.py:33-40, decoder.py:56-60)
    fed the host-regenerated noise, and the carried GRU state."""
    from ddsp_pytorch_amd.realtime import RealtimeGraph
    m, g = _g8_model(dd, "cuda")
    sd = {k[3:]: torch.as_tensor(v).clone() for k, v in g.items() if k.startswith("sd.")}
    cache = sd["decoder.cache_gru"].clone()
    mean, std, seed = float(g["mean_loudness"]), float(g["std_loudness"]), 0x1234
    rt = RealtimeGraph(m, N, mean, std, seed=seed, fused=fused)
    gen = torch.Generator().manual_seed(31)
    with torch.no_grad():
        for k in range(5):
            pitch = 80.0 * 10.0 ** torch.rand(1, N, 1, generator=gen)
            loud = torch.randn(1, N, 1, generator=gen) - 2.0
            y = rt(pitch, loud).clone()
            ref = tr.realtime_forward(sd, pitch, loud, mean, std, cache, host_noise(1, N // BS, BS, seed, k), BS,
                                      48000)
            assert rms(y.numpy(), ref.numpy()) < PARITY_RMS, (k, rms(y.numpy(), ref.numpy()))
            np.testing.assert_allclose(C(m.decoder.cache_gru), cache.numpy(), atol=1e-5)
