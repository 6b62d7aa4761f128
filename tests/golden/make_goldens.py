"""Generate the golden parity fixtures by running the REFERENCE implementation.

Test infrastructure only.  Run once, in the development container (the reference
is not present on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_goldens.py

It imports hugofloresgarcia/ddsp_pytorch from /root/reference (read-only).  The
reference's ``ddsp/core.py:5-6`` imports ``librosa`` and ``crepe`` and
``ddsp/data.py:5`` imports ``pytorch_lightning``; none is installed and none is
used on the synthesis path, so empty placeholder modules are put in
``sys.modules`` for them (SURVEY.md §8(c) recipe).  Every number written below is
computed by the reference's own functions and modules:

* ``ddsp/core.py:64-176``   scale_function, remove_above_nyquist, upsample,
                             harmonic_synth, amp_to_impulse_response, fft_convolve
* ``ddsp/models/modules.py:7-128``  Reverb, HarmonicSynth, FilteredNoise
* ``ddsp/models/decoder.py:76-136`` DDSPDecoder.forward
* ``ddsp/models/encoder.py:31-103`` DDSPAutoencoder.forward (MFCC encoder + z-conditioned decoder)

Inputs follow SURVEY.md §8(d): f0 = 50*20**U[0,1) Hz, raw controls N(0,1),
noise U[-1,1) drawn by ``torch.rand`` after ``torch.manual_seed(123)``, reverb
parameters drawn after ``torch.manual_seed(1)``.  Only data (inputs and expected
outputs) is written; nothing from the reference's source is stored.
"""
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def import_reference():
    for name in ("librosa", "crepe"):
        sys.modules.setdefault(name, types.ModuleType(name))
    pl = types.ModuleType("pytorch_lightning")
    pl.LightningDataModule = type("LightningDataModule", (), {})
    sys.modules.setdefault("pytorch_lightning", pl)
    sys.path.insert(0, REF)
    import ddsp  # noqa: E402
    from ddsp.models import modules, decoder  # noqa: E402
    return ddsp, modules, decoder


def synth_inputs(seed, B, F, H, NB):
    g = torch.Generator().manual_seed(seed)
    f0 = 50.0 * 20.0 ** torch.rand(B, F, 1, generator=g)
    loudness = torch.randn(B, F, 1, generator=g)
    param = torch.randn(B, F, H + 1, generator=g)
    mags = torch.randn(B, F, NB, generator=g)
    return f0, loudness, param, mags


def save(name, **arrays):
    meta = {
        "torch": torch.__version__,
        "generator": "tests/golden/make_goldens.py",
    }
    arrays = {k: (v.detach().cpu().numpy() if torch.is_tensor(v) else np.asarray(v))
              for k, v in arrays.items()}
    arrays["_meta"] = np.array(repr(meta))
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **arrays)
    print(f"{name}: {os.path.getsize(path) / 1024:.0f} KiB")


@torch.no_grad()
def main():
    torch.set_num_threads(8)
    ddsp, modules, decoder = import_reference()
    sr = 48000

    # ---------------- g0: elementwise / layout functions ----------------
    g = torch.Generator().manual_seed(10)
    x = torch.randn(3, 7, 33, generator=g) * 4.0
    f0 = 50.0 * 20.0 ** torch.rand(3, 7, 1, generator=g)
    amps = torch.rand(3, 7, 33, generator=g)
    up_in = torch.randn(2, 5, 3, generator=g)
    save("g0_elementwise",
         scale_in=x, scale_out=ddsp.scale_function(x),
         nyq_amps=amps, nyq_f0=f0, nyq_out=ddsp.remove_above_nyquist(amps, f0, sr),
         nyq_out_44k=ddsp.remove_above_nyquist(amps, f0, 44100),
         up_in=up_in, up_out_3=ddsp.upsample(up_in, 3), up_out_441=ddsp.upsample(up_in, 441))

    # ---------------- g1: harmonic_synth (core.py:136) ----------------
    # (a) frame-constant controls, small
    f0, _, param, _ = synth_inputs(0, 2, 8, 16, 65)
    hs = modules.HarmonicSynth(64, sr)
    c = hs.get_controls(param[..., :1], param[..., 1:], f0)
    amp_frames = (c["harmonic_distribution"] * c["amplitudes"]).clone()
    out = ddsp.harmonic_synth(ddsp.upsample(f0, 64), ddsp.upsample(amp_frames, 64), sr)
    save("g1_harmonic_small", f0_frames=f0, amp_frames=amp_frames, block_size=64,
         sample_rate=sr, out=out)

    # (b) per-sample f0 (not frame constant) and per-sample amplitudes
    g = torch.Generator().manual_seed(11)
    T = 1000
    t = torch.arange(T, dtype=torch.float32) / sr
    f0s = torch.stack([220.0 + 180.0 * torch.sin(2 * np.pi * 3.0 * t),
                       1500.0 * torch.rand(T, generator=g) + 40.0]).unsqueeze(-1)
    amps = torch.rand(2, T, 16, generator=g) / 16
    save("g1_harmonic_persample", f0=f0s, amps=amps, sample_rate=sr,
         out=ddsp.harmonic_synth(f0s, amps, sr),
         out_44k=ddsp.harmonic_synth(f0s, amps, 44100))

    # (c) configuration-1 shape: B=1, F=200, bs=512, H=100
    f0, _, param, _ = synth_inputs(0, 1, 200, 100, 65)
    hs = modules.HarmonicSynth(512, sr)
    c = hs.get_controls(param[..., :1], param[..., 1:], f0)
    out = hs(**c)  # mutates c['harmonic_distribution'] in place (modules.py:73)
    save("g1_harmonic_full", f0_frames=f0, amp_frames=c["harmonic_distribution"],
         block_size=512, sample_rate=sr, out=out)

    # (d) configuration-5 harmonic count, long signal: B=1, F=400, H=128 -> |arg| ~ 3e6 rad
    f0, _, param, _ = synth_inputs(5, 1, 400, 128, 65)
    f0 = f0.clamp(max=1000.0)
    hs = modules.HarmonicSynth(512, sr)
    c = hs.get_controls(param[..., :1], param[..., 1:], f0)
    out = hs(**c)
    save("g1_harmonic_h128", f0_frames=f0, amp_frames=c["harmonic_distribution"],
         block_size=512, sample_rate=sr, out=out)

    # ---------------- g2: HarmonicSynth controls + forward (modules.py:44-80) ----------------
    f0, _, param, _ = synth_inputs(1, 2, 16, 100, 65)
    hs = modules.HarmonicSynth(512, sr)
    c = hs.get_controls(param[..., :1], param[..., 1:], f0)
    amp_c = c["amplitudes"].clone()
    dist_c = c["harmonic_distribution"].clone()
    out = hs(**c)
    save("g2_controls", param=param, f0=f0, block_size=512, sample_rate=sr,
         amplitudes=amp_c, distribution=dist_c,
         distribution_after_forward=c["harmonic_distribution"], out=out)
    # realtime configuration 3: bs=256, H=64, 4 frames
    f0, _, param, _ = synth_inputs(3, 1, 4, 64, 65)
    hs = modules.HarmonicSynth(256, sr)
    c = hs.get_controls(param[..., :1], param[..., 1:], f0)
    save("g2_controls_rt", param=param, f0=f0, block_size=256, sample_rate=sr, out=hs(**c))

    # ---------------- g3: FilteredNoise (modules.py:101-128, core.py:144-176) ----------------
    _, _, _, mags = synth_inputs(2, 2, 16, 100, 65)
    fn = modules.FilteredNoise(512, 65)
    nc = fn.get_controls(mags)
    ir = ddsp.amp_to_impulse_response(nc["magnitudes"], 512)
    torch.manual_seed(123)
    noise_in = torch.rand(2, 16, 512) * 2 - 1
    torch.manual_seed(123)
    out = fn(**nc)
    conv = ddsp.fft_convolve(noise_in, ir)
    assert torch.equal(conv.reshape(2, -1, 1), out)
    # odd sizes for the function-level boundary
    g = torch.Generator().manual_seed(12)
    amp_odd = torch.rand(3, 5, 17, generator=g)
    sig_odd = torch.randn(4, 100, generator=g)
    ker_odd = torch.randn(4, 100, generator=g)
    save("g3_noise", mags=mags, block_size=512, magnitudes=nc["magnitudes"], impulse=ir,
         noise_in=noise_in, out=out,
         amp_odd=amp_odd, ir_odd_40=ddsp.amp_to_impulse_response(amp_odd, 40),
         ir_odd_20=ddsp.amp_to_impulse_response(amp_odd, 20),
         sig_odd=sig_odd, ker_odd=ker_odd, conv_odd=ddsp.fft_convolve(sig_odd, ker_odd))

    # ---------------- g4: Reverb (modules.py:7-35) ----------------
    for tag, L, T, B in (("small", 4800, 9600, 2), ("1s", 48000, 102400, 1), ("crop", 48000, 24000, 1)):
        torch.manual_seed(1)
        rv = modules.Reverb(L, sr)
        g = torch.Generator().manual_seed(13)
        x = torch.randn(B, T, 1, generator=g) * 0.3
        save(f"g4_reverb_{tag}", length=L, sample_rate=sr, noise=rv.noise, decay=rv.decay,
             wet=rv.wet, impulse=rv.build_impulse(), x=x, out=rv(x))
    # non-default wet/decay
    torch.manual_seed(1)
    rv = modules.Reverb(4800, sr, initial_wet=1.5, initial_decay=2.0)
    g = torch.Generator().manual_seed(14)
    x = torch.randn(2, 9600, 1, generator=g) * 0.3
    save("g4_reverb_wet", length=4800, sample_rate=sr, noise=rv.noise, decay=rv.decay, wet=rv.wet,
         impulse=rv.build_impulse(), x=x, out=rv(x))

    # ---------------- g5: DDSPDecoder.forward (decoder.py:101) ----------------
    torch.manual_seed(0)
    model = decoder.DDSPDecoder(32, 100, 65, sr, 512, True).eval()
    f0, loudness, _, _ = synth_inputs(4, 1, 16, 100, 65)
    torch.manual_seed(123)
    o = model({"pitch": f0, "loudness": loudness})
    sd = {"sd." + k: v for k, v in model.state_dict().items()}
    save("g5_decoder", hidden_size=32, n_harmonic=100, n_bands=65, sample_rate=sr,
         block_size=512, pitch=f0, loudness=loudness, signal=o["signal"], noise=o["noise"],
         harmonic_audio=o["harmonic_audio"],
         amplitudes=o["harmonic_ctrls"]["amplitudes"],
         distribution=o["harmonic_ctrls"]["harmonic_distribution"],
         magnitudes=o["noise_ctrls"]["magnitudes"], **sd)

    grad_goldens(ddsp, decoder, modules, sr)
    realtime_goldens(decoder, sr)
    autoencoder_golden(sr)
    decoder512_golden(sr)
    autoencoder512_golden(sr)
    grad512_golden(sr)


@torch.no_grad()
def realtime_goldens(decoder, sr):
    # ---------------- g8: the realtime stream (config 3) ----------------
    # export.py:33-40 ScriptDDSP.forward(realtime=True) on successive 1024-sample calls: loudness
    # normalised with the stored mean/std, pitch and loudness decimated by block_size, then the
    # model's realtime_forward (decoder.py:138-158).  That method reads `self.proj_matrices`, which
    # the fork's DDSPDecoder never defines; the projections it names are
    # harmonic_proj / noise_proj (decoder.py:87-88), used here.  Everything else is the
    # reference's own modules: GRUDecoder.forward(realtime=True) carrying cache_gru
    # (decoder.py:56-60), HarmonicSynth, FilteredNoise (its torch.rand draw seeded per call).
    bs, H, N, mean, std = 256, 64, 1024, -3.0, 1.5
    torch.manual_seed(0)
    model = decoder.DDSPDecoder(64, H, 65, sr, bs, False).eval()
    g = torch.Generator().manual_seed(18)
    model.decoder.cache_gru.copy_(torch.randn(1, 1, 64, generator=g) * 0.1)
    sd = {"sd." + k: v.clone() for k, v in model.state_dict().items()}
    calls = {}
    for k in range(3):
        pitch = 80.0 * 10.0 ** torch.rand(1, N, 1, generator=g)
        loud = torch.randn(1, N, 1, generator=g) - 2.0
        p = pitch[:, ::bs]
        lo = ((loud - mean) / std)[:, ::bs]
        hidden = model.decoder(p, lo, realtime=True)
        param = model.harmonic_proj(hidden)
        hc = model.harmonic_synth.get_controls(param[..., :1], param[..., 1:], p)
        harmonic = model.harmonic_synth(**hc)
        nc = model.noise_synth.get_controls(model.noise_proj(hidden))
        torch.manual_seed(200 + k)
        noise_in = torch.rand(1, N // bs, bs) * 2 - 1  # the draw FilteredNoise.forward makes next
        torch.manual_seed(200 + k)
        noise = model.noise_synth(**nc)
        calls.update({f"pitch_{k}": pitch, f"loudness_{k}": loud, f"noise_in_{k}": noise_in,
                      f"signal_{k}": harmonic + noise, f"harmonic_{k}": harmonic,
                      f"cache_{k}": model.decoder.cache_gru.clone()})
    save("g8_realtime", hidden_size=64, n_harmonic=H, n_bands=65, sample_rate=sr, block_size=bs,
         mean_loudness=mean, std_loudness=std, noise_seeds=np.array([200, 201, 202]), **calls, **sd)


@torch.enable_grad()
def grad_goldens(ddsp, decoder, modules, sr):
    # ---------------- g6: gradients (train.py:84-130 back-propagates through the path) ----------------
    # loss = sum(signal * w) with a fixed random w, so d loss / d signal = w exactly.
    torch.manual_seed(0)
    model = decoder.DDSPDecoder(32, 100, 65, sr, 512, True)
    acts = {}

    def keep(name):
        def hook(mod, inp, out):
            out.retain_grad()
            acts[name] = out
        return hook

    model.harmonic_proj.register_forward_hook(keep("param"))
    model.noise_proj.register_forward_hook(keep("mags"))
    f0, loudness, _, _ = synth_inputs(4, 1, 16, 100, 65)
    torch.manual_seed(123)
    o = model({"pitch": f0, "loudness": loudness})
    w = torch.randn(o["signal"].shape, generator=torch.Generator().manual_seed(15))
    (o["signal"] * w).sum().backward()
    grads = {"grad." + k: v.grad for k, v in model.named_parameters() if v.grad is not None}
    sd = {"sd." + k: v for k, v in model.state_dict().items()}
    save("g6_grad_decoder", hidden_size=32, n_harmonic=100, n_bands=65, sample_rate=sr, block_size=512,
         pitch=f0, loudness=loudness, weight=w, signal=o["signal"].detach(),
         param=acts["param"].detach(), mags=acts["mags"].detach(),
         grad_param=acts["param"].grad, grad_mags=acts["mags"].grad, **grads, **sd)
    # reverb alone, incl. the crop case (L > T)
    for tag, L, T, B in (("small", 4800, 9600, 3), ("crop", 48000, 24000, 1)):
        torch.manual_seed(1)
        rv = modules.Reverb(L, sr, initial_wet=0.5, initial_decay=3.0)
        g = torch.Generator().manual_seed(16)
        x = (torch.randn(B, T, 1, generator=g) * 0.3).requires_grad_(True)
        out = rv(x)
        w = torch.randn(out.shape, generator=g)
        (out * w).sum().backward()
        save(f"g6_grad_reverb_{tag}", length=L, sample_rate=sr, noise=rv.noise.detach(), decay=rv.decay.detach(),
             wet=rv.wet.detach(), x=x.detach(), weight=w, out=out.detach(), grad_x=x.grad,
             grad_noise=rv.noise.grad, grad_decay=rv.decay.grad, grad_wet=rv.wet.grad)

    # ---------------- g7: the training loss (core.py:27-41 multiscale_fft, train.py:70-76) ----------------
    g = torch.Generator().manual_seed(17)
    sig = torch.randn(2, 8192, generator=g) * 0.3
    rec = (sig + 0.1 * torch.randn(2, 8192, generator=g)).requires_grad_(True)
    scales, overlap = [4096, 2048, 1024, 512, 256, 128], 0.75
    ori_stft = ddsp.core.multiscale_fft(sig, scales, overlap)
    rec_stft = ddsp.core.multiscale_fft(rec, scales, overlap)
    loss = 0
    for s_x, s_y in zip(ori_stft, rec_stft):  # train.py:70-76
        loss = loss + (s_x - s_y).abs().mean() + (ddsp.core.safe_log(s_x) - ddsp.core.safe_log(s_y)).abs().mean()
    loss.backward()
    save("g7_stft_loss", sig=sig, rec=rec.detach(), scales=np.array(scales), overlap=overlap, loss=loss.detach(),
         grad_rec=rec.grad, **{f"stft_{s}": m.detach() for s, m in zip(scales, rec_stft)})
    masked_loss_golden(ddsp)


@torch.no_grad()
def autoencoder_golden(sr):
    """g9: the reference's second caller of the path, DDSPAutoencoder.forward (encoder.py:63-103): the
    MFCC encoder (LayerNorm -> GRU -> Linear to z, encoder.py:12-28), the z-conditioned GRUDecoder
    (decoder.py:11-66), then the same synthesis section as DDSPDecoder.forward.  Small hidden size,
    seeded; the MFCCs are an input tensor (the encoder needs no librosa)."""
    from ddsp.models import encoder
    torch.manual_seed(0)
    model = encoder.DDSPAutoencoder(32, 100, 65, sr, 512, True).eval()
    f0, loudness, _, _ = synth_inputs(9, 2, 16, 100, 65)
    mfcc = torch.randn(2, 16, 30, generator=torch.Generator().manual_seed(19)) * 10.0
    torch.manual_seed(123)
    noise_in = torch.rand(2, 16, 512) * 2 - 1  # the draw FilteredNoise.forward makes next
    torch.manual_seed(123)
    o = model({"pitch": f0, "loudness": loudness, "mfcc": mfcc})
    sd = {"sd." + k: v for k, v in model.state_dict().items()}
    save("g9_autoencoder", hidden_size=32, n_harmonic=100, n_bands=65, sample_rate=sr, block_size=512,
         pitch=f0, loudness=loudness, mfcc=mfcc, noise_in=noise_in, signal=o["signal"], noise=o["noise"],
         harmonic_audio=o["harmonic_audio"], z=o["z"],
         amplitudes=o["harmonic_ctrls"]["amplitudes"],
         distribution=o["harmonic_ctrls"]["harmonic_distribution"],
         magnitudes=o["noise_ctrls"]["magnitudes"], **sd)


def state_dict_crcs(model):
    """Per-tensor CRC32 of the state_dict's raw bytes (and shape): the fixture pins the parameters a
    seeded constructor draws without storing them (4.3 M floats at the shipped hidden size)."""
    import zlib
    out = {}
    for k, v in model.state_dict().items():
        a = np.ascontiguousarray(v.detach().cpu().numpy())
        out["crc." + k] = np.uint32(zlib.crc32(a.tobytes()))
        out["shape." + k] = np.asarray(a.shape, dtype=np.int64)
    return out


@torch.no_grad()
def decoder512_golden(sr):
    """g10: DDSPDecoder at the reference's shipped network size (config.yaml:16-21: hidden 512,
    n_harmonic 64, n_bands 65, block 512, reverb on), built after torch.manual_seed(0), forward on
    B=2, F=24 with the noise drawn after manual_seed(123).  The state_dict is stored as per-tensor
    CRC32s only: the test rebuilds the module under the same seed and checks them.  At this size the
    GPU route runs the H=512 GRU step kernel, the 512-wide MLP blocks and the projection kernel."""
    from ddsp.models import decoder
    torch.manual_seed(0)
    model = decoder.DDSPDecoder(512, 64, 65, sr, 512, True).eval()
    f0, loudness, _, _ = synth_inputs(20, 2, 24, 64, 65)
    torch.manual_seed(123)
    noise_in = torch.rand(2, 24, 512) * 2 - 1  # the draw FilteredNoise.forward makes next
    torch.manual_seed(123)
    o = model({"pitch": f0, "loudness": loudness})
    save("g10_decoder512", hidden_size=512, n_harmonic=64, n_bands=65, sample_rate=sr, block_size=512,
         model_seed=0, noise_seed=123, pitch=f0, loudness=loudness, noise_in=noise_in,
         signal=o["signal"], noise=o["noise"], harmonic_audio=o["harmonic_audio"],
         amplitudes=o["harmonic_ctrls"]["amplitudes"],
         distribution=o["harmonic_ctrls"]["harmonic_distribution"],
         magnitudes=o["noise_ctrls"]["magnitudes"], **state_dict_crcs(model))


@torch.no_grad()
def autoencoder512_golden(sr):
    """g9b: DDSPAutoencoder (encoder.py:29-103) at hidden 512, seeded like g10, B=2, F=16; the
    state_dict as CRC32s.  Reaches the 30-input encoder GRU and the z-conditioned decoder GRU
    (input 3H) on the step kernels, z_mlp's K=16 block and out_mlp's extras path."""
    from ddsp.models import encoder
    torch.manual_seed(0)
    model = encoder.DDSPAutoencoder(512, 100, 65, sr, 512, True).eval()
    f0, loudness, _, _ = synth_inputs(21, 2, 16, 100, 65)
    mfcc = torch.randn(2, 16, 30, generator=torch.Generator().manual_seed(22)) * 10.0
    torch.manual_seed(123)
    o = model({"pitch": f0, "loudness": loudness, "mfcc": mfcc})
    save("g9b_autoencoder512", hidden_size=512, n_harmonic=100, n_bands=65, sample_rate=sr, block_size=512,
         model_seed=0, noise_seed=123, pitch=f0, loudness=loudness, mfcc=mfcc, signal=o["signal"],
         noise=o["noise"], harmonic_audio=o["harmonic_audio"], z=o["z"],
         amplitudes=o["harmonic_ctrls"]["amplitudes"],
         distribution=o["harmonic_ctrls"]["harmonic_distribution"],
         magnitudes=o["noise_ctrls"]["magnitudes"], **state_dict_crcs(model))


@torch.enable_grad()
def grad512_golden(sr):
    """g6b: the reference's autograd through DDSPDecoder at the shipped size (hidden 512, 64 harmonics),
    B=2, F=8, loss = sum(signal * w).  Stored: the gradients at the two projections' outputs in full, and
    per parameter the gradient's L2 norm plus 2048 entries at seeded indices (every entry for tensors of
    at most 2048 elements) — enough to pin each gradient without storing 4.3 M floats."""
    from ddsp.models import decoder
    torch.manual_seed(0)
    model = decoder.DDSPDecoder(512, 64, 65, sr, 512, True)
    acts = {}

    def keep(name):
        def hook(mod, inp, out):
            out.retain_grad()
            acts[name] = out
        return hook

    model.harmonic_proj.register_forward_hook(keep("param"))
    model.noise_proj.register_forward_hook(keep("mags"))
    f0, loudness, _, _ = synth_inputs(23, 2, 8, 64, 65)
    torch.manual_seed(123)
    o = model({"pitch": f0, "loudness": loudness})
    w = torch.randn(o["signal"].shape, generator=torch.Generator().manual_seed(24))
    (o["signal"] * w).sum().backward()
    arrays = {}
    gi = torch.Generator().manual_seed(25)
    for k, v in model.named_parameters():
        if v.grad is None:
            continue
        flat = v.grad.reshape(-1)
        if flat.numel() <= 2048:
            idx = torch.arange(flat.numel())
        else:
            idx = torch.randperm(flat.numel(), generator=gi)[:2048].sort().values
        arrays["gidx." + k] = idx.to(torch.int32)
        arrays["gval." + k] = flat[idx]
        arrays["gnorm." + k] = flat.double().norm()
    save("g6b_grad_decoder512", hidden_size=512, n_harmonic=64, n_bands=65, sample_rate=sr, block_size=512,
         model_seed=0, noise_seed=123, pitch=f0, loudness=loudness, weight=w, signal=o["signal"].detach(),
         grad_param=acts["param"].grad, grad_mags=acts["mags"].grad, **arrays, **state_dict_crcs(model))


def masked_loss_golden(ddsp):
    """g7b: train.py:70-76's loss restricted to the well-conditioned bins, on g7's signals, computed by
    the reference's multiscale_fft / safe_log (core.py:10-41) in fp32 with autograd.  The bins with
    |X| or |Y| below 1 % of their spectrogram's RMS (0.14 % of the bins; mask from the reference's own
    fp64 magnitudes) are where the log-L1 term's 1/(|Y| + 1e-7) weight makes the fp32 gradient
    ill-conditioned; on the rest the reference's fp32 gradient is within 3e-6 of its fp64 one, so a
    kernel gradient can be held to 1e-5 against this fixture."""
    g7 = np.load(os.path.join(OUT, "g7_stft_loss.npz"))
    sig, rec0 = torch.as_tensor(g7["sig"]), torch.as_tensor(g7["rec"])
    scales, overlap = [int(v) for v in g7["scales"]], float(g7["overlap"])
    ori64 = ddsp.core.multiscale_fft(sig.double(), scales, overlap)
    my64 = ddsp.core.multiscale_fft(rec0.double(), scales, overlap)
    masks = []
    for mx, my in zip(ori64, my64):
        floor = 1e-2 * float(my.pow(2).mean().sqrt())
        masks.append(((my > floor) & (mx > floor)).float())
    rec = rec0.clone().requires_grad_(True)
    ori_stft = ddsp.core.multiscale_fft(sig, scales, overlap)
    rec_stft = ddsp.core.multiscale_fft(rec, scales, overlap)
    loss = 0
    for m, s_x, s_y in zip(masks, ori_stft, rec_stft):
        loss = loss + (m * (s_x - s_y).abs()).mean() + (m * (ddsp.core.safe_log(s_x) - ddsp.core.safe_log(s_y)).abs()).mean()
    loss.backward()
    save("g7b_stft_loss_masked", loss=loss.detach(), grad_rec=rec.grad,
         **{f"mask_{s}": m.to(torch.uint8) for s, m in zip(scales, masks)})


if __name__ == "__main__":
    if sys.argv[1:] == ["g8"]:  # only the realtime fixture
        torch.set_num_threads(8)
        realtime_goldens(import_reference()[2], 48000)
    elif sys.argv[1:] == ["g9"]:  # only the autoencoder fixture
        torch.set_num_threads(8)
        import_reference()
        autoencoder_golden(48000)
    elif sys.argv[1:] == ["g7b"]:  # only the masked-loss fixture (reads g7)
        torch.set_num_threads(8)
        masked_loss_golden(import_reference()[0])
    elif sys.argv[1:] == ["g10"]:  # only the shipped-size fixtures (g10, g9b, g6b)
        torch.set_num_threads(8)
        import_reference()
        decoder512_golden(48000)
        autoencoder512_golden(48000)
        grad512_golden(48000)
    else:
        main()
