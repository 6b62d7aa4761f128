"""CPU oracle (numpy restatement) of the ddsp_pytorch harmonic-plus-noise synthesis path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker.  The product path (``ddsp_pytorch_amd``) never imports or calls it.

Parity is pinned: ``tests/test_oracle.py`` checks every function here against the
golden vectors in ``tests/golden/`` that ``tests/golden/make_goldens.py`` produced
by running the reference itself (hugofloresgarcia/ddsp_pytorch, torch 2.10 CPU).

The restatement spells out the reference's fp32 arithmetic explicitly
(SURVEY.md Appendix A):

* phase increment ``inc = fl32(fl32(fl32(2*pi) * f0) / sr)`` (true fp32 division);
* phase ``omega = fl32(sum_{s<=t} inc[s])`` accumulated in float64 — for the
  pitch ranges of audio the float64 partial sums are exact, so order is free;
* argument ``fl32(omega * k)``, k = 1..H; sine of that fp32 value (here: float64
  ``sin`` rounded, i.e. correctly rounded — the reference's SLEEF ``sinf`` is
  within 6e-8 of it);
* amplitude-weighted sum over harmonics.

Citations are ``file:line`` in /root/reference.
"""
import math

import numpy as np

f32 = np.float32
TWO_PI_F32 = f32(2.0 * math.pi)          # python float scalar cast to fp32 by ATen
LN10_F32 = f32(math.log(10.0))


# ----------------------------------------------------------------------------
# ddsp/core.py
# ----------------------------------------------------------------------------
def scale_function(x):
    """ddsp/core.py:77-78  ``2 * sigmoid(x) ** ln(10) + 1e-7`` (fp32 at every step)."""
    x = np.asarray(x, dtype=f32)
    sig = (1.0 / (1.0 + np.exp(-x.astype(np.float64)))).astype(f32)
    p = np.power(sig.astype(np.float64), float(LN10_F32)).astype(f32)
    return (f32(2.0) * p + f32(1e-7)).astype(f32)


def remove_above_nyquist(amplitudes, f0, sample_rate):
    """ddsp/core.py:70-74  multiply by fl32(1+1e-4) below Nyquist, by fl32(1e-4) at/above."""
    amplitudes = np.asarray(amplitudes, dtype=f32)
    f0 = np.asarray(f0, dtype=f32)
    n_harm = amplitudes.shape[-1]
    pitches = f0 * np.arange(1, n_harm + 1, dtype=f32)           # fp32 product
    below = pitches < f32(sample_rate / 2)
    aa = np.where(below, f32(1.0) + f32(1e-4), f32(0.0) + f32(1e-4)).astype(f32)
    return (amplitudes * aa).astype(f32)


def upsample(signal, factor):
    """ddsp/core.py:64-67  nearest interpolation to F*factor == repeat along time."""
    return np.repeat(np.asarray(signal, dtype=f32), int(factor), axis=1)


def phase_increment(f0, sample_rate):
    """fp32 increment of ddsp/core.py:138: ``2 * math.pi * f0 / sample_rate``."""
    f0 = np.asarray(f0, dtype=f32)
    return ((TWO_PI_F32 * f0).astype(f32) / f32(sample_rate)).astype(f32)


def phase(f0, sample_rate):
    """ddsp/core.py:138  cumsum over time, float64 accumulator, fp32 result."""
    inc = phase_increment(f0, sample_rate)
    return np.cumsum(inc.astype(np.float64), axis=1).astype(f32)


def harmonic_synth(f0, amplitudes, sample_rate, chunk=1 << 16):
    """ddsp/core.py:136-141  additive oscillator bank, f0 [B,T,1], amplitudes [B,T,H] -> [B,T,1]."""
    amplitudes = np.asarray(amplitudes, dtype=f32)
    omega = phase(f0, sample_rate)                               # [B,T,1] fp32
    H = amplitudes.shape[-1]
    k = np.arange(1, H + 1, dtype=f32)
    B, T = omega.shape[:2]
    out = np.empty((B, T, 1), dtype=f32)
    for s in range(0, T, chunk):
        w = omega[:, s:s + chunk]
        arg = (w * k).astype(f32)                                # fl32(omega * k)
        sn = np.sin(arg.astype(np.float64))
        out[:, s:s + chunk, 0] = (sn * amplitudes[:, s:s + chunk].astype(np.float64)).sum(-1)
    return out


def harmonic_synth_frames(f0_frames, amp_frames, block_size, sample_rate):
    """harmonic_synth(upsample(f0), upsample(amps)) without materialising [B,T,H]."""
    return harmonic_synth(upsample(f0_frames, block_size), upsample(amp_frames, block_size),
                          sample_rate)


def hann_window(n):
    """torch.hann_window(n) (periodic): 0.5 - 0.5*cos(2*pi*m/n)."""
    m = np.arange(n, dtype=np.float64)
    return 0.5 - 0.5 * np.cos(2.0 * np.pi * m / n)


def amp_to_impulse_response(amp, target_size):
    """ddsp/core.py:144-166  zero-phase FIR from real magnitudes: irfft, roll, Hann, pad, roll."""
    amp = np.asarray(amp, dtype=np.float64)
    impulse = np.fft.irfft(amp, axis=-1)                         # n = 2*(NB-1)
    n = impulse.shape[-1]
    impulse = np.roll(impulse, n // 2, axis=-1)
    impulse = impulse * hann_window(n)
    target = int(target_size)
    if target >= n:
        pad = [(0, 0)] * (impulse.ndim - 1) + [(0, target - n)]
        impulse = np.pad(impulse, pad)
    else:                                                        # F.pad with a negative pad crops
        impulse = impulse[..., :target]
    impulse = np.roll(impulse, -n // 2, axis=-1)
    return impulse.astype(f32)


def fft_convolve(signal, kernel):
    """ddsp/core.py:169-176  causal linear convolution truncated to N: y[n] = sum_{m<=n} s[m] k[n-m]."""
    signal = np.asarray(signal, dtype=np.float64)
    kernel = np.asarray(kernel, dtype=np.float64)
    N = signal.shape[-1]
    nfft = 1 << int(math.ceil(math.log2(2 * N)))
    S = np.fft.rfft(signal, nfft, axis=-1)
    K = np.fft.rfft(kernel, nfft, axis=-1)
    return np.fft.irfft(S * K, nfft, axis=-1)[..., :N].astype(f32)


# ----------------------------------------------------------------------------
# ddsp/models/modules.py
# ----------------------------------------------------------------------------
def reverb_build_impulse(noise, decay, wet, length, sample_rate):
    """ddsp/models/modules.py:21-26 (t buffer from modules.py:17-19)."""
    noise = np.asarray(noise, dtype=f32).reshape(1, -1, 1)
    t = (np.arange(length, dtype=np.float64) / sample_rate).astype(f32).reshape(1, -1, 1)
    softplus = np.log1p(np.exp(-float(decay)))                   # softplus(-decay)
    env = np.exp(-(f32(softplus) * t).astype(f32).astype(np.float64) * 500.0).astype(f32)
    sig = f32(1.0 / (1.0 + math.exp(-float(wet))))
    imp = ((noise * env).astype(f32) * sig).astype(f32)
    imp[:, 0] = 1.0
    return imp


def reverb(x, impulse):
    """ddsp/models/modules.py:28-35  pad/crop the IR to len(x), then fft_convolve."""
    x = np.asarray(x, dtype=f32)
    lenx = x.shape[1]
    h = np.asarray(impulse, dtype=f32).reshape(-1)
    if h.shape[0] >= lenx:
        h = h[:lenx]
    else:
        h = np.pad(h, (0, lenx - h.shape[0]))
    return fft_convolve(x[..., 0], h[None, :])[..., None]


def harmonic_get_controls(amplitudes, harmonic_distribution, f0, sample_rate):
    """ddsp/models/modules.py:44-67."""
    amplitudes = scale_function(amplitudes)
    dist = scale_function(harmonic_distribution)
    dist = remove_above_nyquist(dist, f0, sample_rate)
    dist = (dist / dist.astype(np.float64).sum(-1, keepdims=True).astype(f32)).astype(f32)
    return {"f0": np.asarray(f0, dtype=f32), "harmonic_distribution": dist,
            "amplitudes": amplitudes}


def harmonic_forward(amplitudes, harmonic_distribution, f0, block_size, sample_rate):
    """ddsp/models/modules.py:69-80 (returns audio, plus dist*amps as the in-place side effect)."""
    dist = (np.asarray(harmonic_distribution, dtype=f32) * np.asarray(amplitudes, dtype=f32)).astype(f32)
    return harmonic_synth_frames(f0, dist, block_size, sample_rate), dist


def noise_get_controls(magnitudes, initial_bias=-5.0):
    """ddsp/models/modules.py:111-114."""
    return {"magnitudes": scale_function(np.asarray(magnitudes, dtype=f32) + f32(initial_bias))}


def noise_forward(magnitudes, noise, block_size):
    """ddsp/models/modules.py:116-128 with the U[-1,1) noise tensor injected."""
    ir = amp_to_impulse_response(magnitudes, block_size)
    out = fft_convolve(noise, ir)
    return out.reshape(out.shape[0], -1, 1)
