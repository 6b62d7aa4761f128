"""Torch-CPU restatement of the reference synthesis path (the "port" CPU baseline).

TEST INFRASTRUCTURE ONLY.  Used by ``tests/`` as a large-size checker and by
``bench.py``'s ``cpu_baseline`` leg to time the reference's algorithm on the GPU
box's host cores (the reference itself never travels to the box).  The product
path never imports it.

It issues the same ATen operator sequence as the reference on CPU tensors, so on
the golden vectors it is bit-exact with the reference (``tests/test_oracle.py``).
Each function cites the reference line it restates.
"""
import math

import torch
import torch.nn.functional as F


def scale_function(x):
    # ddsp/core.py:77-78
    return 2 * torch.sigmoid(x) ** (math.log(10)) + 1e-7


def remove_above_nyquist(amplitudes, f0, sample_rate):
    # ddsp/core.py:70-74
    k = torch.arange(1, amplitudes.shape[-1] + 1).to(f0)
    mask = (f0 * k < sample_rate / 2).float() + 1e-4
    return amplitudes * mask


def upsample(signal, factor):
    # ddsp/core.py:64-67: nearest interpolation along time
    y = F.interpolate(signal.permute(0, 2, 1), size=signal.shape[1] * factor)
    return y.permute(0, 2, 1)


def harmonic_synth(f0, amplitudes, sample_rate):
    # ddsp/core.py:136-141
    omega = torch.cumsum(2 * math.pi * f0 / sample_rate, 1)
    k = torch.arange(1, amplitudes.shape[-1] + 1).to(omega)
    return (torch.sin(omega * k) * amplitudes).sum(-1, keepdim=True)


def amp_to_impulse_response(amp, target_size):
    # ddsp/core.py:144-166
    spec = torch.view_as_complex(torch.stack([amp, torch.zeros_like(amp)], -1))
    h = torch.fft.irfft(spec)
    n = h.shape[-1]
    h = torch.roll(h, n // 2, -1) * torch.hann_window(n, dtype=h.dtype)
    h = F.pad(h, (0, int(target_size) - int(n)))
    return torch.roll(h, -n // 2, -1)


def fft_convolve(signal, kernel):
    # ddsp/core.py:169-176
    s = F.pad(signal, (0, signal.shape[-1]))
    k = F.pad(kernel, (kernel.shape[-1], 0))
    y = torch.fft.irfft(torch.fft.rfft(s) * torch.fft.rfft(k))
    return y[..., y.shape[-1] // 2:]


class Reverb:
    """ddsp/models/modules.py:7-35 (parameters passed in explicitly)."""

    def __init__(self, noise, decay, wet, length, sample_rate):
        self.noise, self.decay, self.wet = noise, decay, wet
        self.length = length
        self.t = (torch.arange(length) / sample_rate).reshape(1, -1, 1)

    def build_impulse(self):
        env = torch.exp(-F.softplus(-self.decay) * self.t * 500)
        imp = self.noise * env * torch.sigmoid(self.wet)
        imp[:, 0] = 1
        return imp

    def __call__(self, x):
        imp = F.pad(self.build_impulse(), (0, 0, 0, x.shape[1] - self.length))
        return fft_convolve(x.squeeze(-1), imp.squeeze(-1)).unsqueeze(-1)


def harmonic_controls(amplitudes, dist, f0, sample_rate):
    # ddsp/models/modules.py:44-67
    amplitudes = scale_function(amplitudes)
    dist = remove_above_nyquist(scale_function(dist), f0, sample_rate)
    dist /= dist.sum(-1, keepdim=True)
    return amplitudes, dist


def harmonic_forward(amplitudes, dist, f0, block_size, sample_rate):
    # ddsp/models/modules.py:69-80
    dist *= amplitudes
    return harmonic_synth(upsample(f0, block_size), upsample(dist, block_size), sample_rate)


def noise_forward(magnitudes, noise, block_size):
    # ddsp/models/modules.py:111-128 (controls already scaled; noise injected)
    ir = amp_to_impulse_response(magnitudes, block_size)
    y = fft_convolve(noise, ir).contiguous()
    return y.reshape(y.shape[0], -1, 1)


def synth_path_autograd(f0, param, mags, noise, reverb, block_size, sample_rate):
    """Frame-rate controls -> audio: the synthesis section of ddsp/models/decoder.py:106-125,
    differentiable (the gradient checker for the backward kernels)."""
    amp, dist = harmonic_controls(param[..., :1], param[..., 1:], f0, sample_rate)
    harmonic = harmonic_forward(amp, dist, f0, block_size, sample_rate)
    mags = scale_function(mags + (-5.0))
    noise_audio = noise_forward(mags, noise, block_size)
    signal = harmonic + noise_audio
    if reverb is not None:
        signal = reverb(signal)
    return signal


synth_path = torch.no_grad()(synth_path_autograd)
synth_path.__doc__ = "synth_path_autograd under torch.no_grad() (the CPU baseline's forward)."


def safe_log(x):
    # ddsp/core.py:10-11
    return torch.log(x + 1e-7)


def multiscale_fft(signal, scales, overlap):
    # ddsp/core.py:27-41
    out = []
    for s in scales:
        S = torch.stft(signal, s, int(s * (1 - overlap)), s, torch.hann_window(s).to(signal), True,
                       normalized=True, return_complex=True).abs()
        out.append(S)
    return out


def multiscale_spec_loss(ori_stft, rec_stft):
    # train.py:70-76
    loss = 0
    for s_x, s_y in zip(ori_stft, rec_stft):
        loss = loss + (s_x - s_y).abs().mean() + (safe_log(s_x) - safe_log(s_y)).abs().mean()
    return loss


# ---------------------------------------------------------------- the control network (decoder.py)
# Restated over a plain state_dict (the reference's keys), so the checker shares no code with
# the product's modules.

def mlp_forward(sd, prefix, x):
    # ddsp/core.py:122-129: (Linear, LayerNorm, LeakyReLU) x 3 -> Sequential indices 0..8
    for i in (0, 3, 6):
        x = F.linear(x, sd[f"{prefix}.{i}.weight"], sd[f"{prefix}.{i}.bias"])
        x = F.layer_norm(x, (x.shape[-1],), sd[f"{prefix}.{i + 1}.weight"], sd[f"{prefix}.{i + 1}.bias"])
        x = F.leaky_relu(x)
    return x


def gru_forward(sd, prefix, x, h0):
    # ddsp/core.py:132-133: nn.GRU(2 * hidden, hidden, batch_first=True) — torch's CPU GRU
    hidden = sd[f"{prefix}.weight_hh_l0"].shape[1]
    g = torch.nn.GRU(x.shape[-1], hidden, batch_first=True)
    g.load_state_dict({k: sd[f"{prefix}.{k}"] for k in ("weight_ih_l0", "weight_hh_l0", "bias_ih_l0",
                                                         "bias_hh_l0")})
    return g(x, h0) if h0 is not None else g(x)


def gru_decoder_forward(sd, f0, loudness, cache=None):
    """ddsp/models/decoder.py:43-68 (z_dim=None).  With ``cache`` ([1,1,hidden], updated in
    place) the realtime branch of decoder.py:56-60: the GRU starts from and writes back the
    cached state."""
    hidden = torch.cat([mlp_forward(sd, "decoder.f0_mlp", f0), mlp_forward(sd, "decoder.loudness_mlp", loudness)],
                       -1)
    if cache is not None:
        gru_out, h = gru_forward(sd, "decoder.gru", hidden, cache)
        cache.copy_(h)
    else:
        gru_out = gru_forward(sd, "decoder.gru", hidden, None)[0]
    return mlp_forward(sd, "decoder.out_mlp", torch.cat([gru_out, f0, loudness], -1))


@torch.no_grad()
def decoder_synthesis(sd, f0, hidden, noise, block_size, sample_rate, reverb=None):
    """ddsp/models/decoder.py:106-125 (and realtime_forward, decoder.py:138-158, with reverb=None):
    projections, both synths with injected noise, the sum, the optional reverb.  Returns
    (signal, harmonic, filtered noise)."""
    param = F.linear(hidden, sd["harmonic_proj.weight"], sd["harmonic_proj.bias"])
    amp, dist = harmonic_controls(param[..., :1], param[..., 1:], f0, sample_rate)
    harmonic = harmonic_forward(amp, dist, f0, block_size, sample_rate)
    mags = scale_function(F.linear(hidden, sd["noise_proj.weight"], sd["noise_proj.bias"]) + (-5.0))
    noise_audio = noise_forward(mags, noise, block_size)
    signal = harmonic + noise_audio
    if reverb is not None:
        signal = reverb(signal)
    return signal, harmonic, noise_audio


@torch.no_grad()
def realtime_forward(sd, pitch, loudness, mean, std, cache, noise, block_size, sample_rate):
    """export.py:33-40 ScriptDDSP.forward with realtime=True on a [1, N, 1] call: loudness
    normalised, both inputs decimated by block_size ([:, ::block_size]), GRU on the cached
    state (decoder.py:56-60, ``cache`` updated in place), harmonic + noise, no reverb
    (decoder.py:138-158).  ``noise`` is the call's [1, N / block_size, block_size] U[-1,1)."""
    loudness = (loudness - mean) / std
    pitch = pitch[:, ::block_size]
    loudness = loudness[:, ::block_size]
    hidden = gru_decoder_forward(sd, pitch, loudness, cache)
    return decoder_synthesis(sd, pitch, hidden, noise, block_size, sample_rate)[0]
