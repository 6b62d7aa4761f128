"""Caller of the hot path: a ``DDSPDecoder`` with the reference's architecture and
state_dict keys (ddsp/models/decoder.py:9-136, ddsp/core.py:122-133), wired to the gfx950
synth modules.

The GRU/MLP control network is plain PyTorch (MIOpen/hipBLASLt underneath) — it is not
part of the accelerated synthesis path.  It exists so that a
reference checkpoint can be loaded and run end to end on the device, and so the
synthesis section of ``forward`` (decoder.py:106-125) can be exercised exactly as the
reference calls it.
"""
import torch
import torch.nn as nn

from . import core
from .modules import FilteredNoise, HarmonicSynth, Reverb


def mlp(in_size, hidden_size, n_layers):
    """ddsp/core.py:122-129: (Linear, LayerNorm, LeakyReLU) x n_layers."""
    sizes = [in_size] + n_layers * [hidden_size]
    layers = []
    for i in range(n_layers):
        layers += [nn.Linear(sizes[i], sizes[i + 1]), nn.LayerNorm(sizes[i + 1]), nn.LeakyReLU()]
    return nn.Sequential(*layers)


class GRUDecoder(nn.Module):
    """ddsp/models/decoder.py:9-68 (z_dim=None form)."""

    def __init__(self, hidden_size: int):
        super().__init__()
        self.register_buffer("cache_gru", torch.zeros(1, 1, hidden_size))
        self.f0_mlp = mlp(1, hidden_size, 3)
        self.loudness_mlp = mlp(1, hidden_size, 3)
        self.gru = nn.GRU(2 * hidden_size, hidden_size, batch_first=True)
        self.out_mlp = mlp(hidden_size + 2, hidden_size, 3)

    def forward(self, f0, loudness, realtime: bool = False):
        return gru_decoder_forward(self, f0, loudness, None, realtime)


def _gru(mod, hidden, h0):
    """mod.gru(hidden[, h0]) with the recurrence (and, under autograd, its BPTT) on the gfx950 step
    kernels; torch's GRU only for shapes outside the kernel's (hidden % 64 != 0)."""
    if hidden.is_cuda and core.gru_supported(mod.gru):
        return core.gru(hidden, mod.gru, h0)
    return mod.gru(hidden, h0) if h0 is not None else mod.gru(hidden)


def gru_decoder_forward(self, f0, loudness, z=None, realtime=False):
    """ddsp/models/decoder.py:43-68 GRUDecoder.forward (incl. the optional z projection), the GRU on
    the step kernel for inference.  install() binds it to the reference's GRUDecoder too."""
    hidden = torch.cat([self.f0_mlp(f0), self.loudness_mlp(loudness)], -1)
    if getattr(self, "add_z", False):
        assert z is not None
        hidden = torch.cat([hidden, self.z_mlp(z)], -1)
    if realtime:
        gru_out, cache = _gru(self, hidden, self.cache_gru)
        self.cache_gru.copy_(cache)
    else:
        gru_out = _gru(self, hidden, None)[0]
    return self.out_mlp(torch.cat([gru_out, f0, loudness], -1))


class DDSPDecoder(nn.Module):
    """ddsp/models/decoder.py:70-136 with the synthesis on gfx950 kernels."""

    def __init__(self, hidden_size: int, n_harmonic: int, n_bands: int, sample_rate: int,
                 block_size: int, has_reverb: bool):
        super().__init__()
        self.register_buffer("sample_rate", torch.tensor(sample_rate))
        self.register_buffer("block_size", torch.tensor(block_size))
        self.decoder = GRUDecoder(hidden_size)
        self.harmonic_proj = nn.Linear(hidden_size, n_harmonic + 1)
        self.noise_proj = nn.Linear(hidden_size, n_bands)
        self.harmonic_synth = HarmonicSynth(block_size=block_size, sample_rate=sample_rate)
        self.noise_synth = FilteredNoise(block_size=block_size, window_size=n_bands)
        self.has_reverb = has_reverb
        self.reverb = Reverb(sample_rate, sample_rate)
        self.register_buffer("phase", torch.zeros(1))

    def synthesize(self, hidden, f0):
        """decoder.py:106-125: controls -> harmonic + noise (+ reverb)."""
        param = self.harmonic_proj(hidden)
        harmonic_ctrls = self.harmonic_synth.get_controls(param[..., :1], param[..., 1:], f0)
        harmonic = self.harmonic_synth(**harmonic_ctrls)
        noise_ctrls = self.noise_synth.get_controls(self.noise_proj(hidden))
        noise = self.noise_synth(**noise_ctrls)
        signal = harmonic + noise
        if self.has_reverb:
            signal = self.reverb(signal)
        return signal, harmonic, noise, harmonic_ctrls, noise_ctrls

    def forward(self, batch: dict):
        f0, loudness = batch["pitch"], batch["loudness"]
        hidden = self.decoder(f0, loudness)
        signal, harmonic, noise, hc, nc = self.synthesize(hidden, f0)
        return {"f0": f0, "loudness": loudness, "signal": signal, "noise": noise,
                "harmonic_audio": harmonic, "noise_ctrls": nc, "harmonic_ctrls": hc}
