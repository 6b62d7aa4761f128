"""TorchScript export of the DDSP model on the gfx950 operators (`torch.ops.ddsp_hip.*`).

The fork's own export is broken (`export.py:46` constructor kwargs,
`export.py:27` `self.ddsp.gru`, `decoder.py:112` `**` expansion, `decoder.py:143,152` the
missing `proj_matrices`).  `ScriptDDSP` restates `ScriptDDSP` of `export.py:23-40` so that
it scripts: `forward(pitch[1,N,1], loudness[1,N,1]) -> audio[1,N,1]`, loudness normalised
with the stored mean/std, and

* non-realtime: the full `DDSPDecoder.forward` synthesis (harmonic + noise + reverb);
* realtime (the `ddsp~` Pd external's model, `realtime/ddsp_tilde/ddsp_model.cpp:32-52`):
  inputs decimated by block_size (`export.py:37-38`), the GRU run with its cached state
  (`decoder.py:56-60`), harmonic + noise without reverb — what the fork's
  `realtime_forward` (`decoder.py:138-158`) intends.

Every synthesis step in the scripted graph is a `ddsp_hip` operator; the GRU/MLP control
network stays aten (MIOpen/hipBLASLt).  State dict keys are the reference's
(`DDSPDecoder` under `ddsp.`), so a reference `state.pth` loads unchanged.
"""
import os

import torch
import torch.nn as nn

_HERE = os.path.dirname(os.path.abspath(__file__))
OPS_LIB = os.path.join(_HERE, "lib", "libddsp_hip_torch.so")
_loaded = False


def load_ops():
    """Register torch.ops.ddsp_hip.* (raises if the operator library is not built)."""
    global _loaded
    if not _loaded:
        if not os.path.exists(OPS_LIB):
            raise RuntimeError(f"ddsp_hip: TorchScript operator library missing at {OPS_LIB}; run `make`")
        torch.ops.load_library(OPS_LIB)
        _loaded = True


class ScriptReverb(nn.Module):
    """modules.py:7-35 on torch.ops.ddsp_hip (shares the source module's parameters)."""

    def __init__(self, rv):
        super().__init__()
        self.noise = rv.noise
        self.decay = rv.decay
        self.wet = rv.wet
        self.register_buffer("t", rv.t)
        self.length = int(rv.length)
        self.sample_rate = float(rv.sample_rate)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        imp = torch.ops.ddsp_hip.reverb_build_impulse(self.noise, self.decay, self.wet, self.sample_rate)
        spec = torch.ops.ddsp_hip.reverb_spectrum(imp, x.shape[1])
        return torch.ops.ddsp_hip.reverb_apply(x, spec, self.length)


class ScriptGRUDecoder(nn.Module):
    """GRUDecoder (decoder.py:9-68) for TorchScript: the recurrence through torch.ops.ddsp_hip.gru
    (shares the source module's submodules and parameters)."""

    def __init__(self, d):
        super().__init__()
        self.f0_mlp = d.f0_mlp
        self.loudness_mlp = d.loudness_mlp
        self.gru = d.gru
        self.out_mlp = d.out_mlp
        self.register_buffer("cache_gru", d.cache_gru)
        self.native = bool(d.gru.hidden_size % 64 == 0)  # the step kernel's shapes (core.gru_supported)

    def forward(self, f0: torch.Tensor, loudness: torch.Tensor, realtime: bool = False) -> torch.Tensor:
        hidden = torch.cat([self.f0_mlp(f0), self.loudness_mlp(loudness)], -1)
        g = self.gru
        h0 = self.cache_gru if realtime else None
        if self.native:
            out, h_last = torch.ops.ddsp_hip.gru(hidden, g.weight_ih_l0, g.weight_hh_l0, g.bias_ih_l0, g.bias_hh_l0,
                                                 h0)
        else:
            out, h_last = g(hidden, h0)
        if realtime:
            self.cache_gru.copy_(h_last)
        return self.out_mlp(torch.cat([out, f0, loudness], -1))


class ScriptDecoder(nn.Module):
    """DDSPDecoder (decoder.py:70-136) restated for TorchScript; same parameter/buffer names."""

    def __init__(self, m, noise_mode: str = "torch"):
        super().__init__()
        self.register_buffer("sample_rate", m.sample_rate.clone())
        self.register_buffer("block_size", m.block_size.clone())
        self.decoder = ScriptGRUDecoder(m.decoder)
        self.harmonic_proj = m.harmonic_proj
        self.noise_proj = m.noise_proj
        self.reverb = ScriptReverb(m.reverb)
        self.register_buffer("phase", m.phase.clone())
        self.has_reverb = bool(m.has_reverb)
        self.bs = int(m.block_size)
        self.sr = float(m.sample_rate)
        self.initial_bias = float(m.noise_synth.initial_bias)
        self.device_noise = noise_mode == "device"
        self.noise_calls = 0

    def synthesize(self, f0: torch.Tensor, hidden: torch.Tensor, with_reverb: bool) -> torch.Tensor:
        # decoder.py:106-125: both synths, their controls and the sum in one launch
        # (torch.ops.ddsp_hip.synth_frames, the fused kernel), then the reverb
        param = self.harmonic_proj(hidden)
        mags = self.noise_proj(hidden)
        B, F = mags.shape[0], mags.shape[1]
        if self.device_noise:
            self.noise_calls += 1
            signal = torch.ops.ddsp_hip.synth_frames(f0, param, mags, self.bs, self.sr, self.initial_bias, None,
                                                     0x5EEDDD5B, self.noise_calls)
        else:
            noise = (torch.rand(B, F, self.bs) * 2 - 1).to(mags)  # modules.py:119-123
            signal = torch.ops.ddsp_hip.synth_frames(f0, param, mags, self.bs, self.sr, self.initial_bias, noise, 0,
                                                     0)
        if with_reverb:
            signal = self.reverb(signal)
        return signal

    def forward(self, pitch: torch.Tensor, loudness: torch.Tensor, realtime: bool = False) -> torch.Tensor:
        hidden = self.decoder(pitch, loudness, realtime)
        return self.synthesize(pitch.contiguous(), hidden, self.has_reverb and not realtime)


class ScriptDDSP(nn.Module):
    """Scriptable (pitch, loudness) -> audio model over torch.ops.ddsp_hip (export.py:23-40)."""

    def __init__(self, ddsp, mean_loudness: float = 0.0, std_loudness: float = 1.0,
                 realtime: bool = False, noise_mode: str = "torch"):
        super().__init__()
        load_ops()
        self.ddsp = ScriptDecoder(ddsp, noise_mode)
        self.register_buffer("mean_loudness", torch.tensor(float(mean_loudness)))
        self.register_buffer("std_loudness", torch.tensor(float(std_loudness)))
        self.realtime = realtime
        self.block_size = int(ddsp.block_size)

    def forward(self, pitch: torch.Tensor, loudness: torch.Tensor) -> torch.Tensor:
        loudness = (loudness - self.mean_loudness) / self.std_loudness
        if self.realtime:
            pitch = pitch[:, ::self.block_size]
            loudness = loudness[:, ::self.block_size]
        return self.ddsp(pitch, loudness, self.realtime)


def export(ddsp, path, mean_loudness=0.0, std_loudness=1.0, realtime=False, noise_mode="torch"):
    """Script and save a model the way export.py:43-65 intends; returns the ScriptModule."""
    m = torch.jit.script(ScriptDDSP(ddsp, mean_loudness, std_loudness, realtime, noise_mode).eval())
    m.save(path)
    return m
