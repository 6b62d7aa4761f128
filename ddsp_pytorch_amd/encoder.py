"""The reference's second caller of the hot path: ``ddsp/models/encoder.py`` — ``MFCCEncoder`` and
``DDSPAutoencoder`` with the reference's constructors and state_dict keys, wired to the gfx950 path.

``DDSPAutoencoder.forward`` (encoder.py:63-103) runs the same synthesis section as
``DDSPDecoder.forward`` (projections -> both synths' controls -> harmonic + noise -> reverb), here as
``decoder.decoder_synthesize``: the two projections as one GEMM and the synthesis as ONE fused launch
that also writes the parts and the control dicts.  The encoder's GRU (encoder.py:19) and the
z-conditioned decoder's run on the GRU step kernels (``csrc/gru.hip``); LayerNorm and the Linear
layers stay torch (hipBLASLt).  ``install()`` binds ``autoencoder_forward`` and
``mfcc_encoder_forward`` to the reference's classes.
"""
import torch
import torch.nn as nn

from .decoder import GRUDecoder, _gru, decoder_synthesize
from .modules import FilteredNoise, HarmonicSynth, Reverb


def mfcc_encoder_forward(self, mfccs):
    """encoder.py:22-26: LayerNorm -> GRU -> Linear to z, the GRU on the step kernel."""
    x = self.norm(mfccs)
    x = _gru(self, x, None)[0]
    return self.proj(x)


class MFCCEncoder(nn.Module):
    """encoder.py:10-26."""

    def __init__(self, sample_rate: int, block_size: int, hidden_size: int, n_mfccs: int, z_dim: int = None):
        super().__init__()
        self.hidden_size = hidden_size
        self.z_dim = z_dim
        self.norm = nn.LayerNorm(n_mfccs)
        self.gru = nn.GRU(n_mfccs, hidden_size, batch_first=True)
        self.proj = nn.Linear(hidden_size, z_dim)

    forward = mfcc_encoder_forward


def autoencoder_forward(self, batch: dict):
    """encoder.py:63-103 DDSPAutoencoder.forward: z = encoder(mfcc), hidden = decoder(f0, loudness, z),
    then the synthesis section on the fused kernel (decoder_synthesize).  Returns the reference's dict,
    incl. ``z``."""
    f0, loudness, mfcc = batch["pitch"], batch["loudness"], batch["mfcc"]
    z = self.encoder(mfcc)
    hidden = self.decoder(f0, loudness, z=z)
    signal, harmonic, noise, hc, nc = decoder_synthesize(self, hidden, f0)
    return {"f0": f0, "loudness": loudness, "signal": signal, "noise": noise, "harmonic_audio": harmonic,
            "noise_ctrls": nc, "harmonic_ctrls": hc, "z": z}


class DDSPAutoencoder(nn.Module):
    """encoder.py:29-61: MFCC encoder (30 coefficients -> z of 16), z-conditioned GRU decoder, the two
    projections, the synths and the reverb."""

    def __init__(self, hidden_size: int, n_harmonic: int, n_bands: int, sample_rate: int, block_size: int,
                 has_reverb: bool):
        super().__init__()
        self.register_buffer("sample_rate", torch.tensor(sample_rate))
        self.register_buffer("block_size", torch.tensor(block_size))
        self.encoder = MFCCEncoder(sample_rate, block_size, hidden_size, n_mfccs=30, z_dim=16)
        self.decoder = GRUDecoder(hidden_size=hidden_size, z_dim=16)
        self.harmonic_proj = nn.Linear(hidden_size, n_harmonic + 1)
        self.noise_proj = nn.Linear(hidden_size, n_bands)
        self.harmonic_synth = HarmonicSynth(block_size=block_size, sample_rate=sample_rate)
        self.noise_synth = FilteredNoise(block_size=block_size, window_size=n_bands)
        self.has_reverb = has_reverb
        self.reverb = Reverb(sample_rate, sample_rate)
        self.register_buffer("phase", torch.zeros(1))

    synthesize = decoder_synthesize
    forward = autoencoder_forward

