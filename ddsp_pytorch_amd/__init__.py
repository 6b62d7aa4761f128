"""ddsp_pytorch_amd — MI355X (gfx950) backend for the DDSP harmonic-plus-noise synthesis path.

Drop-in for hugofloresgarcia/ddsp_pytorch's synthesis hot path:

* function level — ``ddsp_pytorch_amd.core``: scale_function, remove_above_nyquist,
  upsample, harmonic_synth, amp_to_impulse_response, fft_convolve (ddsp/core.py);
* module level — ``ddsp_pytorch_amd.modules``: HarmonicSynth, FilteredNoise, Reverb
  (ddsp/models/modules.py), fused kernels;
* ``install(ddsp)`` rebinds both inside an imported reference package;
* ``DDSPDecoder`` and ``DDSPAutoencoder`` — the reference's two models (same state_dicts) running
  on these kernels.

All compute goes through the C-ABI library (include/ddsp_hip.h, lib/libddsp_hip.so);
nothing falls back to CPU.
"""
from . import core
from .core import (amp_to_impulse_response, fft_convolve, harmonic_synth, remove_above_nyquist,
                   scale_function, upsample)
from .decoder import DDSPDecoder
from .encoder import DDSPAutoencoder
from .install import install
from .modules import FilteredNoise, HarmonicSynth, Reverb
from . import synth  # noqa: E402  (SynthPath, make_inputs: the bench's and the tests' synthesis-path driver)

__version__ = "0.1.0"
