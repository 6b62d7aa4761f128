"""Function-level drop-ins for ``ddsp/core.py`` — same names, arguments and return shapes.

``ddsp/models/modules.py`` looks these up late-bound through the ``ddsp`` package
(``modules.py:33,53-56,74-78,113,117,125``), so rebinding the package attributes to the
functions below (``ddsp_pytorch_amd.install``) moves the reference's own
``DDSPDecoder.forward`` onto the gfx950 kernels without editing it.

Every function here runs on the HIP device through the C-ABI (include/ddsp_hip.h) and
raises — never falls back to CPU — on tensors it cannot take (CPU tensors, non-fp32).
Shape errors raise ``RuntimeError`` as the reference's torch ops would.

Besides the six reference functions, the fused frame-rate ops used by the module-level
drop-ins (``modules.py``) live here: ``harmonic_controls``, ``harmonic_synth_frames``,
``filtered_noise``, ``reverb_build_impulse``, ``reverb_spectrum``, ``reverb_apply``.
"""
import atexit
import ctypes
import itertools
import math

import torch

from . import _lib

__all__ = [
    "scale_function", "remove_above_nyquist", "upsample", "harmonic_synth",
    "amp_to_impulse_response", "fft_convolve", "phase", "harmonic_controls",
    "harmonic_synth_frames", "harmonic_synth_params", "synth_frames", "filtered_noise", "reverb_build_impulse", "reverb_spectrum_floats",
    "reverb_spectrum", "reverb_impulse_spectrum", "reverb_apply", "reverb_forward", "reverb_cache_bytes", "set_noise_seed", "safe_log", "stft_magnitude", "multiscale_fft",
]


def _dev(*tensors):
    for t in tensors:
        if not isinstance(t, torch.Tensor):
            raise TypeError(f"ddsp_hip: expected a torch.Tensor, got {type(t).__name__}")
        if t.device.type != "cuda":
            raise RuntimeError("ddsp_hip: tensors must be on a HIP device (no CPU fallback); "
                               f"got a tensor on {t.device}")
        if t.dtype != torch.float32:
            raise TypeError(f"ddsp_hip: kernels compute in float32; got {t.dtype}")
    dev = tensors[0].device
    for t in tensors[1:]:
        if t.device != dev:
            raise RuntimeError(f"ddsp_hip: tensors on different devices {dev} and {t.device}")
    return dev


def _wants_grad(*tensors):
    """autograd must record this call: dispatch to the Function in grad.py (backward kernels)."""
    return torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in tensors)


def _c(t):
    """contiguous and 16-byte aligned (the kernels use float4 accesses)."""
    t = t.contiguous()
    if t.data_ptr() % 16:
        t = t.clone()
    return t


def _workspace(nbytes, device):
    return torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=device)


# ------------------------------------------------------------------------------------
# ddsp/core.py functions
# ------------------------------------------------------------------------------------
def scale_function(x):
    """ddsp/core.py:77-78  ``2 * sigmoid(x) ** ln(10) + 1e-7``."""
    return scale_with_bias(x, 0.0)


def scale_with_bias(x, bias):
    """``scale_function(x + bias)`` in one kernel (FilteredNoise.get_controls, modules.py:111-114)."""
    _dev(x)
    if _wants_grad(x):
        return _grad.ScaleFn.apply(x, float(bias))
    x = _c(x)
    y = torch.empty_like(x)
    _lib.call("scale_function", _lib.ptr(x), _lib.ptr(y), x.numel(), float(bias), _lib.stream_of(x))
    return y


def remove_above_nyquist(amplitudes, f0, sample_rate):
    """ddsp/core.py:70-74  amplitudes[..., H] * ((f0 * k < sr/2) + 1e-4), k = 1..H."""
    _dev(amplitudes, f0)
    if _wants_grad(amplitudes, f0):
        return _grad.NyquistFn.apply(amplitudes, f0, sample_rate)
    H = amplitudes.shape[-1]
    lead = amplitudes.shape[:-1]
    if f0.shape[-1] != 1:
        raise RuntimeError(f"remove_above_nyquist: f0 must end in a size-1 dim, got {tuple(f0.shape)}")
    out_lead = torch.broadcast_shapes(lead, f0.shape[:-1])
    amplitudes = _c(amplitudes.expand(*out_lead, H))
    f0 = _c(f0.expand(*out_lead, 1))
    out = torch.empty_like(amplitudes)
    rows = amplitudes.numel() // max(H, 1)
    _lib.call("remove_above_nyquist", _lib.ptr(amplitudes), _lib.ptr(f0), _lib.ptr(out), rows, H,
              float(sample_rate), _lib.stream_of(out))
    return out


def upsample(signal, factor):
    """ddsp/core.py:64-67  nearest upsampling [B, F, C] -> [B, F*factor, C]."""
    _dev(signal)
    if _wants_grad(signal):
        return _grad.UpsampleFn.apply(signal, int(factor))
    if signal.dim() != 3:
        raise RuntimeError(f"upsample: expected [batch, frames, channels], got {tuple(signal.shape)}")
    factor = int(factor)
    B, F, C = signal.shape
    x = _c(signal)
    y = torch.empty(B, F * factor, C, dtype=x.dtype, device=x.device)
    _lib.call("upsample", _lib.ptr(x), _lib.ptr(y), B, F, C, factor, _lib.stream_of(x))
    return y


def harmonic_synth(f0, amplitudes, sample_rate):
    """ddsp/core.py:136-141  f0[B, T, 1], amplitudes[B, T, H] -> [B, T, 1]."""
    _dev(f0, amplitudes)
    if _wants_grad(f0, amplitudes):
        _grad.refuse_f0_grad(f0, "harmonic_synth")
        return _grad.HarmonicSynthFn.apply(f0, amplitudes, sample_rate)
    if amplitudes.dim() != 3 or f0.dim() != 3 or f0.shape[-1] != 1:
        raise RuntimeError("harmonic_synth: expected f0 [B,T,1] and amplitudes [B,T,H], got "
                           f"{tuple(f0.shape)} and {tuple(amplitudes.shape)}")
    B, T, H = amplitudes.shape
    if f0.shape[:2] != (B, T):
        raise RuntimeError(f"harmonic_synth: shape mismatch {tuple(f0.shape)} vs {tuple(amplitudes.shape)}")
    f0 = _c(f0)
    amplitudes = _c(amplitudes)
    out = torch.empty(B, T, 1, dtype=torch.float32, device=f0.device)
    nbytes = _lib.query("harmonic_synth_workspace_size", B, T)
    ws = _workspace(nbytes, f0.device)
    _lib.call("harmonic_synth", _lib.ptr(f0), _lib.ptr(amplitudes), _lib.ptr(out), B, T, H,
              float(sample_rate), _lib.ptr(ws), ws.numel(), _lib.stream_of(out))
    return out


def phase(f0, sample_rate):
    """The fp32 phase ``cumsum(2*pi*f0/sr, 1)`` of ddsp/core.py:138 (exposed for exactness tests)."""
    _dev(f0)
    B, T = f0.shape[0], f0.shape[1]
    f0 = _c(f0)
    out = torch.empty(B, T, 1, dtype=torch.float32, device=f0.device)
    ws = _workspace(_lib.query("harmonic_synth_workspace_size", B, T), f0.device)
    _lib.call("phase", _lib.ptr(f0), _lib.ptr(out), B, T, float(sample_rate), _lib.ptr(ws),
              ws.numel(), _lib.stream_of(out))
    return out


def amp_to_impulse_response(amp, target_size):
    """ddsp/core.py:144-166  zero-phase FIR of length target_size from NB magnitudes."""
    _dev(amp)
    if _wants_grad(amp):
        return _grad.ImpulseResponseFn.apply(amp, int(target_size))
    NB = amp.shape[-1]
    if NB < 2:
        raise RuntimeError("amp_to_impulse_response: need at least 2 frequency bands")
    target = int(target_size)
    x = _c(amp)
    rows = x.numel() // NB
    out = torch.empty(*amp.shape[:-1], target, dtype=torch.float32, device=x.device)
    _lib.call("amp_to_impulse_response", _lib.ptr(x), _lib.ptr(out), rows, NB, target,
              _lib.stream_of(x))
    return out


def fft_convolve(signal, kernel):
    """ddsp/core.py:169-176  causal linear convolution truncated to N (last dim), with broadcasting."""
    _dev(signal, kernel)
    if _wants_grad(signal, kernel):
        return _grad.FFTConvolveFn.apply(signal, kernel)
    N = signal.shape[-1]
    if kernel.shape[-1] != N:
        raise RuntimeError(f"fft_convolve: signal and kernel lengths differ ({N} vs {kernel.shape[-1]})")
    lead = torch.broadcast_shapes(signal.shape[:-1], kernel.shape[:-1])
    rows = math.prod(lead) if len(lead) else 1
    s = _c(signal.expand(*lead, N))
    if kernel.numel() == N:
        k, krows = _c(kernel.reshape(N)), 1
    else:
        k, krows = _c(kernel.expand(*lead, N)), rows
    out = torch.empty(*lead, N, dtype=torch.float32, device=s.device)
    ws = _workspace(_lib.query("fft_convolve_workspace_size", rows, krows, N), s.device)
    _lib.call("fft_convolve", _lib.ptr(s), _lib.ptr(k), _lib.ptr(out), rows, krows, N,
              _lib.ptr(ws), ws.numel(), _lib.stream_of(out))
    return out


# ------------------------------------------------------------------------------------
# fused module-level ops (ddsp/models/modules.py)
# ------------------------------------------------------------------------------------
def _rows_view(t, name):
    """[B, F, C] view with unit stride on C and a single row stride over (B, F)."""
    if t.dim() != 3 or t.stride(-1) != 1 or t.stride(0) != t.shape[1] * t.stride(1):
        t = t.contiguous()
    return t, t.stride(1)


def harmonic_controls(amplitudes, harmonic_distribution, f0, sample_rate):
    """modules.py:44-67 HarmonicSynth.get_controls, fused: returns (amplitudes, distribution)."""
    _dev(amplitudes, harmonic_distribution, f0)
    if _wants_grad(amplitudes, harmonic_distribution, f0):
        _grad.refuse_f0_grad(f0, "harmonic_controls")
        return _grad.ControlsFn.apply(amplitudes, harmonic_distribution, f0, sample_rate)
    B, F, H = harmonic_distribution.shape
    if amplitudes.shape != (B, F, 1) or f0.shape != (B, F, 1):
        raise RuntimeError("harmonic_controls: expected amplitudes/f0 [B,F,1] matching "
                           f"distribution {tuple(harmonic_distribution.shape)}")
    a, a_ld = _rows_view(amplitudes, "amplitudes")
    d, d_ld = _rows_view(harmonic_distribution, "harmonic_distribution")
    f0c = _c(f0)
    amp_out = torch.empty(B, F, 1, dtype=torch.float32, device=f0.device)
    dist_out = torch.empty(B, F, H, dtype=torch.float32, device=f0.device)
    _lib.call("harmonic_controls", _lib.ptr(a), a_ld, _lib.ptr(d), d_ld, _lib.ptr(f0c),
              _lib.ptr(amp_out), _lib.ptr(dist_out), B * F, H, float(sample_rate),
              _lib.stream_of(f0c))
    return amp_out, dist_out


def harmonic_synth_frames(f0, amplitudes, harmonic_distribution, block_size, sample_rate,
                          write_back=True):
    """modules.py:69-80 HarmonicSynth.forward, fused at frame rate.

    f0, amplitudes: [B, F, 1]; harmonic_distribution: [B, F, H] (scaled and normalised).
    Returns audio [B, F*block_size, 1].  With ``write_back`` the distribution is multiplied
    by the amplitudes in place, exactly like ``harmonic_distribution *= amplitudes``
    (modules.py:73), which the reference's caller sees through its controls dict.
    """
    _dev(f0, amplitudes, harmonic_distribution)
    if _wants_grad(f0, amplitudes, harmonic_distribution):
        _grad.refuse_f0_grad(f0, "harmonic_synth_frames")
        out = _grad.SynthFramesHarmonicFn.apply(f0, amplitudes, harmonic_distribution, block_size, sample_rate)
        if write_back:  # modules.py:73, recorded by autograd like the reference's in-place multiply
            harmonic_distribution.mul_(amplitudes)
        return out
    B, F, H = harmonic_distribution.shape
    f0c, ac = _c(f0), _c(amplitudes)
    dist = harmonic_distribution
    if write_back and not (dist.is_contiguous() and dist.data_ptr() % 16 == 0):
        raise RuntimeError("harmonic_synth_frames: in-place write-back needs a contiguous distribution")
    if not write_back:
        dist = _c(dist)
    bs = int(block_size)
    out = torch.empty(B, F * bs, 1, dtype=torch.float32, device=f0.device)
    _lib.call("harmonic_synth_frames", _lib.ptr(f0c), _lib.ptr(ac), _lib.ptr(dist), int(bool(write_back)),
              _lib.ptr(out), B, F, H, bs, float(sample_rate), _lib.stream_of(out))
    return out


class _NoiseCounter:
    """Philox (seed, offset) for on-device noise: each call consumes a fresh offset."""

    def __init__(self):
        self.seed = 0x5EED_DD5B
        self._offsets = itertools.count()

    def next(self):
        return self.seed, next(self._offsets)


_noise_counter = _NoiseCounter()


def set_noise_seed(seed):
    """Seed the on-device noise generator (throughput mode)."""
    _noise_counter.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    _noise_counter._offsets = itertools.count()


def harmonic_synth_params(f0, param, block_size, sample_rate):
    """decoder.py:106-113 + modules.py:44-80 in one kernel: raw harmonic projection
    param[B, F, H+1] (column 0 amplitude, 1..H distribution) and f0 [B, F, 1] -> audio
    [B, F*block_size, 1].  The controls (scale, Nyquist mask, normalisation) never reach HBM."""
    _dev(f0, param)
    if _wants_grad(f0, param):
        _grad.refuse_f0_grad(f0, "harmonic_synth_params")
        return _grad.HarmonicParamsFn.apply(f0, param, block_size, sample_rate)
    B, F, H1 = param.shape
    if f0.shape != (B, F, 1) or H1 < 2:
        raise RuntimeError(f"harmonic_synth_params: f0 {tuple(f0.shape)} / param {tuple(param.shape)}")
    f0c, pc = _c(f0), _c(param)
    bs = int(block_size)
    out = torch.empty(B, F * bs, 1, dtype=torch.float32, device=f0.device)
    _lib.call("harmonic_synth_params", _lib.ptr(f0c), _lib.ptr(pc), _lib.ptr(out), B, F, H1 - 1, bs,
              float(sample_rate), _lib.stream_of(out))
    return out


def filtered_noise(magnitudes, block_size, noise=None, add=None, return_noise=False, raw_bias=None):
    """modules.py:116-128 FilteredNoise.forward, fused.

    magnitudes: [B, F, NB] (already scaled by get_controls; with ``raw_bias`` the raw
    projection, scaled in the kernel as scale_function(x + raw_bias)).  ``noise``
    [B, F, block_size] injects the U[-1,1) samples (parity mode, e.g. the reference's
    ``torch.rand`` stream); ``None`` draws them on the device with Philox4x32-10.  ``add``
    [B, F*bs, 1] is added to the result (fuses ``harmonic + noise``); with ``return_noise`` the
    filtered noise alone is returned as a second tensor.
    """
    _dev(magnitudes)
    if _wants_grad(magnitudes, add):
        outs = _grad.FilteredNoiseFn.apply(magnitudes, add, int(block_size), noise, raw_bias,
                                           bool(return_noise))
        if return_noise and not isinstance(outs, tuple):
            return outs, outs
        return outs
    seed, offset = _noise_counter.next() if noise is None else (0, 0)
    out = _filtered_noise_launch(magnitudes, block_size, noise, add, return_noise, raw_bias, seed, offset)
    if return_noise and not isinstance(out, tuple):
        return out, out
    return out


def _filtered_noise_launch(magnitudes, block_size, noise, add, return_noise, raw_bias, seed, offset):
    B, F, NB = magnitudes.shape
    bs = int(block_size)
    m = _c(magnitudes)
    if noise is not None:
        _dev(noise)
        if tuple(noise.shape) != (B, F, bs):
            raise RuntimeError(f"filtered_noise: noise must be [B, F, block_size] = {(B, F, bs)}")
        noise = _c(noise)
    if add is not None:
        _dev(add)
        add = _c(add)
        if add.numel() != B * F * bs:
            raise RuntimeError("filtered_noise: `add` must have B*F*block_size elements")
    out = torch.empty(B, F * bs, 1, dtype=torch.float32, device=m.device)
    nout = torch.empty_like(out) if (return_noise and add is not None) else None
    if raw_bias is None:
        _lib.call("filtered_noise", _lib.ptr(m), _lib.ptr(noise), seed, offset, _lib.ptr(add),
                  _lib.ptr(out), _lib.ptr(nout), B, F, NB, bs, _lib.stream_of(m))
    else:
        _lib.call("filtered_noise_params", _lib.ptr(m), float(raw_bias), _lib.ptr(noise), seed, offset,
                  _lib.ptr(add), _lib.ptr(out), _lib.ptr(nout), B, F, NB, bs, _lib.stream_of(m))
    return (out, nout) if nout is not None else out


EWORKSPACE = 4  # DDSP_HIP_EWORKSPACE
# the fused synthesis kernel's frames sum their phase prefix themselves up to this many frames per item
# (O(F) per frame); past it one ddsp_hip_frame_phase_prefix launch precomputes every frame's prefix
FRAME_PREFIX_MIN_FRAMES = 512
ERANGE = 5


def synth_frames_in_envelope(n_harmonic, n_bands, block_size, batch=1):
    """The fused kernel's shape envelope (mirrors ddsp_hip_synth_frames' DDSP_HIP_ERANGE checks)."""
    H, NB, bs = int(n_harmonic), int(n_bands), int(block_size)
    if bs % 4 or bs > 1024 or H > 1024 or NB > 1025 or batch > 65535:
        return False
    n = 2 * (NB - 1)
    half = n // 2
    if bs >= n:
        lo_end, tail_start = (half + 3) & ~3, bs - half
        if tail_start < lo_end:
            lo_end = bs
    else:
        lo_end = bs
    pad = (lo_end + 4 + 3) & ~3
    H4, n4 = (H + 3) & ~3, (n + 3) & ~3
    floats = 8 * H4 + n4 + ((NB + 3) & ~3) + ((half + 4) & ~3) + bs + ((half + 3) & ~3) + pad + bs
    return 4 * floats <= 120 * 1024


def synth_frames(f0, param, mags, block_size, sample_rate, bias=-5.0, noise=None, parts=False, controls=False):
    """decoder.py:106-121 in one kernel: raw harmonic projection param[B,F,H+1], pitch f0[B,F,1]
    and raw noise projection mags[B,F,NB] -> signal = harmonic + noise [B,F*bs,1].

    ``noise`` [B,F,bs] injects the U[-1,1) samples (else on-device Philox).  With ``parts`` the
    harmonic and noise signals are returned too: (signal, harmonic, noise).  With ``controls``
    the controls ``DDSPDecoder.forward`` returns (decoder.py:127-135) are appended as a dict
    ``{"amplitudes" [B,F,1], "harmonic_distribution" [B,F,H], "magnitudes" [B,F,NB]}`` — the
    distribution as the reference's caller sees it after ``modules.py:73``'s in-place
    ``*= amplitudes``; written by the same launch (or, under autograd, by the differentiable
    control ops).  Returns None when the shape is outside the fused kernel's envelope
    (block_size % 4 == 0 and <= 1024, H <= 1024, NB <= 1025)."""
    _dev(f0, param, mags)
    B, F, H1 = param.shape
    NB = mags.shape[-1]
    bs = int(block_size)
    if f0.shape != (B, F, 1) or mags.shape[:2] != (B, F) or H1 < 2:
        raise RuntimeError("synth_frames: f0 [B,F,1], param [B,F,H+1], mags [B,F,NB] expected")
    if not synth_frames_in_envelope(H1 - 1, NB, bs, B):
        return None
    if _wants_grad(f0, param, mags):
        _grad.refuse_f0_grad(f0, "synth_frames")
        outs = _grad.SynthFramesFn.apply(f0, param, mags, bs, float(sample_rate), float(bias), noise,
                                         bool(parts))
        if not controls:
            return outs
        amps, dist = harmonic_controls(param[..., :1], param[..., 1:], f0, sample_rate)
        ctrl = {"amplitudes": amps, "harmonic_distribution": dist * amps,
                "magnitudes": scale_with_bias(mags, bias)}
        return (*outs, ctrl) if parts else (outs, ctrl)
    seed, offset = _noise_counter.next() if noise is None else (0, 0)
    return _synth_frames_launch(f0, param, mags, bs, sample_rate, bias, noise, parts, seed, offset, controls)


def _frame_rows(t):
    """(tensor, row stride) for a [B, F, C] tensor read row by row: unit stride on C and one row stride
    over (B, F) — a column slice of a wider projection output qualifies as it is — else a contiguous copy
    (broadcast rows, stride 0, and overlapping rows included).  The kernels read these rows with scalar
    loads only (no 16-byte vector loads), so a view's row base needs no more than 4-byte alignment."""
    if (t.dim() == 3 and t.stride(-1) == 1 and t.stride(1) >= max(t.shape[-1], 1)
            and t.stride(0) == t.shape[1] * t.stride(1)):
        return t, t.stride(1)
    t = t.contiguous()
    return t, t.shape[-1]


def _synth_frames_launch(f0, param, mags, block_size, sample_rate, bias, noise, parts, seed, offset,
                         controls=False):
    B, F, H1 = param.shape
    NB = mags.shape[-1]
    bs = int(block_size)
    f0c = _c(f0)
    (pc, ldp), (mc, ldm) = _frame_rows(param), _frame_rows(mags)
    if noise is not None:
        _dev(noise)
        if tuple(noise.shape) != (B, F, bs):
            raise RuntimeError(f"synth_frames: noise must be [B, F, block_size] = {(B, F, bs)}")
        noise = _c(noise)
    out = torch.empty(B, F * bs, 1, dtype=torch.float32, device=f0.device)
    harm = torch.empty_like(out) if parts else None
    nz = torch.empty_like(out) if parts else None
    ctrl = (torch.empty(B * F * (1 + (H1 - 1) + NB), dtype=torch.float32, device=f0.device)
            if controls else None)
    prefix = None
    if F > FRAME_PREFIX_MIN_FRAMES:  # long renders: each frame reads its phase prefix instead of summing
        prefix = torch.empty(B * F, dtype=torch.float64, device=f0.device)
        _lib.call("frame_phase_prefix", _lib.ptr(f0c), B, F, bs, float(sample_rate), _lib.ptr(prefix),
                  _lib.stream_of(out))
    _lib.call("synth_frames_controls_prefix", _lib.ptr(f0c), _lib.ptr(pc), ldp, _lib.ptr(mc), ldm, float(bias),
              _lib.ptr(noise), seed, offset, _lib.ptr(out), _lib.ptr(harm), _lib.ptr(nz), _lib.ptr(ctrl),
              _lib.ptr(prefix), B, F, H1 - 1, NB, bs, float(sample_rate), _lib.stream_of(out))
    res = (out, harm, nz) if parts else out
    if not controls:
        return res
    BF, H = B * F, H1 - 1
    cd = {"amplitudes": ctrl[:BF].view(B, F, 1), "harmonic_distribution": ctrl[BF:BF * (1 + H)].view(B, F, H),
          "magnitudes": ctrl[BF * (1 + H):].view(B, F, NB)}
    return (*res, cd) if parts else (res, cd)


def synth_frames_counter(f0, param, mags, block_size, sample_rate, counter, seed, bias=-5.0):
    """synth_frames with on-device noise whose Philox offset is the device word counter[0]
    (int64, advanced by one on the stream after the launch): for calls replayed from a captured
    HIP graph, where by-value offsets would freeze.  Call k equals
    synth_frames(..., noise=None) drawn with (seed, offset=k).  Inference only."""
    _dev(f0, param, mags)
    B, F, H1 = param.shape
    NB = mags.shape[-1]
    bs = int(block_size)
    if f0.shape != (B, F, 1) or mags.shape[:2] != (B, F) or H1 < 2:
        raise RuntimeError("synth_frames_counter: f0 [B,F,1], param [B,F,H+1], mags [B,F,NB] expected")
    if counter.dtype != torch.int64 or counter.numel() < 1 or counter.device != f0.device:
        raise RuntimeError("synth_frames_counter: counter must be a device int64 tensor")
    if not synth_frames_in_envelope(H1 - 1, NB, bs, B):
        raise RuntimeError("synth_frames_counter: shape outside the fused kernel's envelope")
    out = torch.empty(B, F * bs, 1, dtype=torch.float32, device=f0.device)
    _lib.call("synth_frames_counter", _lib.ptr(_c(f0)), _lib.ptr(_c(param)), _lib.ptr(_c(mags)), float(bias),
              int(seed) & 0xFFFFFFFFFFFFFFFF, _lib.ptr(counter), _lib.ptr(out), B, F, H1 - 1, NB, bs,
              float(sample_rate), _lib.stream_of(out))
    return out


def reverb_build_impulse(noise, decay, wet, sample_rate):
    """modules.py:21-26 Reverb.build_impulse: noise[L,1] -> impulse [1, L, 1]."""
    _dev(noise, decay, wet)
    if _wants_grad(noise, decay, wet):
        return _grad.BuildImpulseFn.apply(noise, decay, wet, sample_rate)
    L = noise.shape[0]
    n = _c(noise)
    imp = torch.empty(1, L, 1, dtype=torch.float32, device=n.device)
    _lib.call("reverb_build_impulse", _lib.ptr(n), _lib.ptr(_c(decay)), _lib.ptr(_c(wet)),
              _lib.ptr(imp), L, float(sample_rate), _lib.stream_of(n))
    return imp


def reverb_spectrum_floats(n_samples, ir_length):
    return int(_lib.query("reverb_spectrum_floats", int(n_samples), int(ir_length)))


def reverb_spectrum(impulse, n_samples):
    """Partitioned-convolution spectra of the IR cropped/padded to n_samples (for reverb_apply)."""
    _dev(impulse)
    h = _c(impulse.reshape(-1))
    L = h.numel()
    spec = torch.empty(reverb_spectrum_floats(n_samples, L), dtype=torch.float32, device=h.device)
    _lib.call("reverb_spectrum", _lib.ptr(h), L, int(n_samples), _lib.ptr(spec), _lib.stream_of(h))
    return spec


def reverb_impulse_spectrum(noise, decay, wet, sample_rate, n_samples):
    """modules.py:21-35: Reverb.build_impulse and its partition spectra for n_samples in one launch
    (equal to reverb_spectrum(reverb_build_impulse(...), n_samples) bit for bit).  No autograd: the
    module's backward differentiates through noise/decay/wet itself."""
    _dev(noise, decay, wet)
    L = noise.shape[0]
    n = _c(noise)
    spec = torch.empty(reverb_spectrum_floats(n_samples, L), dtype=torch.float32, device=n.device)
    _lib.call("reverb_impulse_spectrum", _lib.ptr(n), _lib.ptr(_c(decay)), _lib.ptr(_c(wet)), L,
              float(sample_rate), int(n_samples), _lib.ptr(spec), _lib.stream_of(n))
    return spec


def reverb_cache_bytes(n_samples, ir_length):
    return int(_lib.query("reverb_cache_bytes", int(n_samples), int(ir_length)))


def reverb_forward(x, noise, decay, wet, ir_length, sample_rate, cache, force=False, n_samples=None):
    """modules.py:21-35 Reverb.forward over a device IR cache that the launch validates against the
    parameters (ddsp_hip_reverb_forward) -> (out [B, T, 1], workspace, spectrum view of the cache).  With
    x None only the cache is validated (for inputs of n_samples).  No autograd (grad.ReverbFn wraps it)."""
    _dev(noise, decay, wet)
    if x is not None:
        _dev(x)
        B, T = x.shape[0], x.shape[1]
        xc = _c(x)
    else:
        B, T, xc = 0, int(n_samples), None
    L = int(ir_length)
    if cache.device != noise.device or cache.numel() < reverb_cache_bytes(T, L):
        raise RuntimeError("reverb_forward: cache on another device or too small")
    out = torch.empty(B, T, 1, dtype=torch.float32, device=noise.device) if B else None
    ws = _workspace(_lib.query("reverb_workspace_size", B, T, L), noise.device) if B else None
    _lib.call("reverb_forward", _lib.ptr(xc), _lib.ptr(_c(noise)), _lib.ptr(_c(decay)), _lib.ptr(_c(wet)), L,
              float(sample_rate), int(bool(force)), _lib.ptr(cache), cache.numel(), _lib.ptr(out), B, T,
              _lib.ptr(ws), ws.numel() if ws is not None else 0, _lib.stream_of(cache))
    spec = cache[:4 * reverb_spectrum_floats(T, L)].view(torch.float32)
    return out, ws, spec


def reverb_apply(x, spectrum, ir_length):
    """modules.py:28-35 Reverb.forward given the cached IR spectrum: x [B, T, 1] -> [B, T, 1]."""
    _dev(x, spectrum)
    if _wants_grad(x, spectrum):
        if spectrum.requires_grad:
            raise NotImplementedError("reverb_apply: the IR spectrum is not differentiable; use "
                                      "modules.Reverb (gradients for noise/decay/wet) instead")
        return _grad.ReverbApplyFn.apply(x, spectrum, int(ir_length))
    return _reverb_apply_launch(x, spectrum, ir_length)[0]


# ------------------------------------------------------------------------------------
# the decoder network's recurrence (decoder.py:33-68)
# ------------------------------------------------------------------------------------
def gru_supported(gru_module):
    """Shapes the step kernel takes: one layer, batch_first, unidirectional, biased, hidden % 64 == 0."""
    g = gru_module
    return (g.num_layers == 1 and g.batch_first and not g.bidirectional and g.bias and
            g.hidden_size % 64 == 0 and g.hidden_size <= 4096)


def gru(x, gru_module, h0=None, persistent_flags=0):
    """torch.nn.GRU(x, h0) forward (1 layer, batch_first) -> (out [B,T,H], h_T [1,B,H]): the input
    projection for all steps as one GEMM, the recurrence on the gfx950 kernels (gru_layer_launch); under
    autograd the backward (BPTT) runs on the step kernels too (grad.GRUFn).  ``persistent_flags``:
    the persistent launch's test hooks (GRU_SPREAD, GRU_NO_MASK_CHECK, GRU_FORCE_ABORT; 0 in use)."""
    _dev(x)
    if not gru_supported(gru_module):
        raise RuntimeError("gru: one layer, batch_first, unidirectional, with bias and hidden % 64 == 0 expected")
    g = gru_module
    params = (g.weight_ih_l0, g.weight_hh_l0, g.bias_ih_l0, g.bias_hh_l0)
    if _wants_grad(x, h0, *params):
        return _grad.GRUFn.apply(x, *params, h0)
    B, T, _ = x.shape
    H = g.hidden_size
    w_ih, w_hh, b_ih, b_hh = params
    out = torch.empty(B, T, H, dtype=torch.float32, device=x.device)
    h_last = torch.empty(1, B, H, dtype=torch.float32, device=x.device)
    h0c = _c(h0.reshape(B, H)) if h0 is not None else None
    gru_layer_launch(x, w_ih, b_ih, w_hh, b_hh, h0c, out, h_last, None, persistent_flags)
    return out, h_last


# include/ddsp_hip.h: ddsp_hip_gru_forward_persistent's flags (test hooks) and status bits
GRU_SPREAD, GRU_NO_MASK_CHECK, GRU_FORCE_ABORT = 1, 2, 4
GRU_STATUS_LOCAL, GRU_STATUS_RESCUED = 1, 2
_GRU_LAST = {}  # device index -> (route, persistent workspace or None) of the last gru_layer_launch


def gru_layer_launch(x, w_ih, b_ih, w_hh, b_hh, h0c, out, h_last, gates, persistent_flags=0):
    """The layer's forward on the device: the input projection for every step as one GEMM, then the
    recurrence as one persistent launch (ddsp_hip_gru_forward_persistent: hidden 512, batch <= 64, a stream
    that may use every CU) or on ddsp_hip_gru_forward's step kernels (a form with each step's projection
    inside the step launch measured slower: 13.3 vs 7.4-7.8 us per step).  A persistent launch
    that cannot get its workgroups resident aborts and its outputs are recomputed, on the same stream, with
    the step kernels' arithmetic (gru_rescue_kernel): the values are right on every route;
    ``gru_last_route`` tells which one ran.  Returns the route taken ("persistent" or "steps")."""
    B, T, I = x.shape
    H = w_hh.shape[1]
    xp = linear(_c(x).reshape(B * T, I), w_ih, b_ih).view(B, T, 3 * H)
    args = (_lib.ptr(xp), _lib.ptr(_c(w_hh)), _lib.ptr(_c(b_hh)), _lib.ptr(h0c), _lib.ptr(out), _lib.ptr(h_last),
            _lib.ptr(gates), B, T, H)
    # hidden 512, batch <= 64: the whole recurrence as one persistent launch (W_hh resident in registers, h
    # handed between the workgroups of a group); otherwise (ERANGE) one launch per step
    ws = _workspace(_lib.query("gru_persistent_workspace_size"), out.device)
    st = _lib.call("gru_forward_persistent", *args, int(persistent_flags), _lib.ptr(ws), ws.numel(),
                   _lib.stream_of(out), allow=(ERANGE,))
    dev = out.device.index if out.device.index is not None else torch.cuda.current_device()
    if st == ERANGE:
        _lib.call("gru_forward", *args, _lib.stream_of(out))
        _GRU_LAST[dev] = ("steps", None)
        return "steps"
    _GRU_LAST[dev] = ("persistent", ws)
    return "persistent"


def gru_last_route(device=None):
    """Which recurrence the last gru_layer_launch on ``device`` ran, read after a device synchronize:
    {"route": "persistent" | "steps" | None, "hand_off": "xcd_local" | "write_through" | None,
    "rescued": bool (the persistent launch aborted and the rescue kernel produced the outputs)}."""
    dev = torch.cuda.current_device() if device is None else torch.device(device).index or 0
    route, ws = _GRU_LAST.get(dev, (None, None))
    info = {"route": route, "hand_off": None, "rescued": False}
    if ws is not None:
        torch.cuda.synchronize(dev)
        off = int(_lib.query("gru_persistent_status_offset"))
        word = int(ws[off:off + 4].cpu().view(torch.int32)[0])
        info["rescued"] = bool(word & GRU_STATUS_RESCUED)
        if not info["rescued"]:
            info["hand_off"] = "xcd_local" if word & GRU_STATUS_LOCAL else "write_through"
    return info


def linear(x, weight, bias):
    """x [rows, in] @ weight[out, in]^T + bias -> [rows, out] (no autograd): ddsp_hip_linear — the bf16 matrix
    cores with the fp32-accurate three-term split — where it applies (in 512 / 1024, out a multiple of 512),
    else torch.addmm (hipBLASLt)."""
    _dev(x, weight, bias)
    rows, K = x.shape
    N = weight.shape[0]
    xc, wc, bc = _c(x), _c(weight), _c(bias)
    y = torch.empty(rows, N, dtype=torch.float32, device=x.device)
    st = _lib.call("linear", _lib.ptr(xc), K, K, _lib.ptr(wc), K, _lib.ptr(bc), _lib.ptr(y), N, rows, N,
                   _lib.stream_of(y), allow=(ERANGE,))
    return torch.addmm(bias, x, weight.t()) if st == ERANGE else y


def linear_weight_grad(grad_y, x):
    """grad_y [rows, out]^T @ x [rows, in] -> [out, in], a Linear's weight gradient (no autograd):
    ddsp_hip_linear_weight_grad — the bf16 matrix cores with the fp32-accurate three-term split, split over
    row ranges summed in a fixed order (any widths; torch.mm only past its 32-bit range offsets)."""
    _dev(grad_y, x)
    rows, M = grad_y.shape
    N = x.shape[1]
    gc, xc = _c(grad_y), _c(x)
    dw = torch.empty(M, N, dtype=torch.float32, device=x.device)
    ws = _workspace(_lib.query("linear_weight_grad_workspace_size", max(rows, 1), M, N), x.device)
    st = _lib.call("linear_weight_grad", _lib.ptr(gc), M, _lib.ptr(xc), N, _lib.ptr(dw), N, rows, M, N,
                   _lib.ptr(ws), ws.numel(), _lib.stream_of(dw), allow=(ERANGE,))
    return grad_y.t().mm(x) if st == ERANGE else dw


MLP_EXACT_F32 = 1  # include/ddsp_hip.h DDSP_HIP_MLP_EXACT_F32


def mlp_block(x, linear, norm, act, out=None, extras=(), flags=0):
    """ddsp/core.py:122-129, one whole block: LeakyReLU(LayerNorm(linear(x))) in one launch
    (ddsp_hip_mlp_block: the Linear on the matrix cores — at 512 inputs fp32-accurate bf16x3 products,
    ``flags=MLP_EXACT_F32`` the f32-input MFMA — LayerNorm + LeakyReLU in its epilogue).
    ``extras``: up to two [..., 1] tensors that are the Linear's LAST input features (the decoder's
    out_mlp input [gru_out, f0, loudness], decoder.py:68, given as x = gru_out, extras = (f0, loudness)).
    Returns None where the kernel does not apply (it is built for 512 output features);
    inference only."""
    _dev(x, linear.weight, linear.bias, norm.weight, norm.bias, *extras)
    n_out, n_in = linear.weight.shape
    K = x.shape[-1]
    if (len(extras) > 2 or K + len(extras) != n_in or n_out != 512 or tuple(norm.normalized_shape) != (n_out,)
            or any(e.shape != x.shape[:-1] + (1,) for e in extras)):
        return None
    xc = _c(x)
    lead = tuple(x.shape[:-1])
    rows = xc.numel() // K if K else 0
    if out is None:
        out = torch.empty(*lead, n_out, dtype=torch.float32, device=x.device)
    elif (tuple(out.shape) != lead + (n_out,) or out.stride(-1) != 1 or
          any(out.stride(i) != out.stride(i + 1) * out.shape[i + 1] for i in range(out.dim() - 2))):
        return None
    y_ld = out.stride(-2) if out.dim() >= 2 else n_out
    ec = [_c(e) for e in extras]
    st = _lib.call("mlp_block", _lib.ptr(xc), K, K, _lib.ptr(_c(linear.weight)), n_in, _lib.ptr(_c(linear.bias)),
                   _lib.ptr(ec[0] if ec else None), _lib.ptr(ec[1] if len(ec) > 1 else None), 1,
                   _lib.ptr(_c(norm.weight)), _lib.ptr(_c(norm.bias)), float(norm.eps), float(act.negative_slope),
                   _lib.ptr(out), int(y_ld), int(rows), n_out, int(flags), _lib.stream_of(out), allow=(ERANGE,))
    return None if st == ERANGE else out


def projections(x, lin1, lin2, pad_to=64):
    """decoder.py:106-117 in ONE launch: ddsp_hip_projections — both Linears on the bf16 matrix cores with the
    fp32-accurate three-term split, reading each layer's parameters where they lie (at 512 inputs, 16-byte
    aligned rows).  Elsewhere ONE library GEMM: both layers' parameters stacked, fresh every call, into a
    zero-padded [n_pad, K] buffer (ddsp_hip_stack_rows, one launch; n_pad a multiple of ``pad_to``:
    hipBLASLt runs 192 outputs in 28-30 us, the unpadded 166 in 38-39), then F.linear.  Returns the two
    outputs as column slices of one [..., n] result.  Nothing is cached on the modules."""
    _dev(x, lin1.weight, lin1.bias, lin2.weight, lin2.bias)
    n1, n2, K = lin1.out_features, lin2.out_features, x.shape[-1]
    xc, w1, w2 = _c(x), _c(lin1.weight), _c(lin2.weight)
    rows = xc.numel() // K if K else 0
    n4 = -(-(n1 + n2) // 4) * 4  # row stride of the result: 16-byte aligned rows
    y = torch.empty(*x.shape[:-1], n4, dtype=torch.float32, device=x.device)
    st = _lib.call("projections", _lib.ptr(xc), K, K, _lib.ptr(w1), w1.stride(0), _lib.ptr(_c(lin1.bias)), n1,
                   _lib.ptr(w2), w2.stride(0), _lib.ptr(_c(lin2.bias)), n2, _lib.ptr(y), n4, rows,
                   _lib.stream_of(y), allow=(ERANGE,))
    if st != ERANGE:
        return y[..., :n1], y[..., n1:n1 + n2]
    n_pad = -(-(n1 + n2) // pad_to) * pad_to
    w = torch.empty(n_pad, K, dtype=torch.float32, device=x.device)
    b = torch.empty(n_pad, dtype=torch.float32, device=x.device)
    _lib.call("stack_rows", _lib.ptr(w1), w1.stride(0), _lib.ptr(_c(lin1.bias)), n1, _lib.ptr(w2), w2.stride(0),
              _lib.ptr(_c(lin2.bias)), n2, K, _lib.ptr(w), _lib.ptr(b), n_pad, _lib.stream_of(w))
    y = torch.nn.functional.linear(x, w, b)  # (this package's matrix-core projection kernel ran 40-44 us)
    return y[..., :n1], y[..., n1:n1 + n2]


def layer_norm_leaky_relu(h, norm, act, out=None, w1=None, b1=None):
    """ddsp/core.py:122-129 after one block's Linear: LeakyReLU(LayerNorm(h)) in one pass
    (ddsp_hip_layer_norm_leaky_relu).  h [..., cols] contiguous; or, with w1/b1 (a Linear with one input
    feature), h [..., 1] is that Linear's input and the block's pre-activation is h * w1 + b1.  ``out``
    (optional) may be a column slice of a wider buffer with one row stride.  Returns None where the
    kernel does not apply (the caller runs torch's modules); inference only."""
    _dev(h, norm.weight, norm.bias)
    cols = int(norm.normalized_shape[-1])
    if len(norm.normalized_shape) != 1 or (w1 is None and h.shape[-1] != cols) or (w1 is not None and h.shape[-1] != 1):
        return None
    if not h.is_contiguous():
        h = h.contiguous()
    lead = tuple(h.shape[:-1])
    rows = h.numel() // h.shape[-1] if h.shape[-1] else 0
    if out is None:
        out = torch.empty(*lead, cols, dtype=torch.float32, device=h.device)
    elif (tuple(out.shape) != lead + (cols,) or out.stride(-1) != 1 or
          any(out.stride(i) != out.stride(i + 1) * out.shape[i + 1] for i in range(out.dim() - 2))):
        return None
    y_ld = out.stride(-2) if out.dim() >= 2 else cols
    g, b = _c(norm.weight), _c(norm.bias)
    w1c = _c(w1) if w1 is not None else None
    b1c = _c(b1) if b1 is not None else None
    st = _lib.call("layer_norm_leaky_relu", _lib.ptr(h), int(h.shape[-1]), _lib.ptr(w1c), _lib.ptr(b1c), _lib.ptr(g),
                   _lib.ptr(b), float(norm.eps), float(act.negative_slope), _lib.ptr(out), int(y_ld), int(rows), cols,
                   _lib.stream_of(out), allow=(ERANGE,))
    return None if st == ERANGE else out


def dense_input(x, width=None, ld=None, scale=1.0, shift=0.0, first=None, norm=None, x_copy=None):
    """One input segment of dense_rows: x [rows, ld] (or, with `first` = a K=1 nn.Linear, one value
    per row at x[r * ld]); `norm` = an nn.LayerNorm applied with LeakyReLU(0.01) after it."""
    inp = _lib.DenseInput()
    inp.x = x.data_ptr()
    inp.scale, inp.shift = float(scale), float(shift)
    if first is not None:
        inp.w1, inp.b1 = first.weight.data_ptr(), first.bias.data_ptr()
        inp.width = first.out_features
    else:
        inp.width = int(width if width is not None else x.shape[-1])
    inp.ld = int(ld if ld is not None else inp.width)
    if norm is not None:
        if norm.eps != 1e-5 or norm.weight is None:
            raise RuntimeError("dense_input: LayerNorm(eps=1e-5, elementwise_affine) expected")
        inp.gamma, inp.beta = norm.weight.data_ptr(), norm.bias.data_ptr()
    if x_copy is not None:
        inp.x_copy = x_copy.data_ptr()
    return inp


def dense_rows(problems, rows, device):
    """ddsp_hip_dense_rows: up to two Linears (each `(inputs, linear, y)`, inputs from dense_input,
    y [rows, out_features] contiguous) over `rows` <= 8 rows in one launch (core.py:122-129 blocks
    with the LayerNorm/LeakyReLU of the previous block folded into the input)."""
    arr = (_lib.DenseProblem * len(problems))()
    for i, (inputs, lin, y) in enumerate(problems):
        P = arr[i]
        for j, inp in enumerate(inputs):
            P.inputs[j] = inp
        P.n_inputs = len(inputs)
        if sum(inp.width for inp in inputs) != lin.in_features:
            raise RuntimeError("dense_rows: inputs do not add up to the Linear's in_features")
        P.weight = lin.weight.data_ptr()
        P.bias = lin.bias.data_ptr() if lin.bias is not None else None
        P.y = y.data_ptr()
        P.ldy = y.shape[-1]
        P.out_features = lin.out_features
    _lib.call("dense_rows", arr, len(problems), int(rows),
              ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream))


# ------------------------------------------------------------------------------------
# training loss (ddsp/core.py:10-41; train.py:70-76)
# ------------------------------------------------------------------------------------
def safe_log(x):
    """ddsp/core.py:10-11."""
    return torch.log(x + 1e-7)


def stft_magnitude(signal, n_fft, hop):
    """|torch.stft(signal, n_fft, hop, n_fft, hann_window(n_fft), center=True, normalized=True)|
    for signal [B, T] -> [B, n_fft/2+1, frames] (a transposed view of the kernel's frame-major
    output; the values and shape are the reference's)."""
    _dev(signal)
    if signal.dim() != 2:
        raise RuntimeError(f"stft_magnitude: expected [batch, time], got {tuple(signal.shape)}")
    if _wants_grad(signal):
        return _grad.StftMagFn.apply(signal, int(n_fft), int(hop))
    B, T = signal.shape
    x = _c(signal)
    frames = int(_lib.query("stft_frames", T, int(hop)))
    M = torch.empty(B, frames, int(n_fft) // 2 + 1, dtype=torch.float32, device=x.device)
    _lib.call("stft_magnitude", _lib.ptr(x), _lib.ptr(M), B, T, int(n_fft), int(hop), _lib.stream_of(x))
    return M.transpose(1, 2)


def multiscale_fft(signal, scales, overlap):
    """ddsp/core.py:27-41: one magnitude spectrogram per scale, hop int(s * (1 - overlap))."""
    return [stft_magnitude(signal, s, int(s * (1 - overlap))) for s in scales]


def _reverb_apply_launch(x, spectrum, ir_length):
    """-> (out, workspace); on return the workspace's first reverb_input_spectra_bytes hold x's
    partition spectra (reused by the backward)."""
    B, T = x.shape[0], x.shape[1]
    if spectrum.numel() != reverb_spectrum_floats(T, ir_length):
        raise RuntimeError("reverb_apply: spectrum was computed for a different length")
    xc = _c(x)
    out = torch.empty(B, T, 1, dtype=torch.float32, device=x.device)
    ws = _workspace(_lib.query("reverb_workspace_size", B, T, int(ir_length)), x.device)
    _lib.call("reverb_apply", _lib.ptr(xc), _lib.ptr(spectrum), _lib.ptr(out), B, T, int(ir_length),
              _lib.ptr(ws), ws.numel(), _lib.stream_of(out))
    return out, ws


from . import grad as _grad  # noqa: E402  (autograd Functions over the backward kernels)


_MASKED_STREAMS = {}


@atexit.register
def _release_masked_streams():
    """Destroy the CU-masked streams before the HIP runtime tears down (left to the runtime's own
    teardown they crashed rocprofv3's finalisation)."""
    if not _MASKED_STREAMS:
        return
    try:
        torch.cuda.synchronize()
        lib = _lib.load()
        for s in _MASKED_STREAMS.values():
            lib.ddsp_hip_stream_destroy(s.cuda_stream)
    except Exception:  # teardown path: nothing left to report to
        pass
    _MASKED_STREAMS.clear()


def cu_mask_words(cus, n_cu):
    """The 32-bit mask words of ddsp_hip_stream_create_cu_masked: bit c of word c // 32 set for
    every CU index c in ``cus`` (indices must lie in [0, n_cu))."""
    words = [0] * ((int(n_cu) + 31) // 32)
    for c in cus:
        c = int(c)
        if not 0 <= c < n_cu:
            raise ValueError(f"CU index {c} outside [0, {n_cu})")
        words[c // 32] |= 1 << (c % 32)
    return words


def cu_masked_stream(cus, n_cu=None):
    """A torch stream whose kernels run only on the CUs with the given indices
    (ddsp_hip_stream_create_cu_masked; see synth.PipelinedSynthPath for how indices map to XCDs).
    One stream per (device, mask), kept for the life of the process: the caching allocator may
    still hold blocks tagged with it, so it is never destroyed under them."""
    dev = torch.cuda.current_device()
    cus = tuple(sorted(set(int(c) for c in cus)))
    n_cu = n_cu or torch.cuda.get_device_properties(dev).multi_processor_count
    if not cus or cus[0] < 0 or cus[-1] >= n_cu:
        raise ValueError("CU indices out of range")
    key = (dev, cus)
    if key not in _MASKED_STREAMS:
        words = (ctypes.c_uint32 * ((n_cu + 31) // 32))(*cu_mask_words(cus, n_cu))
        handle = ctypes.c_void_p()
        _lib.call("stream_create_cu_masked", words, len(words), ctypes.byref(handle))
        _MASKED_STREAMS[key] = torch.cuda.ExternalStream(handle.value, device=torch.device("cuda", dev))
    return _MASKED_STREAMS[key]
