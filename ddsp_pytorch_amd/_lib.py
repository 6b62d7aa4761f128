"""ctypes binding of the C-ABI library ``lib/libddsp_hip.so`` (declared in include/ddsp_hip.h).

This is the host side of the drop-in boundary: torch supplies device memory and the
current HIP stream; every entry point is a plain C function taking device pointers,
sizes and a ``hipStream_t``.  There is no CPU fallback: if the library is missing or a
tensor is not on a HIP device, the call raises.
"""
import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DDSP_HIP_LIB", os.path.join(_HERE, "lib", "libddsp_hip.so"))

_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_F = ctypes.c_float
_I = ctypes.c_int
_U64 = ctypes.c_uint64
_SZ = ctypes.c_size_t



class DenseInput(ctypes.Structure):
    """ddsp_hip_dense_input (include/ddsp_hip.h)."""
    _fields_ = [("x", _P), ("ld", _I64), ("width", _I64), ("scale", _F), ("shift", _F), ("w1", _P),
                ("b1", _P), ("gamma", _P), ("beta", _P), ("x_copy", _P)]


DENSE_MAX_INPUTS = 3
DENSE_MAX_PROBLEMS = 2


class DenseProblem(ctypes.Structure):
    """ddsp_hip_dense_problem (include/ddsp_hip.h)."""
    _fields_ = [("inputs", DenseInput * DENSE_MAX_INPUTS), ("n_inputs", _I), ("weight", _P), ("bias", _P),
                ("y", _P), ("ldy", _I64), ("out_features", _I64)]


# name -> (restype, argtypes); must match include/ddsp_hip.h exactly
SIGNATURES = {
    "ddsp_hip_status_string": (ctypes.c_char_p, [_I]),
    "ddsp_hip_version": (_I, []),
    "ddsp_hip_stream_create_cu_masked": (_I, [ctypes.POINTER(ctypes.c_uint32), _I, ctypes.POINTER(_P)]),
    "ddsp_hip_stream_destroy": (_I, [_P]),
    "ddsp_hip_scale_function": (_I, [_P, _P, _I64, _F, _P]),
    "ddsp_hip_remove_above_nyquist": (_I, [_P, _P, _P, _I64, _I64, _F, _P]),
    "ddsp_hip_upsample": (_I, [_P, _P, _I64, _I64, _I64, _I64, _P]),
    "ddsp_hip_harmonic_synth_workspace_size": (_SZ, [_I64, _I64]),
    "ddsp_hip_harmonic_synth": (_I, [_P, _P, _P, _I64, _I64, _I64, _F, _P, _SZ, _P]),
    "ddsp_hip_phase": (_I, [_P, _P, _I64, _I64, _F, _P, _SZ, _P]),
    "ddsp_hip_amp_to_impulse_response": (_I, [_P, _P, _I64, _I64, _I64, _P]),
    "ddsp_hip_fft_convolve_workspace_size": (_SZ, [_I64, _I64, _I64]),
    "ddsp_hip_fft_convolve": (_I, [_P, _P, _P, _I64, _I64, _I64, _P, _SZ, _P]),
    "ddsp_hip_harmonic_controls": (_I, [_P, _I64, _P, _I64, _P, _P, _P, _I64, _I64, _F, _P]),
    "ddsp_hip_harmonic_synth_frames": (_I, [_P, _P, _P, _I, _P, _I64, _I64, _I64, _I64, _F, _P]),
    "ddsp_hip_harmonic_synth_params": (_I, [_P, _P, _P, _I64, _I64, _I64, _I64, _F, _P]),
    "ddsp_hip_filtered_noise": (_I, [_P, _P, _U64, _U64, _P, _P, _P, _I64, _I64, _I64, _I64, _P]),
    "ddsp_hip_filtered_noise_params": (_I, [_P, _F, _P, _U64, _U64, _P, _P, _P, _I64, _I64, _I64, _I64, _P]),
    "ddsp_hip_synth_frames": (_I, [_P, _P, _P, _F, _P, _U64, _U64, _P, _P, _P, _I64, _I64, _I64, _I64,
                                   _I64, _F, _P]),
    "ddsp_hip_synth_frames_controls": (_I, [_P, _P, _I64, _P, _I64, _F, _P, _U64, _U64, _P, _P, _P, _P, _I64,
                                            _I64, _I64, _I64, _I64, _F, _P]),
    "ddsp_hip_synth_frames_controls_prefix": (_I, [_P, _P, _I64, _P, _I64, _F, _P, _U64, _U64, _P, _P, _P, _P, _P,
                                                   _I64, _I64, _I64, _I64, _I64, _F, _P]),
    "ddsp_hip_frame_phase_prefix": (_I, [_P, _I64, _I64, _I64, _F, _P, _P]),
    "ddsp_hip_synth_frames_counter": (_I, [_P, _P, _P, _F, _U64, _P, _P, _I64, _I64, _I64, _I64, _I64, _F, _P]),
    "ddsp_hip_reverb_build_impulse": (_I, [_P, _P, _P, _P, _I64, _F, _P]),
    "ddsp_hip_reverb_spectrum_floats": (_SZ, [_I64, _I64]),
    "ddsp_hip_reverb_workspace_size": (_SZ, [_I64, _I64, _I64]),
    "ddsp_hip_reverb_spectrum": (_I, [_P, _I64, _I64, _P, _P]),
    "ddsp_hip_reverb_impulse_spectrum": (_I, [_P, _P, _P, _I64, _F, _I64, _P, _P]),
    "ddsp_hip_reverb_apply": (_I, [_P, _P, _P, _I64, _I64, _I64, _P, _SZ, _P]),
    "ddsp_hip_reverb_cache_bytes": (_SZ, [_I64, _I64]),
    "ddsp_hip_reverb_forward": (_I, [_P, _P, _P, _P, _I64, _F, _I, _P, _SZ, _P, _I64, _I64, _P, _SZ, _P]),
    "ddsp_hip_dense_rows": (_I, [_P, _I, _I64, _P]),
    "ddsp_hip_mlp_block": (_I, [_P, _I64, _I64, _P, _I64, _P, _P, _P, _I64, _P, _P, _F, _F, _P, _I64, _I64, _I64, _I,
                                _P]),
    "ddsp_hip_linear": (_I, [_P, _I64, _I64, _P, _I64, _P, _P, _I64, _I64, _I64, _P]),
    "ddsp_hip_layer_norm_leaky_relu": (_I, [_P, _I64, _P, _P, _P, _P, _F, _F, _P, _I64, _I64, _I64, _P]),
    "ddsp_hip_layer_norm_leaky_relu_backward_workspace_size": (_SZ, [_I64]),
    "ddsp_hip_linear_weight_grad_workspace_size": (_SZ, [_I64, _I64, _I64]),
    "ddsp_hip_linear_weight_grad": (_I, [_P, _I64, _P, _I64, _P, _I64, _I64, _I64, _I64, _P, _SZ, _P]),
    "ddsp_hip_layer_norm_leaky_relu_backward": (_I, [_P, _I64, _P, _P, _F, _F, _P, _I64, _P, _I64, _P, _P, _I64, _I64, _P, _SZ, _P]),
    "ddsp_hip_projections": (_I, [_P, _I64, _I64, _P, _I64, _P, _I64, _P, _I64, _P, _I64, _P, _I64, _I64, _P]),
    "ddsp_hip_stack_rows": (_I, [_P, _I64, _P, _I64, _P, _I64, _P, _I64, _I64, _P, _P, _I64, _P]),
    "ddsp_hip_gru_forward": (_I, [_P, _P, _P, _P, _P, _P, _P, _I64, _I64, _I64, _P]),
    "ddsp_hip_gru_persistent_workspace_size": (_SZ, []),
    "ddsp_hip_gru_persistent_status_offset": (_SZ, []),
    "ddsp_hip_gru_forward_persistent": (_I, [_P, _P, _P, _P, _P, _P, _P, _I64, _I64, _I64, _I, _P, _SZ, _P]),
    "ddsp_hip_gru_backward_persistent": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _I64, _I64, _I64, _I, _P, _SZ, _P]),
    "ddsp_hip_gru_backward_workspace_size": (_SZ, [_I64, _I64]),
    "ddsp_hip_gru_backward": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _I64, _I64, _I64, _P, _SZ, _P]),
    # multiscale STFT (training loss)
    "ddsp_hip_stft_frames": (_I64, [_I64, _I64]),
    "ddsp_hip_stft_magnitude": (_I, [_P, _P, _I64, _I64, _I64, _I64, _P]),
    "ddsp_hip_stft_backward_workspace_size": (_SZ, [_I64, _I64, _I64, _I64]),
    "ddsp_hip_stft_magnitude_backward": (_I, [_P, _P, _P, _I64, _I64, _I64, _I64, _P, _SZ, _P]),
    "ddsp_hip_spectral_loss_workspace_size": (_SZ, [_I64, _I64, _P, _P, _I]),
    "ddsp_hip_spectral_loss": (_I, [_P, _P, _I64, _I64, _P, _P, _I, _P, _P, _P, _SZ, _P]),
    # backward
    "ddsp_hip_scale_function_backward": (_I, [_P, _P, _P, _I64, _F, _P]),
    "ddsp_hip_upsample_backward": (_I, [_P, _P, _I64, _I64, _I64, _I64, _P]),
    "ddsp_hip_harmonic_synth_backward": (_I, [_P, _P, _P, _I64, _I64, _I64, _P]),
    "ddsp_hip_amp_to_impulse_response_backward": (_I, [_P, _P, _I64, _I64, _I64, _P]),
    "ddsp_hip_harmonic_controls_backward": (_I, [_P, _I64, _P, _I64, _P, _P, _P, _P, _P, _I64, _I64, _F, _P]),
    "ddsp_hip_harmonic_synth_frames_backward": (_I, [_P, _P, _P, _P, _P, _P, _I64, _I64, _I64, _I64, _F, _P]),
    "ddsp_hip_harmonic_synth_params_backward": (_I, [_P, _P, _P, _P, _I64, _I64, _I64, _I64, _F, _P]),
    "ddsp_hip_synth_frames_backward": (_I, [_P, _P, _P, _F, _P, _U64, _U64, _P, _P, _P, _P, _I64, _I64, _I64,
                                            _I64, _I64, _F, _P]),
    "ddsp_hip_filtered_noise_backward": (_I, [_P, _P, _U64, _U64, _I, _F, _P, _P, _I64, _I64, _I64, _I64, _P]),
    "ddsp_hip_reverb_apply_transposed": (_I, [_P, _P, _P, _I64, _I64, _I64, _P, _SZ, _P]),
    "ddsp_hip_reverb_input_spectra_bytes": (_SZ, [_I64, _I64]),
    "ddsp_hip_reverb_backward_workspace_size": (_SZ, [_I64, _I64, _I64, _I]),
    "ddsp_hip_reverb_backward": (_I, [_P, _P, _P, _P, _P, _P, _I64, _I64, _I64, _P, _SZ, _P]),
    "ddsp_hip_reverb_backward_params": (_I, [_P, _P, _P, _P, _P, _P, _P, _F, _P, _P, _P, _P, _I64, _I64, _I64, _P,
                                            _SZ, _P]),
    "ddsp_hip_reverb_impulse_backward_workspace_size": (_SZ, [_I64]),
    "ddsp_hip_reverb_impulse_backward": (_I, [_P, _P, _P, _P, _I64, _I64, _F, _P, _P, _P, _P, _SZ, _P]),
}

_lib = None
_lock = threading.Lock()


def load():
    """Load (once) and return the C-ABI library; raises if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(
                    f"ddsp_hip: native library not found at {LIB_PATH}; run `make` "
                    "(or __graft_entry__.build()) — there is no CPU fallback")
            lib = ctypes.CDLL(LIB_PATH)
            variant = "DDSP_HIP_LIB" in os.environ  # an A/B build of another revision (tools/ab_*.sh)
            for name, (res, args) in SIGNATURES.items():
                if variant and not hasattr(lib, name):
                    continue  # an entry point that revision does not have: absent, not an error
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _lib = lib
    return _lib


ERANGE = 5  # DDSP_HIP_ERANGE


def call(name, *args, allow=()):
    """Invoke ddsp_hip_<name>; map a non-zero status (other than those in `allow`) to RuntimeError.
    An A/B build of an older revision (DDSP_HIP_LIB) that lacks an entry point whose caller has a
    fallback (ERANGE allowed) answers ERANGE, so that the caller's fallback runs."""
    lib = load()
    fn = getattr(lib, "ddsp_hip_" + name, None)
    if fn is None:
        if ERANGE in allow and "DDSP_HIP_LIB" in os.environ:
            return ERANGE
        raise RuntimeError(f"ddsp_hip: entry point ddsp_hip_{name} is missing from {LIB_PATH}")
    st = fn(*args)
    if st in allow:
        return st
    if st != 0:
        msg = lib.ddsp_hip_status_string(st).decode()
        raise RuntimeError(f"ddsp_hip_{name} failed with status {st}: {msg}")
    return 0


def query(name, *args):
    return getattr(load(), "ddsp_hip_" + name)(*args)


def stream_of(t):
    """The current HIP stream of tensor t's device, as a void*."""
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


class _TensorPtr(ctypes.c_void_p):
    """A device pointer that keeps its tensor alive: callers write ``ptr(_c(x))``, and the contiguous
    temporary must not return its memory to torch's caching allocator (which could hand it to the
    next temporary) before the launch that reads it has been enqueued."""


def ptr(t):
    if t is None:
        return ctypes.c_void_p(0)
    p = _TensorPtr(t.data_ptr())
    p._tensor = t
    return p
