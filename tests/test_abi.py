"""CPU-side checks of the drop-in boundary: the C-ABI library builds, loads and exports every
symbol include/ddsp_hip.h declares (no compute: there is no GPU here), and the host layer
refuses CPU tensors instead of falling back."""
import os
import re
import subprocess

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ddsp_hip.h")


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"\b(ddsp_hip_\w+)\s*\(", text)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    assert "ddsp_hip_harmonic_synth" in syms and "ddsp_hip_filtered_noise" in syms
    assert len(syms) >= 19


def test_library_exports_every_declared_symbol():
    from ddsp_pytorch_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        subprocess.run(["make", "-C", ROOT, "-j4"], check=True)
    lib = _lib.load()
    nm = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                        text=True, check=True).stdout
    exported = set(re.findall(r"\b(ddsp_hip_\w+)\b", nm))
    missing = [s for s in declared_symbols() if s not in exported]
    assert not missing, missing
    # and nothing beyond it: the exported ddsp_hip_* set IS the header's
    undeclared = sorted(exported - set(declared_symbols()))
    assert not undeclared, undeclared
    # the ctypes table binds exactly the declared set
    assert set(_lib.SIGNATURES) == set(declared_symbols())
    assert lib.ddsp_hip_version() >= 100
    assert lib.ddsp_hip_status_string(1) == b"invalid argument or shape"


def test_abi_rejects_bad_arguments_without_launching():
    from ddsp_pytorch_amd import _lib
    lib = _lib.load()
    import ctypes
    null = ctypes.c_void_p(0)
    # negative sizes / missing buffers are rejected before any HIP call
    assert lib.ddsp_hip_scale_function(null, null, -1, 0.0, null) == 1
    assert lib.ddsp_hip_upsample(null, null, 1, 1, 1, 0, null) == 1
    assert lib.ddsp_hip_harmonic_synth(null, null, null, 1, 10, 4, 48000.0, null, 0, null) == 1
    assert lib.ddsp_hip_filtered_noise(null, null, 0, 0, null, null, null, 1, 1, 1, 512, null) == 1
    assert lib.ddsp_hip_fft_convolve(null, null, null, 4, 3, 100, null, 0, null) == 1
    # empty inputs are a no-op success
    assert lib.ddsp_hip_scale_function(null, null, 0, 0.0, null) == 0
    assert lib.ddsp_hip_harmonic_synth_frames(null, null, null, 0, null, 0, 5, 4, 512, 48000.0, null) == 0


def test_no_cpu_fallback():
    import ddsp_pytorch_amd as dd
    x = torch.zeros(1, 4, 3)
    with pytest.raises(RuntimeError, match="HIP device"):
        dd.core.scale_function(x)
    with pytest.raises(RuntimeError, match="HIP device"):
        dd.core.harmonic_synth(torch.zeros(1, 8, 1), torch.zeros(1, 8, 4), 48000)
    with pytest.raises(RuntimeError, match="HIP device"):
        dd.HarmonicSynth(512, 48000).get_controls(x[..., :1], x, x[..., :1])


def test_library_has_no_process_global_state():
    """The boundary contract: no mutable process-wide state, no
    environment switches and no library-owned device allocations in the product sources —
    workspaces come from the caller, so every entry point is reentrant."""
    csrc = os.path.join(ROOT, "ddsp_pytorch_amd", "csrc")
    pat = re.compile(r"static\s+std::(atomic|map|mutex)|getenv|hipMalloc|DDSP_PROBE_")
    hits = []
    for f in sorted(os.listdir(csrc)):
        if f.endswith((".hip", ".h", ".cpp")):
            for i, line in enumerate(open(os.path.join(csrc, f)), 1):
                if pat.search(line):
                    hits.append(f"{f}:{i}: {line.strip()}")
    assert not hits, hits


def test_module_state_dict_keys_match_reference_layout():
    import ddsp_pytorch_amd as dd
    m = dd.DDSPDecoder(32, 100, 65, 48000, 512, True)
    keys = set(m.state_dict())
    for k in ("sample_rate", "block_size", "phase", "decoder.cache_gru", "decoder.gru.weight_ih_l0",
              "decoder.f0_mlp.0.weight", "decoder.out_mlp.7.bias", "harmonic_proj.weight",
              "noise_proj.bias", "reverb.noise", "reverb.decay", "reverb.wet", "reverb.t"):
        assert k in keys, k


def test_training_entry_points_reject_bad_arguments_without_launching():
    """The backward / loss / GRU entry points validate before any HIP call (status codes only)."""
    import ctypes
    from ddsp_pytorch_amd import _lib
    lib = _lib.load()
    null = ctypes.c_void_p(0)
    EINVAL, EWS, ERANGE = 1, 4, 5
    # scale / upsample backward
    assert lib.ddsp_hip_scale_function_backward(null, null, null, -1, 0.0, null) == EINVAL
    assert lib.ddsp_hip_scale_function_backward(null, null, null, 0, 0.0, null) == 0
    assert lib.ddsp_hip_upsample_backward(null, null, 1, 1, 1, 0, null) == EINVAL
    # harmonic / noise / fused backward
    assert lib.ddsp_hip_harmonic_synth_params_backward(null, null, null, null, 1, 2, 4, 64, 48000.0, null) == EINVAL
    assert lib.ddsp_hip_harmonic_synth_params_backward(null, null, null, null, 0, 2, 4, 64, 48000.0, null) == 0
    assert lib.ddsp_hip_filtered_noise_backward(null, null, 0, 0, 0, 0.0, null, null, 1, 1, 1, 512, null) == EINVAL
    assert lib.ddsp_hip_synth_frames_backward(null, null, null, 0.0, null, 0, 0, null, null, null, null,
                                              1, 2, 4, 65, 512, 48000.0, null) == EINVAL
    # reverb backward: nothing requested / workspace
    assert lib.ddsp_hip_reverb_backward(null, null, null, null, null, null, 1, 100, 10, null, 0, null) == EINVAL
    # reverb backward with the parameters' gradients: parameter pointers missing, negative batch, bad rate
    assert lib.ddsp_hip_reverb_backward_params(null, null, null, null, null, null, null, 48000.0, null, null, null,
                                               null, 1, 100, 10, null, 0, null) == EINVAL
    assert lib.ddsp_hip_reverb_backward_params(null, null, null, null, null, null, null, 0.0, null, null, null,
                                               null, -1, 100, 10, null, 0, null) == EINVAL
    # the decoder's projections: missing parameters, a result narrower than both layers, K outside the kernel
    assert lib.ddsp_hip_projections(null, 512, 512, null, 512, null, 101, null, 512, null, 65, null, 166, 10,
                                    null) == EINVAL
    assert lib.ddsp_hip_projections(null, 512, 512, null, 512, null, 101, null, 512, null, 65, null, 166, 0,
                                    null) == EINVAL
    dummy = ctypes.c_void_p(256)  # never dereferenced: every call below returns before any launch
    assert lib.ddsp_hip_projections(dummy, 512, 512, dummy, 512, dummy, 101, dummy, 512, dummy, 65, dummy, 100, 10,
                                    null) == EINVAL
    assert lib.ddsp_hip_projections(dummy, 256, 256, dummy, 256, dummy, 101, dummy, 256, dummy, 65, dummy, 168, 10,
                                    null) == ERANGE
    assert lib.ddsp_hip_projections(dummy, 512, 512, dummy, 512, dummy, 101, dummy, 512, dummy, 65, dummy, 168, 0,
                                    null) == 0
    # a Linear's weight gradient: missing operands, sizes outside the kernel (32-bit offsets over a row range),
    # a short workspace (ragged widths are in range)
    assert lib.ddsp_hip_linear_weight_grad(null, 512, null, 512, null, 512, 10, 512, 512, null, 0, null) == EINVAL
    assert lib.ddsp_hip_linear_weight_grad(dummy, 512, dummy, 512, dummy, 500, 10, 512, 512, null, 0, null) == EINVAL
    assert lib.ddsp_hip_linear_weight_grad(dummy, 1 << 27, dummy, 512, dummy, 512, 10, 512, 512, null, 0, null) == ERANGE
    assert lib.ddsp_hip_linear_weight_grad(dummy, 166, dummy, 512, dummy, 512, 10, 166, 512, null, 0, null) == EWS
    assert lib.ddsp_hip_linear_weight_grad(dummy, 512, dummy, 514, dummy, 514, 10, 512, 514, null, 0, null) == EWS
    assert lib.ddsp_hip_linear_weight_grad(dummy, 512, dummy, 512, dummy, 512, 10, 512, 512, null, 0, null) == EWS
    assert lib.ddsp_hip_linear_weight_grad_workspace_size(12800, 512, 512) >= 4 * 512 * 512
    assert lib.ddsp_hip_linear_weight_grad_workspace_size(0, 512, 512) == 0
    # STFT: sizes outside the kernel's range, padding longer than the signal
    assert lib.ddsp_hip_stft_magnitude(null, null, 1, 1000, 100, 25, null) == ERANGE
    assert lib.ddsp_hip_stft_magnitude(null, null, 1, 1000, 8192, 2048, null) == ERANGE
    assert lib.ddsp_hip_stft_magnitude(null, null, 1, 100, 256, 64, null) == EINVAL
    assert lib.ddsp_hip_stft_frames(102400, 1024) == 101
    n = (ctypes.c_int64 * 1)(512)
    h = (ctypes.c_int64 * 1)(128)
    assert lib.ddsp_hip_spectral_loss(null, null, 1, 1000, n, h, 1, null, null, null, 0, null) == EINVAL
    assert lib.ddsp_hip_spectral_loss_workspace_size(2, 1000, n, h, 1) > 0
    # GRU: hidden not a multiple of 64 is outside the step kernel's range
    assert lib.ddsp_hip_gru_forward(null, null, null, null, null, null, null, 1, 4, 0, null) == EINVAL
    assert lib.ddsp_hip_gru_forward(null, null, null, null, null, null, null, 0, 4, 64, null) == 0
    one = ctypes.c_void_p(16)  # non-null placeholders: the range check comes first
    assert lib.ddsp_hip_gru_forward(one, one, one, null, one, null, null, 1, 4, 96, null) == ERANGE
    assert lib.ddsp_hip_gru_backward(one, one, one, null, null, null, one, one, null, 1, 4, 64, null, 0, null) == EWS
    # persistent GRU: unknown flags, then the range checks, before any HIP call
    assert lib.ddsp_hip_gru_forward_persistent(one, one, one, null, one, null, null, 1, 4, 512, 8, one, 4096,
                                               null) == EINVAL
    assert lib.ddsp_hip_gru_forward_persistent(one, one, one, null, one, null, null, 65, 4, 512, 0, one, 4096,
                                               null) == ERANGE
    assert lib.ddsp_hip_gru_forward_persistent(one, one, one, null, one, null, null, 1, 4, 512, 0, one, 4,
                                               null) == EWS
    assert lib.ddsp_hip_gru_persistent_status_offset() + 4 <= lib.ddsp_hip_gru_persistent_workspace_size()
    assert lib.ddsp_hip_gru_backward_persistent(one, one, one, null, null, null, one, one, null, 1, 4, 512, 8, one,
                                                4096, null) == EINVAL
    assert lib.ddsp_hip_gru_backward_persistent(one, one, one, null, null, null, one, one, null, 65, 4, 512, 0, one,
                                                4096, null) == ERANGE
