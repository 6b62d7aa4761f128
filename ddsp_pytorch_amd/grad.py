"""Autograd for the gfx950 synthesis path (training).

The reference trains by back-propagating a multiscale spectral loss through
``DDSPDecoder.forward`` (train.py:84-130).  Every differentiable entry point of
``core.py`` dispatches here when autograd needs it; each ``torch.autograd.Function``
runs the forward kernel and, in ``backward``, the matching vector-Jacobian kernel of
``csrc/backward.hip`` / ``csrc/upols.hip`` through the C-ABI (include/ddsp_hip.h).

Pitch (f0) is an input feature in the reference's training loop (``batch['pitch']``,
train.py:84-99): no gradient flows to it.  ``remove_above_nyquist`` gives f0 the zero
gradient the reference's comparison gives; the oscillator ops refuse an f0 that
requires grad rather than silently returning a wrong (zero) gradient.
"""
import torch

from . import _lib
from . import core

_F = torch.autograd.Function


def _g(t):
    """contiguous, 16-byte aligned upstream gradient."""
    return core._c(t)


def refuse_f0_grad(f0, name):
    if torch.is_grad_enabled() and f0.requires_grad:
        raise NotImplementedError(
            f"ddsp_hip {name}: no gradient w.r.t. f0 (pitch is an input feature in the reference's "
            "training loop, train.py:84-99); pass f0.detach()")


def wants_grad(*tensors):
    return torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in tensors)


# ------------------------------------------------------------------------------------------
class ScaleFn(_F):
    """core.py:77-78 (+ the bias of modules.py:113)."""

    @staticmethod
    def forward(ctx, x, bias):
        ctx.save_for_backward(x)
        ctx.bias = float(bias)
        return core.scale_with_bias(x, bias)

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        x, g = core._c(x), _g(g)
        dx = torch.empty_like(x)
        _lib.call("scale_function_backward", _lib.ptr(x), _lib.ptr(g), _lib.ptr(dx), x.numel(), ctx.bias,
                  _lib.stream_of(x))
        return dx, None


class NyquistFn(_F):
    """core.py:70-74: d amplitudes = grad * mask; f0 enters only through a comparison (zero grad)."""

    @staticmethod
    def forward(ctx, amplitudes, f0, sample_rate):
        ctx.save_for_backward(f0)
        ctx.sr = sample_rate
        ctx.shape = amplitudes.shape
        return core.remove_above_nyquist(amplitudes, f0, sample_rate)

    @staticmethod
    def backward(ctx, g):
        (f0,) = ctx.saved_tensors
        d = core.remove_above_nyquist(g, f0.detach(), ctx.sr)
        if d.shape != ctx.shape:
            d = d.sum_to_size(ctx.shape)
        return d, None, None


class UpsampleFn(_F):
    """core.py:64-67: nearest upsampling; backward sums each block."""

    @staticmethod
    def forward(ctx, signal, factor):
        ctx.shape = signal.shape
        ctx.factor = int(factor)
        return core.upsample(signal, factor)

    @staticmethod
    def backward(ctx, g):
        B, F, C = ctx.shape
        g = _g(g)
        d = torch.empty(B, F, C, dtype=torch.float32, device=g.device)
        _lib.call("upsample_backward", _lib.ptr(g), _lib.ptr(d), B, F, C, ctx.factor, _lib.stream_of(g))
        return d, None


class HarmonicSynthFn(_F):
    """core.py:136-141 at the op boundary: d amplitudes[b,t,k] = g[b,t] sin(fl32(w[b,t] k))."""

    @staticmethod
    def forward(ctx, f0, amplitudes, sample_rate):
        ctx.save_for_backward(f0)
        ctx.sr = sample_rate
        ctx.H = amplitudes.shape[-1]
        return core.harmonic_synth(f0, amplitudes, sample_rate)

    @staticmethod
    def backward(ctx, g):
        (f0,) = ctx.saved_tensors
        B, T = f0.shape[0], f0.shape[1]
        omega = core.phase(f0.detach(), ctx.sr)
        g = _g(g)
        dA = torch.empty(B, T, ctx.H, dtype=torch.float32, device=g.device)
        _lib.call("harmonic_synth_backward", _lib.ptr(omega), _lib.ptr(g), _lib.ptr(dA), B, T, ctx.H,
                  _lib.stream_of(g))
        return None, dA, None


class ImpulseResponseFn(_F):
    """core.py:144-166: the transposed filter design (a cosine transform of the windowed taps)."""

    @staticmethod
    def forward(ctx, amp, target_size):
        ctx.shape = amp.shape
        ctx.target = int(target_size)
        return core.amp_to_impulse_response(amp, target_size)

    @staticmethod
    def backward(ctx, g):
        NB = ctx.shape[-1]
        g = _g(g)
        rows = g.numel() // ctx.target
        d = torch.empty(ctx.shape, dtype=torch.float32, device=g.device)
        _lib.call("amp_to_impulse_response_backward", _lib.ptr(g), _lib.ptr(d), rows, NB, ctx.target,
                  _lib.stream_of(g))
        return d, None


class FFTConvolveFn(_F):
    """core.py:169-176: y = (s (*) k)[:N].  Both gradients are correlations with g:
    d s = flip((flip g) (*) k), d k = flip((flip g) (*) s), each on the same convolution kernels."""

    @staticmethod
    def forward(ctx, signal, kernel):
        ctx.save_for_backward(signal, kernel)
        return core.fft_convolve(signal, kernel)

    @staticmethod
    def backward(ctx, g):
        s, k = ctx.saved_tensors
        gr = torch.flip(g, (-1,))
        ds = dk = None
        if ctx.needs_input_grad[0]:
            ds = torch.flip(core.fft_convolve(gr, k.detach()), (-1,)).sum_to_size(s.shape)
        if ctx.needs_input_grad[1]:
            dk = torch.flip(core.fft_convolve(gr, s.detach()), (-1,)).sum_to_size(k.shape)
        return ds, dk


# ------------------------------------------------------------------------------------------
class ControlsFn(_F):
    """modules.py:44-67 HarmonicSynth.get_controls."""

    @staticmethod
    def forward(ctx, amplitudes, distribution, f0, sample_rate):
        ctx.save_for_backward(amplitudes, distribution, f0)
        ctx.sr = sample_rate
        return core.harmonic_controls(amplitudes, distribution, f0, sample_rate)

    @staticmethod
    def backward(ctx, g_amp, g_dist):
        a, d, f0 = ctx.saved_tensors
        B, F, H = d.shape
        a_v, a_ld = core._rows_view(a, "amplitudes")
        d_v, d_ld = core._rows_view(d, "harmonic_distribution")
        g_amp = _g(g_amp) if g_amp is not None else torch.zeros(B, F, 1, device=d.device)
        g_dist = _g(g_dist) if g_dist is not None else torch.zeros(B, F, H, device=d.device)
        da = torch.empty(B, F, 1, dtype=torch.float32, device=d.device)
        dd = torch.empty(B, F, H, dtype=torch.float32, device=d.device)
        _lib.call("harmonic_controls_backward", _lib.ptr(a_v), a_ld, _lib.ptr(d_v), d_ld, _lib.ptr(core._c(f0)),
                  _lib.ptr(g_amp), _lib.ptr(g_dist), _lib.ptr(da), _lib.ptr(dd), B * F, H, float(ctx.sr),
                  _lib.stream_of(dd))
        return da, dd, None, None


class SynthFramesHarmonicFn(_F):
    """modules.py:69-80 HarmonicSynth.forward (frame-rate controls in, audio out)."""

    @staticmethod
    def forward(ctx, f0, amplitudes, distribution, block_size, sample_rate):
        ctx.f0 = f0.detach()
        ctx.amp = core._c(amplitudes.detach())
        # the caller multiplies `distribution` in place afterwards (modules.py:73): keep its
        # pre-multiplication value for the amplitude gradient
        ctx.dist = core._c(distribution.detach()).clone()
        ctx.bs, ctx.sr = int(block_size), float(sample_rate)
        return core.harmonic_synth_frames(f0, amplitudes, distribution, block_size, sample_rate,
                                          write_back=False)

    @staticmethod
    def backward(ctx, g):
        B, F, H = ctx.dist.shape
        g = _g(g)
        da = torch.empty(B, F, 1, dtype=torch.float32, device=g.device)
        dd = torch.empty(B, F, H, dtype=torch.float32, device=g.device)
        _lib.call("harmonic_synth_frames_backward", _lib.ptr(core._c(ctx.f0)), _lib.ptr(ctx.amp),
                  _lib.ptr(ctx.dist), _lib.ptr(g), _lib.ptr(da), _lib.ptr(dd), B, F, H, ctx.bs, ctx.sr,
                  _lib.stream_of(g))
        return None, da, dd, None, None


def params_backward(f0, param, g, block_size, sample_rate):
    B, F, H1 = param.shape
    dp = torch.empty(B, F, H1, dtype=torch.float32, device=param.device)
    _lib.call("harmonic_synth_params_backward", _lib.ptr(core._c(f0)), _lib.ptr(core._c(param)), _lib.ptr(g),
              _lib.ptr(dp), B, F, H1 - 1, int(block_size), float(sample_rate), _lib.stream_of(dp))
    return dp


def noise_backward(mags, noise, seed, offset, raw_bias, g, block_size):
    B, F, NB = mags.shape
    dm = torch.empty(B, F, NB, dtype=torch.float32, device=mags.device)
    raw = raw_bias is not None
    _lib.call("filtered_noise_backward", _lib.ptr(core._c(mags) if raw else None), _lib.ptr(noise), seed, offset,
              int(raw), float(raw_bias if raw else 0.0), _lib.ptr(g), _lib.ptr(dm), B, F, NB, int(block_size),
              _lib.stream_of(dm))
    return dm


class HarmonicParamsFn(_F):
    """decoder.py:106-113 + modules.py:44-80 from the raw harmonic projection."""

    @staticmethod
    def forward(ctx, f0, param, block_size, sample_rate):
        ctx.save_for_backward(f0, param)
        ctx.bs, ctx.sr = int(block_size), float(sample_rate)
        return core.harmonic_synth_params(f0, param, block_size, sample_rate)

    @staticmethod
    def backward(ctx, g):
        f0, param = ctx.saved_tensors
        return None, params_backward(f0.detach(), param.detach(), _g(g), ctx.bs, ctx.sr), None, None


class FilteredNoiseFn(_F):
    """modules.py:111-128 (raw_bias given: get_controls fused).  The forward's noise — injected, or
    the Philox (seed, offset) it drew on the device — is what the backward correlates with."""

    @staticmethod
    def forward(ctx, magnitudes, add, block_size, noise, raw_bias, return_noise):
        seed, offset = core._noise_counter.next() if noise is None else (0, 0)
        outs = core._filtered_noise_launch(magnitudes, block_size, noise, add, return_noise, raw_bias, seed,
                                           offset)
        ctx.mags = magnitudes.detach()
        ctx.noise = noise
        ctx.seed, ctx.offset = seed, offset
        ctx.raw_bias = raw_bias
        ctx.bs = int(block_size)
        ctx.two = isinstance(outs, tuple)
        return outs

    @staticmethod
    def backward(ctx, g_out, g_nout=None):
        g = g_out if (g_nout is None) else (g_nout if g_out is None else g_out + g_nout)
        g_f = _g(g)
        dm = noise_backward(ctx.mags, ctx.noise, ctx.seed, ctx.offset, ctx.raw_bias, g_f, ctx.bs)
        d_add = g_out if ctx.needs_input_grad[1] else None
        return dm, d_add, None, None, None, None


class SynthFramesFn(_F):
    """decoder.py:106-121 in one kernel; backward = harmonic params + raw noise VJPs."""

    @staticmethod
    def forward(ctx, f0, param, mags, block_size, sample_rate, bias, noise, parts):
        seed, offset = core._noise_counter.next() if noise is None else (0, 0)
        outs = core._synth_frames_launch(f0, param, mags, block_size, sample_rate, bias, noise, parts, seed,
                                         offset)
        ctx.save_for_backward(f0, param, mags)
        ctx.noise, ctx.seed, ctx.offset = noise, seed, offset
        ctx.bs, ctx.sr, ctx.bias = int(block_size), float(sample_rate), float(bias)
        return outs

    @staticmethod
    def backward(ctx, g_out, g_harm=None, g_nz=None):
        f0, param, mags = ctx.saved_tensors
        gh = _g(g_out if g_harm is None else g_out + g_harm)
        gn = None if g_nz is None else _g(g_out + g_nz)
        B, F, H1 = param.shape
        NB = mags.shape[-1]
        dp = torch.empty(B, F, H1, dtype=torch.float32, device=param.device)
        dm = torch.empty(B, F, NB, dtype=torch.float32, device=param.device)
        # both halves in one C-ABI call (two launches: harmonic, then noise VJP)
        _lib.call("synth_frames_backward", _lib.ptr(core._c(f0.detach())), _lib.ptr(core._c(param.detach())),
                  _lib.ptr(core._c(mags.detach())), ctx.bias, _lib.ptr(ctx.noise), ctx.seed, ctx.offset,
                  _lib.ptr(gh), _lib.ptr(gn), _lib.ptr(dp), _lib.ptr(dm), B, F, H1 - 1, NB, ctx.bs, ctx.sr,
                  _lib.stream_of(dp))
        return (None, dp if ctx.needs_input_grad[1] else None, dm if ctx.needs_input_grad[2] else None,
                None, None, None, None, None)


# ------------------------------------------------------------------------------------------
def reverb_backward(x, x_spectra, spectrum, g, ir_length, want_dx, want_dimp):
    """-> (dx or None, dimp or None) from one transform of g (csrc/upols.hip, upols_backward)."""
    B, T = g.shape[0], g.shape[1]
    dx = torch.empty(B, T, 1, dtype=torch.float32, device=g.device) if want_dx else None
    dimp = torch.empty(int(ir_length), dtype=torch.float32, device=g.device) if want_dimp else None
    have = x_spectra is not None
    ws = core._workspace(_lib.query("reverb_backward_workspace_size", B, T, int(ir_length), int(have)), g.device)
    _lib.call("reverb_backward", _lib.ptr(x), _lib.ptr(x_spectra), _lib.ptr(spectrum), _lib.ptr(g), _lib.ptr(dx),
              _lib.ptr(dimp), B, T, int(ir_length), _lib.ptr(ws), ws.numel(), _lib.stream_of(g))
    return dx, dimp


def reverb_backward_params(x_spectra, spectrum, g, noise, decay, wet, ir_length, sample_rate, want_dx):
    """-> (dx or None, d_noise, d_decay, d_wet): reverb_backward + impulse_backward without the impulse
    gradient round trip (csrc/upols.hip, upols_corr_finish_impulse_kernel)."""
    B, T = g.shape[0], g.shape[1]
    dx = torch.empty(B, T, 1, dtype=torch.float32, device=g.device) if want_dx else None
    dn = torch.empty_like(core._c(noise))
    dd = torch.empty((), dtype=torch.float32, device=g.device)
    dw = torch.empty((), dtype=torch.float32, device=g.device)
    ws = core._workspace(_lib.query("reverb_backward_workspace_size", B, T, int(ir_length), 1), g.device)
    _lib.call("reverb_backward_params", _lib.ptr(None), _lib.ptr(x_spectra), _lib.ptr(spectrum), _lib.ptr(g),
              _lib.ptr(core._c(noise)), _lib.ptr(core._c(decay)), _lib.ptr(core._c(wet)), float(sample_rate),
              _lib.ptr(dx), _lib.ptr(dn), _lib.ptr(dd), _lib.ptr(dw), B, T, int(ir_length), _lib.ptr(ws), ws.numel(),
              _lib.stream_of(g))
    return dx, dn.reshape(noise.shape), dd.reshape(decay.shape), dw.reshape(wet.shape)


def impulse_backward(noise, decay, wet, dimp, grad_length, sample_rate):
    L = noise.shape[0]
    dn = torch.empty_like(core._c(noise))
    dd = torch.empty((), dtype=torch.float32, device=noise.device)
    dw = torch.empty((), dtype=torch.float32, device=noise.device)
    ws = core._workspace(_lib.query("reverb_impulse_backward_workspace_size", L), noise.device)
    _lib.call("reverb_impulse_backward", _lib.ptr(core._c(noise)), _lib.ptr(core._c(decay)), _lib.ptr(core._c(wet)),
              _lib.ptr(dimp), L, int(grad_length), float(sample_rate), _lib.ptr(dn), _lib.ptr(dd), _lib.ptr(dw),
              _lib.ptr(ws), ws.numel(), _lib.stream_of(dn))
    return dn.reshape(noise.shape), dd.reshape(decay.shape), dw.reshape(wet.shape)


class ReverbApplyFn(_F):
    """modules.py:28-35 with a fixed (cached) IR spectrum: gradient w.r.t. the signal only."""

    @staticmethod
    def forward(ctx, x, spectrum, ir_length):
        ctx.spectrum = spectrum
        ctx.L = int(ir_length)
        return core.reverb_apply(x, spectrum, ir_length)

    @staticmethod
    def backward(ctx, g):
        dx, _ = reverb_backward(None, None, ctx.spectrum, _g(g), ctx.L, True, False)
        return dx, None, None


class ReverbFn(_F):
    """modules.py:21-35 Reverb.build_impulse + forward: gradients for the signal and for the
    reverb's parameters (noise, decay, wet).  The forward runs on the module's validated device IR
    cache (modules.Reverb._forward_cached); its input spectra are kept for the impulse gradient."""

    @staticmethod
    def forward(ctx, x, noise, decay, wet, run, ir_length, sample_rate):
        out, ws, spectrum = run(x)  # modules.Reverb._forward_cached: (out, workspace, spectrum of the cache)
        ctx.save_for_backward(noise, decay, wet)
        ctx.ws = ws if any(ctx.needs_input_grad[1:4]) else None
        # a view of the module's cache, rebuilt in place by a later forward only if noise / decay / wet
        # have changed by then.  In-place changes through autograd-visible ops are refused at backward
        # (they are saved tensors, version-checked); a write through .data between this forward and its
        # backward is not, and then the backward uses the new values — for the spectrum exactly as torch's
        # own autograd does for every saved tensor so modified (the .data hazard of any torch module).
        # Forwards on other streams are ordered with this one by Reverb._ir_cache.
        ctx.spectrum = spectrum
        ctx.T = x.shape[1]
        ctx.L, ctx.sr = int(ir_length), float(sample_rate)
        return out

    @staticmethod
    def backward(ctx, g):
        noise, decay, wet = ctx.saved_tensors
        want_p = any(ctx.needs_input_grad[1:4])
        dn = dd = dw = None
        if want_p:  # the impulse gradient never materialised (ddsp_hip_reverb_backward_params)
            dx, dn, dd, dw = reverb_backward_params(ctx.ws, ctx.spectrum, _g(g), noise.detach(), decay.detach(),
                                                    wet.detach(), ctx.L, ctx.sr, ctx.needs_input_grad[0])
        else:
            dx, _ = reverb_backward(None, None, ctx.spectrum, _g(g), ctx.L, True, False)
        ctx.ws = None
        return dx, dn, dd, dw, None, None, None


class BuildImpulseFn(_F):
    """modules.py:21-26 Reverb.build_impulse."""

    @staticmethod
    def forward(ctx, noise, decay, wet, sample_rate):
        ctx.save_for_backward(noise, decay, wet)
        ctx.sr = float(sample_rate)
        return core.reverb_build_impulse(noise, decay, wet, sample_rate)

    @staticmethod
    def backward(ctx, g):
        noise, decay, wet = ctx.saved_tensors
        g = _g(g).reshape(-1)
        dn, dd, dw = impulse_backward(noise.detach(), decay.detach(), wet.detach(), g, noise.shape[0], ctx.sr)
        return dn, dd, dw, None


# ------------------------------------------------------------------------------------------
class StftMagFn(_F):
    """ddsp/core.py:27-41 (one scale): |STFT| of signal [B, T]; backward through the magnitude,
    the transform, the window and the reflect padding (csrc/stft.hip)."""

    @staticmethod
    def forward(ctx, signal, n_fft, hop):
        ctx.save_for_backward(signal)
        ctx.n_fft, ctx.hop = n_fft, hop
        return core.stft_magnitude(signal, n_fft, hop)

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        B, T = x.shape
        gM = core._c(g.transpose(1, 2))  # frame-major, the kernel's layout
        dx = torch.empty(B, T, dtype=torch.float32, device=x.device)
        ws = core._workspace(_lib.query("stft_backward_workspace_size", B, T, ctx.n_fft, ctx.hop), x.device)
        _lib.call("stft_magnitude_backward", _lib.ptr(core._c(x.detach())), _lib.ptr(gM), _lib.ptr(dx), B, T,
                  ctx.n_fft, ctx.hop, _lib.ptr(ws), ws.numel(), _lib.stream_of(dx))
        return dx, None, None


# ------------------------------------------------------------------------------------------
GRU_BPTT_FLAGS = 0  # ddsp_hip_gru_backward_persistent's test hooks (core.GRU_*); 0 in use


class LinearFn(_F):
    """nn.Linear under autograd for the decoder's MLP blocks (ddsp/core.py:122-129, decoder.py:43-68): the
    forward and the input gradient on ddsp_hip_linear (core.linear: the bf16 matrix cores with the exact
    three-term split, fp32-accurate; torch.addmm outside its shapes) — y = x W^T + b and dx = dy W (the same
    kernel over W^T) — and the weight gradient dW = dy^T x on ddsp_hip_linear_weight_grad (core.linear_weight_grad,
    same split; torch.mm outside its shapes); db = sum dy on torch."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        K = x.shape[-1]
        x2 = core._c(x).reshape(-1, K)
        y = core.linear(x2, weight, bias)
        ctx.save_for_backward(x2, weight)
        ctx.x_shape = x.shape
        return y.view(*x.shape[:-1], weight.shape[0])

    @staticmethod
    def backward(ctx, gy):
        x2, w = ctx.saved_tensors
        g2 = _g(gy).reshape(-1, w.shape[0])
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            wt = w.t().contiguous()
            gx = core.linear(g2, wt, torch.zeros(wt.shape[0], dtype=wt.dtype, device=wt.device)).view(ctx.x_shape)
        if ctx.needs_input_grad[1]:
            gw = core.linear_weight_grad(g2, x2)
        if ctx.needs_input_grad[2]:
            gb = g2.sum(0)
        return gx, gw, gb


class ProjectionsFn(_F):
    """decoder.py:106-117's harmonic_proj and noise_proj under autograd: the forward in ONE launch of
    ddsp_hip_projections (both layers on the bf16 matrix cores, parameters read where they lie), returned as the
    [..., n4] buffer the two outputs are column slices of; the backward dx = dy [W1; W2] on torch (166-wide K),
    [dW1; dW2] on ddsp_hip_linear_weight_grad, the biases' sums on torch.  x [..., 512] (decoder_projections
    checks; elsewhere it keeps one differentiable GEMM)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2):
        K = x.shape[-1]
        x2 = core._c(x).reshape(-1, K)
        n1, n2 = w1.shape[0], w2.shape[0]
        n4 = -(-(n1 + n2) // 4) * 4
        y = torch.empty(x2.shape[0], n4, dtype=torch.float32, device=x.device)
        w1c, w2c = core._c(w1), core._c(w2)
        st = _lib.call("projections", _lib.ptr(x2), K, K, _lib.ptr(w1c), K, _lib.ptr(core._c(b1)), n1, _lib.ptr(w2c),
                       K, _lib.ptr(core._c(b2)), n2, _lib.ptr(y), n4, x2.shape[0], _lib.stream_of(y),
                       allow=(core.ERANGE,))
        if st == core.ERANGE:  # (unaligned rows) one library GEMM
            y[:, :n1 + n2] = torch.addmm(torch.cat([b1, b2]), x2, torch.cat([w1c, w2c]).t())
        ctx.save_for_backward(x2, w1c, w2c)
        ctx.x_shape = x.shape
        return y.view(*x.shape[:-1], n4)

    @staticmethod
    def backward(ctx, gy):
        x2, w1, w2 = ctx.saved_tensors
        n1, n2 = w1.shape[0], w2.shape[0]
        g = gy.reshape(-1, gy.shape[-1])[:, :n1 + n2].contiguous()
        gx = gw1 = gb1 = gw2 = gb2 = None
        if ctx.needs_input_grad[0]:
            gx = g.mm(torch.cat([w1, w2])).view(ctx.x_shape)
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[3]:
            gw = core.linear_weight_grad(g, x2)
            gw1, gw2 = gw[:n1], gw[n1:]
        if ctx.needs_input_grad[2] or ctx.needs_input_grad[4]:
            gb = g.sum(0)
            gb1, gb2 = gb[:n1], gb[n1:]
        return (gx, gw1 if ctx.needs_input_grad[1] else None, gb1 if ctx.needs_input_grad[2] else None,
                gw2 if ctx.needs_input_grad[3] else None, gb2 if ctx.needs_input_grad[4] else None)


class LNLeakyFn(_F):
    """LeakyReLU(LayerNorm(g)) under autograd for the decoder's MLP blocks (ddsp/core.py:122-129): the forward on
    ddsp_hip_layer_norm_leaky_relu, the backward — dg, dgamma, dbeta from the saved g — on
    ddsp_hip_layer_norm_leaky_relu_backward (one pass instead of torch's LeakyReLU and LayerNorm backward kernels
    and its separate parameter-gradient reductions).  g [..., cols] with cols 512 or 1024 (mlp_forward checks)."""

    @staticmethod
    def forward(ctx, g, gamma, beta, eps, slope):
        gc = core._c(g)
        cols = gc.shape[-1]
        rows = gc.numel() // cols
        y = torch.empty_like(gc)
        _lib.call("layer_norm_leaky_relu", _lib.ptr(gc), cols, None, None, _lib.ptr(core._c(gamma)),
                  _lib.ptr(core._c(beta)), float(eps), float(slope), _lib.ptr(y), cols, rows, cols, _lib.stream_of(y))
        ctx.save_for_backward(gc, gamma, beta)
        ctx.eps, ctx.slope = float(eps), float(slope)
        return y

    @staticmethod
    def backward(ctx, gy):
        gc, gamma, beta = ctx.saved_tensors
        cols = gc.shape[-1]
        rows = gc.numel() // cols
        dy = _g(gy)
        dg = torch.empty_like(gc)  # (the kernel always writes it)
        want = ctx.needs_input_grad[1] or ctx.needs_input_grad[2]
        dgam = torch.empty_like(gamma) if ctx.needs_input_grad[1] else None
        dbet = torch.empty_like(beta) if ctx.needs_input_grad[2] else None
        ws = core._workspace(_lib.query("layer_norm_leaky_relu_backward_workspace_size", cols), gc.device) if want else None
        _lib.call("layer_norm_leaky_relu_backward", _lib.ptr(gc), cols, _lib.ptr(core._c(gamma)), _lib.ptr(core._c(beta)),
                  ctx.eps, ctx.slope, _lib.ptr(dy), cols, _lib.ptr(dg), cols, _lib.ptr(dgam), _lib.ptr(dbet), rows, cols,
                  _lib.ptr(ws), ws.numel() if ws is not None else 0, _lib.stream_of(dg))
        return (dg if ctx.needs_input_grad[0] else None), dgam, dbet, None, None


class GRUFn(_F):
    """decoder.py:33-68's nn.GRU (1 layer, batch_first) with BPTT on the gfx950 kernels (csrc/gru.hip); the input
    projection and its input gradient on the matrix-core linear kernel (core.linear), the weight gradients on
    its weight-gradient kernel (core.linear_weight_grad)."""

    @staticmethod
    def forward(ctx, x, w_ih, w_hh, b_ih, b_hh, h0):
        B, T, I = x.shape
        H = w_hh.shape[1]
        out = torch.empty(B, T, H, dtype=torch.float32, device=x.device)
        h_last = torch.empty(1, B, H, dtype=torch.float32, device=x.device)
        gates = torch.empty(4, B, T, H, dtype=torch.float32, device=x.device)
        h0c = core._c(h0.reshape(B, H)) if h0 is not None else None
        core.gru_layer_launch(x, w_ih, b_ih, w_hh, b_hh, h0c, out, h_last, gates)
        ctx.save_for_backward(x, w_ih, w_hh, out, gates, h0c if h0c is not None else torch.empty(0))
        ctx.has_h0 = h0 is not None
        ctx.h0_shape = h0.shape if h0 is not None else None
        return out, h_last

    @staticmethod
    def backward(ctx, g_out, g_hlast):
        x, w_ih, w_hh, out, gates, h0c = ctx.saved_tensors
        B, T, I = x.shape
        H = w_hh.shape[1]
        h0p = h0c if ctx.has_h0 else None
        dxp = torch.empty(B, T, 3 * H, dtype=torch.float32, device=x.device)
        dgn = torch.empty(B, T, H, dtype=torch.float32, device=x.device)
        dh0 = torch.empty(B, H, dtype=torch.float32, device=x.device) if ctx.has_h0 else None
        go = core._c(g_out) if g_out is not None else None
        gh = core._c(g_hlast.reshape(B, H)) if g_hlast is not None else None
        args = (_lib.ptr(core._c(w_hh)), _lib.ptr(gates), _lib.ptr(out), _lib.ptr(h0p), _lib.ptr(go), _lib.ptr(gh),
                _lib.ptr(dxp), _lib.ptr(dgn), _lib.ptr(dh0), B, T, H)
        # hidden 512, batch <= 64: the whole BPTT as one persistent launch; otherwise (ERANGE) one launch per step
        ws = core._workspace(_lib.query("gru_persistent_workspace_size"), x.device)
        st = _lib.call("gru_backward_persistent", *args, int(GRU_BPTT_FLAGS), _lib.ptr(ws), ws.numel(),
                       _lib.stream_of(dxp), allow=(core.ERANGE,))
        dev = x.device.index if x.device.index is not None else torch.cuda.current_device()
        core._GRU_LAST[dev] = ("persistent", ws) if st == 0 else ("steps", None)
        if st == core.ERANGE:
            ws = core._workspace(_lib.query("gru_backward_workspace_size", B, H), x.device)
            _lib.call("gru_backward", *args, _lib.ptr(ws), ws.numel(), _lib.stream_of(dxp))
        dxp2 = dxp.view(B * T, 3 * H)
        dG = torch.cat([dxp[..., :2 * H], dgn], -1).view(B * T, 3 * H)
        hprev = torch.cat([(h0p.view(B, 1, H) if h0p is not None else torch.zeros(B, 1, H, device=x.device)),
                           out[:, :-1]], 1).reshape(B * T, H)
        dx = None
        if ctx.needs_input_grad[0]:  # dx = dxp W_ih on the matrix-core kernel (W_ih^T as its weight; addmm outside it)
            wt = w_ih.t().contiguous()
            dx = core.linear(dxp2, wt, torch.zeros(wt.shape[0], dtype=wt.dtype, device=wt.device)).view(B, T, I)
        dw_ih = core.linear_weight_grad(dxp2, x.reshape(B * T, I)) if ctx.needs_input_grad[1] else None
        dw_hh = core.linear_weight_grad(dG, hprev) if ctx.needs_input_grad[2] else None
        db_ih = dxp2.sum(0) if ctx.needs_input_grad[3] else None
        db_hh = dG.sum(0) if ctx.needs_input_grad[4] else None
        dh0r = dh0.view(ctx.h0_shape) if (ctx.has_h0 and ctx.needs_input_grad[5]) else None
        return dx, dw_ih, dw_hh, db_ih, db_hh, dh0r
