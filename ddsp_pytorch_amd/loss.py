"""The training loss of the reference (train.py:70-76) over the gfx950 multiscale STFT.

``multiscale_spec_loss(ori_stft, rec_stft)`` restates train.py:70-76 (sum over scales of the
mean absolute linear and log-magnitude differences) on spectrograms from ``core.multiscale_fft``.
``spectral_loss(sig, rec, scales, overlap)`` is the whole step of train.py:91-104 in one fused
kernel per scale (csrc/stft.hip, ``ddsp_hip_spectral_loss``): no spectrogram is materialised, and
the gradient w.r.t. ``rec`` comes out of the same pass.  A target that itself requires grad takes
the unfused route (spectrograms + autograd).
"""
import ctypes

import torch

from . import _lib, core


def multiscale_spec_loss(ori_stft, rec_stft):
    """train.py:70-76."""
    loss = 0
    for s_x, s_y in zip(ori_stft, rec_stft):
        lin_loss = (s_x - s_y).abs().mean()
        log_loss = (core.safe_log(s_x) - core.safe_log(s_y)).abs().mean()
        loss = loss + lin_loss + log_loss
    return loss


def _fused(sig, rec, scales, overlap, want_grad):
    B, T = rec.shape
    n = len(scales)
    nffts = (ctypes.c_int64 * n)(*[int(s) for s in scales])
    hops = (ctypes.c_int64 * n)(*[int(s * (1 - overlap)) for s in scales])
    ws = core._workspace(_lib.query("spectral_loss_workspace_size", B, T, nffts, hops, n), rec.device)
    loss = torch.empty((), dtype=torch.float32, device=rec.device)
    grad = torch.empty(B, T, dtype=torch.float32, device=rec.device) if want_grad else None
    _lib.call("spectral_loss", _lib.ptr(core._c(sig)), _lib.ptr(core._c(rec)), B, T, nffts, hops, n, _lib.ptr(loss),
              _lib.ptr(grad), _lib.ptr(ws), ws.numel(), _lib.stream_of(rec))
    return loss, grad


class _SpectralLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, sig, rec, scales, overlap):
        loss, grad = _fused(sig, rec, scales, overlap, True)
        ctx.grad = grad
        return loss

    @staticmethod
    def backward(ctx, g):
        return None, ctx.grad * g, None, None


def spectral_loss(sig, rec, scales=(4096, 2048, 1024, 512, 256, 128), overlap=0.75):
    """train.py:91-104 with config.yaml's scales and overlap: sig (target), rec [B, T] -> scalar."""
    core._dev(sig, rec)
    if sig.dim() != 2 or rec.shape != sig.shape:
        raise RuntimeError(f"spectral_loss: expected two [batch, time] signals, got {tuple(sig.shape)}, "
                           f"{tuple(rec.shape)}")
    scales = tuple(int(s) for s in scales)
    if core._wants_grad(sig):
        return multiscale_spec_loss(core.multiscale_fft(sig, scales, overlap),
                                    core.multiscale_fft(rec, scales, overlap))
    if core._wants_grad(rec):
        return _SpectralLossFn.apply(sig.detach(), rec, scales, float(overlap))
    return _fused(sig, rec, scales, overlap, False)[0]
