"""Caller of the hot path: a ``DDSPDecoder`` with the reference's architecture and
state_dict keys (ddsp/models/decoder.py:9-136, ddsp/core.py:122-133), wired to the gfx950
synth modules.

The control network before the path runs at inference on gfx950 kernels
too: each MLP block is one matrix-core launch with its LayerNorm + LeakyReLU (core.mlp_block), the
GRU's input projection for every step one matrix-core launch (core.linear) and its recurrence one
persistent launch per layer (core.gru), the two projections one matrix-core launch reading both layers'
parameters in place (core.projections), and the synthesis section of ``forward`` (decoder.py:106-125) one
fused launch before the reverb.  Under autograd the MLP blocks' Linears run their forward, input gradient
and weight gradient on the matrix-core kernels (grad.LinearFn), their LayerNorm + LeakyReLU forward and
backward on this package's kernels (grad.LNLeakyFn), the projections one grad.ProjectionsFn (forward in one
matrix-core launch, weight gradient on the matrix cores), and the GRU's BPTT is one persistent
launch with its weight gradients on the matrix cores.
"""
import torch
import torch.nn as nn

from . import core
from .modules import NOISE_MODES, FilteredNoise, HarmonicSynth, Reverb


def mlp(in_size, hidden_size, n_layers):
    """ddsp/core.py:122-129: (Linear, LayerNorm, LeakyReLU) x n_layers."""
    sizes = [in_size] + n_layers * [hidden_size]
    layers = []
    for i in range(n_layers):
        layers += [nn.Linear(sizes[i], sizes[i + 1]), nn.LayerNorm(sizes[i + 1]), nn.LeakyReLU()]
    return nn.Sequential(*layers)


class GRUDecoder(nn.Module):
    """ddsp/models/decoder.py:9-68, incl. the optional z conditioning (z_dim: a z_mlp whose output joins
    the GRU input, decoder.py:31-39) that DDSPAutoencoder uses."""

    def __init__(self, hidden_size: int, z_dim: int = None):
        super().__init__()
        self.register_buffer("cache_gru", torch.zeros(1, 1, hidden_size))
        self.f0_mlp = mlp(1, hidden_size, 3)
        self.loudness_mlp = mlp(1, hidden_size, 3)
        self.add_z = z_dim is not None
        if self.add_z:
            self.z_mlp = mlp(z_dim, hidden_size, 3)
        self.gru = nn.GRU((3 if self.add_z else 2) * hidden_size, hidden_size, batch_first=True)
        self.out_mlp = mlp(hidden_size + 2, hidden_size, 3)

    def forward(self, f0, loudness, z=None, realtime: bool = False):
        return gru_decoder_forward(self, f0, loudness, z, realtime)


def _gru(mod, hidden, h0):
    """mod.gru(hidden[, h0]) with the recurrence (and, under autograd, its BPTT) on the gfx950 step
    kernels; torch's GRU only for shapes outside the kernel's (hidden % 64 != 0)."""
    if hidden.is_cuda and core.gru_supported(mod.gru) and _fp32_inference_ok(hidden, (mod.gru,)):
        return core.gru(hidden, mod.gru, h0)
    return mod.gru(hidden, h0) if h0 is not None else mod.gru(hidden)


def _mlp_fusable(seq, x):
    """An unobserved (Linear, LayerNorm, LeakyReLU) x n block chain (ddsp/core.py:122-129) on the GPU at
    inference (see _mlp_plain); the LayerNorm + LeakyReLU pairs may run as one kernel."""
    if torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in seq.parameters())):
        return False
    return _mlp_plain(seq, x)


def _mlp_plain(seq, x):
    """An unobserved (Linear, LayerNorm, LeakyReLU) x n block chain (ddsp/core.py:122-129) in fp32 on the GPU:
    no module or global hooks, the plain torch classes, affine LayerNorms, Linears with biases."""
    from torch.nn.modules import module as _m
    if not x.is_cuda:
        return False
    if _m._global_forward_hooks or _m._global_forward_pre_hooks or seq._forward_hooks or seq._forward_pre_hooks:
        return False
    if type(seq) is not nn.Sequential or type(seq).forward is not nn.Sequential.forward:
        return False
    if not _fp32_inference_ok(x, (seq,)):
        return False
    mods = list(seq)
    if len(mods) % 3:
        return False
    for i in range(0, len(mods), 3):
        lin, ln, act = mods[i:i + 3]
        if (type(lin) is not nn.Linear or type(ln) is not nn.LayerNorm or type(act) is not nn.LeakyReLU or
                lin.bias is None or not ln.elementwise_affine or ln.bias is None or
                any(m._forward_hooks or m._forward_pre_hooks for m in (lin, ln, act))):
            return False
    return True


def mlp_forward(seq, x, out=None, extras=()):
    """seq(torch.cat([x, *extras], -1)) for a core.py:122-129 MLP.  On the GPU at inference a block with
    512 outputs is ONE launch (core.mlp_block: the Linear on the matrix cores, LayerNorm + LeakyReLU in
    its epilogue; ``extras`` — per-row [..., 1] inputs appended to x, the out_mlp's f0 and loudness —
    enter the first block's epilogue, so the concatenation is never built), a one-feature first Linear
    folds into the LayerNorm kernel (core.layer_norm_leaky_relu), other blocks run their GEMM then that
    kernel; the last block may write into ``out`` (e.g. a column slice of the GRU input concatenation)."""
    if not _mlp_fusable(seq, x):
        xin = torch.cat([x, *extras], -1) if extras else x
        if _mlp_plain(seq, xin):
            # under autograd: each block's Linear on grad.LinearFn (the one-feature first Linear stays torch's) and
            # its LayerNorm + LeakyReLU on grad.LNLeakyFn (512 / 1024 features; else torch's modules)
            from .grad import LinearFn, LNLeakyFn
            y = xin
            mods = list(seq)
            for i in range(0, len(mods), 3):
                lin, ln, act = mods[i:i + 3]
                g = LinearFn.apply(y, lin.weight, lin.bias) if lin.in_features >= 16 else lin(y)
                if lin.out_features in (512, 1024) and tuple(ln.normalized_shape) == (lin.out_features,):
                    y = LNLeakyFn.apply(g, ln.weight, ln.bias, ln.eps, act.negative_slope)
                else:
                    y = act(ln(g))
        else:
            y = seq(xin)
        if out is None:
            return y
        out.copy_(y)
        return out
    mods = list(seq)
    h = x
    for i in range(0, len(mods), 3):
        lin, ln, act = mods[i:i + 3]
        dst = out if i + 3 == len(mods) else None
        ext = extras if i == 0 else ()
        y = None
        if lin.in_features == 1 and not ext:
            y = core.layer_norm_leaky_relu(h, ln, act, out=dst, w1=lin.weight[:, 0], b1=lin.bias)
        elif lin.in_features >= 16:
            y = core.mlp_block(h, lin, ln, act, out=dst, extras=ext)
        if y is None:
            hin = torch.cat([h, *ext], -1) if ext else h
            g = torch.nn.functional.linear(hin, lin.weight, lin.bias)
            y = core.layer_norm_leaky_relu(g, ln, act, out=dst)
            if y is None:
                y = act(ln(g))
        if dst is not None and y is not dst:
            dst.copy_(y)
            y = dst
        h = y
    return h


def gru_decoder_forward(self, f0, loudness, z=None, realtime=False):
    """ddsp/models/decoder.py:43-68 GRUDecoder.forward (incl. the optional z projection), the GRU on
    the step kernel for inference.  install() binds it to the reference's GRUDecoder too.  At inference
    on the GPU the MLP blocks' LayerNorm + LeakyReLU run fused and the input MLPs write straight into
    the GRU's input concatenation (mlp_forward)."""
    mlps = [(self.f0_mlp, f0), (self.loudness_mlp, loudness)]
    if getattr(self, "add_z", False):
        assert z is not None
        mlps.append((self.z_mlp, z))
    widths = [m[-3].out_features if len(m) >= 3 else -1 for m, _ in mlps]
    if all(_mlp_fusable(m, x) for m, x in mlps) and len(set(widths)) == 1:
        W = widths[0]
        hidden = torch.empty(*f0.shape[:-1], W * len(mlps), dtype=torch.float32, device=f0.device)
        for i, (m, x) in enumerate(mlps):
            mlp_forward(m, x, out=hidden[..., i * W:(i + 1) * W])
    else:
        hidden = torch.cat([mlp_forward(m, x) for m, x in mlps], -1)
    if realtime:
        gru_out, cache = _gru(self, hidden, self.cache_gru)
        self.cache_gru.copy_(cache)
    else:
        gru_out = _gru(self, hidden, None)[0]
    return mlp_forward(self.out_mlp, gru_out, extras=(f0, loudness))


def _hooked(m):
    """A module call that must stay a module call: forward (pre-)hooks registered on it or globally, or
    a subclass / wrapper whose forward is not nn.Linear's."""
    from torch.nn.modules import module as _m
    return bool(m._forward_hooks or m._forward_pre_hooks or _m._global_forward_hooks or
                _m._global_forward_pre_hooks or type(m).forward is not torch.nn.Linear.forward)


def _synth_overridden(m, cls):
    """The synth module's calls must stay module calls: forward (pre-)hooks on it or globally, or a class
    whose forward / get_controls is not this package's (``cls``; install() binds the same functions to
    the reference's classes, so an installed reference module is not overridden)."""
    from torch.nn.modules import module as _m
    if m._forward_hooks or m._forward_pre_hooks or _m._global_forward_hooks or _m._global_forward_pre_hooks:
        return True
    t = type(m)
    return any(getattr(t, n, None) is not cls.__dict__[n] for n in ("forward", "get_controls"))


def _fp32_inference_ok(x, mods):
    """The fp32 network kernels apply: float32 input and parameters, and no autocast region (under
    torch.autocast torch's modules run in the autocast dtype; these kernels compute in fp32 only)."""
    if x.dtype != torch.float32 or any(p.dtype != torch.float32 for m in mods for p in m.parameters()):
        return False
    return not torch.is_autocast_enabled(x.device.type)


def decoder_projections(self, hidden):
    """decoder.py:106-117: harmonic_proj(hidden), noise_proj(hidden).  On the GPU at inference ONE GEMM
    (core.projections: both layers' parameters stacked fresh on every call into a zero-padded buffer, then
    hipBLASLt — nothing is cached on or rebound in the modules, so every write to a parameter, through
    ``.data`` included, is seen by the next call); the two outputs are column slices of one buffer, which
    the fused synthesis kernel reads with its row stride.  Under autograd the concatenated weights keep the call
    differentiable, so the parameters receive their gradients as the reference's do: at 512 inputs
    grad.ProjectionsFn (the forward on ddsp_hip_projections, the weight gradient on ddsp_hip_linear_weight_grad),
    elsewhere grad.LinearFn over the concatenated parameters."""
    hp, npj = self.harmonic_proj, self.noise_proj
    if not hidden.is_cuda or hp.bias is None or npj.bias is None or _hooked(hp) or _hooked(npj):
        return hp(hidden), npj(hidden)  # (module hooks see the calls the reference makes)
    ps = (hp.weight, hp.bias, npj.weight, npj.bias)
    h1, n = hp.out_features, hp.out_features + npj.out_features
    if torch.is_grad_enabled() and (hidden.requires_grad or any(p.requires_grad for p in ps)):
        from .grad import LinearFn, ProjectionsFn
        if hidden.shape[-1] == 512 and all(p.dtype == torch.float32 and p.dim() and p.stride(-1) == 1 for p in ps) \
                and hidden.dtype == torch.float32 and hp.in_features == npj.in_features == 512:
            out = ProjectionsFn.apply(hidden, hp.weight, hp.bias, npj.weight, npj.bias)
        else:
            w, b = torch.cat([hp.weight, npj.weight]), torch.cat([hp.bias, npj.bias])  # differentiable
            out = LinearFn.apply(hidden, w, b)
        return out[..., :h1], out[..., h1:n]
    if _fp32_inference_ok(hidden, (hp, npj)):
        r = core.projections(hidden, hp, npj)
        if r is not None:
            return r
    return hp(hidden), npj(hidden)


def decoder_synthesize(self, hidden, f0):
    """decoder.py:106-125, the synthesis section of DDSPDecoder.forward: controls -> harmonic + noise
    (+ reverb).  On the fused kernel (one launch for both synths, their controls, the sum and the
    returned control dicts) whenever the shapes are in its envelope: the reference's noise stream
    (``noise_mode = "torch"``: torch.rand(B, F, bs) drawn as modules.py:119-123 draws it, injected)
    or on-device Philox (``"device"``).  Outside the envelope the modules run one by one (still on the
    gfx950 kernels).  Works on this package's DDSPDecoder and, through install(), on the reference's.
    Returns (signal, harmonic, noise, harmonic_ctrls, noise_ctrls)."""
    hs, ns = self.harmonic_synth, self.noise_synth
    param, mags = decoder_projections(self, hidden)
    H, NB, bs = param.shape[-1] - 1, mags.shape[-1], int(hs.block_size)
    fused = (param.is_cuda and int(ns.block_size) == bs and param.shape[0] <= 65535
             and core.synth_frames_in_envelope(H, NB, bs, param.shape[0])
             and not _synth_overridden(hs, HarmonicSynth) and not _synth_overridden(ns, FilteredNoise))
    if fused:
        mode = getattr(ns, "noise_mode", "torch")
        if mode not in NOISE_MODES:
            raise ValueError(f"noise_mode must be one of {NOISE_MODES}")
        noise_in = FilteredNoise.draw_noise(ns, mags) if mode == "torch" else None
        signal, harmonic, noise, ctrl = core.synth_frames(
            f0, param, mags, bs, hs.sample_rate, bias=float(ns.initial_bias), noise=noise_in, parts=True,
            controls=True)
        harmonic_ctrls = {"f0": f0, "harmonic_distribution": ctrl["harmonic_distribution"],
                          "amplitudes": ctrl["amplitudes"]}
        noise_ctrls = {"magnitudes": ctrl["magnitudes"]}
    else:
        harmonic_ctrls = hs.get_controls(param[..., :1], param[..., 1:], f0)
        harmonic = hs(**harmonic_ctrls)
        noise_ctrls = ns.get_controls(mags)
        noise = ns(**noise_ctrls)
        signal = harmonic + noise
    if self.has_reverb:
        signal = self.reverb(signal)
    return signal, harmonic, noise, harmonic_ctrls, noise_ctrls


def decoder_forward(self, batch: dict):
    """decoder.py:101-136 DDSPDecoder.forward with the synthesis section fused (decoder_synthesize);
    install() binds it to the reference's DDSPDecoder."""
    f0, loudness = batch["pitch"], batch["loudness"]
    hidden = self.decoder(f0, loudness)
    signal, harmonic, noise, hc, nc = decoder_synthesize(self, hidden, f0)
    return {"f0": f0, "loudness": loudness, "signal": signal, "noise": noise,
            "harmonic_audio": harmonic, "noise_ctrls": nc, "harmonic_ctrls": hc}


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

    synthesize = decoder_synthesize
    forward = decoder_forward
