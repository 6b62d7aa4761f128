"""Realtime streaming on a captured HIP graph (BASELINE.json config 3).

The reference's realtime host, the `ddsp~` Pd external, calls the exported model once per
1024-sample buffer from a worker thread (`realtime/ddsp_tilde/ddsp_model.cpp:32-52`,
`ddsp_tilde.cpp:67-98`): pitch and loudness at audio rate in, audio out, the GRU state carried
between calls in `cache_gru` (`decoder.py:56-60`), no reverb (`export.py:37-40`).  At batch 1
and 4 frames per call that forward is ~25 short launches (MLPs, LayerNorms, the GRU steps, the
synthesis), so its latency is launch-bound, not compute-bound.

`RealtimeGraph` captures one call — loudness normalisation, decimation by block_size, the
control network with the cached GRU state, the fused synthesis kernel — into a HIP graph
(`torch.cuda.CUDAGraph` is hipGraph on ROCm) over static device buffers, and replays it per
call: one graph launch plus the two host<->device copies.  With `fused=True` (default) the
control network runs on `ddsp_hip_dense_rows` (csrc/dense.hip): each Linear one launch with the
previous block's LayerNorm + LeakyReLU, the first K=1 Linear, the loudness normalisation and
the concatenations folded into its input — 7 launches + the GRU steps + the synthesis instead
of ~30 torch kernels.  The on-device noise takes its
Philox offset from a device counter the graph advances (`ddsp_hip_synth_frames_counter`), so
every replay draws fresh noise; call k equals the eager model run with noise offset k.
"""
from collections import namedtuple

import torch

from . import core
from .decoder import gru_decoder_forward

_Linear = namedtuple("_Linear", "weight bias in_features out_features")


class RealtimeGraph:
    """Graph-replayed realtime forward of a `DDSPDecoder` (the ScriptDDSP realtime model of
    export.py:23-40: `forward(pitch[1,N,1], loudness[1,N,1]) -> audio[1,N,1]`).

    The model's `decoder.cache_gru` is the stream state (updated in place by every call, as in
    decoder.py:56-60); `reset()` zeroes it and rewinds the noise counter.  The returned tensor
    is a static buffer overwritten by the next call (the host copies it out, as `ddsp~` does
    with memcpy)."""

    def __init__(self, model, call_samples=1024, mean_loudness=0.0, std_loudness=1.0,
                 seed=0x5EEDDD5B, device=None, warmup=3, fused=True, gru_route="steps"):
        device = torch.device(device) if device is not None else next(model.parameters()).device
        if device.type != "cuda":
            raise RuntimeError("RealtimeGraph: the model must be on a HIP device")
        bs = int(model.block_size)
        N = int(call_samples)
        if N % bs:
            raise RuntimeError(f"RealtimeGraph: call_samples {N} must be a multiple of block_size {bs}")
        if not core.synth_frames_in_envelope(model.harmonic_proj.out_features - 1,
                                             model.noise_proj.out_features, bs, 1):
            raise RuntimeError("RealtimeGraph: model shape outside the fused synthesis kernel's envelope")
        self.model = model
        self.device = device
        self.block_size = bs
        self.call_samples = N
        self.sample_rate = float(model.sample_rate)
        self.mean_loudness = float(mean_loudness)
        self.std_loudness = float(std_loudness)
        self.seed = int(seed)
        self.bias = float(model.noise_synth.initial_bias)
        # pitch and loudness share one buffer: one host->device copy per call
        self._inp = torch.zeros(2, N, 1, device=device)
        self.pitch, self.loudness = self._inp[0:1], self._inp[1:2]
        self.counter = torch.zeros(1, dtype=torch.int64, device=device)
        self._inp_h = torch.zeros(2, N, 1).pin_memory()
        self._out_h = torch.zeros(1, N, 1).pin_memory()
        self.fused = bool(fused)
        if gru_route not in ("steps", "persistent"):
            raise ValueError("RealtimeGraph: gru_route must be 'steps' or 'persistent'")
        self.gru_route = gru_route  # the route requested; gru_route_taken: the one the graph holds
        self.gru_route_taken = None
        if self.fused:
            self._setup_fused()
        self.graph = torch.cuda.CUDAGraph()
        cache0 = model.decoder.cache_gru.detach().clone()
        side = torch.cuda.Stream(device)
        side.wait_stream(torch.cuda.current_stream(device))
        with torch.no_grad(), torch.cuda.stream(side):
            for _ in range(max(1, int(warmup))):  # library handles / workspaces before capture
                self._forward()
        torch.cuda.current_stream(device).wait_stream(side)
        with torch.no_grad(), torch.cuda.graph(self.graph):
            self.out = self._forward()
        torch.cuda.synchronize(device)
        model.decoder.cache_gru.copy_(cache0)
        self.counter.zero_()

    def _setup_fused(self):
        m, dev = self.model, self.device
        d = m.decoder
        if not core.gru_supported(d.gru):
            raise RuntimeError("RealtimeGraph(fused=True): GRU shape outside the step kernel's")
        for seq in (d.f0_mlp, d.loudness_mlp, d.out_mlp):
            if len(seq) != 9 or any(seq[i].negative_slope != 0.01 for i in (2, 5, 8)):
                raise RuntimeError("RealtimeGraph(fused=True): mlp(.., .., 3) blocks of core.py:122-129 expected")
        R = self.call_samples // self.block_size
        if R > 8:
            raise RuntimeError("RealtimeGraph(fused=True): at most 8 frames per call")
        Hd = d.gru.hidden_size
        z = lambda n: torch.zeros(R, n, device=dev)
        self._buf = {"y2f": z(Hd), "y2l": z(Hd), "y3f": z(Hd), "y3l": z(Hd), "xp": z(3 * Hd),
                     "gru": z(Hd), "y4": z(Hd), "y5": z(Hd), "y6": z(Hd),
                     "param": z(m.harmonic_proj.out_features), "mags": z(m.noise_proj.out_features),
                     "f0": z(1), "loud": z(1), "h_last": z(Hd)[:1]}
        # the persistent recurrence's sync words (ddsp_hip_gru_forward_persistent), zeroed by the call itself
        self._gru_ws = torch.zeros(int(core._lib.query("gru_persistent_workspace_size")), dtype=torch.uint8,
                                   device=dev)

    def _forward_fused(self):
        """The same forward on ddsp_hip_dense_rows: decoder.py:43-68 + the projections
        (decoder.py:107-114) in 7 launches, the GRU on its step kernels (``gru_route="steps"``: R launches)
        or as one persistent launch (``"persistent"``: zeroing + persistent + rescue-check launches), then
        the synthesis."""
        m, d, bs, b = self.model, self.model.decoder, self.block_size, self._buf
        R, dev = self.call_samples // bs, self.device
        di = core.dense_input
        inv = 1.0 / self.std_loudness
        f0m, lm, om = d.f0_mlp, d.loudness_mlp, d.out_mlp
        core.dense_rows([  # mlp layers 1-2 (core.py:122-129), f0 and loudness
            ([di(self.pitch, ld=bs, first=f0m[0], norm=f0m[1], x_copy=b["f0"])], f0m[3], b["y2f"]),
            ([di(self.loudness, ld=bs, scale=inv, shift=-self.mean_loudness * inv, first=lm[0], norm=lm[1],
                 x_copy=b["loud"])], lm[3], b["y2l"])], R, dev)
        core.dense_rows([([di(b["y2f"], norm=f0m[4])], f0m[6], b["y3f"]),
                         ([di(b["y2l"], norm=lm[4])], lm[6], b["y3l"])], R, dev)
        # GRU input projection of cat([f0_mlp(f0), loudness_mlp(loudness)]) (decoder.py:49)
        g = d.gru
        w_ih = _Linear(g.weight_ih_l0, g.bias_ih_l0, g.input_size, 3 * g.hidden_size)
        core.dense_rows([([di(b["y3f"], norm=f0m[7]), di(b["y3l"], norm=lm[7])], w_ih, b["xp"])], R, dev)
        cache = d.cache_gru
        L = core._lib
        args = (L.ptr(b["xp"]), L.ptr(g.weight_hh_l0), L.ptr(g.bias_hh_l0), L.ptr(cache), L.ptr(b["gru"]))
        st = core.ERANGE
        if self.gru_route == "persistent":  # h_T into its own buffer: the rescue kernel re-reads h0
            st = L.call("gru_forward_persistent", *args, L.ptr(b["h_last"]), None, 1, R, g.hidden_size, 0,
                        L.ptr(self._gru_ws), self._gru_ws.numel(), L.stream_of(cache), allow=(core.ERANGE,))
            if st == 0:
                cache.view(1, -1).copy_(b["h_last"])
        if st == core.ERANGE:  # one launch per step, h_T written over h0 (the step kernels allow it)
            L.call("gru_forward", *args, L.ptr(cache), None, 1, R, g.hidden_size, L.stream_of(cache))
        self.gru_route_taken = "persistent" if st == 0 else "steps"
        # out_mlp(cat([gru_out, f0, loudness])) (decoder.py:68), then the projections
        core.dense_rows([([di(b["gru"]), di(b["f0"]), di(b["loud"])], om[0], b["y4"])], R, dev)
        core.dense_rows([([di(b["y4"], norm=om[1])], om[3], b["y5"])], R, dev)
        core.dense_rows([([di(b["y5"], norm=om[4])], om[6], b["y6"])], R, dev)
        core.dense_rows([([di(b["y6"], norm=om[7])], m.harmonic_proj, b["param"]),
                         ([di(b["y6"], norm=om[7])], m.noise_proj, b["mags"])], R, dev)
        return core.synth_frames_counter(b["f0"].view(1, R, 1), b["param"].view(1, R, -1),
                                         b["mags"].view(1, R, -1), bs, self.sample_rate, self.counter,
                                         self.seed, bias=self.bias)

    def _forward(self):
        """export.py:33-40 realtime ScriptDDSP.forward with the model's synthesis fused."""
        if self.fused:
            return self._forward_fused()
        m, bs = self.model, self.block_size
        pitch = self.pitch[:, ::bs]
        loudness = (self.loudness[:, ::bs] - self.mean_loudness) / self.std_loudness
        hidden = gru_decoder_forward(m.decoder, pitch, loudness, None, realtime=True)
        param = m.harmonic_proj(hidden)
        mags = m.noise_proj(hidden)
        return core.synth_frames_counter(pitch, param, mags, bs, self.sample_rate, self.counter,
                                         self.seed, bias=self.bias)

    def reset(self):
        self.model.decoder.cache_gru.zero_()
        self.counter.zero_()

    @torch.no_grad()
    def __call__(self, pitch, loudness):
        """pitch, loudness [1, N, 1] on the host (returns a host tensor) or on the device (returns
        the device output buffer)."""
        if tuple(pitch.shape) != (1, self.call_samples, 1) or tuple(loudness.shape) != tuple(pitch.shape):
            raise RuntimeError(f"RealtimeGraph: pitch and loudness must be [1, {self.call_samples}, 1]")
        stream = torch.cuda.current_stream(self.device)
        if pitch.is_cuda:
            self.pitch.copy_(pitch)
            self.loudness.copy_(loudness)
            self.graph.replay()
            return self.out
        self._inp_h[0:1].copy_(pitch)
        self._inp_h[1:2].copy_(loudness)
        self._inp.copy_(self._inp_h, non_blocking=True)
        self.graph.replay()
        self._out_h.copy_(self.out, non_blocking=True)
        stream.synchronize()
        return self._out_h
