"""The synthesis section of ``DDSPDecoder.forward`` (decoder.py:106-125) as one fused pipeline:
frame-rate controls -> harmonic + filtered noise -> reverb -> audio.

This is the unit the benchmark times (SURVEY.md §8(d) "End-to-end unit"): raw
harmonic parameters [B,F,H+1], pitch [B,F,1] and raw noise magnitudes [B,F,NB] in,
audio [B,F*bs,1] out.  Kernels per call: one synthesis-frame kernel (both synths, their controls, the sum)
and the reverb (partitioned FFT convolution: forward, MAC, inverse).
"""
import torch
import torch.nn as nn

from . import core
from .modules import Reverb


def make_inputs(batch, frames, n_harmonic, n_bands, block_size, seed=0, device="cpu",
                with_noise=True):
    """Seeded synthetic controls of SURVEY.md §8(d): f0 = 50*20**U[0,1) Hz, raw controls
    N(0,1), noise U[-1,1) from torch.manual_seed(123) (as the reference's torch.rand)."""
    g = torch.Generator().manual_seed(seed)
    f0 = 50.0 * 20.0 ** torch.rand(batch, frames, 1, generator=g)
    loudness = torch.randn(batch, frames, 1, generator=g)
    param = torch.randn(batch, frames, n_harmonic + 1, generator=g)
    mags = torch.randn(batch, frames, n_bands, generator=g)
    out = {"f0": f0, "loudness": loudness, "param": param, "mags": mags}
    if with_noise:
        gn = torch.Generator().manual_seed(123 + seed)
        out["noise"] = torch.rand(batch, frames, block_size, generator=gn) * 2 - 1
    return {k: v.to(device) for k, v in out.items()}


class SynthPath(nn.Module):
    """Controls -> audio on gfx950.  noise_mode: "inject" (noise tensor given) or "device"."""

    def __init__(self, block_size, sample_rate, reverb_length=None, noise_mode="device",
                 initial_bias=-5.0, reverb_seed=1):
        super().__init__()
        self.block_size = block_size
        self.sample_rate = sample_rate
        self.initial_bias = initial_bias
        self.noise_mode = noise_mode
        self.reverb = None
        if reverb_length:
            state = torch.random.get_rng_state()
            torch.manual_seed(reverb_seed)  # Reverb built after manual_seed(1)
            self.reverb = Reverb(reverb_length, sample_rate)
            torch.random.set_rng_state(state)
        self.timer = None  # optional callable(name) -> context manager, used by bench.py

    def _t(self, name):
        if self.timer is None:
            return _Null()
        return self.timer(name)

    @torch.no_grad()
    def synthesize(self, f0, param, mags, noise=None):
        """decoder.py:106-121: harmonic + filtered noise (both synths, their controls and the sum)
        in one kernel — the path before the reverb."""
        if self.noise_mode == "inject" and noise is None:
            raise ValueError("noise_mode='inject' needs a noise tensor")
        nz = noise if self.noise_mode == "inject" else None
        with self._t("synth_frames"):
            signal = core.synth_frames(f0, param, mags, self.block_size, self.sample_rate,
                                       bias=self.initial_bias, noise=nz)
        if signal is None:  # outside the fused kernel's envelope: two kernels
            with self._t("synth_frames"):
                harmonic = core.harmonic_synth_params(f0, param, self.block_size, self.sample_rate)
                signal = core.filtered_noise(mags, self.block_size, noise=nz, add=harmonic,
                                             raw_bias=self.initial_bias)
        return signal

    @torch.no_grad()
    def forward(self, f0, param, mags, noise=None):
        signal = self.synthesize(f0, param, mags, noise)
        if self.reverb is not None:
            with self._t("reverb"):
                signal = self.reverb(signal)
        return signal


class PipelinedSynthPath:
    """Two-stage serving pipeline over consecutive batches: the synthesis of batch i+1 runs on one
    CU partition while the reverb of batch i runs on the other (CU-masked HIP streams,
    ``ddsp_hip_stream_create_cu_masked``).  The two stages are complementary — the fused synthesis
    kernel is VALU-bound, the reverb's transforms and MAC memory- and latency-bound — and on one
    stream each waits for the other's tail.  Measured at config 2 (tools/exp_cumask.py): 190.7 us
    per batch against 217.7-220.8 us for the one-stream step; the latency of one batch grows to
    synthesis on 192 CUs + reverb on 64 (~0.31 ms).

    Every call returns that batch's audio, complete once ``join()`` has made the caller's stream
    wait for the reverb stream (or after a device synchronize).  Outputs are those of
    ``path(f0, param, mags, noise)`` bit for bit (same kernels; device noise advances per call in
    call order).  ``reverb_cus``: CU indices 0..reverb_cus-1 take the reverb (HIP spreads them
    evenly over the XCDs; keep it a multiple of 64 — unbalanced partitions run at the pace of
    their smallest shader engine), the rest the synthesis."""

    def __init__(self, path, reverb_cus=64, device=None):
        if path.reverb is None:
            raise ValueError("PipelinedSynthPath needs a SynthPath with a reverb")
        self.path = path
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
        if not 0 < reverb_cus < n_cu:
            raise ValueError(f"reverb_cus must be in (0, {n_cu})")
        self.reverb_cus, self.n_cu = reverb_cus, n_cu
        with torch.cuda.device(dev):
            self.s_reverb = core.cu_masked_stream(range(reverb_cus), n_cu)
            self.s_synth = core.cu_masked_stream(range(reverb_cus, n_cu), n_cu)

    @torch.no_grad()
    def __call__(self, f0, param, mags, noise=None):
        # Ordering with the caller's stream.  The masked streams are blocking streams, so work on the
        # legacy default stream is ordered with them implicitly (both ways); an event recorded there
        # on every call would serialise the two stages (measured 450 vs 184 us per batch), so the
        # explicit waits are only for a caller on a non-default stream.
        cur = torch.cuda.current_stream()
        on_default = cur == torch.cuda.default_stream(cur.device)
        if not on_default:
            self.s_synth.wait_stream(cur)  # inputs written on the caller's stream
            # ... and not handed to the caller's stream's next allocations (the caller may drop them as
            # soon as this returns) before the synthesis stream has read them
            for t in (f0, param, mags, noise):
                if t is not None:
                    t.record_stream(self.s_synth)
        with torch.cuda.stream(self.s_synth):
            signal = self.path.synthesize(f0, param, mags, noise)
            done = torch.cuda.Event()
            done.record(self.s_synth)
        rv = self.path.reverb
        with torch.cuda.stream(self.s_reverb):
            self.s_reverb.wait_event(done)
            signal.record_stream(self.s_reverb)  # its memory is not reused before the reverb read it
            # the IR spectrum the reverb reads: cached by the module, possibly allocated on another stream
            # and freed by a later invalidate() / parameter change while this stream still reads it
            spec = rv._spectrum(signal.shape[1])
            spec.record_stream(self.s_reverb)
            out = core.reverb_apply(signal, spec, rv.length)
        if not on_default:
            out.record_stream(cur)
        return out

    def join(self):
        """Make the caller's current stream wait for every batch submitted so far."""
        cur = torch.cuda.current_stream()
        cur.wait_stream(self.s_reverb)
        cur.wait_stream(self.s_synth)


class SynthGraph:
    """A fixed-shape SynthPath step captured into one HIP graph (torch.cuda.CUDAGraph is hipGraph
    on ROCm) and replayed per call: the serving form of the path for a batch whose shape does not
    change (SURVEY.md §8(b) asks for HIP streams and graphs instead of a tracing compiler).

    The graph holds the fused synthesis kernel and the reverb's three UPOLS kernels; replay
    launches them back to back with no host work between them.  Inputs are the static tensors
    given here (update them in place between replays); ``out`` is a static buffer overwritten by
    every replay.

    * Device noise (``noise=None``): drawn with the offset held in the device counter ``counter``
      (``ddsp_hip_synth_frames_counter``), advanced on the stream by every replay — replay k draws
      the noise of ``core.synth_frames`` at offset k (parity: tests/test_gpu_device_noise.py).
    * ``rebuild_ir=True`` also captures ``Reverb.build_impulse`` and the IR spectrum
      (modules.py:30-33 rebuilds them on every forward); by default the spectrum of the reverb's
      parameters at capture time is copied into a buffer the graph owns (the module's cached
      spectrum may be freed and its memory reused by invalidate() or a forward of another length),
      so re-capture after changing the reverb's parameters.
    """

    def __init__(self, path, f0, param, mags, noise=None, seed=0x5EEDDD5B, rebuild_ir=False, warmup=2):
        if f0.device.type != "cuda":
            raise RuntimeError("SynthGraph: inputs must be on a HIP device")
        self.path = path
        self.f0, self.param, self.mags, self.noise = f0, param, mags, noise
        self.seed = int(seed)
        self.rebuild_ir = bool(rebuild_ir)
        self.counter = torch.zeros(1, dtype=torch.int64, device=f0.device)
        self.spec = None
        if path.reverb is not None and not self.rebuild_ir:
            with torch.no_grad():
                self.spec = path.reverb._spectrum(f0.shape[1] * path.block_size).clone()
        if noise is None and not core.synth_frames_in_envelope(param.shape[-1] - 1, mags.shape[-1],
                                                               path.block_size, param.shape[0]):
            raise RuntimeError("SynthGraph: device noise needs the fused kernel's shape envelope")
        self.graph = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream(f0.device)
        side.wait_stream(torch.cuda.current_stream(f0.device))
        with torch.no_grad(), torch.cuda.stream(side):
            for _ in range(max(1, int(warmup))):  # workspaces and library state before capture
                self._step()
        torch.cuda.current_stream(f0.device).wait_stream(side)
        with torch.no_grad(), torch.cuda.graph(self.graph):
            self.out = self._step()
        self.reset()

    def _step(self):
        p = self.path
        if self.noise is None:
            sig = core.synth_frames_counter(self.f0, self.param, self.mags, p.block_size, p.sample_rate,
                                            self.counter, self.seed, bias=p.initial_bias)
        else:
            sig = core.synth_frames(self.f0, self.param, self.mags, p.block_size, p.sample_rate,
                                    bias=p.initial_bias, noise=self.noise)
            if sig is None:
                harmonic = core.harmonic_synth_params(self.f0, self.param, p.block_size, p.sample_rate)
                sig = core.filtered_noise(self.mags, p.block_size, noise=self.noise, add=harmonic,
                                          raw_bias=p.initial_bias)
        rv = p.reverb
        if rv is None:
            return sig
        if self.rebuild_ir:
            spec = core.reverb_spectrum(rv.build_impulse(), sig.shape[1])
        else:
            spec = self.spec  # owned by the graph
        return core.reverb_apply(sig, spec, rv.length)

    def reset(self):
        """Rewind the device-noise counter (the next replay draws offset 0)."""
        self.counter.zero_()

    def replay(self):
        self.graph.replay()
        return self.out


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
