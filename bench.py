"""Benchmark: DDSP harmonic-plus-noise synthesis on MI355X (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A step = one pass of the synthesis path (decoder.py:106-125: frame-rate controls ->
harmonic + filtered noise -> 1 s reverb -> audio) over one batch of configuration 2
(batch 64 per GPU, 200 frames, block_size 512, 100 harmonics, 65 noise bands, 48 kHz).
Inputs are resident in HBM before the timed region.  Multi-GPU: one process per GPU,
each synthesising its own 64-item shard (batch items are independent — no collective on
the data path; weak scaling); the timed region is bracketed by barrier + synchronize and
the max over ranks is reported.  Rank 0 prints ONE JSON line.

Rooflines:
  * "roofline"    — the dominant kernel of the timed step, the fused synthesis kernel, against its
    real bound, VALU issue: issue slots per launch (PMC instruction counts, the sine at 4 slots) /
    launch duration (HIP events on its stream inside the timed region) / the chip's issue peak;
    "traffic" is its PMC HBM bytes (it reads only frame-rate controls);
  * "op_boundary_effective" — SURVEY.md §8(d)'s convention, the oscillator's op-boundary bytes
    4*(H+2) B/sample divided by the fused kernel's time (not a roofline: fusion removed them);
  * "roofline_op" — the op-boundary harmonic_synth kernel (per-sample f0 [B,T,1] and amplitudes
    [B,T,H] read from HBM), HBM-bound, timed in a separate leg after the timed region.
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)
# VALU issue model of gfx950, measured by tools/issue_probe.hip (profiles/r02_issue_probe.log): with
# two or more waves per SIMD an fp32 VALU op (v_fma/v_mul/v_add) issues every ~2 cycles per SIMD
# (2.26 at 8 waves/SIMD; 4-5 with a single wave, MI355X_MICROARCH.md's one-wave row), and the
# transcendental v_sin_f32 every 8 cycles regardless of waves.  One issue SLOT = 2 SIMD cycles:
# fp32 VALU op = 1 slot, v_sin_f32 = 4 slots.  Peak = 256 CUs x 4 SIMDs x 2.4 GHz / 2 cycles.
VALU_PEAK_SLOTS = 256 * 4 * 2.4e9 / 2      # 1.2288e12 wave-instruction slots/s
SIN_SLOTS = 4
OSC_SLOTS_PER_SINE = 6 + SIN_SLOTS         # per (sample, harmonic): 6 fp32 VALU ops + one v_sin_f32
                                           # (synth_frame.hip inner loop; tools/loop_align.py counts it)

DOMINANT_KERNEL = "synth_frame_kernelILb1ELb0ELb0ELb0EE"   # device noise, 4 samples/thread, no control dicts


def kernel_source_sha():
    """sha256 (16 hex) of the dominant kernel's instruction stream in the built library
    (tools/loop_align.kernel_sha): PMC instruction counts recorded for another build of that kernel
    (profiles/pmc_valu.json "kernel_sha") are stale and not used."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    try:
        import loop_align
        from ddsp_pytorch_amd import _lib
        return loop_align.kernel_sha(_lib.LIB_PATH, DOMINANT_KERNEL)
    except Exception:  # no llvm-objdump: counts cannot be matched to the build
        return None


def fir_macs_per_frame(n_bands, block_size):
    """Multiply-adds of one frame's causal, truncated noise convolution (core.py:169-176 keeps the first
    block_size outputs of signal (*) h): sum over the filter's nonzero taps m of (block_size - m).  The
    taps follow amp_to_impulse_response (core.py:158-164): h[j] = ir[(q - n/2) mod n] * hann_n[q] with
    q = (j + n/2) rolled into the block, zero where q >= n or hann_n[q] = 0 (q = 0).  At 65 bands and
    block 512: taps [0, 64) and (448, 512) -> 64 x 512 MACs, i.e. n/2 = 64 per sample (the filter has
    127 nonzero taps, but causality truncates the wrapped ones to the block's last samples)."""
    n, half, bs = 2 * (n_bands - 1), n_bands - 1, block_size
    total = 0
    for j in range(bs):
        q = j + half
        if q >= bs:
            q = q - bs if half < bs else q % bs
        if 0 < q < n:
            total += bs - j
    return total


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--settle", type=float, default=0.25,
                   help="minimum seconds of untimed warmup (clock/power settling), on top of --warmup steps")
    p.add_argument("--config", type=int, default=2, choices=(2, 4, 5),
                   help="BASELINE.json configuration: 2 (default; batch 64, 200 frames, 100 "
                        "harmonics, 1 s IR), 4 (batch 16, 2 s IR), 5 (per-GPU shard of the 8-GPU "
                        "job: batch 64, 400 frames, 128 harmonics)")
    p.add_argument("--batch", type=int, default=None, help="items per GPU")
    p.add_argument("--frames", type=int, default=None)
    p.add_argument("--block-size", type=int, default=512)
    p.add_argument("--harmonics", type=int, default=None)
    p.add_argument("--bands", type=int, default=65)
    p.add_argument("--sample-rate", type=int, default=48000)
    p.add_argument("--reverb-length", type=int, default=None)
    p.add_argument("--noise", choices=("device", "inject"), default="device")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-op-leg", action="store_true")
    p.add_argument("--chunks", type=int, default=4,
                   help="N>1 scatter/gather leg: batch chunks pipelined through the collectives")
    p.add_argument("--no-gather", action="store_true",
                   help="N>1: skip the synth + RCCL gather-to-rank-0 leg (reported separately as "
                        "'gathered'; value is always the left-sharded throughput)")
    p.add_argument("--no-train-leg", action="store_true",
                   help="skip the training-step leg (synthesis forward + backward kernels)")
    p.add_argument("--no-loss-leg", action="store_true",
                   help="skip the multiscale spectral loss leg (forward + backward, both signals)")
    p.add_argument("--no-model-train-leg", action="store_true",
                   help="skip the full training step of train.py (DDSPDecoder + spectral loss + backward + Adam)")
    p.add_argument("--no-decoder-leg", action="store_true",
                   help="skip the full DDSPDecoder.forward leg (GRU/MLP + synthesis)")
    p.add_argument("--no-realtime-leg", action="store_true",
                   help="skip config 3's realtime leg (1024-sample calls through the HIP-graph stream)")
    p.add_argument("--realtime-calls", type=int, default=400)
    p.add_argument("--cpu-batch", type=int, default=None, help="items in the CPU-baseline sample")
    p.add_argument("--cpu-reps", type=int, default=3)
    p.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"),
                   help="PMC HBM bytes per launch (tools/pmc_traffic.py output)")
    p.add_argument("--valu-counts", default=os.path.join(ROOT, "profiles", "pmc_valu.json"),
                   help="PMC SQ_INSTS_VALU per launch of the dominant kernel (tools/pmc_valu.py output)")
    p.add_argument("--no-pipelined-leg", action="store_true",
                   help="skip the two-stage serving pipeline leg (synth.PipelinedSynthPath)")
    p.add_argument("--reverb-cus", type=int, default=64,
                   help="CUs of the pipelined leg's reverb partition (the rest run the synthesis)")
    p.add_argument("--no-uncached-leg", action="store_true",
                   help="skip the step with the IR spectrum rebuilt on every call (as modules.py:30-33)")
    a = p.parse_args()
    cfg = {2: (64, 200, 100, 48000), 4: (16, 200, 100, 96000), 5: (64, 400, 128, 48000)}[a.config]
    if a.cpu_batch is None:
        a.cpu_batch = 8 if a.config == 5 else 16
    for name, v in zip(("batch", "frames", "harmonics", "reverb_length"), cfg):
        if getattr(a, name) is None:
            setattr(a, name, v)
    return a


class EventTimer:
    """Per-kernel HIP-event timing on the launching stream (torch's current stream)."""

    def __init__(self, names):
        self.names = set(names)
        self.pairs = {n: [] for n in names}
        self.enabled = False

    def __call__(self, name):
        timer = self

        class Ctx:
            def __enter__(self):
                if timer.enabled and name in timer.names:
                    self.e0 = torch.cuda.Event(enable_timing=True)
                    self.e0.record()
                return self

            def __exit__(self, *a):
                if timer.enabled and name in timer.names:
                    e1 = torch.cuda.Event(enable_timing=True)
                    e1.record()
                    timer.pairs[name].append((self.e0, e1))
                return False

        return Ctx()

    def mean_ms(self, name):
        ps = self.pairs[name]
        return sum(a.elapsed_time(b) for a, b in ps) / len(ps) if ps else float("nan")


def load_traffic(path):
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def cpu_baseline(args, rank_inputs_seed=0):
    """The reference's algorithm on the host cores: oracle/torch_ref.py (the same ATen op
    sequence as ddsp/core.py + modules.py, bit-exact to the reference's goldens).

    Thread counts (BASELINE.md's plan: torch.set_num_threads(os.cpu_count())): a sweep over
    {16, 32, 64, 128, 256} threads capped at os.cpu_count(), plus the process's CPU share
    (OMP_NUM_THREADS / the affinity mask; a GPU box gives one process a 16-core share of a larger
    host), each timed on a 4-item sample; the fastest thread count is then timed on the full
    sample and reported, with every sweep point and the host's core count."""
    from oracle import torch_ref as tr
    from ddsp_pytorch_amd.synth import make_inputs
    host = os.cpu_count() or 1
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = host
    share = int(os.environ.get("OMP_NUM_THREADS", "0")) or affinity
    torch.manual_seed(1)
    noise = (torch.rand(args.reverb_length) * 2 - 1).unsqueeze(-1)
    rv = tr.Reverb(noise, torch.tensor(5.0), torch.tensor(0.0), args.reverb_length, args.sample_rate)

    def runner(B):
        inp = make_inputs(B, args.frames, args.harmonics, args.bands, args.block_size, seed=0)
        return lambda: tr.synth_path(inp["f0"], inp["param"], inp["mags"], inp["noise"], rv,
                                     args.block_size, args.sample_rate)

    prev = torch.get_num_threads()
    sweep_b = min(4, args.cpu_batch)
    run = runner(sweep_b)
    by_threads = {}
    for threads in sorted({t for t in (16, 32, 64, 128, 256) if t <= host} | {share}):
        torch.set_num_threads(threads)
        run()  # warm-up
        t0 = time.perf_counter()
        run()
        by_threads[threads] = sweep_b * args.frames * args.block_size / (time.perf_counter() - t0)
    best = max(by_threads, key=by_threads.get)
    torch.set_num_threads(best)
    B = args.cpu_batch
    run = runner(B)
    run()  # warm-up
    times = []
    budget = time.perf_counter() + 15.0
    for _ in range(args.cpu_reps):
        t0 = time.perf_counter()
        run()
        times.append(time.perf_counter() - t0)
        if time.perf_counter() > budget:
            break
    torch.set_num_threads(prev)
    t = sorted(times)[len(times) // 2]
    samples = B * args.frames * args.block_size
    return {"value": samples / t, "unit": "samples/s", "cores": best, "kind": "port",
            "host_cpu_count": host, "affinity_cpus": affinity,
            "by_threads": {str(k): round(v, 1) for k, v in sorted(by_threads.items())},
            "sample": f"oracle/torch_ref.synth_path (reference ATen op sequence), batch {B} of "
                      f"config {args.config} (F={args.frames}, bs={args.block_size}, H={args.harmonics}, "
                      f"NB={args.bands}, {args.reverb_length}-tap reverb), median of {len(times)} runs, "
                      f"{t:.3f} s each at {best} threads (the fastest of the by_threads sweep, timed on "
                      f"{sweep_b} items; host os.cpu_count() = {host})"}


def train_leg(args, inp, dev, reps=100):
    """one training step of the synthesis path — forward (synth_frames +
    reverb) and backward (reverb input/IR gradients, harmonic and noise VJPs) for an upstream
    gradient w, i.e. what train.py:84-130 runs below the decoder network.  Timed at steady state, as a
    training loop runs it: 10 untimed steps, then `reps` (0.05 s of steps at config 2; 20 steps read about
    1 % higher on one box: 0.5289-0.5340 vs 0.5234-0.5277 ms)."""
    from ddsp_pytorch_amd import core
    from ddsp_pytorch_amd.modules import Reverb
    B, F, H, NB, bs, sr = (args.batch, args.frames, args.harmonics, args.bands, args.block_size,
                           args.sample_rate)
    torch.manual_seed(1)
    rv = Reverb(args.reverb_length, sr).to(dev)
    param = inp["param"].clone().requires_grad_(True)
    mags = inp["mags"].clone().requires_grad_(True)
    w = torch.randn(B, F * bs, 1, device=dev)
    ev = {k: [] for k in ("forward", "backward")}

    def step(timed):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        param.grad = mags.grad = None
        for p_ in rv.parameters():
            p_.grad = None
        e[0].record()
        sig = core.synth_frames(inp["f0"], param, mags, bs, sr)
        out = rv(sig)
        e[1].record()
        out.backward(w)
        e[2].record()
        if timed:
            ev["forward"].append((e[0], e[1]))
            ev["backward"].append((e[1], e[2]))

    for _ in range(10):
        step(False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        step(True)
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / reps
    assert torch.isfinite(param.grad).all() and torch.isfinite(mags.grad).all()
    ms = {k: round(sum(a.elapsed_time(b) for a, b in v) / len(v), 4) for k, v in ev.items()}
    return {"value": round(B * F * bs / t, 1), "unit": "samples/s", "ms_per_step": round(t * 1e3, 4),
            "event_ms": ms, "gradients": "param [B,F,H+1], mags [B,F,NB], reverb noise/decay/wet",
            "workload": f"config {args.config} synthesis forward + backward, batch {B}/GPU"}


def loss_leg(args, dev, reps=10):
    """train.py:91-104's multiscale spectral loss (scales 4096..128, 75%
    overlap) of a target and a reconstruction [B, T], forward + backward w.r.t. the
    reconstruction — on the gfx950 STFT kernels, and on torch.stft (rocFFT) for comparison."""
    from ddsp_pytorch_amd import core
    from ddsp_pytorch_amd.loss import multiscale_spec_loss
    B, T = args.batch, args.frames * args.block_size
    scales = (4096, 2048, 1024, 512, 256, 128)
    g = torch.Generator(device=dev).manual_seed(5)
    sig = torch.randn(B, T, device=dev, generator=g) * 0.3
    rec = (sig + 0.05 * torch.randn(B, T, device=dev, generator=g)).requires_grad_(True)

    def torch_fft(x):
        return [torch.stft(x, s, s // 4, s, torch.hann_window(s, device=dev), True, normalized=True,
                           return_complex=True).abs() for s in scales]

    def run(fn):
        for _ in range(3):
            rec.grad = None
            multiscale_spec_loss(fn(sig), fn(rec)).backward()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            rec.grad = None
            multiscale_spec_loss(fn(sig), fn(rec)).backward()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps

    def run_fused():
        from ddsp_pytorch_amd.loss import spectral_loss
        for _ in range(3):
            rec.grad = None
            spectral_loss(sig, rec, scales, 0.75).backward()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            rec.grad = None
            spectral_loss(sig, rec, scales, 0.75).backward()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps

    t_fused = run_fused()
    t_ours = run(lambda x: core.multiscale_fft(x, scales, 0.75))
    t_torch = run(torch_fft)
    return {"value": round(B * T / t_fused, 1), "unit": "samples/s", "ms_per_step": round(t_fused * 1e3, 4),
            "spectrogram_route_ms_per_step": round(t_ours * 1e3, 4),
            "torch_stft_ms_per_step": round(t_torch * 1e3, 4),
            "workload": f"multiscale spectral loss fwd+bwd, batch {B} x {T} samples, scales {list(scales)}; "
                        "value: fused ddsp_hip_spectral_loss; spectrogram route: core.multiscale_fft + "
                        "train.py's loss in torch; torch_stft: the reference's torch.stft (rocFFT) on the GPU"}


def model_train_leg(args, inp, dev, reps=5):
    """train.py:84-130's step at config 2's shape: DDSPDecoder.forward (hidden 512) -> fused spectral
    loss -> backward -> Adam step, all gradients on the gfx950 kernels (synthesis VJPs, GRU BPTT,
    STFT loss, the MLP blocks' Linear / LayerNorm + LeakyReLU forward and backward, the Linears' and the
    GRU's weight gradients; the one-feature first Linears, the 514-input out_mlp block and the output
    projections stay on torch under autograd).  Random-init weights and a synthetic target signal."""
    from ddsp_pytorch_amd.decoder import DDSPDecoder
    from ddsp_pytorch_amd.loss import spectral_loss
    B, F, bs = args.batch, args.frames, args.block_size
    torch.manual_seed(0)
    model = DDSPDecoder(512, args.harmonics, args.bands, args.sample_rate, bs, True).to(dev).train()
    model.noise_synth.noise_mode = "device"
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    sig = torch.randn(B, F * bs, device=dev) * 0.1
    batch = {"pitch": inp["f0"], "loudness": torch.randn(B, F, 1, device=dev)}

    def step():
        out = model(batch)
        loss = spectral_loss(sig, out["signal"].squeeze(-1))
        opt.zero_grad()
        loss.backward()
        opt.step()
        return loss

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        loss = step()
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / reps
    assert torch.isfinite(loss)
    del model, opt
    return {"value": round(B * F * bs / t, 1), "unit": "samples/s", "ms_per_step": round(t * 1e3, 3),
            "workload": f"train.py step: DDSPDecoder(hidden 512, H {args.harmonics}) fwd + spectral loss "
                        f"(6 scales) + backward + Adam, batch {B} x {F} frames"}


def decoder_leg(args, inp, dev, reps=10):
    """the full DDSPDecoder.forward rate, reported beside the synthesis path —
    GRU/MLP control network (hidden 512, torch on MIOpen/hipBLASLt) + the gfx950 synthesis."""
    from ddsp_pytorch_amd.decoder import DDSPDecoder
    B, F = args.batch, args.frames
    torch.manual_seed(0)
    model = DDSPDecoder(512, args.harmonics, args.bands, args.sample_rate, args.block_size, True)
    model = model.to(dev).eval()
    model.noise_synth.noise_mode = "device"
    if args.reverb_length != args.sample_rate:
        model.reverb = type(model.reverb)(args.reverb_length, args.sample_rate).to(dev)
    batch = {"pitch": inp["f0"], "loudness": torch.randn(B, F, 1, device=dev)}
    with torch.no_grad():
        for _ in range(3):
            model(batch)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            out = model(batch)
        torch.cuda.synchronize()
        t = (time.perf_counter() - t0) / reps
    assert torch.isfinite(out["signal"]).all()
    del model
    return {"value": round(B * F * args.block_size / t, 1), "unit": "samples/s",
            "ms_per_forward": round(t * 1e3, 4),
            "model": f"DDSPDecoder(hidden 512, H {args.harmonics}, NB {args.bands}, reverb "
                     f"{args.reverb_length}), random init, batch {B} x {F} frames"}


def decoder_synthesis_leg(args, inp, dev, reps=50):
    """The synthesis section of DDSPDecoder.forward (decoder.py:106-125: the two projections, both
    synths with their controls, the sum, the returned parts and control dicts, the 1 s reverb) as the
    decoder runs it (decoder.decoder_synthesize, the fused kernel; install() binds the same function
    under the reference's DDSPDecoder.forward), from a fixed GRU output; device noise."""
    from ddsp_pytorch_amd.decoder import DDSPDecoder, decoder_projections, decoder_synthesize
    B, F, bs = args.batch, args.frames, args.block_size
    torch.manual_seed(0)
    model = DDSPDecoder(512, args.harmonics, args.bands, args.sample_rate, bs, True).to(dev).eval()
    model.noise_synth.noise_mode = "device"
    if args.reverb_length != args.sample_rate:
        model.reverb = type(model.reverb)(args.reverb_length, args.sample_rate).to(dev)
    def timed(fn):
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            r = fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps, r

    from ddsp_pytorch_amd import core
    with torch.no_grad():
        hidden = model.decoder(inp["f0"], torch.randn(B, F, 1, device=dev))
        t, out = timed(lambda: decoder_synthesize(model, hidden, inp["f0"]))
        t_proj, _ = timed(lambda: decoder_projections(model, hidden))
        param, mags = decoder_projections(model, hidden)

        def synth_rev():
            sig = core.synth_frames(inp["f0"], param, mags, bs, args.sample_rate, parts=True, controls=True)[0]
            return model.reverb(sig)
        t_syn, _ = timed(synth_rev)
    assert torch.isfinite(out[0]).all()
    del model
    return {"value": round(B * F * bs / t, 1), "unit": "samples/s", "ms_per_step": round(t * 1e3, 4),
            "split_ms": {"projections (one GEMM)": round(t_proj * 1e3, 4),
                         "synthesis_parts_controls_reverb": round(t_syn * 1e3, 4)},
            "workload": f"decoder.py:106-125 synthesis section of DDSPDecoder(hidden 512, H {args.harmonics}, "
                        f"NB {args.bands}, reverb {args.reverb_length}) from a fixed GRU output: projections, "
                        "fused synthesis writing signal + harmonic + noise + control dicts, reverb; batch "
                        f"{B} x {F} frames, device noise"}


def realtime_leg(dev, calls=400, warm=40):
    """BASELINE config 3: the realtime stream at the shipped model size — DDSPDecoder(512, 64, 65, 48000, 256,
    False) (config.yaml's decoder with block 256, no reverb, export.py:33-40's realtime forward), batch 1,
    one 1024-sample call at a time as the ddsp~ host makes them (realtime/ddsp_tilde/ddsp_model.cpp:32-52:
    host pitch/loudness in, host audio out, the GRU state carried between calls), through
    realtime.RealtimeGraph (one HIP-graph replay per call).  Per call: p50 / p99 wall time from the host's
    buffers to the host's audio, and the device time of one replay.  Realtime factor as the reference's
    performance.py:28-34 computes it: samples per call / (mean call time x sample rate).  The GRU runs on
    both routes (step kernels, one persistent launch); the faster by p50 is reported."""
    from ddsp_pytorch_amd.decoder import DDSPDecoder
    from ddsp_pytorch_amd.realtime import RealtimeGraph
    N, sr, bs = 1024, 48000, 256
    torch.manual_seed(0)
    m = DDSPDecoder(512, 64, 65, sr, bs, False).to(dev).eval()
    g = torch.Generator().manual_seed(3)
    ins = [(80.0 * 10.0 ** torch.rand(1, N, 1, generator=g), torch.randn(1, N, 1, generator=g) - 2.0)
           for _ in range(16)]
    by_route = {}
    for route in ("steps", "persistent"):
        rt = RealtimeGraph(m, N, fused=True, gru_route=route)
        lat = []
        with torch.no_grad():
            for i in range(warm + calls):
                p, l = ins[i % len(ins)]
                t0 = time.perf_counter()
                y = rt(p, l)
                if i >= warm:
                    lat.append((time.perf_counter() - t0) * 1e3)
            assert torch.isfinite(y).all()
            pd, ld = ins[0][0].to(dev), ins[0][1].to(dev)
            for _ in range(20):
                rt(pd, ld)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(200):
                rt(pd, ld)
            e1.record()
            torch.cuda.synchronize()
        lat.sort()
        mean = sum(lat) / len(lat)
        by_route[route] = {"p50_ms": round(lat[len(lat) // 2], 4), "p99_ms": round(lat[int(0.99 * len(lat))], 4),
                           "mean_ms": round(mean, 4), "device_ms_per_replay": round(e0.elapsed_time(e1) / 200, 4),
                           "realtime_factor": round(N / (mean * 1e-3 * sr), 1),
                           "gru_route_taken": rt.gru_route_taken}
        del rt
    best = min(by_route, key=lambda r: by_route[r]["p50_ms"])
    b = by_route[best]
    return {"value": b["realtime_factor"], "unit": "x realtime (performance.py:28-34)", "p50_ms": b["p50_ms"],
            "p99_ms": b["p99_ms"], "device_ms_per_replay": b["device_ms_per_replay"], "gru_route": best,
            "by_route": by_route, "budget_ms": round(N / sr * 1e3, 3), "calls_timed": calls,
            "workload": "config 3: DDSPDecoder(hidden 512, H 64, NB 65, 48 kHz, block 256, no reverb), batch 1, "
                        "1024-sample calls (4 frames) host -> HIP-graph replay -> host, GRU state carried, "
                        "device noise; random-init weights, synthetic pitch/loudness"}


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def _max_over_ranks(seconds, dev, dist):
    t = torch.tensor([seconds], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gathered_leg(step, global_batch, samples_per_step, steps, dev, dist):
    """N>1 leg (SURVEY 8(e) "gathered to rank 0"): every rank synthesises its shard (``step()``
    returns this rank's [b_r, T, 1] slice of a ``global_batch``-item batch, ragged shards allowed)
    and the audio is gathered on rank 0 (torch.distributed.gather: RCCL over xGMI on MI355X, gloo
    in the CPU tests).  Timed between barrier + device sync on both sides, max over ranks.
    Returns (result dict, the last gathered batch on rank 0 / None elsewhere)."""
    from ddsp_pytorch_amd.shard import gather_audio
    _sync(dev)
    dist.barrier()
    t0 = time.perf_counter()
    g = None
    for _ in range(steps):
        g = gather_audio(step(), global_batch)
    _sync(dev)
    dist.barrier()
    t = _max_over_ranks(time.perf_counter() - t0, dev, dist)
    backend = "RCCL" if dist.get_backend() == "nccl" else dist.get_backend()
    return ({"value": round(samples_per_step * steps / t, 1), "unit": "samples/s",
             "collective": f"torch.distributed.gather ({backend})",
             "ms_per_step": round(t / steps * 1e3, 4)}, g)


def scatter_gather_leg(synth, held, global_batch, tails, samples_per_step, steps, chunks, dev, dist,
                       reverb=None, warm=2):
    """N>1 leg (SURVEY 8(e) root-held batch): rank 0 holds the frame-rate controls of all
    ``global_batch`` items (``held``: full-batch tensors in the order ``synth`` takes them, None on
    the other ranks; ``tails``: their per-item shapes), scatters them in ``chunks`` pieces, every
    rank synthesises its shard and the audio is gathered back on rank 0, the collectives of one
    chunk overlapping the synthesis of its neighbours (shard.synthesize_pipelined).  The reverb IR
    is broadcast once first.  Returns (result dict, the last gathered batch on rank 0)."""
    from ddsp_pytorch_amd.shard import broadcast_module, synthesize_pipelined
    if reverb is not None:
        broadcast_module(reverb)
    pipe = lambda: synthesize_pipelined(synth, held, global_batch, tails, chunks=chunks, device=dev)
    for _ in range(warm):
        pipe()
    _sync(dev)
    dist.barrier()
    t0 = time.perf_counter()
    g = None
    for _ in range(steps):
        g = pipe()
    _sync(dev)
    dist.barrier()
    t = _max_over_ranks(time.perf_counter() - t0, dev, dist)
    backend = "RCCL" if dist.get_backend() == "nccl" else dist.get_backend()
    return ({"value": round(samples_per_step * steps / t, 1), "unit": "samples/s",
             "ms_per_step": round(t / steps * 1e3, 4), "chunks": chunks,
             "collective": f"torch.distributed scatter (controls) + gather (audio), {backend}, async per chunk"},
            g)


PIPELINE_MIN_BATCHES = 200


def pipelined_leg(syn, run_args, samples_per_step, steps, reverb_cus, dev, dist, warm=40):
    """Serving form over consecutive batches (synth.PipelinedSynthPath): the synthesis of batch i+1
    on one CU partition beside the reverb of batch i on the other.  Same work per batch as the
    headline step; reported beside it, never as it.  A steady-state rate: at least
    PIPELINE_MIN_BATCHES batches are timed whatever --steps is (at the driver's 20 the pipeline's fill
    and drain and the host's start-up dominate: 0.222 vs 0.189 ms per batch at 200, profiles/
    r04c_pipelined_steps.log).  Timed between barrier + device sync, max over ranks; latency = one batch
    alone through both stages (best of 5).  The warmup runs until the caching allocator holds the
    blocks the two streams cycle through (fresh blocks are hipMalloc'd while signals still wait for
    the reverb stream: the first ~10-20 batches run slower)."""
    from ddsp_pytorch_amd.synth import PipelinedSynthPath
    steps = max(int(steps), PIPELINE_MIN_BATCHES)
    pipe = PipelinedSynthPath(syn, reverb_cus=reverb_cus, device=dev)
    for _ in range(warm):
        pipe(*run_args)
    pipe.join()
    _sync(dev)
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        pipe(*run_args)
    pipe.join()
    _sync(dev)
    t = time.perf_counter() - t0
    if dist:
        dist.barrier()
        t = _max_over_ranks(t, dev, dist)
    lat = []
    for _ in range(5):
        _sync(dev)
        t1 = time.perf_counter()
        pipe(*run_args)
        pipe.join()
        _sync(dev)
        lat.append(time.perf_counter() - t1)
    return {"value": round(samples_per_step * steps / t, 1), "unit": "samples/s", "batches_timed": steps,
            "ms_per_step": round(t / steps * 1e3, 4), "latency_ms": round(min(lat) * 1e3, 4),
            "cu_split": {"reverb": reverb_cus, "synthesis": pipe.n_cu - reverb_cus},
            "note": "two-stage pipeline over consecutive batches on CU-masked streams (synthesis of "
                    "batch i+1 beside the reverb of batch i); same work per batch as the headline "
                    "step, reported beside it"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # launched by torch.distributed.run (WORLD_SIZE set, 1 included): one process per GPU over RCCL
    if "WORLD_SIZE" in os.environ:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist = None
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    import ddsp_pytorch_amd  # noqa: F401  (loads the C-ABI library; raises if missing)
    from ddsp_pytorch_amd import core
    from ddsp_pytorch_amd.synth import SynthPath, make_inputs

    B, F, H, NB, bs, sr = (args.batch, args.frames, args.harmonics, args.bands, args.block_size,
                           args.sample_rate)
    inp = make_inputs(B, F, H, NB, bs, seed=rank, device=dev, with_noise=(args.noise == "inject"))
    syn = SynthPath(bs, sr, reverb_length=args.reverb_length, noise_mode=args.noise).to(dev)
    # timed region: events only around the dominant kernel (the roofline's launch duration);
    # the per-kernel breakdown is measured in a separate loop afterwards
    timer = EventTimer(["synth_frames"])
    syn.timer = timer
    core.set_noise_seed(1234 + rank)

    def step():
        return syn(inp["f0"], inp["param"], inp["mags"], inp.get("noise"))

    # W untimed warmup steps, continued until the GPU has run the step for --settle seconds:
    # a cold MI355X runs the VALU-bound synthesis kernel ~12% slower for its first ~50 ms
    # (0.194 vs 0.172 ms per launch, measured) while clocks and power state settle
    warm_steps, tw = 0, time.perf_counter()
    while warm_steps < args.warmup or time.perf_counter() - tw < args.settle:
        step()
        warm_steps += 1
        if warm_steps % 32 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    warm_s = time.perf_counter() - tw
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    timer.enabled = True
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    timer.enabled = False
    if dist:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    assert torch.isfinite(out).all()

    # per-kernel breakdown: one event pair per step, one kernel group per loop (events around
    # every group of a step add their own gaps and read high against rocprofv3)
    kern_ms = {}
    for name in ("synth_frames", "reverb"):
        breakdown = EventTimer([name])
        syn.timer = breakdown
        for _ in range(20):  # back at the loaded clock before the events are read
            step()
        breakdown.enabled = True
        for _ in range(50):
            step()
        torch.cuda.synchronize()
        breakdown.enabled = False
        kern_ms[name] = breakdown.mean_ms(name)
    syn.timer = None

    samples_per_step = B * F * bs * world
    value = samples_per_step * args.steps / elapsed
    traffic = load_traffic(args.traffic)

    # dominant kernel: the fused synthesis kernel (per launch = B*F*bs samples of this rank).  Its
    # bound is VALU issue (it reads only frame-rate controls): achieved = issue slots per launch
    # (PMC SQ_INSTS_VALU of this kernel, each v_sin_f32 counted at 4 slots) / launch duration.
    osc_ms = timer.mean_ms("synth_frames")
    n_sin = B * F * bs * H
    osc_slots = n_sin / 64 * OSC_SLOTS_PER_SINE
    vc = load_traffic(args.valu_counts).get(f"config{args.config}", {})
    src_sha = kernel_source_sha()
    stale = bool(vc) and (src_sha is None or vc.get("kernel_sha") != src_sha)
    if vc.get("SQ_INSTS_VALU") and not stale:
        slots = vc["SQ_INSTS_VALU"] + (SIN_SLOTS - 1) * n_sin / 64
        slots_src = (f"PMC SQ_INSTS_VALU {vc['SQ_INSTS_VALU']:.4g} wave-instructions per launch "
                     f"({args.valu_counts.replace(ROOT + os.sep, '')}) + {SIN_SLOTS - 1} extra slots per "
                     "v_sin_f32 wave-instruction")
    else:
        slots = osc_slots
        slots_src = ("oscillator model only (" + ("the PMC counts were taken on another build of the kernel"
                     if stale else "no PMC counts for this configuration") + ")")
    # algorithmic issue slots: per sample H x (6 VALU + v_sin_f32 at 4 slots) for the oscillator + the
    # causal noise FIR's multiply-adds (one FMA each: n/2 = 64 per sample at 65 bands, fir_macs_per_frame);
    # no controls, RNG or addressing.  Rounds 2-3 counted the filter's 127 nonzero taps for every sample
    # (kept as frac_algorithmic_r03_convention for comparison)
    fir_macs = fir_macs_per_frame(NB, bs) / bs
    alg_slots = B * F * bs / 64 * (H * OSC_SLOTS_PER_SINE + fir_macs)
    alg_slots_r03 = B * F * bs / 64 * (H * OSC_SLOTS_PER_SINE + 2 * (NB - 1) - 1)
    achieved = slots / (osc_ms * 1e-3)
    osc_bytes = 4 * (H + 2) * B * F * bs
    roofline = {"bound": "valu", "achieved": round(achieved / 1e12, 4), "peak": VALU_PEAK_SLOTS / 1e12,
                "unit": "T issue slots/s (wave64 VALU: fp32 op 1 slot = 2 SIMD cycles, v_sin_f32 4 slots)",
                "frac": round(achieved / VALU_PEAK_SLOTS, 4),
                "frac_algorithmic": round(alg_slots / (osc_ms * 1e-3) / VALU_PEAK_SLOTS, 4),
                "algorithmic_slots_per_launch": round(alg_slots),
                "algorithmic_slots_note": f"samples/64 x (H x {OSC_SLOTS_PER_SINE} + {fir_macs:g}): per (sample, "
                                          "harmonic) 6 VALU + v_sin_f32 (4 slots), per sample the causal noise "
                                          "FIR's multiply-adds (bench.fir_macs_per_frame)",
                "frac_algorithmic_r03_convention": round(alg_slots_r03 / (osc_ms * 1e-3) / VALU_PEAK_SLOTS, 4),
                "valu_counts_kernel_sha": vc.get("kernel_sha"), "kernel_sha": src_sha,
                "traffic": traffic.get("synth_frame_kernel"),
                "kernel": "synth_frame_kernel (oscillator bank + filtered noise + their controls, fused)",
                "avg_launch_ms": round(osc_ms, 4), "slots_per_launch": round(slots),
                "slots_source": slots_src,
                "oscillator_frac": round(osc_slots / (osc_ms * 1e-3) / VALU_PEAK_SLOTS, 4),
                "sines_per_s": round(n_sin / (osc_ms * 1e-3), 1),
                "peak_note": "256 CU x 4 SIMD x 2.4 GHz / 2 cycles per wave64 fp32 VALU op (issue rate "
                             "at >=2 waves/SIMD measured by tools/issue_probe.hip, profiles/"
                             "r02_issue_probe.log; v_sin_f32 issues every 8 cycles)"}
    # SURVEY 8(d)'s effective-bandwidth convention (op-boundary bytes 4*(H+2) B/sample credited to
    # the fused kernel): NOT a roofline fraction - the fused kernel never moves these bytes
    op_boundary_effective = {"gbs": round(osc_bytes / (osc_ms * 1e-3) / 1e9, 1),
                             "algorithmic_bytes_per_launch": osc_bytes,
                             "note": "SURVEY 8(d) convention: op-boundary bytes / fused-kernel time; "
                                     "exceeds HBM peak because fusion removed that traffic"}

    # the reverb group (forward transform + IR-cache check, MAC, inverse) against HBM: SURVEY 8(d)'s 8 B per
    # sample (x in, y out) over the group's event-timed duration, beside its PMC bytes (the two spectra round
    # trips of the partitioned convolution, DESIGN.md 3a, make the physical traffic ~5x the algorithmic bytes)
    roofline_reverb = None
    if syn.reverb is not None and kern_ms.get("reverb"):
        rev_s = kern_ms["reverb"] * 1e-3
        rev_bytes = 8 * B * F * bs
        rt = traffic.get("reverb")
        roofline_reverb = {"bound": "hbm", "achieved": round(rev_bytes / rev_s / 1e9, 1), "peak": 8000.0,
                           "unit": "GB/s", "frac": round(rev_bytes / rev_s / 8e12, 4), "traffic": rt,
                           "physical_gbs": round(rt / rev_s / 1e9, 1) if rt else None,
                           "algorithmic_bytes_per_launch": rev_bytes, "avg_group_ms": round(kern_ms["reverb"], 4),
                           "kernels": "upols_forward_ir_kernel + upols_mac_stream_kernel + upols_inverse_kernel",
                           "note": "8 B/sample (x in, y out; the cached IR spectrum aside) over the group's "
                                   "event-timed duration (kernel_ms.reverb); traffic = PMC FETCH_SIZE + WRITE_SIZE "
                                   "per group (profiles/pmc_traffic.json)"}

    result = {
        "metric": "audio samples/sec (48 kHz, 100 harm, blk=512) at 1/2/4/8 GPU; % HBM roofline",
        "value": round(value, 1), "unit": "samples/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "warmup_steps_run": warm_steps, "warmup_s": round(warm_s, 3),
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
        "data": f"synthetic (SURVEY 8(d) seeded controls; noise {'on-device Philox' if args.noise == 'device' else 'injected'})",
        "config": {"workload": f"config {args.config} synth path: batch {B}/GPU, frames {F}, block_size {bs}, "
                               f"n_harmonic {H}, n_bands {NB}, sr {sr}, reverb {args.reverb_length} taps",
                   "global_batch": B * world, "seq_len": F * bs, "parallelism": f"batch-shard x{world}"},
        "roofline": roofline,
        "op_boundary_effective": op_boundary_effective,
        "roofline_reverb": roofline_reverb,
        "kernel_ms": {k: round(v, 4) for k, v in kern_ms.items()},
        "kernel_ms_note": "HIP events, one kernel group per loop, measured after the timed region; "
                          "roofline.avg_launch_ms is from inside it.  The synthesis kernel's time depends "
                          "on what ran before it (the shader clock it gets after the reverb's MAC, "
                          "DESIGN.md 3c)",
    }

    if syn.reverb is not None and not args.no_uncached_leg:
        # the reference rebuilds the impulse and its transform on every Reverb.forward
        # (modules.py:30-33); the module caches the spectrum between calls.  Same step with the
        # cache off: build_impulse + partition spectra + the rest, every call.
        # timed at steady state over at least 200 steps (20 steps of a 0.2 ms step are a 4 ms window in
        # which one host hiccup moves the mean by several per cent)
        syn.reverb.cache_spectrum = False
        n_unc = max(args.steps, 200)
        for _ in range(5):
            step()
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        tu = time.perf_counter()
        for _ in range(n_unc):
            step()
        torch.cuda.synchronize()
        tu = time.perf_counter() - tu
        syn.reverb.cache_spectrum = True
        syn.reverb.invalidate()
        if dist:
            tt = torch.tensor([tu], device=dev, dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            tu = float(tt.item())
        result["uncached_ir"] = {"value": round(samples_per_step * n_unc / tu, 1), "unit": "samples/s",
                                 "ms_per_step": round(tu / n_unc * 1e3, 4), "steps_timed": n_unc,
                                 "note": "step with the reverb IR and its partition spectra rebuilt every call "
                                         "(Reverb.cache_spectrum = False), as the reference's Reverb.forward does"}

    if syn.reverb is not None and world == 1 and not args.no_pipelined_leg:
        try:
            result["pipelined"] = pipelined_leg(
                syn, (inp["f0"], inp["param"], inp["mags"], inp.get("noise")), samples_per_step,
                args.steps, args.reverb_cus, dev, dist)
        except Exception as e:  # a refused CU mask must not cost the headline line
            result["pipelined"] = {"error": f"{type(e).__name__}: {e}"}

    if dist and not args.no_gather:
        r, g = gathered_leg(step, B * world, samples_per_step, args.steps, dev, dist)
        if args.noise == "inject":  # deterministic: rank 0's shard of the gathered batch vs its own step
            if rank == 0:
                ref = step()
                r["check_vs_local_step"] = {"equal": bool(torch.equal(g[:B], ref)),
                                            "max_abs_diff": float((g[:B] - ref).abs().max())}
        result["gathered"] = r
        del g
        # root-held batch: controls scattered from rank 0 in chunks, audio gathered back,
        # scatter(i+1) || synth(i) || gather(i-1) (shard.synthesize_pipelined); IR broadcast once
        keys = ["f0", "param", "mags"] + (["noise"] if args.noise == "inject" else [])
        tails = [tuple(inp[k].shape[1:]) for k in keys]
        held = None
        if rank == 0:
            full = make_inputs(B * world, F, H, NB, bs, seed=0, device=dev,
                               with_noise=(args.noise == "inject"))
            held = [full[k] for k in keys]
        r, g = scatter_gather_leg(syn, held, B * world, tails, samples_per_step, args.steps, args.chunks,
                                  dev, dist, reverb=syn.reverb)
        if args.noise == "inject" and rank == 0:  # the gathered batch vs one process synthesising it all
            with torch.no_grad():
                ref = syn(*held)
            r["check_vs_one_process_step"] = {"equal": bool(torch.equal(g, ref)),
                                              "max_abs_diff": float((g - ref).abs().max())}
        result["scatter_gather"] = r
        del g, held
        # the three N>1 rates side by side: left sharded (value), gathered on rank 0, and
        # root-held controls scattered + audio gathered
        result["value_gathered"] = result["gathered"]["value"]
        result["value_scatter_gather"] = result["scatter_gather"]["value"]

    if rank == 0 and not args.no_op_leg:
        # op-boundary oscillator (core.py:136): per-sample inputs materialised in HBM
        with torch.no_grad():
            f0s = core.upsample(inp["f0"], bs)
            amps = core.upsample(torch.rand(B, F, H, device=dev) / H, bs)
            for _ in range(3):
                core.harmonic_synth(f0s, amps, sr)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 10
            e0.record()
            for _ in range(reps):
                core.harmonic_synth(f0s, amps, sr)
            e1.record()
            torch.cuda.synchronize()
            op_ms = e0.elapsed_time(e1) / reps
            del f0s, amps
        op_gbs = osc_bytes / (op_ms * 1e-3) / 1e9
        result["roofline_op"] = {"bound": "hbm", "achieved": round(op_gbs, 1), "peak": HBM_PEAK_GBS,
                                 "unit": "GB/s", "frac": round(op_gbs / HBM_PEAK_GBS, 4),
                                 "traffic": traffic.get("harmonic_samples_kernel"),
                                 "kernel": "phase_chunk_sums_kernel + harmonic_samples_tiled_kernel",
                                 "avg_launch_ms": round(op_ms, 4)}

    if rank == 0 and not args.no_train_leg:
        result["train_step"] = train_leg(args, inp, dev)

    if rank == 0 and not args.no_loss_leg:
        result["spectral_loss"] = loss_leg(args, dev)

    if rank == 0 and not args.no_decoder_leg:
        result["decoder_forward"] = decoder_leg(args, inp, dev)
        result["decoder_synthesis"] = decoder_synthesis_leg(args, inp, dev)

    if rank == 0 and not args.no_realtime_leg:
        result["realtime"] = realtime_leg(dev, args.realtime_calls)

    if rank == 0 and not args.no_model_train_leg:
        result["model_train_step"] = model_train_leg(args, inp, dev)

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args)
    elif rank == 0:
        result["cpu_baseline"] = None

    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
