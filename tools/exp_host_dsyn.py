"""Development experiment: host (CPU) cost per call of the pieces of decoder_synthesize at config 2 —
each piece called after a device synchronize, so the time is the Python + launch work alone, not
queueing behind the GPU — against the same pieces' device time (HIP events)."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddsp_pytorch_amd import core
from ddsp_pytorch_amd.decoder import DDSPDecoder, decoder_projections, decoder_synthesize

dev = "cuda"
B, F, bs, sr = 64, 200, 512, 48000
torch.manual_seed(0)
m = DDSPDecoder(512, 100, 65, sr, bs, True).to(dev).eval()
m.noise_synth.noise_mode = "device"
f0 = 50.0 * 20.0 ** torch.rand(B, F, 1, device=dev)
hidden = torch.randn(B, F, 512, device=dev)


def host(fn, reps=100):
    for _ in range(10):
        fn()
    tot = 0.0
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        tot += time.perf_counter() - t0
    torch.cuda.synchronize()
    return round(tot / reps * 1e6, 1)


def dev_us(fn, reps=50):
    for _ in range(10):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) / reps * 1e3, 1)


with torch.no_grad():
    param, mags = decoder_projections(m, hidden)
    sig = core.synth_frames(f0, param, mags, bs, sr, parts=True, controls=True)[0]
    pieces = {
        "decoder_synthesize": lambda: decoder_synthesize(m, hidden, f0),
        "projections": lambda: decoder_projections(m, hidden),
        "synth_frames_parts_controls": lambda: core.synth_frames(f0, param, mags, bs, sr, parts=True, controls=True),
        "synth_frames_plain": lambda: core.synth_frames(f0, param, mags, bs, sr),
        "reverb_forward": lambda: m.reverb(sig),
        "empty_kernel_torch": lambda: torch.empty(1, device=dev).zero_(),
    }
    res = {k: {"host_us": host(fn), "device_us": dev_us(fn)} for k, fn in pieces.items()}
print(json.dumps(res), flush=True)
