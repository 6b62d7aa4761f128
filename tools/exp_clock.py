"""SCLK seen by the fused synthesis kernel in different stream contexts (development experiment):
a one-wave probe kernel (tools/clock_probe.hip) measures the shader clock right after each kernel.

    python tools/exp_clock.py          (build first: hipcc -shared tools/clock_probe.hip -o build/clock_probe.so)
"""
import ctypes
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ddsp_pytorch_amd import core  # noqa: E402
from ddsp_pytorch_amd.synth import SynthPath, make_inputs  # noqa: E402


def main():
    lib = ctypes.CDLL(os.path.join(ROOT, "build", "clock_probe.so"))
    lib.clock_probe.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    B, F, H, NB, bs, sr = 64, 200, 100, 65, 512, 48000
    inp = make_inputs(B, F, H, NB, bs, device="cuda", with_noise=False)
    syn = SynthPath(bs, sr, reverb_length=48000).to("cuda")
    synth = lambda: core.synth_frames(inp["f0"], inp["param"], inp["mags"], bs, sr)
    sig = synth()
    spec = syn.reverb._spectrum(F * bs)
    reverb = lambda: core.reverb_apply(sig, spec, 48000)
    out = torch.zeros(4096, device="cuda")
    stream = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def probe(i):
        lib.clock_probe(4000, ctypes.c_void_p(out.data_ptr()), i, stream())

    def pattern(name, body, n=60):
        t = time.perf_counter()
        while time.perf_counter() - t < 0.3:
            body(None)
        torch.cuda.synchronize()
        out.zero_()
        for i in range(n):
            body(i)
        torch.cuda.synchronize()
        v = out[:n].cpu().tolist()
        print(f"{name:44s}: SCLK median {statistics.median(v):7.0f} MHz (min {min(v):.0f}, max {max(v):.0f})",
              flush=True)

    def p(i):
        if i is not None:
            probe(i)

    pattern("after synth, synth back-to-back", lambda i: (synth(), p(i)))
    pattern("after synth, step (reverb, synth)", lambda i: (reverb(), synth(), p(i)))
    pattern("after reverb, step (synth, reverb)", lambda i: (synth(), reverb(), p(i)))
    pattern("after reverb, reverb back-to-back", lambda i: (reverb(), p(i)))

    def idle(i):
        torch.cuda.synchronize()
        time.sleep(0.0005)
        p(i)
    pattern("after 0.5 ms idle", idle)



def in_kernel():
    """With the DDSP_PROBE_CLOCK library (tools/ab_build.sh clk synth_frame -DDDSP_PROBE_CLOCK, loaded
    through DDSP_HIP_LIB): each workgroup's shader clocks / 100 MHz ticks over its life, so the SCLK
    the fused kernel itself ran at, back to back and in the step's (reverb, synth) order."""
    B, F, H, NB, bs, sr = 64, 200, 100, 65, 512, 48000
    inp = make_inputs(B, F, H, NB, bs, device="cuda", with_noise=False)
    syn = SynthPath(bs, sr, reverb_length=48000).to("cuda")
    synth = lambda: core.synth_frames(inp["f0"], inp["param"], inp["mags"], bs, sr, parts=True)
    sig = synth()[0]
    spec = syn.reverb._spectrum(F * bs)
    reverb = lambda: core.reverb_apply(sig, spec, 48000)

    def run(name, body, n=20):
        t = time.perf_counter()
        while time.perf_counter() - t < 0.3:
            body()
        torch.cuda.synchronize()
        res, runs = [], []
        for _ in range(n):  # queued back to back; read after one synchronize
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            runs.append((e0, e1, body(e0, e1)))
        torch.cuda.synchronize()
        for e0, e1, h in runs:
            r = h[1].view(B * F, bs)[:, :6].double().cpu() / 100.0  # us (100 MHz ticks)
            start = r[:, 0] - r[:, 0].min()
            end = start + r[:, 3]
            span = float(end.max())
            # concurrency over the launch: resident workgroups in 1 us bins
            bins = torch.arange(0, span + 1, 1.0, dtype=torch.float64)
            occ = ((start[None, :] <= bins[:, None]) & (end[None, :] > bins[:, None])).sum(1).double()
            res.append({"kernel": e0.elapsed_time(e1) * 1e3, "span": span,
                        "clk": float(r[:, 5].sum() / r[:, 3].sum()) * 100.0, "clk_lo": float((r[:, 5] / r[:, 3]).quantile(0.05)) * 100.0, "clk_hi": float((r[:, 5] / r[:, 3]).quantile(0.95)) * 100.0,
                        "pro": float(r[:, 1].mean()), "osc": float((r[:, 2] - r[:, 1]).mean()),
                        "post": float((r[:, 4] - r[:, 2]).mean()), "store": float((r[:, 3] - r[:, 4]).mean()),
                        "occ_mean": float(occ.mean()), "occ": occ,
                        "first_end": float(end.min()), "last_start": float(start.max())})
        md = lambda k: statistics.median(x[k] for x in res)
        print(f"{name:30s}: kernel {md('kernel'):6.1f} us (workgroup span {md('span'):6.1f}), SCLK {md('clk'):6.0f} MHz (5-95 % of workgroups {md('clk_lo'):5.0f}-{md('clk_hi'):5.0f});"
              f" workgroup life: prologue {md('pro'):5.2f} + sine loop {md('osc'):5.2f} + FIR/tail {md('post'):4.2f}"
              f" + store {md('store'):4.2f} us; resident workgroups mean {md('occ_mean'):6.0f} of 4096; first"
              f" end {md('first_end'):5.1f} us, last start {md('last_start'):6.1f} us", flush=True)
        occ = res[len(res) // 2]["occ"]
        print("   resident per 10 us: " + " ".join(f"{int(occ[i:i + 10].mean())}" for i in range(0, len(occ), 10)),
              flush=True)

    def b2b(e0=None, e1=None):
        if e0 is not None:
            e0.record()
        h = synth()
        if e1 is not None:
            e1.record()
        return h

    def step(e0=None, e1=None):
        reverb()
        return b2b(e0, e1)

    run("synth back-to-back", b2b)
    run("step order (reverb, synth)", step)
    run("synth back-to-back", b2b)

    def idle(e0=None, e1=None):
        torch.cuda.synchronize()
        return b2b(e0, e1)
    run("after a host sync (idle)", idle)




def overlap():
    """Do two fused-kernel launches queued back to back on one stream overlap in time?  (probe
    library) Workgroup start/end timestamps of both launches on the 100 MHz clock."""
    B, F, H, NB, bs, sr = 64, 200, 100, 65, 512, 48000
    inp = make_inputs(B, F, H, NB, bs, device="cuda", with_noise=False)
    synth = lambda: core.synth_frames(inp["f0"], inp["param"], inp["mags"], bs, sr, parts=True)
    tiny = torch.zeros(16, device="cuda")
    for between in ("nothing", "tiny fill kernel"):
        for _ in range(50):
            synth()
        torch.cuda.synchronize()
        for rep in range(3):
            a = synth()
            if between != "nothing":
                tiny.fill_(1.0)
            b = synth()
            torch.cuda.synchronize()
            ra = a[1].view(B * F, bs)[:, :4].double().cpu()
            rb = b[1].view(B * F, bs)[:, :4].double().cpu()
            t0 = ra[:, 0].min()
            sa, ea = ra[:, 0] - t0, ra[:, 0] - t0 + ra[:, 3]
            sb, eb = rb[:, 0] - t0, rb[:, 0] - t0 + rb[:, 3]
            print(f"between: {between:16s} launch 1 {float(sa.min()) / 100:7.1f}..{float(ea.max()) / 100:7.1f} us, "
                  f"launch 2 {float(sb.min()) / 100:7.1f}..{float(eb.max()) / 100:7.1f} us; launch-2 workgroups started "
                  f"before launch 1 ended: {int((sb < ea.max()).sum())}", flush=True)


if __name__ == "__main__":
    if "--in-kernel" in sys.argv:
        in_kernel()
    elif "--overlap" in sys.argv:
        overlap()
    else:
        main()
