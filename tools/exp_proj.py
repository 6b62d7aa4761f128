"""Development experiment: the decoder's stacked projections (hidden [12800, 512] -> 166 outputs) on
hipBLASLt for padded output widths and both weight layouts (device time, HIP events)."""
import json, torch
dev = "cuda"
h = torch.randn(64 * 200, 512, device=dev)


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


res = {}
with torch.no_grad():
    for n in (166, 168, 176, 192, 224, 256):
        w = torch.randn(n, 512, device=dev)
        bvec = torch.randn(n, device=dev)
        wt = w.t().contiguous()
        res[n] = {"linear": dev_us(lambda: torch.nn.functional.linear(h, w, bvec)),
                  "addmm_wT_contig": dev_us(lambda: torch.addmm(bvec, h, wt)),
                  "mm_no_bias": dev_us(lambda: h @ w.t())}
print(json.dumps(res), flush=True)
