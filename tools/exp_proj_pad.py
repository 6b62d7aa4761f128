"""Projection GEMM (config 2 rows: 12800 x 512 -> n outputs) on hipBLASLt through torch: F.linear (NT) at several
padded output counts, and the NN (weight stored K x n) and transposed-output forms at n = 192."""
import torch

dev = torch.device("cuda", 0)
torch.manual_seed(0)
x = torch.randn(12800, 512, device=dev)


def timed(fn):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = []
    for _ in range(3):
        e0.record()
        for _ in range(100):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best.append(e0.elapsed_time(e1) / 100 * 1e3)
    return round(min(best), 2)


res = {}
for n in (166, 168, 176, 192, 208, 224, 256):
    w = torch.randn(n, 512, device=dev)
    b = torch.randn(n, device=dev)
    res[f"linear_{n}"] = timed(lambda: torch.nn.functional.linear(x, w, b))
w = torch.randn(192, 512, device=dev)
b = torch.randn(192, device=dev)
wt = w.t().contiguous()
res["addmm_nn_192"] = timed(lambda: torch.addmm(b, x, wt))
res["mm_outT_192"] = timed(lambda: torch.mm(w, x.t()))
xt = x.t().contiguous()
res["mm_outT_xT_192"] = timed(lambda: torch.mm(w, xt))
print(res)
