"""Development experiment: the decoder's two projections (hidden [12800, 512] -> 101 + 65 outputs) as the
package's one-launch kernel (core.projections) vs hipBLASLt (F.linear on the stacked / padded weights),
device time by HIP events; and the kernel's error vs an fp64 host matmul."""
import json
import sys

import torch

sys.path.insert(0, ".")
from ddsp_pytorch_amd import core  # noqa: E402

dev = "cuda"


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
    return round(a.elapsed_time(b) / reps * 1e3, 2)


res = {}
torch.manual_seed(0)
with torch.no_grad():
    for H, rows in ((100, 12800), (64, 12800), (128, 25600)):
        h = torch.randn(rows, 512, device=dev)
        l1, l2 = torch.nn.Linear(512, H + 1).to(dev), torch.nn.Linear(512, 65).to(dev)
        w = torch.cat([l1.weight, l2.weight])
        b = torch.cat([l1.bias, l2.bias])
        n_pad = -(-w.shape[0] // 64) * 64
        wp = torch.zeros(n_pad, 512, device=dev)
        wp[:w.shape[0]] = w
        bp = torch.zeros(n_pad, device=dev)
        bp[:b.shape[0]] = b
        r = {"kernel": dev_us(lambda: core.projections(h, l1, l2)),
             "hipblaslt_stacked": dev_us(lambda: torch.nn.functional.linear(h, w, b)),
             "hipblaslt_padded": dev_us(lambda: torch.nn.functional.linear(h, wp, bp))}
        p, m = core.projections(h, l1, l2)
        ref = h.double() @ w.double().t() + b.double()
        got = torch.cat([p, m], -1).double()
        r["max_err"] = float((got - ref).abs().max())
        r["tflops"] = round(2 * rows * 512 * w.shape[0] / (r["kernel"] * 1e-6) / 1e12, 1)
        res[f"H{H}_rows{rows}"] = r
print(json.dumps(res), flush=True)
