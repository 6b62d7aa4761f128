"""mlp_block at config 2's shape (12,800 rows x 512 -> 512): the x-resident kernel (contiguous x) against the
staged kernel (x rows 514 floats apart), device time per launch by HIP events over back-to-back launches."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ddsp_pytorch_amd as dd  # noqa: E402

L = dd._lib
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 12800
torch.manual_seed(0)
lin = torch.nn.Linear(512, 512).cuda()
ln = torch.nn.LayerNorm(512).cuda()
wide = torch.randn(rows, 514, device="cuda")
x = wide[:, :512].contiguous()
y = torch.empty(rows, 512, device="cuda")


def run(buf, ld, flags):
    L.call("mlp_block", L.ptr(buf), ld, 512, L.ptr(lin.weight), 512, L.ptr(lin.bias), None, None, 1,
           L.ptr(ln.weight), L.ptr(ln.bias), 1e-5, 0.01, L.ptr(y), 512, rows, 512, flags, L.stream_of(y))


res = {}
for name, buf, ld, fl in (("bf16x3", x, 512, 0), ("resident", x, 512, 1), ("staged", wide, 514, 0),
                          ("bf16x3_2", x, 512, 0), ("resident2", x, 512, 1), ("staged2", wide, 514, 0)):
    for _ in range(20):
        run(buf, ld, fl)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        run(buf, ld, fl)
    e1.record()
    torch.cuda.synchronize()
    res[name + "_us"] = round(e0.elapsed_time(e1) / 50 * 1e3, 2)
flop = 2.0 * rows * 512 * 512
res["tflops_resident"] = round(flop / (res["resident_us"] * 1e-6) / 1e12, 1)
res["tflops_bf16x3"] = round(flop / (res["bf16x3_us"] * 1e-6) / 1e12, 1)
print(json.dumps(res))

# the GRU input projection: 12,800 x 1024 -> 1536 (decoder.py:41) on ddsp_hip_linear vs torch.addmm
xg = torch.randn(rows, 1024, device="cuda")
wg = torch.randn(1536, 1024, device="cuda") * 0.03
bg = torch.randn(1536, device="cuda")
res2 = {}
for name, fn in (("linear_bf16x3", lambda: dd.core.linear(xg, wg, bg)), ("addmm", lambda: torch.addmm(bg, xg, wg.t())),
                 ("linear_bf16x3_2", lambda: dd.core.linear(xg, wg, bg)), ("addmm_2", lambda: torch.addmm(bg, xg, wg.t()))):
    for _ in range(10):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        fn()
    e1.record()
    torch.cuda.synchronize()
    res2[name + "_us"] = round(e0.elapsed_time(e1) / 20 * 1e3, 2)
print(json.dumps(res2))
