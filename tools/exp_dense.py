"""Latency of ddsp_hip_dense_rows (realtime control network) in isolation: back-to-back launches
of one Linear at 4 rows, with and without the LayerNorm prologue, vs torch's Linear.
    python tools/exp_dense.py"""
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddsp_pytorch_amd import core  # noqa: E402


def t_us(fn, reps=100):
    """GPU time per call: `reps` calls captured in one HIP graph (no host launch cost)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (10 * reps) * 1e3


dev = torch.device("cuda", 0)
R = 4
nul = torch.zeros(1, dtype=torch.int64, device=dev)
with torch.no_grad():
    print(f"empty kernel (x += 1): {t_us(lambda: nul.add_(1)):6.2f} us", flush=True)
for K, N in ((512, 512), (1024, 1536), (512, 65)):
    lin, ln = nn.Linear(K, N).to(dev), nn.LayerNorm(K).to(dev)
    x = torch.randn(R, K, device=dev)
    y = torch.empty(R, N, device=dev)
    with torch.no_grad():
        a = t_us(lambda: core.dense_rows([([core.dense_input(x, norm=ln)], lin, y)], R, dev))
        b = t_us(lambda: core.dense_rows([([core.dense_input(x)], lin, y)], R, dev))
        c = t_us(lambda: lin(x))
        d = t_us(lambda: lin(nn.functional.leaky_relu(ln(x), 0.01)))
    print(f"K={K} N={N}: dense+LN {a:6.2f} us  dense raw {b:6.2f} us  torch linear {c:6.2f} us  torch LN+lrelu+linear {d:6.2f} us",
          flush=True)
