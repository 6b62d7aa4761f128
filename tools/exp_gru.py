"""Development experiment: the GRU recurrence at the decoder's config-2 shape (B=64, T=200, H=512)."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddsp_pytorch_amd import core

torch.manual_seed(0)
B, T, I, H = 64, 200, 1024, 512
g = torch.nn.GRU(I, H, batch_first=True).cuda()
x = torch.randn(B, T, I, device="cuda")


def t(fn, reps=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t0) / reps * 1e3, 4)


with torch.no_grad():
    print(json.dumps({"native_ms": t(lambda: core.gru(x, g)), "miopen_ms": t(lambda: g(x)),
                      "input_gemm_ms": t(lambda: torch.addmm(g.bias_ih_l0, x.reshape(B * T, I), g.weight_ih_l0.t()))}))
