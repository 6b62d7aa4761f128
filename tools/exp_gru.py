"""Development experiment: the GRU at the decoder's config-2 shape (B=64, T=200, I=1024, H=512):
the whole layer on ddsp_hip_gru_layer_forward (each step's input projection inside its launch,
when the loaded library has it: round 4's r04n build), the split route (one hipBLASLt GEMM for the projection +
ddsp_hip_gru_forward's step kernels), the GEMM alone, and MIOpen's nn.GRU.  Runs against any
library revision loaded through DDSP_HIP_LIB (tools/ab_time.sh)."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddsp_pytorch_amd import _lib, core

torch.manual_seed(0)
B, T, I, H = 64, 200, 1024, 512
g = torch.nn.GRU(I, H, batch_first=True).cuda()
x = torch.randn(B, T, I, device="cuda")
lib = _lib.load()


def t(fn, reps=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t0) / reps * 1e3, 4)


out = torch.empty(B, T, H, device="cuda")
w_ih, w_hh, b_ih, b_hh = g.weight_ih_l0, g.weight_hh_l0, g.bias_ih_l0, g.bias_hh_l0


def split():
    xp = torch.addmm(b_ih, x.reshape(B * T, I), w_ih.t())
    _lib.call("gru_forward", _lib.ptr(xp), _lib.ptr(w_hh), _lib.ptr(b_hh), None, _lib.ptr(out), None, None, B, T, H,
              _lib.stream_of(out))


def layer():
    _lib.call("gru_layer_forward", _lib.ptr(x), _lib.ptr(w_ih), _lib.ptr(b_ih), _lib.ptr(w_hh), _lib.ptr(b_hh), None,
              _lib.ptr(out), None, None, B, T, I, H, _lib.stream_of(out))


with torch.no_grad():
    res = {"split_ms": t(split)}
    if hasattr(lib, "ddsp_hip_gru_layer_forward"):
        res["layer_ms"] = t(layer)
    res["input_gemm_ms"] = t(lambda: torch.addmm(b_ih, x.reshape(B * T, I), w_ih.t()))
    res["miopen_ms"] = t(lambda: g(x))
print(json.dumps(res), flush=True)
