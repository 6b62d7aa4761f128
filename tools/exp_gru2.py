"""Development experiment: the decoder's GRU recurrence at config 2 (B=64, T=200, I=1024, H=512) as one
persistent launch (ddsp_hip_gru_forward_persistent) vs the per-step launches (ddsp_hip_gru_forward), the
recurrence alone on a fixed input projection, device time by HIP events; plus core.gru end to end."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddsp_pytorch_amd import _lib, core  # noqa: E402

torch.manual_seed(0)
B, T, I, H = 64, 200, 1024, 512
g = torch.nn.GRU(I, H, batch_first=True).cuda()
x = torch.randn(B, T, I, device="cuda")
w_ih, w_hh, b_ih, b_hh = g.weight_ih_l0, g.weight_hh_l0, g.bias_ih_l0, g.bias_hh_l0
out = torch.empty(B, T, H, device="cuda")
ws = torch.empty(_lib.query("gru_persistent_workspace_size"), dtype=torch.uint8, device="cuda")


def dev_ms(fn, reps=20):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) / reps, 4)


with torch.no_grad():
    xp = torch.addmm(b_ih, x.reshape(B * T, I), w_ih.t()).view(B, T, 3 * H)
    st = lambda: _lib.stream_of(out)  # noqa: E731

    def steps():
        _lib.call("gru_forward", _lib.ptr(xp), _lib.ptr(w_hh), _lib.ptr(b_hh), None, _lib.ptr(out), None, None, B, T,
                  H, st())

    def persistent():
        _lib.call("gru_forward_persistent", _lib.ptr(xp), _lib.ptr(w_hh), _lib.ptr(b_hh), None, _lib.ptr(out), None,
                  None, B, T, H, 0, _lib.ptr(ws), ws.numel(), st())
    res = {"steps_ms": dev_ms(steps)}
    ref = out.clone()
    res["persistent_ms"] = dev_ms(persistent)
    res["max_diff_vs_steps"] = float((out - ref).abs().max())
    res["abort_word"] = int(ws.view(torch.int32)[17 * 32].item())
    res["census"] = ws.view(torch.int32)[8 * 32:17 * 32:32].tolist()
    res["core_gru_ms"] = dev_ms(lambda: core.gru(x, g))
    res["input_gemm_ms"] = dev_ms(lambda: torch.addmm(b_ih, x.reshape(B * T, I), w_ih.t()))
    for b in (1, 16):
        xb = xp[:b].contiguous()
        ob = torch.empty(b, T, H, device="cuda")
        res[f"persistent_B{b}_ms"] = dev_ms(lambda: _lib.call(
            "gru_forward_persistent", _lib.ptr(xb), _lib.ptr(w_hh), _lib.ptr(b_hh), None, _lib.ptr(ob), None, None,
            b, T, H, 0, _lib.ptr(ws), ws.numel(), st()))
print(json.dumps(res), flush=True)

# the BPTT (training): ddsp_hip_gru_backward_persistent vs the per-step backward launches, on saved gates
gates = torch.empty(4, B, T, H, device="cuda")
with torch.no_grad():
    _lib.call("gru_forward", _lib.ptr(xp), _lib.ptr(w_hh), _lib.ptr(b_hh), None, _lib.ptr(out), None, _lib.ptr(gates),
              B, T, H, _lib.stream_of(out))
gout = torch.randn(B, T, H, device="cuda")
dxp = torch.empty(B, T, 3 * H, device="cuda")
dgn = torch.empty(B, T, H, device="cuda")
wsb = torch.empty(_lib.query("gru_backward_workspace_size", B, H), dtype=torch.uint8, device="cuda")
bargs = lambda: (_lib.ptr(w_hh), _lib.ptr(gates), _lib.ptr(out), None, _lib.ptr(gout), None, _lib.ptr(dxp),  # noqa: E731
                 _lib.ptr(dgn), None, B, T, H)
res2 = {"bptt_steps_ms": dev_ms(lambda: _lib.call("gru_backward", *bargs(), _lib.ptr(wsb), wsb.numel(),
                                                    _lib.stream_of(out)))}
ref = dxp.clone()
res2["bptt_persistent_ms"] = dev_ms(lambda: _lib.call("gru_backward_persistent", *bargs(), 0, _lib.ptr(ws), ws.numel(),
                                                        _lib.stream_of(out)))
res2["bptt_rel_diff"] = float((dxp - ref).norm() / ref.norm())
print(json.dumps(res2), flush=True)
