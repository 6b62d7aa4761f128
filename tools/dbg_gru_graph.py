"""Development check: the persistent GRU recurrence captured in a HIP graph, replayed several times,
against eager calls; prints the sync words after each replay (census total 256 = the memset node ran)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddsp_pytorch_amd import _lib  # noqa: E402

torch.manual_seed(0)
B, T, H = 1, 4, 512
w_hh = torch.randn(3 * H, H, device="cuda") * 0.04
b_hh = torch.randn(3 * H, device="cuda") * 0.1
xp = torch.randn(B, T, 3 * H, device="cuda")
h0 = torch.randn(B, H, device="cuda") * 0.5
out = torch.empty(B, T, H, device="cuda")
hl = torch.empty(B, H, device="cuda")
ws = torch.zeros(_lib.query("gru_persistent_workspace_size"), dtype=torch.uint8, device="cuda")


def run():
    _lib.call("gru_forward_persistent", _lib.ptr(xp), _lib.ptr(w_hh), _lib.ptr(b_hh), _lib.ptr(h0), _lib.ptr(out),
              _lib.ptr(hl), None, B, T, H, 0, _lib.ptr(ws), ws.numel(), _lib.stream_of(out))


def words():
    w = ws.view(torch.int32)
    return [int(w[g * 32]) for g in range(8)], int(w[16 * 32]), int(w[17 * 32])


s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    run()
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
ref = out.clone()
print("eager", words(), flush=True)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    run()
torch.cuda.synchronize()
for k in range(3):
    out.zero_()
    g.replay()
    torch.cuda.synchronize()
    print("replay", k, float((out - ref).abs().max()), words(), flush=True)
