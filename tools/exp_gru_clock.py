"""Development experiment: per-step phase times of the persistent GRU recurrence (workgroup 0), from the
gruclk probe build (tools/probe_build.py gruclk -> build/ab_gruclk.so, loaded through DDSP_HIP_LIB)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddsp_pytorch_amd import _lib  # noqa: E402

torch.manual_seed(0)
B, T, H = int(sys.argv[1]) if len(sys.argv) > 1 else 64, 200, 512
w_hh = torch.randn(3 * H, H, device="cuda") * 0.04
b_hh = torch.randn(3 * H, device="cuda") * 0.1
xp = torch.randn(B, T, 3 * H, device="cuda")
out = torch.empty(B, T, H, device="cuda")
ws = torch.zeros(_lib.query("gru_persistent_workspace_size"), dtype=torch.uint8, device="cuda")
for _ in range(3):
    _lib.call("gru_forward_persistent", _lib.ptr(xp), _lib.ptr(w_hh), _lib.ptr(b_hh), None, _lib.ptr(out), None, None,
              B, T, H, 0, _lib.ptr(ws), ws.numel(), _lib.stream_of(out))
torch.cuda.synchronize()
st = ws.view(torch.int32)[17 * 32 + 64:17 * 32 + 64 + 8 * T].view(T, 8)[:, :6].cpu().long()
st = (st - st[0, 0]) * 10  # ns
d = st[1:, :] - st[:-1, :]
ph = {"step_ns": float(d[10:, 0].float().median()), "wait_poll_ns": float((st[10:, 1] - st[10:, 0]).float().median()),
      "load_compute_ns": float((st[10:, 2] - st[10:, 1]).float().median()),
      "stage_ns": float((st[10:, 5] - st[10:, 1]).float().median()),
      "compute_ns": float((st[10:, 2] - st[10:, 5]).float().median()),
      "gates_store_ns": float((st[10:, 3] - st[10:, 2]).float().median()),
      "publish_ns": float((st[10:, 4] - st[10:, 3]).float().median()),
      "total_us": float(st[-1, 4]) / 1e3}
print(json.dumps(ph), flush=True)
