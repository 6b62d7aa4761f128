"""Development experiment: time the fused synthesis backward (harmonic + noise VJP) at config 2."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddsp_pytorch_amd import core, grad
from ddsp_pytorch_amd.synth import make_inputs

B, F, H, NB, bs, sr = 64, 200, 100, 65, 512, 48000
inp = make_inputs(B, F, H, NB, bs, device="cuda", with_noise=False)
g = torch.randn(B, F * bs, 1, device="cuda")
param = inp["param"].requires_grad_(True)
mags = inp["mags"].requires_grad_(True)
mode = sys.argv[1] if len(sys.argv) > 1 else "fused"
if mode == "fused":
    out = core.synth_frames(inp["f0"], param, mags, bs, sr)
elif mode == "harm":
    out = core.harmonic_synth_params(inp["f0"], param, bs, sr)
else:
    out = core.filtered_noise(mags, bs, raw_bias=-5.0)
def bwd():
    out.backward(g, retain_graph=True)
import time
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.5:  # clocks / power state settle
    bwd()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(50):
    bwd()
e1.record()
torch.cuda.synchronize()
print(json.dumps({"mode": mode, "threads": os.environ.get("DDSP_HIP_BWD_THREADS", "default"), "ms": round(e0.elapsed_time(e1) / 50, 4)}))
