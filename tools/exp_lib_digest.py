"""Digest of the reverb's output at config 2 (seeded input) for the library DDSP_HIP_LIB points at: same-box
bit-identity check of a kernel variant against the shipped library (tools/ab_build.sh / tools/ab_src.sh builds).

    DDSP_HIP_LIB=build/ab_<name>.so python tools/exp_lib_digest.py [B]
"""
import hashlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddsp_pytorch_amd.synth import SynthPath  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
dev = torch.device("cuda", 0)
torch.manual_seed(0)
syn = SynthPath(512, 48000, reverb_length=48000).to(dev)
x = torch.randn(B, 200 * 512, 1, device=dev)
with torch.no_grad():
    y = syn.reverb(x)
    y2 = syn.reverb(x * 0.5)  # a second call on the cached IR spectrum
torch.cuda.synchronize()
h = hashlib.sha256(y.cpu().numpy().tobytes() + y2.cpu().numpy().tobytes()).hexdigest()[:16]
print(json.dumps({"lib": os.environ.get("DDSP_HIP_LIB", "in-tree"), "B": B, "digest": h,
                  "rms": float(y.pow(2).mean().sqrt()), "finite": bool(torch.isfinite(y).all())}))
