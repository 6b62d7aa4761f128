"""The reverb at config-2 rows for batch B (one UPOLS MAC wave per 64 bins of a pair): run under
rocprofv3 once per B to read how the streaming MAC's time scales with its waves per SIMD.

    python tools/exp_mac_scaling.py B [reps]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddsp_pytorch_amd.synth import SynthPath  # noqa: E402

B = int(sys.argv[1])
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
dev = torch.device("cuda", 0)
syn = SynthPath(512, 48000, reverb_length=48000).to(dev)
x = torch.randn(B, 200 * 512, 1, device=dev)
with torch.no_grad():
    for _ in range(reps):
        syn.reverb(x)
torch.cuda.synchronize()
