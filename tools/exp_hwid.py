"""Which SIMD does each wave of the persistent synthesis kernel land on?  (development experiment;
library built with -DDDSP_PROBE_HWID, loaded through DDSP_HIP_LIB)"""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddsp_pytorch_amd import core  # noqa: E402
from ddsp_pytorch_amd.synth import make_inputs  # noqa: E402


def main():
    B, F, H, NB, bs = 64, 200, 100, 65, 512
    inp = make_inputs(B, F, H, NB, bs, device="cuda", with_noise=False)
    for wpc in (5, 8):
        core.set_persistent_workgroups(wpc)
        out = core.synth_frames(inp["f0"], inp["param"], inp["mags"], bs, 48000, parts=True)
        torch.cuda.synchronize()
        n = torch.cuda.get_device_properties(0).multi_processor_count * wpc
        hw = out[1].view(-1)[:4 * n].view(torch.int32).view(n, 4)[:, :3].cpu()
        per_simd = collections.Counter()
        per_cu = collections.Counter()
        for g in range(n):
            for w in range(3):
                v = int(hw[g, w])
                simd, cu, sh, se = (v >> 4) & 3, (v >> 8) & 15, (v >> 12) & 1, (v >> 13) & 7
                key = (se, sh, cu)
                per_cu[key] += 1
                if w < 2:
                    per_simd[key + (simd,)] += 1
        synth_counts = collections.Counter(per_simd.values())
        print(f"wpc={wpc}: {len(per_cu)} CUs seen; waves per CU {collections.Counter(per_cu.values())}; "
              f"synthesis waves per SIMD (count of SIMDs): {sorted(synth_counts.items())}; SIMDs with synthesis "
              f"waves {len(per_simd)}", flush=True)
        print("   first workgroups' (wave0, wave1, wave2) SIMDs:",
              [tuple((int(hw[g, w]) >> 4) & 3 for w in range(3)) for g in range(12)], flush=True)


if __name__ == "__main__":
    main()
