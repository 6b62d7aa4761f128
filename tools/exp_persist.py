"""Phase timing of the persistent synthesis kernel (development experiment; library built with
-DDDSP_PROBE_CLOCK, loaded through DDSP_HIP_LIB): per frame the preparation wave's phases (loads +
controls + noise, filter taps, windowed filter, noise tail) and the synthesis waves' frame time and
barrier wait, in us (100 MHz ticks)."""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddsp_pytorch_amd import core  # noqa: E402
from ddsp_pytorch_amd.synth import make_inputs  # noqa: E402


def main():
    B, F, H, NB, bs = 64, 200, 100, 65, 512
    inp = make_inputs(B, F, H, NB, bs, device="cuda", with_noise=False)
    for wpc in (4, 5, 6):
        core.set_persistent_workgroups(wpc)
        run = lambda: core.synth_frames(inp["f0"], inp["param"], inp["mags"], bs, 48000, controls=True)
        t = time.perf_counter()
        while time.perf_counter() - t < 0.3:
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            out, c = run()
        e1.record()
        torch.cuda.synchronize()
        v = c["amplitudes"].untyped_storage()
        raw = torch.empty(0, device="cuda").set_(v).view(-1)[:8 * B * F].view(B * F, 8).double().cpu() / 100.0
        names = ["prep: loads+controls+noise", "prep: irfft taps", "prep: windowed taps", "prep: noise tail",
                 "synth: frame", "synth: barrier wait"]
        print(f"wpc={wpc}: kernel {e0.elapsed_time(e1) / 10 * 1e3:.1f} us; " +
              ", ".join(f"{n} {statistics.mean(raw[:, i].tolist()):.2f}" for i, n in enumerate(names)), flush=True)
        G = torch.cuda.get_device_properties(0).multi_processor_count * wpc
        firsts = torch.nonzero(raw[:, 7] > 0).flatten()  # each workgroup's first frame holds its record
        st = raw[firsts, 6]
        st = st - st.min()
        en = st + raw[firsts, 7]
        bins = torch.arange(0, float(en.max()) + 1, 2.0, dtype=torch.float64)
        occ = ((st[None, :] <= bins[:, None]) & (en[None, :] > bins[:, None])).sum(1)
        print(f"   workgroups {G}: start spread {float(st.max()):.1f} us, life mean {float(raw[firsts, 7].mean()):.1f} "
              f"us, span {float(en.max()):.1f} us; resident per 10 us: "
              + " ".join(str(int(occ[i:i + 5].double().mean())) for i in range(0, len(occ), 5)), flush=True)


if __name__ == "__main__":
    main()
