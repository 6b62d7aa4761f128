"""Is the fused synthesis kernel's slowdown after the reverb tied to where its output lands (the
caching allocator hands it a different block once the reverb's buffers come and go)?  Launches
through the C-ABI into fixed output buffers.  (development experiment)

    python tools/exp_addr.py
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddsp_pytorch_amd import _lib, core  # noqa: E402
from ddsp_pytorch_amd.synth import SynthPath, make_inputs  # noqa: E402


def main():
    B, F, H, NB, bs, sr = 64, 200, 100, 65, 512, 48000
    inp = make_inputs(B, F, H, NB, bs, device="cuda", with_noise=False)
    syn = SynthPath(bs, sr, reverb_length=48000).to("cuda")
    f0, param, mags = inp["f0"].contiguous(), inp["param"].contiguous(), inp["mags"].contiguous()
    sig = core.synth_frames(f0, param, mags, bs, sr)
    spec = syn.reverb._spectrum(F * bs)
    ptrs = set()

    def synth_into(out):
        _lib.call("synth_frames_controls", _lib.ptr(f0), _lib.ptr(param), H + 1, _lib.ptr(mags), NB, -5.0,
                  _lib.ptr(None), 0, 0, _lib.ptr(out), _lib.ptr(None), _lib.ptr(None), _lib.ptr(None), B, F, H, NB, bs, float(sr), _lib.stream_of(out))

    def synth_alloc():
        o = core.synth_frames(f0, param, mags, bs, sr)
        ptrs.add(o.data_ptr())
        return o

    fixed = torch.empty_like(sig)
    yfix = [None]
    E = lambda: torch.cuda.Event(enable_timing=True)

    def per_launch(fn, between, n=120):
        for _ in range(20):
            fn(); between()
        ps = []
        for _ in range(n):
            e0, e1 = E(), E()
            e0.record()
            fn()
            e1.record()
            between()
            ps.append((e0, e1))
        torch.cuda.synchronize()
        return statistics.median(a.elapsed_time(b) * 1e3 for a, b in ps)

    rv = lambda: core.reverb_apply(sig, spec, 48000)
    def rv_keep():
        yfix[0] = core.reverb_apply(sig, spec, 48000)
    cases = [
        ("alloc, back to back", synth_alloc, lambda: None),
        ("fixed out, back to back", lambda: synth_into(fixed), lambda: None),
        ("alloc, reverb between", synth_alloc, rv),
        ("fixed out, reverb between", lambda: synth_into(fixed), rv),
        ("fixed out, reverb kept alive", lambda: synth_into(fixed), rv_keep),
        ("into sig (reverb reads it)", lambda: synth_into(sig), rv),
    ]
    for name, fn, between in cases:
        ptrs.clear()
        t = per_launch(fn, between)
        print(f"{name:32s}: synth {t:7.1f} us   output blocks used {len(ptrs)}", flush=True)


if __name__ == "__main__":
    main()
