"""Guard of the oscillator loops' code placement: the fused synthesis kernel ran
~10 % faster on MI355X (135-137 vs 148-149 us at config 2) when the 8-byte instructions of its
sine loop sit at odd dword addresses (address % 8 == 4).  Any edit to synth_frame.hip, common.h,
noise_dsp.h or backward.hip, or a compiler update, can move the loop; this test reads the built
library's ISA (llvm-objdump, no GPU) and fails when a throughput kernel lost the fast placement.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
LIB = os.path.join(ROOT, "ddsp_pytorch_amd", "lib", "libddsp_hip.so")

# the throughput instantiations (one wave owns 4 samples x all harmonics): device-noise and
# injected-noise forward, the harmonic half of the synthesis backward (the training step's
# kernel since the backward runs as two launches) and the frame-control harmonic backward.  The
# one-sample-per-thread SPLIT forms run only for launches of few frames (the realtime stream),
# which are latency-bound: reported, not pinned.
PINNED = ("synth_frame_kernelILb1ELb0ELb0ELb0EE", "synth_frame_kernelILb0ELb0ELb0ELb0EE",
          "synth_frame_kernelILb1ELb0ELb1ELb0EE", "synth_frame_kernelILb0ELb0ELb1ELb0EE",
          "frame_backward_kernelILi2ELi0ELb0EE", "frame_backward_kernelILi1ELi0ELb0EE")


@pytest.mark.skipif(not os.path.exists(LIB), reason="libddsp_hip.so not built (make)")
@pytest.mark.skipif(not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump"),
                    reason="llvm-objdump not available")
@pytest.mark.parametrize("kernel", PINNED)
def test_sine_loop_at_fast_placement(kernel):
    import loop_align
    rs = loop_align.analyze_all(LIB, kernel)
    assert rs, f"no hardware-sine loop found in {kernel}"
    for r in rs:  # every copy of the loop the kernel carries
        assert r["sines"] >= 8
        frac = r["odd_dword"] / max(r["eight_byte"], 1)
        assert frac >= 0.9, (f"{kernel}: only {r['odd_dword']} of {r['eight_byte']} 8-byte loop instructions at odd "
                             f"dword addresses (loop @{r['start']:#x}); re-pad the loop (DESIGN.md §3)")
