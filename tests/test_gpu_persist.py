"""The persistent, wave-specialised form of the fused synthesis kernel (synth_frame.hip,
synth_persist_kernel: launches of >= 2 x CUs x 8 frames) against the one-workgroup-per-frame form
(ddsp_hip_set_persistent_workgroups(0)) and the CPU oracle: same arithmetic per sample, so the two
agree to the last bits (the controls' normalisation sum and the noise filter's centre tap are summed
in another order; tolerance 2e-7 relative), device noise included; control dicts, parts, the
graph-replayed counter, ragged frame ranges (frames not a multiple of the workgroups)."""
import numpy as np
import pytest
import torch

from conftest import rms
from oracle import torch_ref as tr
from ddsp_pytorch_amd.synth import make_inputs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dd():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import ddsp_pytorch_amd
    ddsp_pytorch_amd._lib.load()
    yield ddsp_pytorch_amd
    ddsp_pytorch_amd.core.set_persistent_workgroups(-1)


def _both(dd, fn):
    """fn() with the persistent kernel (6 workgroups per CU) and with one workgroup per frame."""
    prev = dd.core.set_persistent_workgroups(6)
    try:
        a = fn()
        dd.core.set_persistent_workgroups(0)
        b = fn()
    finally:
        dd.core.set_persistent_workgroups(prev)
    return a, b


def _close(a, b, rel=2e-7):
    a, b = a.double(), b.double()
    assert float((a - b).abs().max()) <= rel * max(1.0, float(b.abs().max())), float((a - b).abs().max())


@pytest.mark.parametrize("B,F,H,NB,bs", [(64, 200, 100, 65, 512), (23, 211, 37, 33, 256), (9, 480, 128, 65, 512),
                                         (40, 128, 64, 17, 1024)])
def test_persistent_matches_per_frame(dd, B, F, H, NB, bs):
    inp = make_inputs(B, F, H, NB, bs, seed=B + F, device="cuda")
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    assert B * F >= 2 * cus * 6 or bs == 1024, "shape must take the persistent kernel"

    def run():
        with torch.no_grad():
            dd.core.set_noise_seed(11)
            inj = dd.core.synth_frames(inp["f0"], inp["param"], inp["mags"], bs, 48000, noise=inp["noise"],
                                       parts=True, controls=True)
            dev = dd.core.synth_frames(inp["f0"], inp["param"], inp["mags"], bs, 48000)
        return inj, dev

    (inj_p, dev_p), (inj_f, dev_f) = _both(dd, run)
    for a, b in zip(inj_p[:3], inj_f[:3]):
        _close(a, b)
    for k in ("amplitudes", "harmonic_distribution", "magnitudes"):
        _close(inj_p[3][k], inj_f[3][k])
    _close(dev_p, dev_f)
    # and against the reference's op sequence on the CPU, for two items
    ref = tr.synth_path(inp["f0"][:2].cpu(), inp["param"][:2].cpu(), inp["mags"][:2].cpu(),
                        inp["noise"][:2].cpu(), None, bs, 48000)
    assert rms(inj_p[0][:2].cpu().numpy(), ref.numpy()) < 1e-6


def test_persistent_counter_replay(dd):
    """The device-counter entry point (graph replay) on the persistent kernel: call k draws offset k."""
    dd.core.set_persistent_workgroups(6)
    B, F, H, NB, bs = 24, 200, 40, 65, 512
    inp = make_inputs(B, F, H, NB, bs, seed=3, device="cuda", with_noise=False)
    counter = torch.zeros(1, dtype=torch.int64, device="cuda")
    with torch.no_grad():
        c0 = dd.core.synth_frames_counter(inp["f0"], inp["param"], inp["mags"], bs, 48000, counter, 99)
        c1 = dd.core.synth_frames_counter(inp["f0"], inp["param"], inp["mags"], bs, 48000, counter, 99)
        dd.core.set_noise_seed(99)
        e0 = dd.core.synth_frames(inp["f0"], inp["param"], inp["mags"], bs, 48000)
        e1 = dd.core.synth_frames(inp["f0"], inp["param"], inp["mags"], bs, 48000)
    assert torch.equal(c0, e0) and torch.equal(c1, e1) and int(counter.item()) == 2


def test_persistent_workgroup_setting_roundtrip(dd):
    prev = dd.core.set_persistent_workgroups(5)
    try:
        assert dd.core.set_persistent_workgroups(3) == 5
        B, F, H, NB, bs = 16, 100, 20, 17, 128  # 1600 frames: persistent at 3 per CU on 256 CUs
        inp = make_inputs(B, F, H, NB, bs, seed=8, device="cuda")
        with torch.no_grad():
            a = dd.core.synth_frames(inp["f0"], inp["param"], inp["mags"], bs, 48000, noise=inp["noise"])
            dd.core.set_persistent_workgroups(0)
            b = dd.core.synth_frames(inp["f0"], inp["param"], inp["mags"], bs, 48000, noise=inp["noise"])
        _close(a, b)
    finally:
        dd.core.set_persistent_workgroups(prev)
