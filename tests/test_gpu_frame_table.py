"""The two-launch form of the fused synthesis (synth_frame.hip: frame_table_kernel writes every frame's
controls, filter taps and phase prefix, synth_tab_kernel synthesises from them; opt-in, measured slower:
DESIGN §3c) against the one-launch form (ddsp_hip_set_frame_table(0), synth_frame_kernel): the
table holds the values frame_synth computes, by the same arithmetic and summation order, so every
output is BIT-identical — signal, parts, control dicts, device and injected noise, the graph counter,
strided projections (the decoder route), odd band counts, H > 128, block sizes 256..1024 — and
against the reference's op sequence on the CPU (oracle/torch_ref.py)."""
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
    prev = ddsp_pytorch_amd.core.set_persistent_workgroups(0)
    yield ddsp_pytorch_amd
    ddsp_pytorch_amd.core.set_persistent_workgroups(prev)
    ddsp_pytorch_amd.core.set_frame_table(-1)


def _both(dd, fn):
    """fn() with the frame table (two launches) and without it (one launch)."""
    prev = dd.core.set_frame_table(1)
    try:
        a = fn()
        dd.core.set_frame_table(0)
        b = fn()
    finally:
        dd.core.set_frame_table(prev)
    return a, b


@pytest.mark.parametrize("B,F,H,NB,bs", [(64, 200, 100, 65, 512), (23, 211, 37, 33, 256), (9, 480, 128, 65, 512),
                                         (40, 128, 64, 17, 1024), (6, 300, 200, 100, 512), (5, 130, 100, 65, 768)])
def test_table_matches_one_launch_bitwise(dd, B, F, H, NB, bs):
    inp = make_inputs(B, F, H, NB, bs, seed=B + F + H, device="cuda")

    def run():
        with torch.no_grad():
            dd.core.set_noise_seed(11)
            inj = dd.core.synth_frames(inp["f0"], inp["param"], inp["mags"], bs, 48000, noise=inp["noise"],
                                       parts=True, controls=True)
            dev = dd.core.synth_frames(inp["f0"], inp["param"], inp["mags"], bs, 48000)
        torch.cuda.synchronize()
        return inj, dev

    (inj_t, dev_t), (inj_o, dev_o) = _both(dd, run)
    for a, b in zip(inj_t[:3], inj_o[:3]):
        assert torch.equal(a, b)
    for k in ("amplitudes", "harmonic_distribution", "magnitudes"):
        assert torch.equal(inj_t[3][k], inj_o[3][k]), k
    assert torch.equal(dev_t, dev_o)
    # and against the reference's op sequence on the CPU, for two items (fp32 path: 1e-6 RMS)
    ref = tr.synth_path(inp["f0"][:2].cpu(), inp["param"][:2].cpu(), inp["mags"][:2].cpu(),
                        inp["noise"][:2].cpu(), None, bs, 48000)
    assert rms(inj_t[0][:2].cpu().numpy(), ref.numpy()) < 1e-6


@pytest.mark.parametrize("B,F,H,NB,bs", [(64, 200, 100, 65, 512), (23, 211, 37, 33, 256)])
def test_persistent_table_matches_one_launch_bitwise(dd, B, F, H, NB, bs):
    """The persistent kernel fed by the frame table (its preparation wave loads the record) against the
    one-launch per-frame kernel: bit-identical too."""
    inp = make_inputs(B, F, H, NB, bs, seed=B * F, device="cuda")

    def run():
        with torch.no_grad():
            dd.core.set_noise_seed(5)
            inj = dd.core.synth_frames(inp["f0"], inp["param"], inp["mags"], bs, 48000, noise=inp["noise"],
                                       parts=True, controls=True)
            dev = dd.core.synth_frames(inp["f0"], inp["param"], inp["mags"], bs, 48000)
        torch.cuda.synchronize()
        return inj, dev

    dd.core.set_persistent_workgroups(6)
    try:
        dd.core.set_frame_table(1)
        inj_t, dev_t = run()
        dd.core.set_persistent_workgroups(0)
        dd.core.set_frame_table(0)
        inj_o, dev_o = run()
    finally:
        dd.core.set_persistent_workgroups(0)
        dd.core.set_frame_table(-1)
    for a, b in zip(inj_t[:3], inj_o[:3]):
        assert torch.equal(a, b)
    for k in ("amplitudes", "harmonic_distribution", "magnitudes"):
        assert torch.equal(inj_t[3][k], inj_o[3][k]), k
    assert torch.equal(dev_t, dev_o)


def test_table_strided_projections(dd):
    """param / magnitudes as column slices of one projection output (the decoder's one-GEMM route)."""
    B, F, H, NB, bs = 16, 200, 100, 65, 512
    inp = make_inputs(B, F, H, NB, bs, seed=5, device="cuda")
    both = torch.cat([inp["param"], inp["mags"]], dim=-1)
    param, mags = both[..., :H + 1], both[..., H + 1:]
    assert not param.is_contiguous() and not mags.is_contiguous()

    def run():
        with torch.no_grad():
            r = dd.core.synth_frames(inp["f0"], param, mags, bs, 48000, noise=inp["noise"], parts=True, controls=True)
        torch.cuda.synchronize()
        return r

    t, o = _both(dd, run)
    for a, b in zip(t[:3], o[:3]):
        assert torch.equal(a, b)
    for k in t[3]:
        assert torch.equal(t[3][k], o[3][k]), k


def test_table_counter_replay(dd):
    """The device-counter entry point: call k draws offset k, equal to the eager seeded calls."""
    dd.core.set_frame_table(1)
    try:
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
    finally:
        dd.core.set_frame_table(-1)


def test_table_buffer_grows_and_streams(dd):
    """A larger launch after a smaller one (the stream's table buffer grows), and the same launch on
    a side stream (its own buffer), both equal to the one-launch results."""
    dd.core.set_frame_table(1)
    try:
        outs = []
        side = torch.cuda.Stream()
        for B, F in ((4, 150), (32, 300)):
            inp = make_inputs(B, F, 60, 65, 512, seed=B, device="cuda")
            with torch.no_grad():
                a = dd.core.synth_frames(inp["f0"], inp["param"], inp["mags"], 512, 48000, noise=inp["noise"])
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    s = dd.core.synth_frames(inp["f0"], inp["param"], inp["mags"], 512, 48000, noise=inp["noise"])
                torch.cuda.current_stream().wait_stream(side)
                dd.core.set_frame_table(0)
                o = dd.core.synth_frames(inp["f0"], inp["param"], inp["mags"], 512, 48000, noise=inp["noise"])
                dd.core.set_frame_table(1)
            outs.append((a, s, o))
        torch.cuda.synchronize()
        for a, s, o in outs:
            assert torch.equal(a, o) and torch.equal(s, o)
    finally:
        dd.core.set_frame_table(-1)


def test_frame_table_setting_roundtrip(dd):
    prev = dd.core.set_frame_table(0)
    try:
        assert dd.core.set_frame_table(1) == 0
        assert dd.core.set_frame_table(-1) == 1
    finally:
        dd.core.set_frame_table(prev)
