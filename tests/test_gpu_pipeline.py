"""Two-stage serving pipeline (synth.PipelinedSynthPath): synthesis of batch i+1 on one CU
partition beside the reverb of batch i on the other.  Every batch's audio must equal the one-stream
SynthPath's bit for bit (same kernels; device noise advancing per call in call order), including
when the caller reuses its input buffers right after submitting, and a full config-2 batch must
match the torch-CPU restatement of the reference."""
import numpy as np
import pytest
import torch

from conftest import rms

pytestmark = pytest.mark.gpu


def _batches(n, B=8, F=200, H=100, NB=65, bs=512, seed=0):
    from ddsp_pytorch_amd.synth import make_inputs
    return [make_inputs(B, F, H, NB, bs, seed=seed + i, device="cuda") for i in range(n)]


def test_masked_stream_rejects_bad_masks():
    from ddsp_pytorch_amd import core
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    with pytest.raises(ValueError):
        core.cu_masked_stream([], n_cu)
    with pytest.raises(ValueError):
        core.cu_masked_stream([n_cu], n_cu)
    s = core.cu_masked_stream(range(64), n_cu)
    assert s is core.cu_masked_stream(range(64), n_cu)  # one stream per mask


@pytest.mark.parametrize("noise_mode", ["inject", "device"])
def test_pipelined_equals_one_stream(noise_mode):
    from ddsp_pytorch_amd import core
    from ddsp_pytorch_amd.synth import PipelinedSynthPath, SynthPath
    batches = _batches(4)
    syn = SynthPath(512, 48000, reverb_length=48000, noise_mode=noise_mode).cuda()
    args = lambda b: (b["f0"], b["param"], b["mags"], b["noise"])
    core.set_noise_seed(77)
    ref = [syn(*args(b)).clone() for b in batches]
    core.set_noise_seed(77)
    pipe = PipelinedSynthPath(syn, reverb_cus=64)
    outs = [pipe(*args(b)) for b in batches]
    pipe.join()
    torch.cuda.synchronize()
    for i, (o, r) in enumerate(zip(outs, ref)):
        assert torch.equal(o, r), i


def test_pipelined_inputs_reusable_after_submit():
    """The caller may overwrite its input buffers on its own stream right after a call: the
    pipeline's synthesis stream waited for the caller's stream before reading them, and the
    caller's later writes are ordered after the reads only if it joins — here it overwrites the
    inputs after join() and submits again."""
    from ddsp_pytorch_amd.synth import PipelinedSynthPath, SynthPath
    a, b = _batches(2, seed=5)
    syn = SynthPath(512, 48000, reverb_length=48000, noise_mode="inject").cuda()
    ref_a, ref_b = syn(a["f0"], a["param"], a["mags"], a["noise"]).clone(), syn(
        b["f0"], b["param"], b["mags"], b["noise"]).clone()
    pipe = PipelinedSynthPath(syn)
    buf = {k: v.clone() for k, v in a.items()}
    out_a = pipe(buf["f0"], buf["param"], buf["mags"], buf["noise"])
    pipe.join()
    for k in buf:
        buf[k].copy_(b[k])
    out_b = pipe(buf["f0"], buf["param"], buf["mags"], buf["noise"])
    pipe.join()
    torch.cuda.synchronize()
    assert torch.equal(out_a, ref_a) and torch.equal(out_b, ref_b)


def test_pipelined_config2_vs_oracle():
    """A config-2 batch (B=64) through the pipeline, two items against the reference's ATen op
    sequence (oracle/torch_ref.py) at the north_star tolerance."""
    from oracle import torch_ref as tr
    from ddsp_pytorch_amd.synth import PipelinedSynthPath, SynthPath, make_inputs
    inp = make_inputs(64, 200, 100, 65, 512, seed=3, device="cuda")
    syn = SynthPath(512, 48000, reverb_length=48000, noise_mode="inject").cuda()
    pipe = PipelinedSynthPath(syn)
    out = pipe(inp["f0"], inp["param"], inp["mags"], inp["noise"])
    pipe.join()
    out = out.cpu().numpy()
    rv = tr.Reverb(syn.reverb.noise.detach().cpu(), syn.reverb.decay.detach().cpu(),
                   syn.reverb.wet.detach().cpu(), 48000, 48000)
    for b in (1, 62):
        sl = slice(b, b + 1)
        ref = tr.synth_path(inp["f0"][sl].cpu(), inp["param"][sl].cpu(), inp["mags"][sl].cpu(),
                            inp["noise"][sl].cpu(), rv, 512, 48000).numpy()
        assert rms(out[sl], ref) < 1e-5, b


def test_pipelined_from_a_side_stream():
    """A caller on a non-default stream: its input writes are waited for, and the outputs are
    ordered before its later work by join()."""
    from ddsp_pytorch_amd.synth import PipelinedSynthPath, SynthPath
    a, b = _batches(2, seed=9)
    syn = SynthPath(512, 48000, reverb_length=48000, noise_mode="inject").cuda()
    ref = [syn(x["f0"], x["param"], x["mags"], x["noise"]).clone() for x in (a, b)]
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    pipe = PipelinedSynthPath(syn)
    with torch.cuda.stream(side):
        bufs = [{k: v.clone() for k, v in x.items()} for x in (a, b)]  # written on the side stream
        outs = [pipe(x["f0"], x["param"], x["mags"], x["noise"]) for x in bufs]
        pipe.join()
        got = [o.clone() for o in outs]
    torch.cuda.synchronize()
    assert all(torch.equal(g, r) for g, r in zip(got, ref))
    # inputs dropped right after the call (temporaries): their blocks must not be handed to the side
    # stream's next allocations, overwritten below, before the synthesis stream has read them
    with torch.cuda.stream(side):
        outs = []
        for x in (a, b):
            outs.append(pipe(*(x[k].clone() for k in ("f0", "param", "mags", "noise"))))
            junk = [torch.full_like(x[k], 1e3) for k in ("f0", "param", "mags", "noise")]  # reuse attempt
            del junk
        pipe.join()
        got = [o.clone() for o in outs]
    torch.cuda.synchronize()
    assert all(torch.equal(g, r) for g, r in zip(got, ref))



@pytest.mark.parametrize("B,F,H,NB,bs,L", [(1, 12, 40, 33, 256, 48000), (3, 10, 17, 9, 441, 2000)])
def test_pipelined_odd_shapes(B, F, H, NB, bs, L):
    """Batch of one and an odd batch; a block size outside the fused kernel's envelope (441: the
    two-kernel fallback) and a reverb longer than the signal (the crop case, modules.py:30-33)."""
    from ddsp_pytorch_amd.synth import PipelinedSynthPath, SynthPath, make_inputs
    batches = [make_inputs(B, F, H, NB, bs, seed=40 + i, device="cuda") for i in range(3)]
    syn = SynthPath(bs, 48000, reverb_length=L, noise_mode="inject").cuda()
    ref = [syn(b["f0"], b["param"], b["mags"], b["noise"]).clone() for b in batches]
    pipe = PipelinedSynthPath(syn)
    outs = [pipe(b["f0"], b["param"], b["mags"], b["noise"]) for b in batches]
    pipe.join()
    torch.cuda.synchronize()
    for i, (o, r) in enumerate(zip(outs, ref)):
        assert o.shape == (B, F * bs, 1) and torch.equal(o, r), i


def test_synth_graph_replays_and_owns_its_spectrum():
    """synth.SynthGraph: replay k equals the eager step drawing device noise at offset k, and the graph
    keeps reading the spectrum it captured after the module's cached spectrum was freed
    (Reverb.invalidate) and its memory reused by an eager forward of another length."""
    from ddsp_pytorch_amd import core
    from ddsp_pytorch_amd.synth import SynthGraph, SynthPath, make_inputs
    inp = make_inputs(4, 16, 24, 65, 512, seed=5, device="cuda", with_noise=False)
    syn = SynthPath(512, 48000, reverb_length=48000).cuda()
    g = SynthGraph(syn, inp["f0"], inp["param"], inp["mags"], seed=77)
    r0, r1 = g.replay().clone(), g.replay().clone()
    core.set_noise_seed(77)
    with torch.no_grad():
        e0 = syn(inp["f0"], inp["param"], inp["mags"])
        e1 = syn(inp["f0"], inp["param"], inp["mags"])
    assert torch.equal(r0, e0) and torch.equal(r1, e1) and not torch.equal(r0, r1)
    syn.reverb.invalidate()
    with torch.no_grad():
        for n in (3, 5, 9):  # fresh spectra of other lengths, allocated where the old one lived
            syn.reverb(torch.randn(2, n * 2048, 1, device="cuda"))
    g.reset()
    assert torch.equal(g.replay(), r0)
