"""The multi-GPU collectives on one MI355X (world size 1, RCCL): scatter / gather / broadcast
issued with device tensors exactly as bench.py's N>1 legs issue them, around the gfx950
synthesis path.  (The N>1 logic — ragged shards, chunking, ordering — is covered on CPU with
gloo in tests/test_shard.py.)"""
import os
import socket

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def pg():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    yield dev
    dist.destroy_process_group()


@pytest.mark.parametrize("B,chunks", [(16, 4), (5, 3)])
def test_rccl_pipelined_synth_matches_unsharded(pg, B, chunks):
    from ddsp_pytorch_amd.shard import broadcast_module, gather_audio, synthesize_pipelined
    from ddsp_pytorch_amd.synth import SynthPath, make_inputs
    dev = pg
    syn = SynthPath(512, 48000, reverb_length=4800, noise_mode="inject").to(dev)
    before = syn.reverb(torch.zeros(1, 8192, 1, device=dev)).clone()
    broadcast_module(syn.reverb)
    inp = make_inputs(B, 20, 100, 65, 512, seed=3, device=dev, with_noise=True)
    keys = ["f0", "param", "mags", "noise"]
    ref = syn(*[inp[k] for k in keys])
    assert torch.equal(syn.reverb(torch.zeros(1, 8192, 1, device=dev)), before)
    assert torch.equal(gather_audio(ref, B), ref)
    tails = [tuple(inp[k].shape[1:]) for k in keys]
    out = synthesize_pipelined(syn, [inp[k] for k in keys], B, tails, chunks=chunks, device=dev)
    torch.cuda.synchronize()
    assert out.shape == ref.shape
    assert float((out - ref).abs().max()) < 1e-6
