"""Multi-rank path on CPU with gloo, world_size 2 and 3.

The HIP kernels cannot run here, so each rank runs the torch-CPU restatement of the
reference synth path (oracle/torch_ref.py) on its shard — the test covers the sharding,
ragged shards and the gather, which are the only multi-GPU logic the path has."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ddsp_pytorch_amd.shard import (broadcast_module, chunk_bounds, gather_audio, pack_items,
                                    shard_range, synthesize_pipelined, synthesize_sharded,
                                    unpack_items)


def test_shard_range_partitions_batch():
    for batch in (1, 2, 7, 64, 512):
        for world in (1, 2, 3, 8):
            spans = [shard_range(batch, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == batch
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_range(4, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, batch, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.set_num_threads(1)
        from oracle import torch_ref as tr
        from ddsp_pytorch_amd.synth import make_inputs
        inp = make_inputs(batch, 4, 16, 9, 64, seed=0)
        torch.manual_seed(1)
        noise = (torch.rand(300) * 2 - 1).unsqueeze(-1)
        rv = tr.Reverb(noise, torch.tensor(5.0), torch.tensor(0.0), 300, 48000)
        synth = lambda f0, p, m, n: tr.synth_path(f0, p, m, n, rv, 64, 48000)
        out = synthesize_sharded(synth, inp, rank, world, gather=True)
        if rank == 0:
            full = synth(inp["f0"], inp["param"], inp["mags"], inp["noise"])
            q.put(("ok", float((out - full).abs().max()), tuple(out.shape)))
        # ragged gather of arbitrary payloads
        a, b = shard_range(batch, rank, world)
        local = torch.arange(a, b, dtype=torch.float32).reshape(-1, 1, 1).repeat(1, 5, 1)
        g = gather_audio(local, batch)
        if rank == 0:
            q.put(("gather", bool(torch.equal(g[:, 0, 0], torch.arange(batch, dtype=torch.float32))), None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,batch", [(2, 4), (2, 5), (3, 7)])
def test_sharded_synth_matches_full_batch(world, batch):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, batch, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    res = {}
    while not q.empty():
        k, v, shape = q.get()
        res[k] = (v, shape)
    # MKL may pick a batch-size dependent FFT algorithm: equal to fp32 rounding
    assert res["ok"][0] < 1e-6 and res["ok"][1][0] == batch
    assert res["gather"][0] is True


def test_pack_and_chunks():
    a, b = torch.randn(5, 3, 1), torch.randn(5, 3, 7)
    pa, pb = unpack_items(pack_items([a, b]), [(3, 1), (3, 7)])
    assert torch.equal(pa, a) and torch.equal(pb, b)
    for batch in (1, 5, 64):
        for c in (1, 3, 8, 100):
            bs = chunk_bounds(batch, c)
            assert bs[0][0] == 0 and bs[-1][1] == batch and all(x[1] > x[0] for x in bs)


def _pipeline_worker(rank, world, port, batch, chunks, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.set_num_threads(1)
        from oracle import torch_ref as tr
        from ddsp_pytorch_amd.synth import make_inputs
        # the reverb IR parameters differ per rank until broadcast from rank 0
        torch.manual_seed(1 + rank)
        ir = torch.nn.Module()
        ir.noise = torch.nn.Parameter(torch.rand(300, 1) * 2 - 1)
        ir.decay = torch.nn.Parameter(torch.tensor(5.0 + rank))
        ir.wet = torch.nn.Parameter(torch.tensor(0.0))
        broadcast_module(ir)
        rv = tr.Reverb(ir.noise.data, ir.decay.data, ir.wet.data, 300, 48000)
        synth = lambda f0, p, m, n: tr.synth_path(f0, p, m, n, rv, 64, 48000)
        inp = make_inputs(batch, 4, 16, 9, 64, seed=0)
        keys = ("f0", "param", "mags", "noise")
        tails = [tuple(inp[k].shape[1:]) for k in keys]
        held = [inp[k] for k in keys] if rank == 0 else None  # only the root holds the batch
        out = synthesize_pipelined(synth, held, batch, tails, chunks=chunks)
        if rank == 0:
            torch.manual_seed(1)
            noise0 = torch.rand(300, 1) * 2 - 1
            rv0 = tr.Reverb(noise0, torch.tensor(5.0), torch.tensor(0.0), 300, 48000)
            full = tr.synth_path(*[inp[k] for k in keys], rv0, 64, 48000)
            q.put(("pipe", float((out - full).abs().max()), tuple(out.shape)))
        else:
            q.put(("none%d" % rank, out is None, None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,batch,chunks", [(2, 8, 3), (3, 7, 2), (2, 5, 8)])
def test_pipelined_scatter_synth_gather(world, batch, chunks):
    """Root-held controls scattered in chunks, synthesised per rank, gathered on the root,
    with the IR parameters broadcast from the root: equals the full-batch synth path."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipeline_worker, args=(r, world, port, batch, chunks, q))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    res = {}
    while not q.empty():
        k, v, shape = q.get()
        res[k] = (v, shape)
    assert res["pipe"][0] < 1e-6 and res["pipe"][1][0] == batch, res
    assert all(res["none%d" % r][0] for r in range(1, world))


def _pipeline_order_worker(rank, world, port, batch, chunks, q):
    """Config-5-shaped items (F=400, H=128, NB=65, bs=512) through synthesize_pipelined at world 4.
    The synth stand-in is cheap and item-local (the kernels cannot run here): audio row i is a fixed
    function of item i's controls, so the gathered batch is checked item by item."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.set_num_threads(1)
        F, H, NB, bs = 400, 128, 65, 512
        tails = [(F, 1), (F, H + 1), (F, NB)]

        def synth(f0, param, mags):  # [b, F*bs, 1], item-local
            v = f0[:, :, 0] + param.sum(-1) - mags.sum(-1)
            return v.repeat_interleave(bs, 1).unsqueeze(-1)

        g = torch.Generator().manual_seed(5)
        full = [torch.rand((batch,) + t, generator=g) for t in tails]
        held = full if rank == 0 else None
        trace = []
        out = synthesize_pipelined(synth, held, batch, tails, chunks=chunks, trace=trace)
        res = {"trace": trace}
        if rank == 0:
            res["err"] = float((out - synth(*full)).abs().max())
            res["shape"] = tuple(out.shape)
        else:
            res["none"] = out is None
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("chunks", [1, 4, 8])
def test_pipelined_world4_config5_items_overlap_order(chunks):
    """SURVEY §8(e) at world 4 with config-5-shaped items: the scatter of chunk c+1 is issued before
    chunk c is synthesised, every gather is issued right after its synth and none is waited before the
    last synth (the collectives of neighbouring chunks overlap the synthesis), and the gathered batch
    equals the one-process result item for item."""
    world, batch = 4, 32
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipeline_order_worker, args=(r, world, port, batch, chunks, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    assert res[0]["err"] == 0.0 and res[0]["shape"] == (batch, 400 * 512, 1)
    assert all(res[r]["none"] for r in range(1, world))
    n = len(chunk_bounds(batch, min(chunks, batch // world)))
    assert n == min(chunks, batch // world)
    for r in range(world):
        tr = res[r]["trace"]
        pos = {e: i for i, e in enumerate(tr)}
        assert len(pos) == 5 * n, tr
        last_synth = pos[("synth", n - 1)]
        for c in range(n):
            assert pos[("scattered", c)] < pos[("synth", c)] < pos[("gather", c)] < pos[("gathered", c)]
            if c + 1 < n:
                assert pos[("scatter", c + 1)] < pos[("synth", c)]   # next chunk's scatter in flight
                assert pos[("gather", c)] < pos[("synth", c + 1)]    # this chunk's gather in flight
            assert pos[("gathered", c)] > last_synth                 # no gather waited early
