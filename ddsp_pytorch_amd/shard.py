"""Batch sharding of the synthesis path across GPUs (one process per GPU).

The synthesis path has no cross-item reduction: batch items are
independent and the only shared state, the reverb IR, is a module parameter every rank
already holds.  So the data path needs no collective — each rank synthesises its own
contiguous slice of the batch.  A collective appears only where a caller wants the audio
in one place: ``gather_audio`` collects the shards on one rank with ``torch.distributed``
``gather`` (RCCL over xGMI on MI355X: each peer's shard crosses its own point-to-point
link to the root; gloo on CPU for tests).
"""
import torch
import torch.distributed as dist


def shard_range(batch, rank, world):
    """[start, stop) of rank's contiguous slice; the first batch % world ranks get one more."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world {rank}/{world}")
    base, extra = divmod(int(batch), world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def shard(t, rank, world):
    """Rank's slice of t along dim 0 (a view)."""
    a, b = shard_range(t.shape[0], rank, world)
    return t[a:b]


def gather_audio(local, batch, dst=0, group=None):
    """Collect every rank's [b_i, T, 1] shard into [batch, T, 1] on rank ``dst`` (None elsewhere).

    Equal shards are received straight into the [batch, T, 1] result (its row blocks); ragged
    shards (batch % world != 0) are padded to the largest shard for the collective and trimmed on
    the root."""
    rank = dist.get_rank(group)
    result = local.new_empty((batch,) + tuple(local.shape[1:])) if rank == dst else None
    work, recv, sizes = _gather_async(local, batch, dst, group, into=result)
    work.wait()
    if rank != dst:
        return None
    if recv is not None:
        for r, (a, b) in zip(recv, sizes):
            result[a:b].copy_(r[: b - a])
    return result


def synthesize_sharded(synth, inputs, rank, world, gather=False, dst=0):
    """Run ``synth(f0, param, mags, noise)`` on this rank's slice of full-batch ``inputs``
    (dict of [B, ...] tensors); optionally gather the audio on ``dst``."""
    batch = inputs["f0"].shape[0]
    local = {k: shard(v, rank, world) for k, v in inputs.items()}
    audio = synth(local["f0"], local["param"], local["mags"], local.get("noise"))
    if gather:
        return gather_audio(audio, batch, dst=dst)
    return audio


# ---------------------------------------------------------------------------------------------
# Root-held batches: the frame-rate controls live on one rank, which scatters
# them, every rank synthesises its shard, and the audio is gathered back.  The reverb IR is
# broadcast once.  The batch is cut into chunks so the collectives of one chunk overlap the
# synthesis of its neighbours: scatter(i+1) || synth(i) || gather(i-1).  With RCCL the
# collectives run on the process group's own HIP stream and the synthesis on the current one;
# async work handles order them (wait() makes the current stream wait, without a host sync).
# ---------------------------------------------------------------------------------------------


def broadcast_module(module, src=0, group=None):
    """Broadcast a module's parameters and buffers (the reverb IR parameters) from ``src``.

    Each tensor is received into a copy and written back with copy_ (the Reverb's device IR cache
    validates itself against the parameters on its next call)."""
    with torch.no_grad():
        for t in list(module.parameters()) + list(module.buffers()):
            tmp = t.detach().clone()
            dist.broadcast(tmp, src, group=group)
            t.copy_(tmp)


def pack_items(tensors):
    """[b, ...] tensors -> one [b, sum of per-item sizes] buffer (a single collective per chunk)."""
    b = tensors[0].shape[0]
    return torch.cat([t.reshape(b, -1) for t in tensors], 1)


def unpack_items(packed, tails):
    """Inverse of pack_items for per-item shapes ``tails``."""
    out, o = [], 0
    for tail in tails:
        n = 1
        for d in tail:
            n *= int(d)
        out.append(packed[:, o:o + n].reshape((packed.shape[0],) + tuple(tail)))
        o += n
    return out


def _scatter_async(full, batch, width_cols, dtype, device, src, group):
    """Start scattering [batch, width_cols] (significant on src only) into ragged shards."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    sizes = [shard_range(batch, r, world) for r in range(world)]
    width = max(b - a for a, b in sizes)
    recv = torch.empty((width, width_cols), dtype=dtype, device=device)
    send = None
    if rank == src:
        send = []
        for a, b in sizes:
            part = full[a:b]
            if b - a < width:
                part = torch.cat([part, part.new_zeros((width - (b - a), width_cols))], 0)
            send.append(part.contiguous())
    work = dist.scatter(recv, send, src=src, group=group, async_op=True)
    a, b = sizes[rank]
    return work, recv, b - a


def _gather_async(local, batch, dst, group, into=None):
    """Start gathering the ragged shards [b_r, ...] of a ``batch``-item chunk on dst.  With ``into``
    (dst's [batch, ...] destination) and equal shards, the receive buffers are its row blocks, so
    the result needs no copy; ragged shards are padded to the widest and compacted afterwards."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    sizes = [shard_range(batch, r, world) for r in range(world)]
    width = max(b - a for a, b in sizes)
    send = local
    if local.shape[0] < width:
        send = torch.cat([local, local.new_zeros((width - local.shape[0],) + tuple(local.shape[1:]))], 0)
    direct = into is not None and all(b - a == width for a, b in sizes)
    if rank != dst:
        recv = None
    elif direct:
        recv = [into[a:b] for a, b in sizes]  # contiguous row blocks of the destination
    else:
        recv = [torch.empty_like(send) for _ in range(world)]
    work = dist.gather(send.contiguous(), recv, dst=dst, group=group, async_op=True)
    return work, (None if direct else recv), sizes


def chunk_bounds(batch, chunks):
    """[start, stop) of each of ``chunks`` near-equal pieces of the global batch (empty ones dropped)."""
    chunks = max(1, min(int(chunks), int(batch)))
    return [r for r in (shard_range(batch, c, chunks) for c in range(chunks)) if r[1] > r[0]]


def synthesize_pipelined(synth, inputs, batch, tails, chunks=4, src=0, dst=0, group=None,
                         device=None, dtype=torch.float32, trace=None):
    """Root-held batch through the sharded synth path with overlapped collectives.

    inputs: list of full-batch [batch, *tail] tensors on ``src`` (ignored elsewhere, may be
    None), in the order ``synth`` takes them; tails: their per-item shapes (every rank knows
    them).  Each of ``chunks`` pieces of the batch is scattered over the ranks, synthesised
    ([b, T, 1] per shard) and gathered on ``dst``.  Returns [batch, T, 1] on dst, None elsewhere.

    ``trace`` (a list, optional) receives the order of events — ("scatter", c) issued, ("scattered", c)
    waited, ("synth", c), ("gather", c) issued, ("gathered", c) waited — so tests can check the overlap:
    scatter(c+1) is issued before synth(c) and no gather is waited before the last synth.
    """
    log = trace.append if trace is not None else (lambda e: None)
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    if batch < world:
        raise ValueError(f"batch {batch} smaller than the world size {world}")
    bounds = chunk_bounds(batch, min(int(chunks), batch // world))  # every shard non-empty
    cols = sum(int(torch.Size(t).numel()) for t in tails)
    packed = pack_items(inputs) if rank == src else None

    def start(c):
        a, b = bounds[c]
        log(("scatter", c))
        return _scatter_async(packed[a:b] if packed is not None else None, b - a, cols, dtype,
                              device, src, group)

    pending = start(0)
    gathers = []
    result = None
    for c in range(len(bounds)):
        work, recv, n = pending
        work.wait()
        log(("scattered", c))
        if c + 1 < len(bounds):
            pending = start(c + 1)  # in flight while this chunk is synthesised
        audio = synth(*unpack_items(recv[:n], tails))
        log(("synth", c))
        a, b = bounds[c]
        if rank == dst and result is None:  # every rank's audio has this item shape
            result = audio.new_empty((batch,) + tuple(audio.shape[1:]))
        gathers.append((a, _gather_async(audio, b - a, dst, group, into=result[a:b] if result is not None else None)))
        log(("gather", c))
    for c, (a, (work, recv, sizes)) in enumerate(gathers):
        work.wait()
        log(("gathered", c))
        if rank == dst and recv is not None:  # ragged shards: compact the padded blocks
            for r, (s0, s1) in zip(recv, sizes):
                result[a + s0:a + s1].copy_(r[: s1 - s0])
    return result if rank == dst else None
