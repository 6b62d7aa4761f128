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

    Shards may be ragged (batch % world != 0): each is padded to the largest shard for the
    collective and trimmed on the root."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    sizes = [shard_range(batch, r, world) for r in range(world)]
    width = max(b - a for a, b in sizes)
    send = local
    if local.shape[0] < width:
        pad = torch.zeros((width - local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype,
                          device=local.device)
        send = torch.cat([local, pad], 0)
    recv = [torch.empty_like(send) for _ in range(world)] if rank == dst else None
    dist.gather(send.contiguous(), recv, dst=dst, group=group)
    if rank != dst:
        return None
    return torch.cat([r[: b - a] for r, (a, b) in zip(recv, sizes)], 0)


def synthesize_sharded(synth, inputs, rank, world, gather=False, dst=0):
    """Run ``synth(f0, param, mags, noise)`` on this rank's slice of full-batch ``inputs``
    (dict of [B, ...] tensors); optionally gather the audio on ``dst``."""
    batch = inputs["f0"].shape[0]
    local = {k: shard(v, rank, world) for k, v in inputs.items()}
    audio = synth(local["f0"], local["param"], local["mags"], local.get("noise"))
    if gather:
        return gather_audio(audio, batch, dst=dst)
    return audio
