"""Host (numpy) restatement of the on-device noise generator (``noise_mode="device"``).

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module, and only as the checker.  It regenerates, on the
host, exactly the U[-1,1) samples the gfx950 kernels draw, so that device-noise outputs can be
compared with the CPU oracle (``oracle/torch_ref.py``) fed the same noise.

The reference draws ``torch.rand(B, F, bs) * 2 - 1`` (ddsp/models/modules.py:119-123):
independent U[-1,1) per (item, frame, sample).  The device mode keeps that distribution with a
counter-based generator so that no host RNG or H2D copy sits in the synthesis step:

* Philox4x32-10 (Salmon, Moraes, Dror, Shaw, "Parallel random numbers: as easy as 1, 2, 3",
  SC'11), multipliers 0xD2511F53 / 0xCD9E8D57, Weyl key increments 0x9E3779B9 / 0xBB67AE85,
  ten rounds — the published algorithm (known-answer vectors in tests/test_philox.py);
* counter layout (ddsp_pytorch_amd/csrc/synth_frame.hip:71-76, noise.hip:96-103,
  backward.hip:173-180): for frame index ``fr = b * F + f`` and sample quad ``t`` (samples
  4t..4t+3 of the frame, ``quads = ceil(bs / 4)``), the 128-bit counter is
  ``(lo32(q), hi32(q), lo32(offset), hi32(offset))`` with ``q = fr * quads + t``, and the key is
  ``(lo32(seed), hi32(seed))``;
* word c of the output → sample 4t+c: ``u = (word >> 8) * 2^-24``, ``u * 2 - 1`` in fp32
  (both steps exact).
"""
import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = 0x9E3779B9, 0xBB67AE85
_MASK = np.uint64(0xFFFFFFFF)
_S32 = np.uint64(32)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Philox4x32-10 of the counters (uint32 arrays, broadcast) under key (k0, k1) (python
    ints).  Returns the four output words as uint32 arrays."""
    c0, c1, c2, c3 = (np.asarray(c, dtype=np.uint64) for c in (c0, c1, c2, c3))
    k0, k1 = int(k0) & 0xFFFFFFFF, int(k1) & 0xFFFFFFFF
    for _ in range(10):
        p0 = M0 * c0  # exact: both factors < 2^32
        p1 = M1 * c2
        hi0, lo0 = p0 >> _S32, p0 & _MASK
        hi1, lo1 = p1 >> _S32, p1 & _MASK
        c0, c1, c2, c3 = hi1 ^ c1 ^ np.uint64(k0), lo1, hi0 ^ c3 ^ np.uint64(k1), lo0
        k0 = (k0 + W0) & 0xFFFFFFFF
        k1 = (k1 + W1) & 0xFFFFFFFF
    return tuple(c.astype(np.uint32) for c in (c0, c1, c2, c3))


def uniform_pm1(words):
    """U[-1,1) from the top 24 bits of each word (common.h uniform_pm1)."""
    u = (np.asarray(words, dtype=np.uint32) >> np.uint32(8)).astype(np.float32) * np.float32(2.0 ** -24)
    return u * np.float32(2.0) - np.float32(1.0)


def device_noise(batch, frames, block_size, seed, offset):
    """The [batch, frames, block_size] fp32 noise tensor the kernels draw for (seed, offset)."""
    quads = (block_size + 3) // 4
    fr = np.arange(batch * frames, dtype=np.uint64)[:, None]
    q = fr * np.uint64(quads) + np.arange(quads, dtype=np.uint64)[None, :]
    off = int(offset) & 0xFFFFFFFFFFFFFFFF
    words = philox4x32_10(q & _MASK, q >> _S32, np.uint64(off & 0xFFFFFFFF), np.uint64(off >> 32),
                          seed & 0xFFFFFFFF, (int(seed) >> 32) & 0xFFFFFFFF)
    x = np.stack([uniform_pm1(w) for w in words], -1).reshape(batch * frames, quads * 4)
    return np.ascontiguousarray(x[:, :block_size]).reshape(batch, frames, block_size)
