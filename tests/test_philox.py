"""The host restatement of the on-device noise generator (oracle/philox.py), pinned to the
published Philox4x32-10 known-answer vectors (Random123, Salmon et al. SC'11) and to the counter
layout the kernels use (synth_frame.hip:71-76, noise.hip:96-103, backward.hip:173-180)."""
import numpy as np
import pytest

from oracle import philox


@pytest.mark.parametrize("ctr,key,expect", [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF, 0xFFFFFFFF), (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
])
def test_philox_known_answers(ctr, key, expect):
    out = philox.philox4x32_10(*[np.uint64(c) for c in ctr], *key)
    assert tuple(int(w) for w in out) == expect


def test_device_noise_layout():
    seed, off = 0x123456789ABCDEF0, (5 << 32) + 7
    x = philox.device_noise(3, 4, 12, seed, off)
    assert x.shape == (3, 4, 12) and x.dtype == np.float32
    # sample 4t+c of frame fr = b*F+f is word c of counter (fr*quads+t, offset), key = seed
    b, f, t, c = 2, 1, 2, 3
    q = (b * 4 + f) * 3 + t
    w = philox.philox4x32_10(np.uint64(q), np.uint64(0), np.uint64(7), np.uint64(5),
                             seed & 0xFFFFFFFF, seed >> 32)[c]
    assert x[b, f, 4 * t + c] == np.float32((int(w) >> 8) * 2.0 ** -24 * 2 - 1)
    # a ragged block (bs % 4 != 0) keeps the per-frame stride ceil(bs/4)
    y = philox.device_noise(3, 4, 10, seed, off)
    z = philox.device_noise(3, 4, 12, seed, off)
    assert np.array_equal(y, z[..., :10])


def test_device_noise_distribution():
    x = philox.device_noise(4, 50, 512, 99, 0).ravel()
    assert x.min() >= -1.0 and x.max() < 1.0
    assert abs(x.mean()) < 5e-3 and abs(x.var() - 1.0 / 3.0) < 5e-3
    # offsets and seeds select disjoint streams
    assert not np.array_equal(philox.device_noise(1, 2, 64, 99, 0), philox.device_noise(1, 2, 64, 99, 1))
    assert not np.array_equal(philox.device_noise(1, 2, 64, 99, 0), philox.device_noise(1, 2, 64, 98, 0))
    # frames of one call are distinct blocks (no counter collision between items / frames)
    a = philox.device_noise(8, 8, 64, 3, 0).reshape(64, 64)
    assert len({r.tobytes() for r in a}) == 64
