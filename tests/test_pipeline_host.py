"""Host logic of the two-stage serving pipeline (no GPU): the CU-mask words handed to
ddsp_hip_stream_create_cu_masked, and the C-ABI's refusal of empty or missing masks."""
import ctypes

import pytest


def test_cu_mask_words_layout():
    from ddsp_pytorch_amd.core import cu_mask_words
    assert cu_mask_words(range(64), 256) == [0xFFFFFFFF, 0xFFFFFFFF, 0, 0, 0, 0, 0, 0]
    assert cu_mask_words(range(64, 256), 256) == [0, 0] + [0xFFFFFFFF] * 6
    assert cu_mask_words([0, 33, 255], 256) == [1, 2, 0, 0, 0, 0, 0, 1 << 31]
    assert cu_mask_words([5], 40) == [1 << 5, 0]
    # the two partitions of the pipeline are complementary
    a, b = cu_mask_words(range(64), 256), cu_mask_words(range(64, 256), 256)
    assert all(x & y == 0 and x | y == 0xFFFFFFFF for x, y in zip(a, b))
    with pytest.raises(ValueError):
        cu_mask_words([256], 256)
    with pytest.raises(ValueError):
        cu_mask_words([-1], 256)


def test_stream_create_rejects_bad_arguments_without_a_device():
    from ddsp_pytorch_amd import _lib
    lib = _lib.load()
    handle = ctypes.c_void_p()
    zeros = (ctypes.c_uint32 * 8)()
    assert lib.ddsp_hip_stream_create_cu_masked(zeros, 8, ctypes.byref(handle)) != 0  # no CU selected
    ones = (ctypes.c_uint32 * 8)(*([0xFFFFFFFF] * 8))
    assert lib.ddsp_hip_stream_create_cu_masked(ones, 0, ctypes.byref(handle)) != 0  # no words
    assert lib.ddsp_hip_stream_create_cu_masked(ones, 8, None) != 0  # nowhere to return it
    assert lib.ddsp_hip_stream_destroy(None) != 0
