"""openfl_amd.hostmem: payload `bytes` made from a host buffer (the one copy a
plugin payload needs) and the opt-in heap policy.  CPU only."""
import sys

import numpy as np
import pytest

from openfl_amd import hostmem


@pytest.mark.parametrize("n", [0, 1, 4095, (8 << 20) - 1, 8 << 20, (8 << 20) + 3, (21 << 20) + 12345])
def test_bytes_from_equals_tobytes(n):
    src = np.random.default_rng(n).integers(0, 256, size=max(n, 1), dtype=np.uint8)
    b = hostmem.bytes_from(src.ctypes.data, n)
    assert type(b) is bytes
    assert b == src[:n].tobytes()
    if n > 1:  # b"" and 1-byte bytes are interned singletons
        assert sys.getrefcount(b) == 2  # no leaked reference from the C-API call


def test_bytes_from_small_threshold_path():
    src = np.arange(256, dtype=np.uint8)
    assert hostmem.bytes_from(src.ctypes.data + 3, 100, huge_min=0) == src[3:103].tobytes()
    assert hostmem.bytes_from(src.ctypes.data + 3, 100) == src[3:103].tobytes()
