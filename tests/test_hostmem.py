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
        # no leaked reference from the C-API call (payloads >= 8 MiB: plus the
        # recycling pool's own)
        pooled = hostmem._RECYCLE and n >= hostmem._RECYCLE_MIN and hostmem._bytes_layout_ok()
        assert sys.getrefcount(b) == (3 if pooled else 2)
    assert len(b) == n and hash(b) == hash(src[:n].tobytes())


def test_bytes_from_small_threshold_path():
    src = np.arange(256, dtype=np.uint8)
    assert hostmem.bytes_from(src.ctypes.data + 3, 100, huge_min=0) == src[3:103].tobytes()
    assert hostmem.bytes_from(src.ctypes.data + 3, 100) == src[3:103].tobytes()


def _src(seed, n):
    return np.random.default_rng(seed).integers(0, 256, size=n, dtype=np.uint8)


needs_recycle = pytest.mark.skipif(not (hostmem._RECYCLE and hostmem._bytes_layout_ok()),
                                   reason="payload recycling off (OFL_HOST_RECYCLE=0 or another Python layout)")


@needs_recycle
def test_recycled_payload_is_reused_only_when_released():
    n = 9 << 20
    a, c = _src(1, n), _src(2, n)
    b1 = hostmem.bytes_from(a.ctypes.data, n)
    h1 = hash(b1)  # cached in the object: must be reset on reuse
    k1 = id(b1)
    b2 = hostmem.bytes_from(c.ctypes.data, n - 4097)  # b1 still held: a new object
    assert id(b2) != k1 and b1 == a.tobytes() and hash(b1) == h1
    assert b2 == c[:n - 4097].tobytes()
    del b1
    b3 = hostmem.bytes_from(c.ctypes.data + 5, n - 777)  # b1's memory, resized
    assert id(b3) == k1
    want = c[5:5 + n - 777].tobytes()
    assert len(b3) == n - 777 and b3 == want and hash(b3) == hash(want)
    assert b3[-1:] == want[-1:] and bytes(memoryview(b3)[-3:]) == want[-3:]


@needs_recycle
@pytest.mark.parametrize("hold", ["memoryview", "ndarray", "slice_view"])
def test_referenced_payload_is_never_rewritten(hold):
    n = 8 << 20
    a = _src(3, n)
    b = hostmem.bytes_from(a.ctypes.data, n)
    k = id(b)
    keep = memoryview(b) if hold == "memoryview" else np.frombuffer(b, np.uint8) if hold == "ndarray" \
        else memoryview(b)[10:20]
    del b
    for s in range(3):
        c = _src(10 + s, n)
        d = hostmem.bytes_from(c.ctypes.data, n)
        assert id(d) != k and d == c.tobytes()
    assert bytes(keep) == (a.tobytes() if hold != "slice_view" else a[10:20].tobytes())


@needs_recycle
def test_recycling_under_threads():
    from concurrent.futures import ThreadPoolExecutor
    n = 8 << 20
    srcs = [_src(20 + i, n + 4096 * i) for i in range(6)]

    def job(i):
        ok = True
        for r in range(4):
            s = srcs[(i + r) % len(srcs)]
            b = hostmem.bytes_from(s.ctypes.data, s.size)
            ok &= b == s.tobytes()
            del b
        return ok
    with ThreadPoolExecutor(4) as ex:
        assert all(ex.map(job, range(8)))


@needs_recycle
def test_pool_capacity_is_bounded():
    n = 8 << 20
    a = _src(5, n)
    held = [hostmem.bytes_from(a.ctypes.data, n) for _ in range(4)]
    assert sum(c for _, c in hostmem._pool) <= hostmem._RECYCLE_CAP
    assert all(h == a.tobytes() for h in held)
