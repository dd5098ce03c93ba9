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
        # (payloads >= 8 MiB: plus the pool's own, recycling or not)
        pooled = n >= hostmem._RECYCLE_MIN and (hostmem._bytes_layout_ok() or not hostmem._RECYCLE)
        assert sys.getrefcount(b) == (3 if pooled else 2)
    assert len(b) == n and hash(b) == hash(src[:n].tobytes())


def test_bytes_from_small_threshold_path():
    src = np.arange(256, dtype=np.uint8)
    assert hostmem.bytes_from(src.ctypes.data + 3, 100, huge_min=0) == src[3:103].tobytes()
    assert hostmem.bytes_from(src.ctypes.data + 3, 100) == src[3:103].tobytes()


def _src(seed, n):
    return np.random.default_rng(seed).integers(0, 256, size=n, dtype=np.uint8)


needs_layout = pytest.mark.skipif(not hostmem._bytes_layout_ok(), reason="another Python object layout")


@pytest.fixture
def recycle_on(monkeypatch):
    """The opt-in in-place recycling (OFL_HOST_RECYCLE=1) for one test."""
    hostmem.release_pool()
    monkeypatch.setattr(hostmem, "_RECYCLE", True)
    yield
    hostmem.release_pool()


needs_recycle = pytest.mark.usefixtures("recycle_on")


@needs_layout
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


@needs_layout
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


@needs_layout
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


@needs_layout
@needs_recycle
def test_pool_capacity_is_bounded():
    n = 8 << 20
    a = _src(5, n)
    held = [hostmem.bytes_from(a.ctypes.data, n) for _ in range(4)]
    assert sum(e[1] for e in hostmem._pool) <= hostmem._RECYCLE_CAP
    assert all(h == a.tobytes() for h in held)


def test_default_mode_never_rewrites_a_payload(monkeypatch):
    """Default (OFL_HOST_RECYCLE unset): a dropped payload is only released
    (off the caller's thread), never refilled; a payload held by a protobuf
    NamedTensor built from it, by a serialized gRPC-style copy of that message
    or by nothing at all keeps its bytes while later payloads are made."""
    from openfl_amd import protocols
    monkeypatch.setattr(hostmem, "_RECYCLE", False)
    hostmem.release_pool()
    n = 9 << 20
    srcs = [_src(10 + k, n) for k in range(4)]
    b1 = hostmem.bytes_from(srcs[0].ctypes.data, n)
    k1, want1 = id(b1), srcs[0].tobytes()
    nt = protocols.NamedTensor(name="w", round_number=1, lossless=False, report=False,
                               data_bytes=b1)
    wire = nt.SerializeToString()
    del b1
    b2 = hostmem.bytes_from(srcs[1].ctypes.data, n)
    b3 = hostmem.bytes_from(srcs[2].ctypes.data, n - 5)
    assert nt.data_bytes == want1
    back = protocols.NamedTensor()
    back.ParseFromString(wire)
    assert back.data_bytes == want1
    assert b2 == srcs[1].tobytes() and b3 == srcs[2][:n - 5].tobytes()
    held = hostmem.bytes_from(srcs[3].ctypes.data, n)
    view = memoryview(held)
    for _ in range(3):
        hostmem.bytes_from(srcs[0].ctypes.data, n)
    assert bytes(view) == srcs[3].tobytes() and held == srcs[3].tobytes()
    hostmem.release_pool()
    assert not hostmem._pool
    assert k1 is not None


def _wait_release_thread():
    if hostmem._reaper is not None:
        hostmem._reaper.submit(lambda: None).result(30)


@needs_layout
@pytest.mark.parametrize("holder", ["local", "attribute"])
def test_idle_payloads_still_held_are_never_discarded(monkeypatch, holder):
    """A payload the caller still holds past the pool's idle window (here
    0.1 s) is only forgotten by the pool, never discarded: a bytes_from
    payload and a seal_payload payload, held directly or only through a plain
    attribute (a pure-python protobuf-style holder), keep their bytes while
    two more large payloads are made after the window has passed."""
    import ctypes
    import time
    monkeypatch.setattr(hostmem, "_RECYCLE", False)
    monkeypatch.setattr(hostmem, "_POOL_IDLE_S", 0.1)
    hostmem.release_pool()
    _wait_release_thread()
    n = 9 << 20
    a, c = _src(31, n), _src(32, n + 11)
    b1 = hostmem.bytes_from(a.ctypes.data, n)
    b2, addr = hostmem.new_payload(n + 4096)
    ctypes.memmove(addr, c.ctypes.data, n + 11)
    hostmem.seal_payload(b2, n + 11)

    class Holder:   # what a pure-python message does with a bytes field
        pass
    h = Holder()
    if holder == "attribute":
        h.data_bytes, h.other = b1, b2
        del b1, b2
        get = lambda: (h.data_bytes, h.other)   # noqa: E731
    else:
        get = lambda: (b1, b2)   # noqa: E731
    time.sleep(0.25)
    for k in range(2):
        s = _src(40 + k, n)
        assert hostmem.bytes_from(s.ctypes.data, n) == s.tobytes()
    _wait_release_thread()
    x1, x2 = get()
    assert x1 == a.tobytes() and x2 == c.tobytes()
    assert not any(e[0] is x1 or e[0] is x2 for e in hostmem._pool)   # forgotten, not freed
    hostmem.release_pool()


@needs_layout
def test_idle_entry_aged_by_hand_is_not_discarded(monkeypatch):
    """The advisor's recipe: age a held payload's pool entry by hand, make
    another payload, check the held bytes."""
    monkeypatch.setattr(hostmem, "_RECYCLE", False)
    hostmem.release_pool()
    _wait_release_thread()
    n = 8 << 20
    a, c = _src(51, n), _src(52, n)
    held = hostmem.bytes_from(a.ctypes.data, n)
    for e in hostmem._pool:
        if e[0] is held:
            e[2] -= 10 * hostmem._POOL_IDLE_S + 1
    hostmem.bytes_from(c.ctypes.data, n)
    _wait_release_thread()
    assert held == a.tobytes()
    hostmem.release_pool()


def test_release_pool_drops_tracked_payloads(monkeypatch):
    monkeypatch.setattr(hostmem, "_RECYCLE", False)
    hostmem.release_pool()
    n = 8 << 20
    src = _src(3, n)
    b = hostmem.bytes_from(src.ctypes.data, n)
    assert sys.getrefcount(b) == 3 and len(hostmem._pool) == 1
    hostmem.release_pool()
    assert sys.getrefcount(b) == 2 and b == src.tobytes()


def test_release_pauses_inside_quiet(monkeypatch):
    """The release thread frees no pages while a quiet() section (a large H2D
    from pageable memory) is open, and frees them once it closes."""
    import threading
    import time
    monkeypatch.setattr(hostmem, "_RECYCLE", False)
    hostmem.release_pool()
    calls = []
    real = hostmem._c()

    class Spy:
        def madvise(self, a, n, adv):
            calls.append(time.monotonic())
            return real.madvise(a, n, adv)
    monkeypatch.setattr(hostmem, "_c", lambda: Spy())
    n = 24 << 20
    src = _src(4, n)
    b = hostmem.bytes_from(src.ctypes.data, n)
    if hostmem._reaper is not None:   # earlier tests' releases finish first
        hostmem._reaper.submit(lambda: None).result(10)
    calls.clear()
    done = threading.Event()
    with hostmem.quiet():
        del b
        hostmem._release_dead()          # hands the dead payload to the release thread
        hostmem._reaper.submit(done.set)
        time.sleep(0.2)
        assert not calls and not done.is_set()
        t_open = time.monotonic()
    assert done.wait(5)
    assert len(calls) >= 3 and min(calls) >= t_open   # 8 MiB slices, all after the section closed


def test_new_payload_seal(monkeypatch):
    """new_payload / seal_payload (the gzip payload filled by the producer in
    place): the sealed object is an ordinary bytes of the written length --
    content, len, hash, slicing and protobuf use match bytes() of the source;
    below 8 MiB or with recycling on the helper declines; a length above the
    capacity is refused."""
    import ctypes
    from openfl_amd import protocols
    monkeypatch.setattr(hostmem, "_RECYCLE", False)
    hostmem.release_pool()
    assert hostmem.new_payload((8 << 20) - 1) is None
    cap, n = 12 << 20, (9 << 20) + 7
    src = _src(21, n)
    b, addr = hostmem.new_payload(cap)
    assert len(b) == cap
    ctypes.memmove(addr, src.ctypes.data, n)
    with pytest.raises(ValueError):
        hostmem.seal_payload(b, cap + 1)
    assert hostmem.seal_payload(b, n) is b
    want = src.tobytes()
    assert len(b) == n and b == want and hash(b) == hash(want)
    assert b[-7:] == want[-7:] and b[n:] == b""
    nt = protocols.NamedTensor(name="w", round_number=1, lossless=False, report=False, data_bytes=b)
    back = protocols.NamedTensor()
    back.ParseFromString(nt.SerializeToString())
    assert back.data_bytes == want
    assert any(e[0] is b for e in hostmem._pool)
    monkeypatch.setattr(hostmem, "_RECYCLE", True)
    assert hostmem.new_payload(cap) is None
    hostmem.release_pool()
