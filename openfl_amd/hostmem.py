"""Host memory of the payload path: payload bytes made from pinned staging
(recycled above 8 MiB) and the opt-in, process-wide heap policy.

Every payload crosses the plugin boundary as a fresh Python `bytes` (the
reference API; protobuf's data_bytes takes nothing else) and every decoded
tensor as a fresh ndarray.  glibc serves blocks above its mmap threshold
with a new mapping each time, so each large payload pays first-touch page
faults: a 144 MiB `bytes` takes ~24 ms to make at ~6 GB/s.  keep_large_blocks()
raises the mmap and trim thresholds (mallopt), so large blocks come from the
heap and freed ones stay there for the next call: the same copy then runs at
~30 GB/s (tools/bytes_copy_probe.py, profiles/r02_bytes_copy_probe_mallopt.txt).
The cost: memory freed by the process is kept by it rather than returned to
the OS.  OFL_HOST_KEEP_LARGE_BLOCKS=1 in the environment applies it at import.

Large payloads (>= 8 MiB) that bytes_from made are tracked in a small pool
for one purpose by default: when the caller has dropped one (the pool holds
the only reference), the pool hands its last reference to a background
thread, so the munmap of the dead payload (~37k pages for a 144 MiB stream,
~8.7 ms on the GPU box) is not paid on the caller's thread.  That thread
frees the pages in slices, pausing while a large H2D from pageable memory
runs (hostmem.quiet(), around gunzip_device's copy): page freeing beside the
runtime's staging slowed the copy ~7x.  No live `bytes` is ever written in
this default mode; hostmem.release_pool() drops
every tracked reference at once, and tracked payloads older than
OFL_HOST_POOL_IDLE_S seconds (default 30) are dropped at the next call.

Opt-in (OFL_HOST_RECYCLE=1): instead of being released, a dead payload is
refilled in place for the next payload of a size that fits (its ob_size /
ob_shash reset; the CPython layout is checked once on a live object), which
also saves the successor's first-touch faults (KC step 43-51 -> 34.3 ms,
profiles/r03_kc_recycle_ab.txt).  The invariant this mode relies on: every
consumer of a payload holds a real reference while it uses the buffer (a
memoryview, an ndarray or protobuf's own copy all do, tests/test_hostmem.py);
C code that keeps a borrowed char* past its last reference would see the
bytes change.  OFL_HOST_RECYCLE_MIB caps the pooled capacity (default 2048).
"""
import ctypes
import ctypes.util
import os
import sys
import threading

import numpy as np

_M_TRIM_THRESHOLD, _M_MMAP_THRESHOLD = -1, -3
_MADV_HUGEPAGE = 14
_HUGE = 2 << 20
_libc = None

_new_bytes = ctypes.pythonapi.PyBytes_FromStringAndSize
_new_bytes.argtypes = [ctypes.c_void_p, ctypes.c_ssize_t]
_new_bytes.restype = ctypes.py_object
_bytes_addr = ctypes.pythonapi.PyBytes_AsString
_bytes_addr.argtypes = [ctypes.py_object]
_bytes_addr.restype = ctypes.c_void_p


def _c():
    global _libc
    if _libc is None:
        _libc = ctypes.CDLL(ctypes.util.find_library("c") or "libc.so.6", use_errno=True)
        _libc.madvise.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    return _libc


_RECYCLE = os.environ.get("OFL_HOST_RECYCLE", "0") == "1"
_RECYCLE_MIN = 8 << 20
_RECYCLE_CAP = int(os.environ.get("OFL_HOST_RECYCLE_MIB", "2048")) << 20
_POOL_IDLE_S = float(os.environ.get("OFL_HOST_POOL_IDLE_S", "30"))
_pool = []  # [[bytes, capacity, made_at]]: payloads this module made, newest last
_pool_lock = threading.Lock()
_layout_ok = None
_reaper = None


def _refcount_is_pool_only(ent):
    # read by address with no local bound to the object (a loop variable
    # holding it would count too): 1 = the pool's entry
    return ctypes.c_ssize_t.from_address(id(ent[0])).value == 1


_MADV_DONTNEED = 4
_SLICE = 8 << 20
_quiet_n = 0
_quiet_cv = threading.Condition()


class quiet:
    """Context manager around a large H2D from pageable memory: while one is
    open, the release thread does not free pages.  Freeing a dead payload's
    ~30k pages (munmap, or madvise) beside the runtime's staging of another
    payload slowed that copy ~7x on the GPU box (tools/h2d_probe.py: a 128 MiB
    H2D 2.8 ms alone, 20 ms median beside a release; KC inflate 7 -> 25 ms)."""

    def __enter__(self):
        global _quiet_n
        with _quiet_cv:
            _quiet_n += 1
        return self

    def __exit__(self, *exc):
        global _quiet_n
        with _quiet_cv:
            _quiet_n -= 1
            _quiet_cv.notify_all()
        return False


def _release(objs):
    """Free dead payloads (the only references are in `objs`): their whole
    pages are discarded in 8 MiB slices (madvise DONTNEED), each slice only
    while no quiet() section is open (waiting at most 1 s per slice), then
    the objects are freed (a munmap of a range with no pages left)."""
    libc = _c()
    for b in objs:
        a = _bytes_addr(b)
        lo = (a + 4095) & ~4095              # the headers sit before the data, in the first page
        hi = (a + len(b)) & ~4095
        for s in range(lo, hi, _SLICE):
            with _quiet_cv:
                _quiet_cv.wait_for(lambda: _quiet_n == 0, timeout=1.0)
            libc.madvise(ctypes.c_void_p(s), min(_SLICE, hi - s), _MADV_DONTNEED)
    with _quiet_cv:
        _quiet_cv.wait_for(lambda: _quiet_n == 0, timeout=1.0)
    objs.clear()


def _drop_later(objs):
    """Release the last references to dead payloads on a background thread
    (their page release and munmap off the caller's thread)."""
    global _reaper
    if not objs:
        return
    if _reaper is None:
        from concurrent.futures import ThreadPoolExecutor
        _reaper = ThreadPoolExecutor(max_workers=1, thread_name_prefix="ofl-hostmem-release")
    _reaper.submit(_release, objs)


def _release_dead():
    """Default mode: hand tracked payloads nobody else references to the
    release thread (their pages are discarded there).  Payloads tracked longer
    than _POOL_IDLE_S that someone still references are only forgotten: the
    pool drops its reference and the caller's own references free the object
    as usual, untouched.  Only a refcount-1 object (the pool's entry is its
    last reference, so nothing outside this module can reach it) is ever
    handed to _release."""
    import time
    now = time.monotonic()
    dead = []
    with _pool_lock:
        keep = []
        for i in range(len(_pool)):
            if _refcount_is_pool_only(_pool[i]):
                dead.append(_pool[i][0])
            elif now - _pool[i][2] <= _POOL_IDLE_S:
                keep.append(_pool[i])
            # else: live and idle -> forgotten (its reference dropped with the old list)
        if len(keep) != len(_pool):
            _pool[:] = keep
        keep = None
    _drop_later(dead)


def release_pool():
    """Drop every payload reference the pool holds (e.g. at round end); the
    payloads still referenced elsewhere live on, the rest are freed."""
    with _pool_lock:
        objs = [e[0] for e in _pool]
        _pool.clear()
    objs.clear()


def _bytes_layout_ok():
    """CPython 3.x PyBytesObject: {refcnt, type, ob_size, ob_shash, ob_sval[]}.
    Checked once on live objects before any in-place reuse."""
    global _layout_ok
    if _layout_ok is None:
        ok = sys.implementation.name == "cpython" and ctypes.sizeof(ctypes.c_void_p) == 8
        if ok:
            b = _new_bytes(None, 100)
            a = id(b)
            ok = (_bytes_addr(b) == a + 32 and ctypes.c_ssize_t.from_address(a + 16).value == 100
                  and ctypes.c_ssize_t.from_address(a).value >= 1)
            if ok:
                h = hash(b)
                ok = ctypes.c_ssize_t.from_address(a + 24).value == h
        _layout_ok = bool(ok)
    return _layout_ok


def _recycled(n):
    """A pooled payload of capacity >= n that nobody else references, resized
    to n bytes (hash reset), or None.  The pool keeps the caller's reference
    out of the count: the object is claimed under the lock and only reached
    through the pool, so no other thread can obtain it meanwhile."""
    with _pool_lock:
        best = -1
        for i in range(len(_pool)):
            ent = _pool[i]
            cap = ent[1]
            if cap < n or cap > 2 * n + (64 << 20):
                continue
            if not _refcount_is_pool_only(ent):
                continue
            if best < 0 or cap < _pool[best][1]:
                best = i
        if best < 0:
            return None
        ent = _pool.pop(best)
        b = ent[0]
        a = id(b)
        ctypes.c_ssize_t.from_address(a + 16).value = n   # ob_size (the allocation stays cap + 1 bytes)
        ctypes.c_ssize_t.from_address(a + 24).value = -1  # ob_shash: not computed
        ctypes.c_char.from_address(a + 32 + n).value = b"\0"
        _pool.append(ent)  # newest last; the caller's reference keeps it from reuse
        return b


def _remember(b, cap):
    import time
    with _pool_lock:
        _pool.append([b, cap, time.monotonic()])
        tot = sum(e[1] for e in _pool)
        i = 0
        while tot > _RECYCLE_CAP and i < len(_pool):  # oldest first
            tot -= _pool[i][1]
            _pool.pop(i)


def bytes_from(src_addr, n, threads=8, huge_min=8 << 20, par_min=1 << 20):
    """A new `bytes` of the n bytes at host address src_addr (pinned staging).

    The object is created uninitialised (PyBytes_FromStringAndSize(NULL, n),
    the CPython idiom for filling a bytes before anyone else holds it); above
    huge_min its 2 MiB-aligned interior is marked MADV_HUGEPAGE (transparent
    huge pages in 'madvise' mode), so first touch costs one fault per 2 MiB
    instead of per 4 KiB; above par_min the copy runs on native threads, so
    those faults are taken in parallel.  Same bytes as bytes(memoryview) of
    the source.  From 8 MiB on the payload is tracked so its release happens
    off the caller's thread; with OFL_HOST_RECYCLE=1 a payload this function
    made earlier and nobody references any more is refilled instead (module
    docstring)."""
    n = int(n)
    if n < par_min:
        return ctypes.string_at(src_addr, n) if n else b""
    piece = 4 << 20 if n >= huge_min else max(256 << 10, -(-n // (2 * threads)) // 4096 * 4096)
    if _RECYCLE and n >= _RECYCLE_MIN and _bytes_layout_ok():
        b = _recycled(n)
        if b is not None:
            _fill(_bytes_addr(b), src_addr, n, threads, 1 << 62, piece)  # pages already resident
            return b
        # a fresh one with 1/8 headroom (untouched pages cost nothing), so the
        # next payload of a slightly larger size still fits
        cap = n + (n >> 3)
        b = _new_bytes(None, cap)
        _fill(_bytes_addr(b), src_addr, n, threads, huge_min, piece)
        a = id(b)
        ctypes.c_ssize_t.from_address(a + 16).value = n
        ctypes.c_char.from_address(a + 32 + n).value = b"\0"
        _remember(b, cap)
        return b
    b = _new_bytes(None, n)
    _fill(_bytes_addr(b), src_addr, n, threads, huge_min, piece)
    if n >= _RECYCLE_MIN:
        _release_dead()
        _remember(b, n)
    return b


def new_payload(cap):
    """(b, addr) for a producer that writes a payload of at most cap bytes
    straight into a new `bytes` (e.g. ofl_gzip_ranks_to, batch by batch while
    the GPU works): an uninitialised object of capacity cap nobody else holds,
    its 2 MiB-aligned interior marked MADV_HUGEPAGE as in bytes_from.  Pages
    the producer never writes are never touched.  Finish it with
    seal_payload(b, n) before anyone else sees it.  None below 8 MiB, with
    OFL_HOST_RECYCLE=1 (that mode refills pooled payloads via bytes_from) or
    when the CPython layout check fails."""
    cap = int(cap)
    if cap < _RECYCLE_MIN or _RECYCLE or not _bytes_layout_ok():
        return None
    b = _new_bytes(None, cap)
    a = _bytes_addr(b)
    lo = (a + _HUGE - 1) // _HUGE * _HUGE
    hi = (a + cap) // _HUGE * _HUGE
    if hi > lo:
        _c().madvise(lo, hi - lo, _MADV_HUGEPAGE)  # advisory: a refusal only costs speed
    return b, a


def seal_payload(b, n):
    """Set a new_payload object's length to the n bytes written (n <= its
    capacity; the allocation keeps its capacity, untouched pages cost
    nothing) and track it like a bytes_from payload.  Returns b."""
    n = int(n)
    a = id(b)
    if not 0 <= n <= ctypes.c_ssize_t.from_address(a + 16).value:
        raise ValueError("seal_payload: length exceeds the capacity")
    ctypes.c_ssize_t.from_address(a + 16).value = n   # ob_size; ob_shash is still -1 (never hashed)
    ctypes.c_char.from_address(a + 32 + n).value = b"\0"
    _release_dead()
    _remember(b, n)
    return b


def _fill(dst, src_addr, n, threads, huge_min, piece):
    if n >= huge_min:
        lo = (dst + _HUGE - 1) // _HUGE * _HUGE
        hi = (dst + n) // _HUGE * _HUGE
        if hi > lo:
            _c().madvise(lo, hi - lo, _MADV_HUGEPAGE)  # advisory: a refusal only costs speed
    from openfl_amd import _lib
    offs = np.arange(0, n, piece, dtype=np.uint64)
    sizes = np.minimum(np.uint64(piece), np.uint64(n) - offs).astype(np.int64)
    d = np.uint64(dst) + offs
    s = np.uint64(src_addr) + offs
    _lib.check(_lib.lib().ofl_host_copy_many(offs.size, d.ctypes.data, s.ctypes.data, sizes.ctypes.data,
                                             int(threads)))


def array_from(src_addr, count, dtype=np.float32, threads=8, par_min=1 << 20, huge_min=4 << 20):
    """A new ndarray of `count` elements copied from host address src_addr
    (pinned staging): a fresh array's first touch is page faults, so above
    par_min bytes the copy runs in pieces on native threads (the faults taken
    in parallel) and above huge_min the array's 2 MiB-aligned interior is
    marked MADV_HUGEPAGE first."""
    dt = np.dtype(dtype)
    out = np.empty(int(count), dt)
    n = out.nbytes
    if n < par_min:
        if n:
            ctypes.memmove(out.ctypes.data, src_addr, n)
        return out
    _fill(out.ctypes.data, src_addr, n, threads, huge_min, max(256 << 10, -(-n // (2 * threads)) // 4096 * 4096))
    return out


def keep_large_blocks(threshold=1 << 30):
    """Serve allocations below `threshold` bytes from the heap and keep up to
    2 x threshold of freed heap memory.  Returns True if glibc accepted both."""
    name = ctypes.util.find_library("c") or "libc.so.6"
    try:
        libc = ctypes.CDLL(name)
        return bool(libc.mallopt(_M_MMAP_THRESHOLD, int(threshold))) and \
            bool(libc.mallopt(_M_TRIM_THRESHOLD, int(2 * threshold)))
    except (OSError, AttributeError):
        return False
