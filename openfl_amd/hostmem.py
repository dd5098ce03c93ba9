"""Host-memory policy for the payload path (opt-in, process-wide).

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
"""
import ctypes
import ctypes.util

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


def bytes_from(src_addr, n, threads=8, huge_min=8 << 20, par_min=1 << 20):
    """A new `bytes` of the n bytes at host address src_addr (pinned staging).

    The object is created uninitialised (PyBytes_FromStringAndSize(NULL, n),
    the CPython idiom for filling a bytes before anyone else holds it); above
    huge_min its 2 MiB-aligned interior is marked MADV_HUGEPAGE (transparent
    huge pages in 'madvise' mode), so first touch costs one fault per 2 MiB
    instead of per 4 KiB; above par_min the copy runs on native threads, so
    those faults are taken in parallel.  Same bytes as bytes(memoryview) of
    the source."""
    n = int(n)
    if n < par_min:
        return ctypes.string_at(src_addr, n) if n else b""
    b = _new_bytes(None, n)
    _fill(_bytes_addr(b), src_addr, n, threads, huge_min, 4 << 20 if n >= huge_min else
          max(256 << 10, -(-n // (2 * threads)) // 4096 * 4096))
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
