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

_M_TRIM_THRESHOLD, _M_MMAP_THRESHOLD = -1, -3


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
