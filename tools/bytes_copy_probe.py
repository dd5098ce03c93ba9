"""How fast a large `bytes` object can be made from pinned memory (the one
host copy a gzip / planes payload needs): first-touch page faults of the
fresh object dominate.  Run with and without GLIBC_TUNABLES=glibc.malloc.hugetlb=1
(glibc >= 2.35: large malloc'd blocks get transparent huge pages)."""
import os
import time

import numpy as np

src = np.ones(142 << 20, np.uint8)
thp = open("/sys/kernel/mm/transparent_hugepage/enabled").read().strip() if os.path.exists(
    "/sys/kernel/mm/transparent_hugepage/enabled") else "n/a"
ts = []
for _ in range(5):
    t0 = time.perf_counter()
    b = src.tobytes()
    ts.append(time.perf_counter() - t0)
    del b
print({"GLIBC_TUNABLES": os.environ.get("GLIBC_TUNABLES"), "thp": thp,
       "ms": [round(1e3 * t, 1) for t in ts], "GBps_best": round(len(src) / min(ts) / 1e9, 2)})

# the same with glibc's mmap threshold raised at run time (mallopt): freed large
# blocks stay in the heap and the next payload reuses already-faulted pages
import ctypes  # noqa: E402
libc = ctypes.CDLL("libc.so.6")
M_TRIM_THRESHOLD, M_MMAP_THRESHOLD = -1, -3
libc.mallopt(M_MMAP_THRESHOLD, 1 << 30)
libc.mallopt(M_TRIM_THRESHOLD, 1 << 31)
ts = []
for _ in range(5):
    t0 = time.perf_counter()
    b = src.tobytes()
    ts.append(time.perf_counter() - t0)
    del b
print({"mallopt": "M_MMAP_THRESHOLD=1GiB, M_TRIM_THRESHOLD=2GiB", "ms": [round(1e3 * t, 1) for t in ts],
       "GBps_best": round(len(src) / min(ts) / 1e9, 2)})
