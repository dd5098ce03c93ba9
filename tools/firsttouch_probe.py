"""First read of a freshly made 144 MiB `bytes` on this box: member-index
walk + staging copy timed on the first and second access, for payloads made
by ndarray.tobytes() and by hostmem.bytes_from (8 / 1 threads)."""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openfl_amd import _lib, hostmem, lossy  # noqa: E402

L = _lib.lib()
x = torch.multinomial(torch.tensor([0.07, 0.2, 0.23, 0.23, 0.2, 0.07], device="cuda"), 1 << 28,
                      replacement=True).to(torch.float32)
z0 = lossy.gzip_ranks(x)
n = len(z0)
pin = torch.empty(n, dtype=torch.uint8).pin_memory()
pin.numpy()[:] = np.frombuffer(z0, np.uint8)
stage = torch.empty(n + (1 << 20), dtype=torch.uint8).pin_memory()
info = {}
for f in ("/proc/sys/kernel/numa_balancing", "/sys/kernel/mm/transparent_hugepage/defrag",
          "/sys/kernel/mm/transparent_hugepage/enabled"):
    try:
        info[f] = open(f).read().strip()
    except OSError as e:
        info[f] = str(e)
info["nodes"] = sorted(d for d in os.listdir("/sys/devices/system/node") if d.startswith("node")) \
    if os.path.isdir("/sys/devices/system/node") else None
info["affinity"] = len(os.sched_getaffinity(0))


def access(z):
    src = np.frombuffer(z, np.uint8)
    nm, tt, mx = ctypes.c_int64(), ctypes.c_size_t(), ctypes.c_uint32()
    cap = src.size // 26 + 1
    idx = np.empty((cap, 4), np.int64)
    t0 = time.perf_counter()
    L.ofl_gzip_member_index(src.ctypes.data, src.size, idx.ctypes.data, cap, ctypes.byref(nm), ctypes.byref(tt),
                            ctypes.byref(mx), None)
    t1 = time.perf_counter()
    lossy._parallel_copy(stage.data_ptr(), src.ctypes.data, src.size)
    t2 = time.perf_counter()
    return round(1e3 * (t1 - t0), 2), round(1e3 * (t2 - t1), 2)


res = {"info": info}
makers = {"tobytes": lambda: pin.numpy().tobytes(),
          "bytes_from_8thr": lambda: hostmem.bytes_from(pin.data_ptr(), n, threads=8),
          "bytes_from_1thr": lambda: hostmem.bytes_from(pin.data_ptr(), n, threads=1),
          "bytes_from_8thr_no_huge": lambda: hostmem.bytes_from(pin.data_ptr(), n, threads=8, huge_min=1 << 62)}
for name, mk in makers.items():
    rows = []
    for rep in range(3):
        t0 = time.perf_counter()
        z = mk()
        t_make = round(1e3 * (time.perf_counter() - t0), 2)
        first = access(z)
        second = access(z)
        t0 = time.perf_counter()
        del z
        t_free = round(1e3 * (time.perf_counter() - t0), 2)
        rows.append({"make": t_make, "first(index,copy)": first, "second(index,copy)": second, "free": t_free})
    res[name] = rows
print(json.dumps(res))
