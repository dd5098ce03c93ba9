"""Fine-grained phases of the KC pipeline step of bench.py (kc_uniform_1gib):
the steps inside lossy.gunzip_device timed with device syncs in between."""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openfl_amd import _lib, lossy  # noqa: E402
from openfl_amd.workloads import WORKLOADS, numel  # noqa: E402

dev = torch.device("cuda:0")
numels = [numel(s) for _, s in WORKLOADS["uniform_1gib"]()]
offs = list(np.cumsum([0] + [(n + 63) // 64 * 64 for n in numels[:-1]]))
tot = offs[-1] + numels[-1]
x = torch.randn(tot, device=dev) * 0.01
ranks = torch.empty_like(x)
rb = ranks.view(torch.uint8)
L = _lib.lib()
ph = {}


def tick(name, t0):
    torch.cuda.synchronize()
    t = time.perf_counter()
    ph[name] = ph.get(name, 0.0) + 1e3 * (t - t0)
    return t


steps = 4
for it in range(steps + 1):
    if it == 1:
        ph = {}
    t = time.perf_counter()
    lossy.kmeans_batch(x, offs, numels, 6, n_init=6, seed=it, ranks_out=ranks)
    t = tick("kmeans", t)
    z = lossy.gzip_ranks(ranks)
    t = tick("gzip_ranks", t)
    src = np.frombuffer(z, np.uint8)
    nm, tt, mx = ctypes.c_int64(), ctypes.c_size_t(), ctypes.c_uint32()
    cap = src.size // 26 + 1
    idx = np.empty((cap, 4), np.int64)
    t = tick("inflate.alloc", t)
    L.ofl_gzip_member_index(src.ctypes.data, src.size, idx.ctypes.data, cap, ctypes.byref(nm), ctypes.byref(tt),
                            ctypes.byref(mx), None)
    t = tick("inflate.index", t)
    idx = idx[:nm.value]
    ioff = (src.size + 7) // 8 * 8
    need = ioff + idx.nbytes
    t_b = time.perf_counter()
    stage = lossy._buf("host", "gz_in", need, pinned=True)
    ph["inflate.stage_buf"] = ph.get("inflate.stage_buf", 0.0) + 1e3 * (time.perf_counter() - t_b)
    sn = stage.numpy()
    lossy._parallel_copy(sn.ctypes.data, src.ctypes.data, src.size)
    sn[ioff:need] = idx.view(np.uint8).reshape(-1)
    t = tick("inflate.stage_copy", t)
    d_in = lossy._buf(dev, "gz_in", need)
    d_in[:need].copy_(stage[:need], non_blocking=True)
    t = tick("inflate.h2d", t)
    ws = lossy._buf(dev, "gz_status", 256)
    with torch.cuda.device(dev):
        _lib.check_gzip(L.ofl_inflate_members(d_in.data_ptr(), d_in.data_ptr() + ioff, nm.value, mx.value,
                                              rb.data_ptr(), rb.numel(), ws.data_ptr(), ws.numel(),
                                              torch.cuda.current_stream(dev).cuda_stream))
    t = tick("inflate.kernels", t)
    t = time.perf_counter()
    lossy.gunzip_device(z, rb)
    t = tick("gunzip_device_whole", t)
    del src, idx, sn
    t = tick("free_views", t)
    z = None
    t = tick("free_payload", t)
print(json.dumps({k: round(v / steps, 2) for k, v in ph.items()}))
