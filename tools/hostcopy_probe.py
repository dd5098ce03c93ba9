"""Host-side copies of a KC-sized payload (144 MiB) on this box:
  * pinned -> new `bytes`: ndarray.tobytes() vs hostmem.bytes_from (uninitialised
    bytes, MADV_HUGEPAGE interior, native threads)
  * bytes -> reused pinned staging (lossy._parallel_copy), the gunzip_device copy
  * H2D of the stream: from pinned staging vs straight from the pageable bytes"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openfl_amd import hostmem, lossy  # noqa: E402


def t_ms(fn, reps=5):
    out = []
    for _ in range(reps):
        t0 = time.perf_counter()
        r = fn()
        out.append(1e3 * (time.perf_counter() - t0))
        del r
    return [round(v, 1) for v in out]


n = 144 << 20
pin = torch.empty(n, dtype=torch.uint8).pin_memory()
pin.numpy()[:] = np.random.default_rng(0).integers(0, 256, n, dtype=np.uint8)
res = {"bytes": n}
res["pinned_to_bytes_tobytes_ms"] = t_ms(lambda: pin.numpy().tobytes())
res["pinned_to_bytes_bytes_from_ms"] = t_ms(lambda: hostmem.bytes_from(pin.data_ptr(), n))
b = hostmem.bytes_from(pin.data_ptr(), n)
assert b == pin.numpy().tobytes()
src = np.frombuffer(b, np.uint8)
stage = torch.empty(n, dtype=torch.uint8).pin_memory()
res["bytes_to_pinned_stage_8thr_ms"] = t_ms(lambda: lossy._parallel_copy(stage.data_ptr(), src.ctypes.data, n))
res["bytes_to_pinned_stage_1thr_ms"] = t_ms(lambda: np.copyto(stage.numpy(), src))
d = torch.empty(n, dtype=torch.uint8, device="cuda")


def h2d(t):
    d.copy_(t, non_blocking=True)
    torch.cuda.synchronize()


res["h2d_pinned_ms"] = t_ms(lambda: h2d(stage))
res["h2d_pageable_ms"] = t_ms(lambda: h2d(torch.from_numpy(src)))
print(json.dumps(res))
