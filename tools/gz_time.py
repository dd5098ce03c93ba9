"""Time lossy.gzip_ranks (device gzip of float32 ranks) on a KC-like 1 GiB
rank array; prints ms per call and the compressed ratio."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openfl_amd import lossy  # noqa: E402

n = 1 << 28
g = torch.Generator(device="cuda").manual_seed(0)
p = torch.tensor([0.07, 0.2, 0.23, 0.23, 0.2, 0.07], device="cuda")
x = torch.multinomial(p, n, replacement=True, generator=g).to(torch.float32)
z = lossy.gzip_ranks(x)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(3):
    z = lossy.gzip_ranks(x)
dt = (time.perf_counter() - t0) / 3
print(f"gzip_ranks 1 GiB: {1e3 * dt:.1f} ms, {4 * n / dt / 2**30:.2f} GiB/s, ratio {len(z) / (4 * n):.4f}")
# the pinned -> bytes copy inside gzip_ranks, timed alone on the same size
buf = torch.empty(len(z), dtype=torch.uint8).pin_memory()
t0 = time.perf_counter()
for _ in range(3):
    b = buf.numpy().tobytes()
print(f"pinned -> bytes copy of {len(z) / 2**20:.1f} MiB: {1e3 * (time.perf_counter() - t0) / 3:.1f} ms")
# decode: device inflate of the same stream (H2D of the compressed bytes included) vs host inflate on 16 threads
out = torch.empty(4 * n, dtype=torch.uint8, device="cuda")
lossy.gunzip_device(z, out)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(3):
    lossy.gunzip_device(z, out)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / 3
ok = torch.equal(out.view(torch.float32), x)
print(f"gunzip_device 1 GiB: {1e3 * dt:.1f} ms, {4 * n / dt / 2**30:.2f} GiB/s, exact {ok}")
stage = torch.empty(4 * n, dtype=torch.uint8).pin_memory()
t0 = time.perf_counter()
for _ in range(3):
    lossy.gunzip(z, 16, out=stage.numpy())
dt = (time.perf_counter() - t0) / 3
print(f"gunzip host (16 threads) 1 GiB: {1e3 * dt:.1f} ms, {4 * n / dt / 2**30:.2f} GiB/s")
# phases of gunzip_device: host member index, pinned staging copy, H2D, kernel
import ctypes  # noqa: E402
from openfl_amd import _lib  # noqa: E402
L = _lib.lib()
src = np.frombuffer(z, np.uint8)
nm, tot, mx = ctypes.c_int64(), ctypes.c_size_t(), ctypes.c_uint32()
t0 = time.perf_counter()
L.ofl_gzip_member_index(src.ctypes.data, src.size, None, 0, ctypes.byref(nm), ctypes.byref(tot), ctypes.byref(mx), None)
idx = np.empty((nm.value, 4), np.int64)
L.ofl_gzip_member_index(src.ctypes.data, src.size, idx.ctypes.data, nm.value, ctypes.byref(nm), ctypes.byref(tot),
                        ctypes.byref(mx), None)
t1 = time.perf_counter()
pin = torch.empty(src.size + idx.nbytes + 8, dtype=torch.uint8).pin_memory()
pn = pin.numpy()
pn[:src.size] = src
t2 = time.perf_counter()
d = torch.empty_like(pin, device="cuda")
torch.cuda.synchronize()
t3 = time.perf_counter()
d.copy_(pin)
torch.cuda.synchronize()
t4 = time.perf_counter()
print(f"gunzip_device phases: index {1e3 * (t1 - t0):.1f} ms ({nm.value} members), staging copy {1e3 * (t2 - t1):.1f} ms, "
      f"H2D {1e3 * (t4 - t3):.1f} ms")
