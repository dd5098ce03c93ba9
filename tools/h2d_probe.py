"""H2D of a freshly received pageable payload and the device inflate around
it, on the GPU:
  - a payload used once (a new `bytes` per call, as a received gzip stream
    is) vs one copied again and again: plain hipMemcpyAsync vs
    ofl_copy_h2d_staged on 2..8 threads vs a pinned source;
  - gunzip_device of the 1 GiB KC stream, a fresh gzip_ranks payload per
    call, with the plain and the staged copy.

  python tools/h2d_probe.py
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openfl_amd import _lib, hostmem, lossy  # noqa: E402


def timed(fn, reps=5, fresh=None):
    ts = []
    for _ in range(reps):
        a = fresh() if fresh else None
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn(a)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return min(ts), float(np.median(ts))


def main():
    dev = torch.device("cuda:0")
    L = _lib.lib()
    n = 128 << 20
    base = np.random.default_rng(0).integers(0, 256, n, dtype=np.uint8)
    d = torch.empty(n + 64, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream

    def fresh():  # a payload as the plugin receives it: a new bytes object
        return hostmem.bytes_from(base.ctypes.data, n)
    reused = fresh()

    def fresh_quiet():  # a new payload, the previous one freed before the copy starts
        b = fresh()
        hostmem.release_pool()
        time.sleep(0.05)
        return b

    def fresh_prefaulted():  # heap-like: the new payload's pages were touched before (no first-touch faults)
        b = fresh()
        hostmem.release_pool()
        time.sleep(0.05)
        np.frombuffer(b, np.uint8).sum()
        return b
    res = {}
    for kind, fr in (("fresh", fresh), ("fresh_quiet", fresh_quiet), ("reused", lambda: reused)):
        res[f"{kind}_plain"] = timed(lambda b: _lib.check(L.ofl_copy_h2d_async(
            d.data_ptr(), np.frombuffer(b, np.uint8).ctypes.data, n, st)), fresh=fr)
        for t in (2, 4, 8):
            res[f"{kind}_staged{t}"] = timed(lambda b: _lib.check(L.ofl_copy_h2d_staged(
                d.data_ptr(), np.frombuffer(b, np.uint8).ctypes.data, n, t, st)), fresh=fr)
    pin = torch.from_numpy(base.copy()).pin_memory()
    res["pinned"] = timed(lambda _: d[:n].copy_(pin, non_blocking=True))
    ok = bool(torch.equal(d[:n].cpu(), pin))
    print(json.dumps({k: {"GBps_best": round(n / v[0] / 1e9, 2), "ms_med": round(1e3 * v[1], 3)} for k, v in res.items()}
                     | {"ok": ok}), flush=True)

    nv = 1 << 28
    g = torch.Generator(device=dev).manual_seed(0)
    p = torch.tensor([0.074, 0.1816, 0.2444, 0.2444, 0.1816, 0.074], device=dev)
    x = torch.empty(nv, dtype=torch.float32, device=dev)
    for o in range(0, nv, 1 << 24):
        x[o:o + (1 << 24)] = torch.multinomial(p, 1 << 24, replacement=True, generator=g).to(torch.float32)
    out = torch.empty(4 * nv + 64, dtype=torch.uint8, device=dev)
    for thr in (0, 4, 8):
        lossy._H2D_THREADS = thr
        t = timed(lambda z: lossy.gunzip_device(z, out), reps=4, fresh=lambda: lossy.gzip_ranks(x))
        okd = bool(torch.equal(out[:4 * nv].view(torch.float32), x))
        print(json.dumps({"gunzip_device": "fresh 1 GiB KC payload", "h2d_threads": thr, "ok": okd,
                          "ms_best": round(1e3 * t[0], 3), "ms_med": round(1e3 * t[1], 3)}), flush=True)


if __name__ == "__main__":
    main()
