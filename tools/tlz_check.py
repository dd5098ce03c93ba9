"""TLZ gzip / inflate check on the GPU (csrc/deflate_kernels.hip, gz::tlz):
round trips through gzip.decompress and the device inflate, the ratio
against gzip -9, and the kernel times on the 1 GiB KC rank set.

  python tools/tlz_check.py [--big]
"""
import argparse
import gzip
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openfl_amd import _lib, lossy  # noqa: E402


def kc_like(n, seed):
    th = np.array([-1.4468, -0.6568, 0.0, 0.6568, 1.4468])
    x = np.random.default_rng(seed).standard_normal(n)
    return np.searchsorted(th, x).astype(np.float32)


def cases():
    rng = np.random.default_rng(1)
    yield "one", np.float32([5.0])
    yield "seven", rng.integers(0, 4, 7).astype(np.float32)
    yield "kc6_200k", kc_like(200_000, 2)
    yield "ternary", rng.choice(3, 300_000, p=[0.05, 0.9, 0.05]).astype(np.float32)
    yield "constant", np.full(100_000, 2.0, np.float32)
    yield "all32", rng.integers(0, 32, 150_000).astype(np.float32)
    yield "runs", np.repeat(rng.integers(0, 6, 3001), 100)[:300_000].astype(np.float32)
    yield "ragged", rng.integers(0, 4, 131072 * 2 + 2049).astype(np.float32)
    yield "kc6_1m", kc_like(1 << 20, 3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--big", action="store_true")
    args = ap.parse_args()
    dev = "cuda:0"
    res = {}
    for name, x in cases():
        xd = torch.from_numpy(x).to(dev)
        t0 = time.perf_counter()
        z = lossy.gzip_ranks(xd)
        t1 = time.perf_counter()
        ok_host = gzip.decompress(z) == x.tobytes()
        out = torch.full((x.nbytes + 64,), 7, dtype=torch.uint8, device=dev)
        try:
            got = lossy.gunzip_device(z, out)
            ok_dev = got.numel() == x.nbytes and got.cpu().numpy().tobytes() == x.tobytes() and bool(out[x.nbytes:].eq(7).all())
            err = None
        except _lib.CodecError as e:
            ok_dev, err = False, str(e)
        ref = len(gzip.compress(x.tobytes(), compresslevel=9))
        res[name] = {"n": int(x.size), "ok_host": ok_host, "ok_dev": ok_dev, "err": err,
                     "ratio": round(len(z) / x.nbytes, 5), "gzip9": round(ref / x.nbytes, 5),
                     "det": z == lossy.gzip_ranks(xd), "ms": round(1e3 * (t1 - t0), 2)}
        print(name, res[name], flush=True)
    if args.big:
        n = 1 << 28
        g = torch.Generator(device=dev).manual_seed(0)
        p = torch.tensor([0.074, 0.1816, 0.2444, 0.2444, 0.1816, 0.074], device=dev)
        x = torch.empty(n, dtype=torch.float32, device=dev)
        for o in range(0, n, 1 << 24):
            x[o:o + (1 << 24)] = torch.multinomial(p, 1 << 24, replacement=True, generator=g).to(torch.float32)
        out = torch.empty(4 * n + 64, dtype=torch.uint8, device=dev)
        L = _lib.lib()
        for it in range(4):
            L.ofl_gzip_profile(1)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            z = lossy.gzip_ranks(x)
            t1 = time.perf_counter()
            got = lossy.gunzip_device(z, out)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            names = ctypes_buf = None
            import ctypes
            nb = ctypes.create_string_buffer(4096)
            ms = np.zeros(16, np.float64)
            ln = np.zeros(16, np.int64)
            nk = ctypes.c_int()
            L.ofl_gzip_profile_collect(nb, 4096, ms.ctypes.data, ln.ctypes.data, 16, ctypes.byref(nk))
            names = nb.value.decode().split("\n")[:nk.value]
            ok = bool(torch.equal(got.view(torch.float32), x))
            print(json.dumps({"it": it, "ok": ok, "ratio": round(len(z) / (4 * n), 5), "gzip_ms": round(1e3 * (t1 - t0), 2),
                              "inflate_ms": round(1e3 * (t2 - t1), 2),
                              "kernels_ms": {k: round(float(v), 3) for k, v in zip(names, ms)},
                              "launches": {k: int(v) for k, v in zip(names, ln)}}), flush=True)
        L.ofl_gzip_profile(0)
        sample = x[:1 << 22].cpu().numpy().tobytes()
        print("gzip9 ratio (16 MiB sample):", len(gzip.compress(sample, 9)) / len(sample))
    bad = [k for k, v in res.items() if not (v["ok_host"] and v["ok_dev"] and v["det"])]
    print("FAILED" if bad else "ALL OK", bad)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
