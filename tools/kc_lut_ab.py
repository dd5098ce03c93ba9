"""A/B of the KC decode on the 1 GiB set, same process: the payload's H2D +
device inflate + lut_decode_batch (unfused) against the inflate with the LUT
fused into its stores (lossy.lut_tables).  Alternated, 10 rounds each; prints
one JSON line with the per-variant medians (ms) and the kernel times."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openfl_amd import _lib, lossy  # noqa: E402
from openfl_amd.workloads import WORKLOADS, numel  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    shapes = WORKLOADS["uniform_1gib"]()
    numels = [numel(s) for _, s in shapes]
    offs = list(np.cumsum([0] + [(n + 63) // 64 * 64 for n in numels[:-1]]))
    tot = offs[-1] + numels[-1]
    x = torch.empty(tot, dtype=torch.float32, device=dev)
    for j, (o, n) in enumerate(zip(offs, numels)):
        g = torch.Generator(device=dev)
        g.manual_seed(j)
        x[o:o + n].normal_(0.0, 0.01, generator=g)
    ranks = torch.empty_like(x)
    _, _, _, uniq = lossy.kmeans_batch(x, offs, numels, 6, n_init=6, seed=7, ranks_out=ranks)
    maps = [{i: u for i, u in enumerate(uq)} for uq in uniq]
    z = lossy.gzip_ranks(ranks)
    y = torch.empty_like(x)
    yb = y.view(torch.uint8)

    def unfused():
        lossy.gunzip_device(z, yb)
        lossy.lut_decode_batch(y, offs, numels, maps, y)

    def fused():
        lossy.gunzip_device(z, yb, lut=lossy.lut_tables(offs, numels, maps, dev))
    res = {"unfused": [], "fused": []}
    outs = {}
    for r in range(12):
        for name, fn in (("unfused", unfused), ("fused", fused)):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            if r >= 2:
                res[name].append(1e3 * (time.perf_counter() - t0))
            outs[name] = y.clone() if r == 11 else None
    same = all(bool(torch.equal(outs["fused"][o:o + n], outs["unfused"][o:o + n])) for o, n in zip(offs, numels))
    print(json.dumps({k: round(float(np.median(v)), 3) for k, v in res.items()} | {"identical": same,
                                                                                     "stream_bytes": len(z)}))


if __name__ == "__main__":
    main()
