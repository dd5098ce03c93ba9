#!/usr/bin/env python3
"""Where the KC step's wall time goes between its timed phases (bench.py's
kc_uniform_1gib loop with a clock around every statement, including the
release of the previous step's stream)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from openfl_amd import lossy, hostmem
    from openfl_amd.workloads import WORKLOADS, numel
    if "--heap" in sys.argv:
        hostmem.keep_large_blocks()
    dev = torch.device("cuda", 0)
    shapes = WORKLOADS["uniform_1gib"]()
    numels = [numel(s) for _, s in shapes]
    offs = list(np.cumsum([0] + [(n + 63) // 64 * 64 for n in numels[:-1]]))
    tot = offs[-1] + numels[-1]
    x = torch.empty(tot, dtype=torch.float32, device=dev)
    g = torch.Generator(device=dev)
    for j, (o, n) in enumerate(zip(offs, numels)):
        g.manual_seed(j)
        x[o:o + n].normal_(0.0, 0.01, generator=g)
    ranks = torch.empty_like(x)
    y = torch.empty_like(x)
    rb = ranks.view(torch.uint8)
    rng = np.random.RandomState(7)
    clk = time.perf_counter
    ph = {}

    def add(k, dt):
        ph[k] = ph.get(k, 0.0) + dt

    z = None
    steps = 8
    for it in range(steps + 2):
        if it == 2:
            ph.clear()
            torch.cuda.synchronize()
            w0 = clk()
        t = [clk()]
        _, _, _, uniq = lossy.kmeans_batch(x, offs, numels, 6, n_init=6, seed=int(rng.randint(0, 2 ** 31 - 1)),
                                           ranks_out=ranks)
        t.append(clk())
        z_new = lossy.gzip_ranks(ranks)
        t.append(clk())
        z = None  # the previous step's stream released here
        t.append(clk())
        maps = [{i: u for i, u in enumerate(uq)} for uq in uniq]
        t.append(clk())
        lossy.gunzip_device(z_new, rb)
        t.append(clk())
        lossy.lut_decode_batch(ranks, offs, numels, maps, y)
        torch.cuda.synchronize()
        t.append(clk())
        z = z_new
        del z_new
        t.append(clk())
        for k, a, b in zip(("kmeans", "gzip", "free_prev", "maps", "inflate", "lut", "rebind"), t[:-1], t[1:]):
            add(k, b - a)
    torch.cuda.synchronize()
    wall = (clk() - w0) / steps
    out = {"ms_per_step": round(1e3 * wall, 3), "phases_ms": {k: round(1e3 * v / steps, 3) for k, v in ph.items()},
           "sum_ms": round(1e3 * sum(ph.values()) / steps, 3), "heap_policy": "--heap" in sys.argv,
           "stream_bytes": len(z)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
