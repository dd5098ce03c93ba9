"""Strong-scaling rehearsal on ONE GPU: every rank's shard of the Llama-3-8B
update (bench.py --scaling strong: LPT weighted by bytes x passes,
openfl_amd/sharding.py) timed alone, back to back.  The path shards with no
exchange, so an N-GPU step takes max over ranks of these times (plus the
barrier); prints per-rank ms/step and the implied whole-job GiB/s and
efficiency against N = 1.  An estimate for the driver's 8-GPU run, not a
replacement for it.

    python tools/shard_sim.py [--ranks 1,2,4,8] [--steps 5]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from openfl_amd.codec import EdenPlan  # noqa: E402
from openfl_amd.sharding import shard_indices  # noqa: E402
from openfl_amd.workloads import WORKLOADS, numel  # noqa: E402


def time_shard(sizes, idx, steps, warmup, dev):
    numels = [sizes[i] for i in idx]
    plan = EdenPlan(numels, 8)
    x = torch.empty(max(plan.arena_numel, 1), dtype=torch.float32, device=dev)
    g = torch.Generator(device=dev)
    for j, i in enumerate(idx):
        g.manual_seed(i)
        o = plan.elem_offsets[j]
        x[o:o + numels[j]].normal_(0.0, 0.01, generator=g)
    y = torch.empty_like(x)
    planes = torch.empty(max(plan.planes_bytes, 1), dtype=torch.uint8, device=dev)
    scales = torch.empty(max(plan.n_slices, 1), dtype=torch.float32, device=dev)
    ws = torch.empty(max(plan.ws_bytes, 256), dtype=torch.uint8, device=dev)
    seeds = torch.tensor(np.random.RandomState(7).randint(0, 2 ** 16, size=len(numels)), dtype=torch.int32,
                         device=dev)
    for _ in range(warmup):
        plan.encode(x, seeds, planes, scales, ws)
        plan.decode(planes, seeds, scales, y, ws)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        plan.encode(x, seeds, planes, scales, ws)
        plan.decode(planes, seeds, scales, y, ws)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    del x, y, planes, scales, ws
    torch.cuda.empty_cache()
    return dt, 4 * sum(numels)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="llama3_8b_fp32_update")
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    sizes = [numel(s) for _, s in WORKLOADS[a.workload]()]
    total = 4 * sum(sizes)
    base = None
    for n in [int(v) for v in a.ranks.split(",")]:
        per = []
        for r in range(n):
            dt, b = time_shard(sizes, shard_indices(sizes, r, n, "strong"), a.steps, a.warmup, dev)
            per.append((round(1e3 * dt, 3), b))
        t = max(ms for ms, _ in per) / 1e3
        v = total / t / 2 ** 30
        base = base or v
        print(json.dumps({"ranks": n, "per_rank_ms": [ms for ms, _ in per], "per_rank_GiB": [round(b / 2 ** 30, 2) for _, b in per],
                          "implied_GiBps": round(v, 1), "efficiency_vs_1": round(v / (n * base), 3)}), flush=True)


if __name__ == "__main__":
    main()
