"""Where the ResNet-50 step goes: the step of the whole set vs its large
tensors alone (every slice > 2^15, the wave streams) vs its small tensors
alone (the small-slice stream), eager and graph-replayed.
  python tools/resnet_split.py [steps]"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openfl_amd.codec import EdenPlan, EdenStepGraph  # noqa: E402
from openfl_amd.workloads import WORKLOADS, numel  # noqa: E402


def step_time(numels, steps, graph):
    dev = torch.device("cuda:0")
    plan = EdenPlan(numels, 8)
    x = torch.randn(max(plan.arena_numel, 1), device=dev) * 0.01
    y = torch.empty_like(x)
    planes = torch.empty(max(plan.planes_bytes, 1), dtype=torch.uint8, device=dev)
    scales = torch.empty(max(plan.n_slices, 1), dtype=torch.float32, device=dev)
    ws = torch.empty(max(plan.ws_bytes, 256), dtype=torch.uint8, device=dev)
    seeds = torch.tensor(np.random.RandomState(1).randint(0, 2 ** 16, size=len(numels)), dtype=torch.int32,
                         device=dev)
    if graph:
        g = EdenStepGraph(plan, x, seeds, planes, scales, y, ws)
        run = g.replay
    else:
        def run():
            plan.encode(x, seeds, planes, scales, ws)
            plan.decode(planes, seeds, scales, y, ws)
    for _ in range(10):
        run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        run()
    torch.cuda.synchronize()
    return 1e6 * (time.perf_counter() - t0) / steps


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    numels = [numel(s) for _, s in WORKLOADS["resnet50_fp32"]()]
    big = [n for n in numels if n > 36045]       # every slice > 2^15 (greedy slicing, 10 % pad rule)
    small = [n for n in numels if n <= 36045]
    if len(sys.argv) > 2 and sys.argv[2] == "large":  # one eager run of the large tensors (for a kernel trace)
        print(json.dumps({"large_only_us": round(step_time(big, steps, False), 1)}))
        return
    out = {}
    for tag, ns in (("all", numels), ("large_only", big), ("small_only", small)):
        for graph in (False, True):
            out[f"{tag}{'_graph' if graph else ''}_us"] = round(step_time(ns, steps, graph), 1)
    out["tensors"] = {"all": len(numels), "large": len(big), "small": len(small)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
