"""A/B: one Eden step (encode + decode of a workload) enqueued launch by
launch vs replayed from a captured hipGraph (torch.cuda.CUDAGraph around
the C-ABI calls; the library's side-stream fork/join is captured as graph
edges).  Prints one JSON line per workload: device ms/step both ways and
whether the outputs are bit-identical.

    python tools/graph_ab.py [--workloads resnet50_fp32,uniform_1gib] [--steps 200]
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
from openfl_amd.workloads import WORKLOADS, numel  # noqa: E402


def run(name, steps, warmup, streams):
    dev = torch.device("cuda", 0)
    numels = [numel(s) for _, s in WORKLOADS[name]()]
    plan = EdenPlan(numels, 8, streams=streams)
    x = torch.empty(max(plan.arena_numel, 1), dtype=torch.float32, device=dev)
    g = torch.Generator(device=dev)
    for j, n in enumerate(numels):
        g.manual_seed(j)
        o = plan.elem_offsets[j]
        x[o:o + n].normal_(0.0, 0.01, generator=g)
    y = torch.zeros_like(x)
    # zero-filled: the alignment gaps between tensors' plane runs are never written
    planes = torch.zeros(max(plan.planes_bytes, 1), dtype=torch.uint8, device=dev)
    scales = torch.empty(max(plan.n_slices, 1), dtype=torch.float32, device=dev)
    ws = torch.empty(max(plan.ws_bytes, 256), dtype=torch.uint8, device=dev)
    seeds = torch.tensor(np.random.RandomState(1).randint(0, 2 ** 16, size=len(numels)), dtype=torch.int32,
                         device=dev)

    def step():
        plan.encode(x, seeds, planes, scales, ws)
        plan.decode(planes, seeds, scales, y, ws)

    def timed(fn):
        for _ in range(warmup):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        for _ in range(steps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / steps, 1e3 * (time.perf_counter() - t0) / steps

    eager_gpu, eager_wall = timed(step)
    y_eager, p_eager = y.clone(), planes.clone()
    y.zero_()
    planes.zero_()
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        step()
    graph.replay()
    torch.cuda.synchronize()
    same_after_first = bool(torch.equal(y, y_eager) and torch.equal(planes, p_eager))
    graph_gpu, graph_wall = timed(graph.replay)
    same = same_after_first and bool(torch.equal(y, y_eager) and torch.equal(planes, p_eager))
    nbytes = 4 * sum(numels)
    return {"workload": name, "streams": plan.n_streams, "launches": len(plan.launches(True)) + len(plan.launches(False)),
            "eager": {"gpu_ms": round(eager_gpu, 4), "wall_ms": round(eager_wall, 4),
                      "GiBps": round(nbytes / (eager_wall / 1e3) / 2 ** 30, 2)},
            "graph": {"gpu_ms": round(graph_gpu, 4), "wall_ms": round(graph_wall, 4),
                      "GiBps": round(nbytes / (graph_wall / 1e3) / 2 ** 30, 2)},
            "bit_identical": same, "steps": steps}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="resnet50_fp32,uniform_1gib")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--streams", type=int, default=0, help="0 = the plan's default schedule")
    a = ap.parse_args()
    for w in a.workloads.split(","):
        print(json.dumps(run(w, a.steps, a.warmup, a.streams or None)), flush=True)


if __name__ == "__main__":
    main()
