"""Host enqueue rate vs GPU time per step (is a workload launch-bound?).
Times N step() enqueues without synchronising, then the drain."""
import sys, time
import numpy as np
import torch
sys.path.insert(0, ".")
from openfl_amd.codec import EdenPlan
from openfl_amd.workloads import WORKLOADS, numel

wl = sys.argv[1] if len(sys.argv) > 1 else "resnet50_fp32"
sizes = [numel(s) for _, s in WORKLOADS[wl]()]
plan = EdenPlan(sizes, 8)
dev = torch.device("cuda", 0)
x = torch.randn(max(plan.arena_numel, 1), device=dev) * 0.01
y = torch.empty_like(x)
planes = torch.empty(plan.planes_bytes, dtype=torch.uint8, device=dev)
scales = torch.empty(plan.n_slices, dtype=torch.float32, device=dev)
ws = torch.empty(max(plan.ws_bytes, 256), dtype=torch.uint8, device=dev)
seeds = torch.tensor(np.random.RandomState(1).randint(0, 2 ** 16, len(sizes)), dtype=torch.int32, device=dev)
for _ in range(5):
    plan.encode(x, seeds, planes, scales, ws); plan.decode(planes, seeds, scales, y, ws)
torch.cuda.synchronize()
for n in (20, 100):
    t0 = time.perf_counter()
    for _ in range(n):
        plan.encode(x, seeds, planes, scales, ws); plan.decode(planes, seeds, scales, y, ws)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{wl} steps={n} host enqueue {1e6*(t1-t0)/n:.1f} us/step, total {1e6*(t2-t0)/n:.1f} us/step, "
          f"launches/step {len(plan.launches(True)) + len(plan.launches(False))}")
