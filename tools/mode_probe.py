#!/usr/bin/env python3
"""The Llama line's two modes (~425 vs ~437 GiB/s, per process): does the
placement of the step's buffers decide it?  One process, one plan; each
trial allocates fresh x / y / planes / ws (after a pad allocation of a
varying size, so the buffers land on other physical pages) and times 6
steps.  Prints one line per trial and a JSON summary."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from openfl_amd.codec import EdenPlan  # noqa: E402
from openfl_amd.workloads import WORKLOADS, numel  # noqa: E402


def main():
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    dev = torch.device("cuda", 0)
    numels = [numel(s) for _, s in WORKLOADS["llama3_8b_fp32_update"]()]
    plan = EdenPlan(numels, 8)
    seeds = torch.tensor(np.random.RandomState(1).randint(0, 2 ** 16, size=len(numels)), dtype=torch.int32, device=dev)
    res = []
    for t in range(trials):
        pad = torch.empty((t * 37 % 11) * (3 << 20) + 1, dtype=torch.uint8, device=dev)
        x = torch.empty(plan.arena_numel, dtype=torch.float32, device=dev).normal_(0, 0.01)
        y = torch.empty_like(x)
        planes = torch.empty(plan.planes_bytes, dtype=torch.uint8, device=dev)
        scales = torch.empty(plan.n_slices, dtype=torch.float32, device=dev)
        ws = torch.empty(max(plan.ws_bytes, 256), dtype=torch.uint8, device=dev)
        for _ in range(2):
            plan.encode(x, seeds, planes, scales, ws)
            plan.decode(planes, seeds, scales, y, ws)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(6):
            plan.encode(x, seeds, planes, scales, ws)
            plan.decode(planes, seeds, scales, y, ws)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 6
        gib = 4 * sum(numels) / 2 ** 30 / (ms / 1e3)
        print(f"trial {t}: {ms:.3f} ms/step {gib:.1f} GiB/s (x at {x.data_ptr():#x}, ws at {ws.data_ptr():#x})", flush=True)
        res.append(ms)
        del x, y, planes, scales, ws, pad
        torch.cuda.empty_cache()
    print(json.dumps({"ms_per_step": [round(m, 3) for m in res]}))


if __name__ == "__main__":
    main()
