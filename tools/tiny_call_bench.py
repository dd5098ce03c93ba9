"""Latency of one-tensor plugin calls (EdenPipeline.forward / backward, what an
unchanged TensorCodec makes per tensor) by tensor size: microseconds per call."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from openfl_amd.pipelines import EdenPipeline  # noqa: E402

pipe = EdenPipeline(n_bits=8, dim_threshold=100, device="cuda:0")
res = {}
for n in (256, 2048, 1 << 15, 1 << 18, 1 << 21):
    x = (np.random.default_rng(n).standard_normal(n) * 0.01).astype(np.float32)
    reps = max(20, min(2000, (1 << 24) // n))
    for _ in range(5):
        d, md = pipe.forward(x)
        pipe.backward(d, list(md))
    t0 = time.perf_counter()
    for _ in range(reps):
        d, md = pipe.forward(x)
    t1 = time.perf_counter()
    for _ in range(reps):
        pipe.backward(d, list(md))
    t2 = time.perf_counter()
    res[n] = {"forward_us": round(1e6 * (t1 - t0) / reps, 1), "backward_us": round(1e6 * (t2 - t1) / reps, 1)}
print(json.dumps(res))
torch.cuda.synchronize()
