"""Phase times of EdenPipeline.forward_batch / backward_batch internals on the
ResNet-50 set (host side of the batched end-to-end path): seed sums, staging
+ H2D, encode + D2H, bytes creation; decode likewise."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from e2e_bench import state_dict  # noqa: E402
from openfl_amd.pipelines import EdenPipeline  # noqa: E402
from openfl_amd.pipelines import eden_pipeline as E  # noqa: E402
from openfl_amd.workloads import WORKLOADS  # noqa: E402

sd = state_dict(WORKLOADS["resnet50_fp32"](), 100)
arrays = [a for _, a in sd]
pipe = EdenPipeline(n_bits=8, dim_threshold=100, device="cuda:0")
tr = pipe.transformers[0]
big = [i for i, a in enumerate(arrays) if a.size > 100]
for rep in range(4):
    torch.cuda.synchronize()
    t = [time.perf_counter()]
    sums = E._serial_sums([a.reshape(-1) for a in arrays]); t.append(time.perf_counter())
    staged = E._batch_stage(tr.eden, [arrays[i] for i in big]); torch.cuda.synchronize(); t.append(time.perf_counter())
    seeds = E.eden_seeds(sums)
    plan, flats, x = staged
    st = tr.eden._stream()
    ph = tr.eden._staging().get("planes", plan.planes_bytes, torch.uint8)
    with torch.cuda.stream(st):
        sdv = torch.tensor([seeds[i] for i in big], dtype=torch.int32).to(tr.eden.device)
        planes, scales = tr.eden.codec.encode_arena(plan, x, sdv, stream=st)
    st.synchronize(); t.append(time.perf_counter())
    with torch.cuda.stream(st):
        ph[:plan.planes_bytes].copy_(planes[:plan.planes_bytes], non_blocking=True)
    st.synchronize(); t.append(time.perf_counter())
    pn = ph.numpy()
    outs = [pn[plan.planes_offsets[k]:plan.planes_offsets[k] + plan.planes_nbytes[k]].tobytes() for k in range(len(big))]
    t.append(time.perf_counter())
    full = pipe.forward_batch(arrays); t.append(time.perf_counter())
    back = pipe.backward_batch(full); t.append(time.perf_counter())
    names = ["sums", "stage+H2D", "encode", "D2H planes", "bytes", "forward_batch total", "backward_batch total"]
    print({n: round(1e3 * (b - a), 2) for n, a, b in zip(names, t[:-1], t[1:])}, flush=True)
