"""Where a one-tensor plugin call's time goes.

For each size: EdenPipeline.forward / backward per call (reference and fast
seed modes), the native floor of the same call (ofl_eden_encode_host /
ofl_eden_decode_host in a loop on prepared buffers: H2D, launches, D2H, sync,
no Python around it), and for n = 2048 a cProfile of the plugin calls.
Prints one JSON object (microseconds per call)."""
import cProfile
import io
import json
import os
import pstats
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from openfl_amd import _lib  # noqa: E402
from openfl_amd.pipelines import EdenPipeline  # noqa: E402
from openfl_amd.pipelines.eden_pipeline import _al256  # noqa: E402


def per_call(fn, reps):
    for _ in range(5):
        fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return 1e6 * (time.perf_counter() - t0) / reps


def native_floor(eden, x):
    """The encode / decode host calls alone, buffers prepared once."""
    n = x.size
    plan = eden.codec.plan([n], streams=1)
    pb, ns = plan.planes_bytes, plan.n_slices
    off_seeds = _al256(4 * plan.arena_numel)
    in_bytes = off_seeds + 4
    off_scales = _al256(pb)
    out_bytes = off_scales + 4 * ns
    ih = torch.empty(in_bytes, dtype=torch.uint8).pin_memory()
    oh = torch.empty(out_bytes, dtype=torch.uint8).pin_memory()
    ih.numpy()[:4 * n].view(np.float32)[:] = x
    idev = torch.empty(in_bytes, dtype=torch.uint8, device=eden.device)
    odev = torch.empty(out_bytes, dtype=torch.uint8, device=eden.device)
    ws = eden.codec.ws.get(plan.ws_bytes, eden.device)
    st = torch.cuda.Stream(device=eden.device)
    L = _lib.lib()
    args = (plan.handle, ih.data_ptr(), idev.data_ptr(), in_bytes, off_seeds, odev.data_ptr(), oh.data_ptr(),
            out_bytes, off_scales, ws.data_ptr(), ws.numel(), st.cuda_stream)
    enc = per_call(lambda: L.ofl_eden_encode_host(*args), max(50, min(3000, (1 << 23) // max(n, 1))))
    # decode: planes + scales + seed
    off_s2 = _al256(pb)
    off_seed2 = _al256(off_s2 + 4 * ns)
    in2 = off_seed2 + 4
    ih2 = torch.zeros(in2, dtype=torch.uint8).pin_memory()
    idev2 = torch.empty(in2, dtype=torch.uint8, device=eden.device)
    ydev = torch.empty(max(plan.arena_numel, 1), dtype=torch.float32, device=eden.device)
    y = np.empty(n, np.float32)
    args2 = (plan.handle, ih2.data_ptr(), idev2.data_ptr(), in2, off_s2, off_seed2, ydev.data_ptr(), y.ctypes.data,
             4 * n, ws.data_ptr(), ws.numel(), st.cuda_stream)
    dec = per_call(lambda: L.ofl_eden_decode_host(*args2), max(50, min(3000, (1 << 23) // max(n, 1))))
    return enc, dec


def main():
    out = {}
    for mode in ("reference", "fast"):
        pipe = EdenPipeline(n_bits=8, dim_threshold=100, device="cuda:0", seed_mode=mode)
        res = {}
        for n in (256, 2048, 1 << 15, 1 << 18, 1 << 21):
            x = (np.random.default_rng(n).standard_normal(n) * 0.01).astype(np.float32)
            reps = max(20, min(2000, (1 << 24) // n))
            d, md = pipe.forward(x)
            f = per_call(lambda: pipe.forward(x), reps)
            b = per_call(lambda: pipe.backward(d, [dict(md[0])]), reps)
            r = {"forward_us": round(f, 1), "backward_us": round(b, 1)}
            if mode == "reference":
                ne, nd = native_floor(pipe.transformers[0].eden, x)
                r.update({"native_encode_host_us": round(ne, 1), "native_decode_host_us": round(nd, 1)})
            res[n] = r
        out[mode] = res
    # cProfile of the plugin calls at n = 2048 (reference seeds)
    pipe = EdenPipeline(n_bits=8, dim_threshold=100, device="cuda:0")
    x = (np.random.default_rng(1).standard_normal(2048) * 0.01).astype(np.float32)
    d, md = pipe.forward(x)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(2000):
        d, md = pipe.forward(x)
        pipe.backward(d, list(md))
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(18)
    out["cprofile_2048"] = s.getvalue().splitlines()[:40]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
