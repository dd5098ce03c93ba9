#!/usr/bin/env python3
"""Where a per-tensor plugin call's host time goes (EdenPipeline.forward /
backward on the ResNet-50 set, 2 rounds, the second timed): every native
call and host copy inside the call wrapped with a clock, summed per size
bucket.  Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch  # noqa: F401
    from openfl_amd import _lib, hostmem, protocols as P
    from openfl_amd.pipelines import EdenPipeline
    from openfl_amd.pipelines import eden_pipeline as EP
    from openfl_amd.workloads import WORKLOADS
    L = _lib.lib()
    acc = {}
    cur = {"b": ""}
    clk = time.perf_counter

    def wrap(owner, name, label):
        f = getattr(owner, name)

        def g(*a, **k):
            t0 = clk()
            try:
                return f(*a, **k)
            finally:
                key = f"{cur['b']} {label}"
                acc[key] = acc.get(key, 0.0) + clk() - t0
        setattr(owner, name, g)

    for n in ("ofl_copy_h2d_chunked", "ofl_eden_encode_seeded", "ofl_eden_decode_host", "ofl_eden_encode_host",
              "ofl_eden_encode_mapped", "ofl_eden_decode_mapped", "ofl_serial_sum_copy_f32"):
        if hasattr(L, n):
            wrap(L, n, n)
    wrap(hostmem, "bytes_from", "bytes_from")
    wrap(hostmem, "array_from", "array_from")
    shapes = WORKLOADS["resnet50_fp32"]()
    rng = np.random.default_rng(1)
    sd = [(nm, rng.standard_normal(s, dtype=np.float32) * np.float32(0.01)) for nm, s in shapes]
    pipe = EdenPipeline(n_bits=8, dim_threshold=100, device="cuda:0")

    def bucket(n):
        return "<=100" if n <= 100 else "<=2^15" if n <= 1 << 15 else "<=2^18" if n <= 1 << 18 else ">2^18"
    for r in range(3):
        if r == 2:
            acc.clear()
        tot = {}
        for name, a in sd:
            cur["b"] = "fwd " + bucket(a.size)
            t0 = clk()
            data, md = pipe.forward(a)
            t1 = clk()
            b = P.construct_named_tensor((name, "col", 1, False, ("trained",)), data, md, False).SerializeToString()
            t2 = clk()
            nt = P.NamedTensor()
            nt.ParseFromString(b)
            mdd = P.transformer_metadata_of(nt)
            cur["b"] = "bwd " + bucket(a.size)
            t3 = clk()
            pipe.backward(nt.data_bytes, mdd)
            t4 = clk()
            for k, v in ((f"fwd {bucket(a.size)} total", t1 - t0), ("protobuf build", t2 - t1),
                         ("protobuf parse", t3 - t2), (f"bwd {bucket(a.size)} total", t4 - t3)):
                tot[k] = tot.get(k, 0.0) + v
    out = {"totals_ms": {k: round(1e3 * v, 3) for k, v in sorted(tot.items())},
           "inside_ms": {k: round(1e3 * v, 3) for k, v in sorted(acc.items())}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
