"""Where a large one-tensor plugin call's time goes:
per size, microseconds per call of
  fwd_ref / fwd_fast   EdenPipeline.forward (reference / fast seed)
  bwd                  EdenPipeline.backward
  sum_mt               the exact serial sum alone (ofl_serial_sum_f32_mt)
  copy_sum             ofl_copy_h2d_chunked with the sum + stream sync
  copy_nosum           the same without the sum
  bytes_from           hostmem.bytes_from of the planes' size (fresh bytes)
  array_from           hostmem.array_from of the tensor (fresh array)
Each call on one of 6 distinct arrays in turn (a model's tensors are
different arrays).  Prints one JSON object."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from openfl_amd import _lib, hostmem  # noqa: E402
from openfl_amd.pipelines import EdenPipeline  # noqa: E402


def per_call(fn, reps):
    for i in range(3):
        fn(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(reps):
        fn(i)
    torch.cuda.synchronize()
    return round(1e6 * (time.perf_counter() - t0) / reps, 1)


def main():
    L = _lib.lib()
    dev = "cuda:0"
    out = {}
    for n in (1 << 18, 1 << 20, 1 << 21, 2359296):
        xs = [np.random.default_rng(k).standard_normal(n).astype(np.float32) * np.float32(0.01) for k in range(6)]
        ref = EdenPipeline(n_bits=8, dim_threshold=100, device=dev)
        fast = EdenPipeline(n_bits=8, dim_threshold=100, device=dev, seed_mode="fast")
        pays = [ref.forward(x) for x in xs]
        r = {}
        r["fwd_ref"] = per_call(lambda i: ref.forward(xs[i % 6]), 30)
        r["fwd_fast"] = per_call(lambda i: fast.forward(xs[i % 6]), 30)

        def bwd(i):
            p, md = pays[i % 6]
            ref.backward(p, [dict(m) for m in md])
        r["bwd"] = per_call(bwd, 30)
        r["sum_mt"] = per_call(lambda i: L.ofl_serial_sum_f32_mt(xs[i % 6].ctypes.data, n, None, 0), 30)
        pin = torch.empty(4 * n, dtype=torch.uint8, pin_memory=True)
        d = torch.empty(4 * n, dtype=torch.uint8, device=dev)
        st = torch.cuda.current_stream().cuda_stream
        import ctypes
        s = ctypes.c_float()

        def cp(i, want):
            _lib.check(L.ofl_copy_h2d_chunked(xs[i % 6].ctypes.data, pin.data_ptr(), d.data_ptr(), n, 1 << 18, want,
                                              ctypes.byref(s), st))
            torch.cuda.current_stream().synchronize()
        r["copy_sum"] = per_call(lambda i: cp(i, 1), 30)
        r["copy_nosum"] = per_call(lambda i: cp(i, 0), 30)
        r["bytes_from"] = per_call(lambda i: hostmem.bytes_from(pin.data_ptr(), n), 30)
        r["array_from"] = per_call(lambda i: hostmem.array_from(pin.data_ptr(), n, np.float32), 30)
        out[str(n)] = r
        print(n, r, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
