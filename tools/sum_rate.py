#!/usr/bin/env python3
"""Rate of the reference seed's serial float32 sum (eden_pipeline.py:771):
the plain left-to-right chain vs its exact multi-threaded evaluation
(csrc/serial_sum.cpp), on update-like data (N(0, 0.01^2), zero mean: the
partial sums random-walk and cross binades often) and biased data."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openfl_amd import _lib  # noqa: E402


def main():
    L = _lib.lib()
    rng = np.random.default_rng(0)
    res = {}
    for dist in ("N(0,.01)", "N(.001,.01)"):
        for lg in (18, 21, 23, 26):
            n = 1 << lg
            x = (rng.standard_normal(n) * 0.01 + (0.001 if dist != "N(0,.01)" else 0.0)).astype(np.float32)
            row = {}
            want = None
            for th in (1, 4, 8, 16):
                reps = max(3, min(50, (1 << 24) // n))
                L.ofl_serial_sum_f32_mt(x.ctypes.data, n, None, th)
                t0 = time.perf_counter()
                for _ in range(reps):
                    v = L.ofl_serial_sum_f32_mt(x.ctypes.data, n, None, th)
                dt = (time.perf_counter() - t0) / reps
                want = v if want is None else want
                assert np.float32(v).tobytes() == np.float32(want).tobytes()
                row[f"threads_{th}_ns_per_elem"] = round(dt / n * 1e9, 4)
            res[f"{dist} 2^{lg}"] = row
            print(f"{dist} 2^{lg}: {row}", flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
