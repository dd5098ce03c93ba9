"""The exact serial sum's phases on this host (OFL_SUM_DEBUG=1 prints A / B /
C and the serial sub-chunks of each call): N(0, 0.01) tensors of 2^20,
2^21 and 2359296 elements at 8 and 16 threads."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openfl_amd import _lib  # noqa: E402

L = _lib.lib()
for n in (1 << 20, 1 << 21, 2359296):
    xs = [(np.random.default_rng(k).standard_normal(n) * 0.01).astype(np.float32) for k in range(4)]
    for th in (1, 8, 16):
        for x in xs:
            L.ofl_serial_sum_f32_mt(x.ctypes.data, n, None, th)
        t0 = time.perf_counter()
        for _ in range(5):
            for x in xs:
                L.ofl_serial_sum_f32_mt(x.ctypes.data, n, None, th)
        print(f"n={n} threads={th} {1e6 * (time.perf_counter() - t0) / 20:.1f} us/call", flush=True)
