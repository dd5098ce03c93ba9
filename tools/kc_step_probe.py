"""Where the KC step's host-visible time goes (GPU box): the bench's KC loop
(tools/kc_bench.py / bench.kc_pipeline) with the library calls inside
lossy.gzip_ranks and lossy.gunzip_device timed one by one (wall clock of
each ctypes call and of hostmem.bytes_from).

  python tools/kc_step_probe.py [--steps 8]
"""
import argparse
import collections
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=8)
    args = ap.parse_args()
    import torch
    from openfl_amd import _lib, hostmem, lossy
    acc = collections.defaultdict(float)
    real = _lib.lib()

    class Timed:
        def __getattr__(self, name):
            f = getattr(real, name)
            if name not in ("ofl_gzip_ranks", "ofl_gzip_ranks_to", "ofl_gzip_member_index", "ofl_inflate_tlz", "ofl_copy_h2d_staged"):
                return f

            def w(*a):
                t0 = time.perf_counter()
                r = f(*a)
                acc[name] += time.perf_counter() - t0
                return r
            return w
    timed = Timed()
    _lib.lib = lambda: timed
    bf = hostmem.bytes_from

    def bytes_from(*a, **k):
        t0 = time.perf_counter()
        r = bf(*a, **k)
        acc["hostmem.bytes_from"] += time.perf_counter() - t0
        return r
    hostmem.bytes_from = bytes_from
    import bench
    dev = torch.device("cuda", 0)
    out = bench.kc_pipeline(2, 1, dev, extras=False)  # warm
    acc.clear()
    out = bench.kc_pipeline(args.steps, 0, dev, extras=False)
    res = {"kc_line": {k: out[k] for k in ("value", "ms_per_step", "phases_ms")},
           "ms_per_step_by_call": {k: round(1e3 * v / args.steps, 3) for k, v in sorted(acc.items())},
           "note": "wall time of each call on the calling thread; ofl_copy_h2d_staged runs on a pool "
                   "thread beside ofl_gzip_member_index"}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
