#!/usr/bin/env python3
"""KCPipeline forward+backward of the 1 GiB set alone (BASELINE config 3),
the steps of bench.py's kc_uniform_1gib line and nothing else, so that a
rocprofv3 --pmc pass over this process counts exactly (warmup + steps)
pipeline steps of KC kernels (tools/pmc_traffic.py KC_DIR STEPS+WARMUP).

    python tools/kc_bench.py [--steps 10] [--warmup 2] [--hostmem]

--hostmem: first apply the opt-in process-wide host-memory policy
(openfl_amd.hostmem.keep_large_blocks) and time the pipeline under it.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--hostmem", action="store_true")
    args = ap.parse_args()
    import torch
    import bench
    if args.hostmem:
        from openfl_amd.hostmem import keep_large_blocks
        if not keep_large_blocks():
            raise SystemExit("keep_large_blocks() is not available here")
    torch.cuda.set_device(0)
    out = bench.kc_pipeline(args.steps, args.warmup, torch.device("cuda", 0), extras=False)
    out["hostmem_policy"] = bool(args.hostmem)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
