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
    ap.add_argument("--no-numa-bind", action="store_true")
    ap.add_argument("--extra-streams", type=int, default=0,
                    help="diagnostics: create and use this many torch streams first (HW queue sharing)")
    ap.add_argument("--ballast-gib", type=float, default=0.0,
                    help="diagnostics: hold this much device memory (written once) during the run")
    ap.add_argument("--hw-queues", type=int, default=0, help="GPU_MAX_HW_QUEUES to set (0: leave HIP's default)")
    args = ap.parse_args()
    if args.hw_queues > 0:
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.hw_queues)
    import torch
    import bench
    if args.hostmem:
        from openfl_amd.hostmem import keep_large_blocks
        if not keep_large_blocks():
            raise SystemExit("keep_large_blocks() is not available here")
    torch.cuda.set_device(0)
    cpus = None
    if not args.no_numa_bind:
        from openfl_amd import numa
        cpus = numa.bind_to_device(0)
    keep = []
    for _ in range(args.extra_streams):
        st = torch.cuda.Stream()
        with torch.cuda.stream(st):
            keep.append(torch.ones(1024, device="cuda:0") * 2)
        keep.append(st)
    torch.cuda.synchronize()
    ballast = None
    if args.ballast_gib > 0:
        ballast = torch.ones(int(args.ballast_gib * 2 ** 28), dtype=torch.float32, device="cuda:0")
        torch.cuda.synchronize()
    out = bench.kc_pipeline(args.steps, args.warmup, torch.device("cuda", 0), extras=False)
    out["hostmem_policy"] = bool(args.hostmem)
    out["ballast_gib"] = args.ballast_gib
    out["numa_cpus"] = f"{cpus[0]}-{cpus[-1]} ({len(cpus)})" if cpus else None
    out["GPU_MAX_HW_QUEUES"] = os.environ.get("GPU_MAX_HW_QUEUES")
    del ballast
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
