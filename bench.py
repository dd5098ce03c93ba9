#!/usr/bin/env python3
"""Device-resident Eden encode+decode throughput (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload NAME]

One step = Eden-encode every tensor of the workload (fp32 arena in HBM ->
bit planes + scales in HBM) and decode them back (-> fp32 arena in HBM), the
per-round codec work of openfl/pipelines/eden_pipeline.py:555-659 for one
model update.  Inputs are resident before the timed region.

Multi-GPU (launched by torch.distributed.run, one rank per GPU): the path
shards with no data exchange, so every rank codes its own update set
("weak" scaling: one collaborator update per GPU; --scaling strong instead
LPT-partitions ONE set over the ranks).  The only collectives are the
barrier and the max-over-ranks of the timed region.

Prints ONE JSON line on rank 0 (fields documented in DESIGN.md section 6).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GiB/s device-resident Eden encode+decode, fp32 update tensors, 1/2/4/8 GPU"
PEAK_HBM_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def cpu_baseline(shapes, x_host_fn, n_bits, sample_mib):
    """The C oracle (oracle/eden_oracle.c, single thread) on a bounded sample
    of the same workload: leading tensors (after a leading embedding, if any)
    until sample_mib is reached."""
    from oracle import eden as O
    from openfl_amd.workloads import numel
    picked, tot = [], 0
    start = 1 if shapes and numel(shapes[0][1]) * 4 > 2 * sample_mib * 2 ** 20 else 0
    for i in range(start, len(shapes)):
        if tot >= sample_mib * 2 ** 20:
            break
        n = numel(shapes[i][1])
        if n * 4 > 2 * sample_mib * 2 ** 20:
            continue
        picked.append(i)
        tot += 4 * n
    t_enc = t_dec = 0.0
    for i in picked:
        x = x_host_fn(i)
        t0 = time.perf_counter()
        planes, scales, dims, total = O.compress(x, 4242, n_bits)
        t1 = time.perf_counter()
        O.decompress(planes, total, scales, dims, 4242, n_bits)
        t2 = time.perf_counter()
        t_enc += t1 - t0
        t_dec += t2 - t1
    gib = tot / 2 ** 30
    return {"value": round(gib / (t_enc + t_dec), 5), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"{len(picked)} tensors ({tot / 2 ** 20:.1f} MiB) of the same workload, "
                      f"oracle/eden_oracle.c single-threaded; enc {t_enc:.2f} s + dec {t_dec:.2f} s"}


def secondary(name, n_bits, steps, warmup, dev, wave_mib, streams):
    """One more workload on this GPU (same step definition, inputs resident):
    the north_star's 1 GiB set and BASELINE config 2 (ResNet-50) next to the
    main line.  Device time from events around the timed steps."""
    import torch
    from openfl_amd.codec import EdenPlan
    from openfl_amd.workloads import WORKLOADS, numel
    numels = [numel(s) for _, s in WORKLOADS[name]()]
    plan = EdenPlan(numels, n_bits, wave_mib=wave_mib, streams=streams)
    x = torch.empty(max(plan.arena_numel, 1), dtype=torch.float32, device=dev)
    gen = torch.Generator(device=dev)
    for j, n in enumerate(numels):
        gen.manual_seed(j)
        off = plan.elem_offsets[j]
        x[off:off + n].normal_(0.0, 0.01, generator=gen)
    y = torch.empty_like(x)
    planes = torch.empty(max(plan.planes_bytes, 1), dtype=torch.uint8, device=dev)
    scales = torch.empty(max(plan.n_slices, 1), dtype=torch.float32, device=dev)
    ws = torch.empty(max(plan.ws_bytes, 256), dtype=torch.uint8, device=dev)
    seeds = torch.tensor(np.random.RandomState(1234).randint(0, 2 ** 16, size=len(numels)), dtype=torch.int32,
                         device=dev)
    for _ in range(warmup):
        plan.encode(x, seeds, planes, scales, ws)
        plan.decode(planes, seeds, scales, y, ws)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(steps):
        plan.encode(x, seeds, planes, scales, ws)
        plan.decode(planes, seeds, scales, y, ws)
    ev1.record()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    gpu_s = ev0.elapsed_time(ev1) / 1e3
    alg = sum(l["bytes_alg"] for e in (True, False) for l in plan.launches(e))
    return {"value": round(4 * sum(numels) * steps / wall / 2 ** 30, 2), "unit": "GiB/s",
            "ms_per_step": round(1e3 * wall / steps, 4), "gpu_ms_per_step": round(1e3 * gpu_s / steps, 4),
            "roofline_frac": round(alg * steps / gpu_s / 1e9 / PEAK_HBM_GBPS, 4),
            "bytes": 4 * sum(numels), "tensors": len(numels), "slices": plan.n_slices, "waves": plan.n_waves,
            "streams": plan.n_streams, "steps": steps}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="llama3_8b_fp32_update")
    ap.add_argument("--n-bits", type=int, default=8)
    ap.add_argument("--scaling", choices=("weak", "strong"), default="weak")
    ap.add_argument("--cpu-sample-mib", type=float, default=384.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-events", action="store_true",
                    help="do not record per-launch HIP events in the timed region")
    ap.add_argument("--traffic-json", default=None,
                    help="rocprofv3 PMC-derived HBM bytes per step (tools/pmc_traffic.py output)")
    ap.add_argument("--wave-mib", type=float, default=None,
                    help="large-slice wave size (ofl_eden_plan_set_schedule; default: library's)")
    ap.add_argument("--streams", type=int, default=None, help="1 or 2 (default: library's)")
    ap.add_argument("--also", default="uniform_1gib,resnet50_fp32",
                    help="secondary workloads timed after the main one (rank 0 line, 'also'); '' = none")
    ap.add_argument("--also-steps", type=int, default=20)
    ap.add_argument("--profile-steps", type=int, default=3,
                    help="steps of the serialized per-kernel profile pass (two-stream schedules)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    import torch
    import torch.distributed as dist
    from openfl_amd.codec import EdenPlan
    from openfl_amd.sharding import max_over_ranks, shard_indices, throughput_gib_s
    from openfl_amd.workloads import WORKLOADS, numel

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    shapes = WORKLOADS[args.workload]()
    sizes = [numel(s) for _, s in shapes]
    mine = shard_indices(sizes, rank, world, args.scaling)
    numels = [sizes[i] for i in mine]
    plan = EdenPlan(numels, args.n_bits, wave_mib=args.wave_mib, streams=args.streams)

    # synthetic update: N(0, 0.01^2) fp32, seeded per (rank, tensor)
    x = torch.empty(max(plan.arena_numel, 1), dtype=torch.float32, device=dev)
    gen = torch.Generator(device=dev)
    for j, i in enumerate(mine):
        gen.manual_seed(1_000_003 * (rank if args.scaling == "weak" else 0) + i)
        off = plan.elem_offsets[j]
        x[off:off + numels[j]].normal_(0.0, 0.01, generator=gen)
    y = torch.empty_like(x)
    planes = torch.empty(max(plan.planes_bytes, 1), dtype=torch.uint8, device=dev)
    scales = torch.empty(max(plan.n_slices, 1), dtype=torch.float32, device=dev)
    ws = torch.empty(max(plan.ws_bytes, 256), dtype=torch.uint8, device=dev)
    rs = np.random.RandomState(1234 + rank)
    seeds = torch.tensor(rs.randint(0, 2 ** 16, size=len(numels)), dtype=torch.int32, device=dev)

    def step():
        plan.encode(x, seeds, planes, scales, ws)
        plan.decode(planes, seeds, scales, y, ws)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    # per-launch events inside the timed region only for a single-stream
    # schedule: with two streams a launch's events also span the other
    # stream's kernel it waits behind (a serialized profile pass follows)
    two = plan.n_streams == 2
    if not args.no_kernel_events and not two:
        plan.profile(True)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(args.steps):
        step()
    ev1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    gpu_ms = ev0.elapsed_time(ev1)
    elapsed = max_over_ranks(elapsed, dev)

    # per-kernel breakdown: events of the timed region (one stream), or of a
    # serialized profile pass over the same tensors (two streams)
    kernels = {}
    kernels_source = None
    if not args.no_kernel_events:
        pplan, pws = plan, ws
        if two:
            pplan = EdenPlan(numels, args.n_bits, wave_mib=args.wave_mib, streams=1)
            pws = torch.empty(max(pplan.ws_bytes, 256), dtype=torch.uint8, device=dev)
            pplan.encode(x, seeds, planes, scales, pws)
            pplan.decode(planes, seeds, scales, y, pws)
            torch.cuda.synchronize()
            pplan.profile(True)
            for _ in range(args.profile_steps):
                pplan.encode(x, seeds, planes, scales, pws)
                pplan.decode(planes, seeds, scales, y, pws)
            torch.cuda.synchronize()
            kernels_source = (f"serialized profile pass after the timed region: {args.profile_steps} steps of "
                              f"the same tensors on one stream ({pplan.n_waves} waves); HIP events around "
                              "every launch")
        else:
            kernels_source = "HIP events around every launch inside the timed region"
        for enc in (True, False):
            ms, calls = pplan.profile_collect(enc)
            for info, m in zip(pplan.launches(enc), ms):
                k = kernels.setdefault(info["name"], {"ms": 0.0, "launches": 0, "bytes_moved": 0,
                                                      "bytes_alg": 0})
                k["ms"] += float(m)
                k["launches"] += calls
                k["bytes_moved"] += info["bytes_moved"] * calls
                k["bytes_alg"] += info["bytes_alg"] * calls
        pplan.profile(False)
        if two:
            del pplan, pws

    # quality check (not timed): relative L2 error of decode(encode(x))
    with torch.no_grad():
        rel = float(torch.linalg.vector_norm((y - x).double()) / torch.linalg.vector_norm(x.double()))

    in_bytes_rank = 4 * sum(numels)
    value = throughput_gib_s(in_bytes_rank, world, args.steps, elapsed, args.scaling, 4 * sum(sizes))

    alg_step = sum(l["bytes_alg"] for e in (True, False) for l in plan.launches(e))
    step_s = gpu_ms / 1e3 / args.steps
    achieved = alg_step / step_s / 1e9
    traffic = None
    traffic_src = args.traffic_json
    if traffic_src is None and args.workload == "llama3_8b_fp32_update" and args.n_bits == 8 \
            and args.scaling == "weak":
        # PMC counters cannot be read from inside this process: default to the
        # committed rocprofv3 --pmc passes of this same workload (tools/pmc_run.sh)
        traffic_src = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles",
                                   "r01_llama3_8b_hbm_traffic_final.json")
    if traffic_src and os.path.exists(traffic_src):
        with open(traffic_src) as f:
            traffic = json.load(f).get("hbm_bytes_per_step")
    else:
        traffic_src = None
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBPS, "unit": "GB/s",
            "frac": round(achieved / PEAK_HBM_GBPS, 4), "traffic": traffic,
            "scope": "one codec step = every encode+decode launch; algorithmic bytes per step = "
                     "sum over tensors of 4n (x read) + b*P/8 (planes write) + b*P/8 (planes read) "
                     "+ 4n (y write) (SURVEY 8(d)); FWHT intermediates not counted",
            "alg_bytes_per_step": alg_step,
            "traffic_unit": "HBM bytes per step (2 x FETCH_SIZE + WRITE_SIZE, gfx950 correction)",
            "traffic_source": (os.path.relpath(traffic_src, os.path.dirname(os.path.abspath(__file__)))
                               + " (rocprofv3 --pmc passes of this workload, not this run)")
                              if traffic_src else None}
    if kernels:
        tot_ms = sum(k["ms"] for k in kernels.values())
        name, k = max(kernels.items(), key=lambda kv: kv[1]["ms"])
        avg_us = 1e3 * k["ms"] / k["launches"]
        roof["dominant_kernel"] = {
            "name": name, "avg_us": round(avg_us, 2), "launches": k["launches"],
            "share_of_step": round(k["ms"] / tot_ms, 3),
            "bytes_moved_per_launch": k["bytes_moved"] // k["launches"],
            "bytes_alg_per_launch": k["bytes_alg"] // k["launches"],
            "moved_GBps": round(k["bytes_moved"] / (k["ms"] / 1e3) / 1e9, 1),
            "moved_frac": round(k["bytes_moved"] / (k["ms"] / 1e3) / 1e9 / PEAK_HBM_GBPS, 4)}
        if traffic_src:
            with open(traffic_src) as f:
                pk = json.load(f).get("kernels", {}).get(name)
            if pk:  # PMC bytes per dispatch of the dominant kernel (same workload)
                roof["dominant_kernel"]["traffic_per_launch"] = (pk["read_bytes_per_dispatch"]
                                                                 + pk["write_bytes_per_dispatch"])
        roof["kernels_source"] = kernels_source
        roof["kernels"] = {n: {"avg_us": round(1e3 * v["ms"] / v["launches"], 2),
                               "share": round(v["ms"] / tot_ms, 3),
                               "moved_GBps": round(v["bytes_moved"] / max(v["ms"], 1e-9) / 1e6, 1)}
                           for n, v in sorted(kernels.items(), key=lambda kv: -kv[1]["ms"])}

    also = {}
    if world == 1 and args.also:
        for name in [a for a in args.also.split(",") if a]:
            also[name] = secondary(name, args.n_bits, args.also_steps, 3, dev, args.wave_mib, args.streams)

    out = None
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            def x_host(i):
                j = mine.index(i)
                off = plan.elem_offsets[j]
                return x[off:off + numels[j]].cpu().numpy()
            cpu = cpu_baseline(shapes, x_host, args.n_bits, args.cpu_sample_mib)
            cpu["cores"] = 1
        out = {
            "metric": METRIC, "value": round(value, 2), "unit": "GiB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: seeded N(0, 0.01^2) fp32 tensors of the workload's shapes, "
                    "resident in HBM; no checkpoint",
            "config": {"workload": args.workload, "tensors": len(numels), "numel_per_rank": sum(numels),
                       "bytes_per_rank": in_bytes_rank, "n_bits": args.n_bits, "slices": plan.n_slices,
                       "planes_bytes_per_rank": plan.planes_bytes, "waves": plan.n_waves,
                       "streams": plan.n_streams, "wave_mib": plan.wave_mib,
                       "parallelism": (f"{world} independent replicas, one update set per GPU"
                                       if args.scaling == "weak" else f"LPT-sharded over {world} GPUs")},
            "gpu_ms_per_step": round(gpu_ms / args.steps, 3),
            "check_rel_l2": round(rel, 6),
            "roofline": roof,
            "cpu_baseline": cpu,
            "also": also or None,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return out


if __name__ == "__main__":
    main()
