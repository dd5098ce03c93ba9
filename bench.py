#!/usr/bin/env python3
"""Device-resident Eden encode+decode throughput (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload NAME]

One step = Eden-encode every tensor of the workload (fp32 arena in HBM ->
bit planes + scales in HBM) and decode them back (-> fp32 arena in HBM), the
per-round codec work of openfl/pipelines/eden_pipeline.py:555-659 for one
model update.  Inputs are resident before the timed region.

Multi-GPU: one process per GPU.  `--gpus N` with N > 1 started directly
spawns N ranks (torch.distributed.run, 127.0.0.1) before anything touches a
GPU; under torch.distributed.run (WORLD_SIZE set) the ranks run as launched.
The default is "strong" scaling -- ONE update set (BASELINE config 4: one
Llama-3-8B update) LPT-partitioned over the ranks per tensor, the unit the
aggregator codes (aggregator.py:816 compress, :826 decompress), balanced by
the bytes each tensor's passes move (openfl_amd.sharding.tensor_cost).
`--scaling weak` gives every rank its own set instead.  The path shards with
no data exchange: the only collectives are the barriers around the timed
region and the max over ranks of its duration.

`--dry-run` runs the sharding and the rank plumbing only (no GPU, gloo).

Prints ONE JSON line on rank 0 (fields documented in DESIGN.md section 4).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GiB/s device-resident Eden encode+decode, fp32 update tensors, 1/2/4/8 GPU"
PEAK_HBM_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
DEFAULT_ALSO = "uniform_1gib,resnet50_fp32,kc_uniform_1gib"


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="llama3_8b_fp32_update")
    ap.add_argument("--n-bits", type=int, default=8)
    ap.add_argument("--scaling", choices=("weak", "strong"), default="strong")
    ap.add_argument("--cpu-budget-s", type=float, default=15.0,
                    help="CPU baseline: oracle time budget on the main workload's tensors")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--numa-bind", action="store_true",
                    help="bind the process to the GPU's NUMA node (openfl_amd.numa); default: the OS placement")
    ap.add_argument("--no-numa-bind", action="store_true", help=argparse.SUPPRESS)  # the default (older scripts)
    ap.add_argument("--no-kc-numa-variant", action="store_true",
                    help="skip the KC line's NUMA-bound variant (tools/kc_bench.py in a child process)")
    ap.add_argument("--hw-queues", type=int, default=0,
                    help="set GPU_MAX_HW_QUEUES before the HIP runtime starts (0 = leave the environment's / "
                         "HIP's default of 4); recorded in the line's host_env")
    ap.add_argument("--no-kernel-events", action="store_true",
                    help="do not record per-launch HIP events in the timed region")
    ap.add_argument("--traffic-json", default=None,
                    help="rocprofv3 PMC-derived HBM bytes per step (tools/pmc_traffic.py output)")
    ap.add_argument("--wave-mib", type=float, default=None,
                    help="large-slice wave size (ofl_eden_plan_set_schedule; default: library's)")
    ap.add_argument("--streams", type=int, default=None, help="1 or 2 (default: library's)")
    ap.add_argument("--also", default=DEFAULT_ALSO,
                    help="secondary workloads timed after the main one (rank 0 line, 'also'); '' = none")
    ap.add_argument("--also-steps", type=int, default=20)
    ap.add_argument("--profile-steps", type=int, default=3,
                    help="steps of the serialized per-kernel profile pass (two-stream schedules)")
    ap.add_argument("--dry-run", action="store_true", help="sharding + rank plumbing only (CPU, gloo)")
    ap.add_argument("--master-port", type=int, default=0)
    return ap.parse_args(argv)


# --------------------------------------------------------------- launcher ---
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n, argv, port=0):
    """Run this script as n ranks under torch.distributed.run (127.0.0.1) and
    return its exit code.  Called before this process touches a GPU: the
    ranks are children, nothing is exec'd over a GPU-initialised process."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port or _free_port()),
           os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


# ---------------------------------------------------------- CPU baselines ---
def _oracle_threads():
    from oracle import eden as O
    cores = O.host_cores()
    O.set_threads(cores)
    return O, cores


def cpu_baseline(shapes, x_host_fn, n_bits, budget_s, indices=None):
    """The C oracle (oracle/eden_oracle.c, OpenMP over the host cores this
    process may use) on the workload's tensors in order until budget_s of
    CPU time has been spent (tensors above 1 GiB are left out; the Llama
    embedding alone would take the whole budget)."""
    from openfl_amd.workloads import numel
    O, cores = _oracle_threads()
    idx = list(range(len(shapes))) if indices is None else list(indices)
    picked, skipped, tot, t_enc, t_dec = [], [], 0, 0.0, 0.0
    for i in idx:
        if t_enc + t_dec >= budget_s:
            break
        n = numel(shapes[i][1])
        if 4 * n > 2 ** 30:
            skipped.append(shapes[i][0])
            continue
        x = x_host_fn(i)
        t0 = time.perf_counter()
        planes, scales, dims, total = O.compress(x, 4242, n_bits)
        t1 = time.perf_counter()
        O.decompress(planes, total, scales, dims, 4242, n_bits)
        t2 = time.perf_counter()
        t_enc += t1 - t0
        t_dec += t2 - t1
        picked.append(i)
        tot += 4 * n
    full = len(picked) == len(idx)
    what = "the whole set" if full else (f"tensors {picked[0]}..{picked[-1]} in workload order "
                                         f"({len(picked)} of {len(idx)}; skipped >1 GiB: {skipped or 'none'})")
    return {"value": round(tot / 2 ** 30 / (t_enc + t_dec), 5), "unit": "GiB/s", "cores": cores, "kind": "port",
            "sample": f"{what}, {tot / 2 ** 20:.1f} MiB; oracle/eden_oracle.c with {cores} OpenMP threads; "
                      f"enc {t_enc:.2f} s + dec {t_dec:.2f} s"}


# --------------------------------------------------- secondary workloads ---
def _fill_arena(plan, numels, dev, seed0=0):
    import torch
    x = torch.empty(max(plan.arena_numel, 1), dtype=torch.float32, device=dev)
    gen = torch.Generator(device=dev)
    for j, n in enumerate(numels):
        gen.manual_seed(seed0 + j)
        off = plan.elem_offsets[j]
        x[off:off + n].normal_(0.0, 0.01, generator=gen)
    return x


def secondary(name, n_bits, steps, warmup, dev, wave_mib, streams, cpu=False, graph=False):
    """One more workload on this GPU (same step definition, inputs resident):
    the north_star's 1 GiB set and BASELINE config 2 (ResNet-50) next to the
    main line.  Device time from events around the timed steps.  cpu=True
    also times the C oracle on the WHOLE set (all host cores)."""
    import torch
    from openfl_amd.codec import EdenPlan
    from openfl_amd.workloads import WORKLOADS, numel
    shapes = WORKLOADS[name]()
    numels = [numel(s) for _, s in shapes]
    plan = EdenPlan(numels, n_bits, wave_mib=wave_mib, streams=streams)
    x = _fill_arena(plan, numels, dev)
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
    out = {"value": round(4 * sum(numels) * steps / wall / 2 ** 30, 2), "unit": "GiB/s",
           "ms_per_step": round(1e3 * wall / steps, 4), "gpu_ms_per_step": round(1e3 * gpu_s / steps, 4),
           "roofline_frac": round(alg * steps / gpu_s / 1e9 / PEAK_HBM_GBPS, 4),
           "bytes": 4 * sum(numels), "tensors": len(numels), "slices": plan.n_slices, "waves": plan.n_waves,
           "streams": plan.n_streams, "steps": steps}
    if graph:
        # the same step replayed from a captured hipGraph (EdenStepGraph):
        # every launch of the step, submitted as one graph
        from openfl_amd.codec import EdenStepGraph
        g = EdenStepGraph(plan, x, seeds, planes, scales, y, ws)
        for _ in range(warmup):
            g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev0.record()
        for _ in range(steps):
            g.replay()
        ev1.record()
        torch.cuda.synchronize()
        gw = time.perf_counter() - t0
        gg = ev0.elapsed_time(ev1) / 1e3
        out["graph"] = {"value": round(4 * sum(numels) * steps / gw / 2 ** 30, 2),
                        "ms_per_step": round(1e3 * gw / steps, 4), "gpu_ms_per_step": round(1e3 * gg / steps, 4),
                        "roofline_frac": round(alg * steps / gg / 1e9 / PEAK_HBM_GBPS, 4),
                        "scope": "the same encode+decode step replayed from a captured hipGraph"}
    if cpu:
        def x_host(i):
            off = plan.elem_offsets[i]
            return x[off:off + numels[i]].cpu().numpy()
        out["cpu_baseline"] = cpu_baseline(shapes, x_host, n_bits, budget_s=float("inf"))
    return out


def _newest_profile(*names):
    """The first of the committed profile files that exists (newest round first)."""
    paths = [os.path.join(ROOT, "profiles", n) for n in names]
    return next((p for p in paths if os.path.exists(p)), paths[-1])


KC_TRAFFIC_JSON = _newest_profile("r06_final_kc_pipeline_hbm_traffic.json", "r05_final_kc_pipeline_hbm_traffic.json")
KC_SQ_JSON = _newest_profile("r06_final_kc_sq.json", "r05_final_kc_sq.json")


def _valu_busy(sq):
    """VALU issue share of a dispatch from rocprofv3 SQ counters (means per
    dispatch): wave64 VALU instructions x 4 cycles over the 1024 SIMDs,
    against SQ_BUSY_CYCLES summed over the 32 shader engines (8 XCDs x 4)."""
    if not sq or not sq.get("SQ_BUSY_CYCLES"):
        return None
    return round(sq["SQ_INSTS_VALU"] * 4 / 1024 / (sq["SQ_BUSY_CYCLES"] / 32), 3)


def _kc_kernel_profile(encode, decode, dev, steps=2):
    """Per-kernel time of the KC step, measured: HIP events around every
    gzip / inflate launch inside the library (ofl_gzip_profile) and torch
    events around the k-means and LUT calls (several small kernels each), in
    a serialized pass right after the timed region.  -> {name: {...}}."""
    import ctypes
    import torch
    from openfl_amd import _lib
    L = _lib.lib()
    calls = {}

    def timed(name, fn, *a, **kw):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r = fn(*a, **kw)
        e1.record()
        calls.setdefault(name, []).append((e0, e1))
        return r
    _lib.check_gzip(L.ofl_gzip_profile(1))
    try:
        for _ in range(steps):
            decode(*encode(timed), timed)
        torch.cuda.synchronize()
        names = ctypes.create_string_buffer(8192)
        ms = np.zeros(64, np.float64)
        ln = np.zeros(64, np.int64)
        nk = ctypes.c_int()
        _lib.check_gzip(L.ofl_gzip_profile_collect(names, 8192, ms.ctypes.data, ln.ctypes.data, 64, ctypes.byref(nk)))
    finally:
        L.ofl_gzip_profile(0)
    out = {}
    for name, t, k in zip(names.value.decode().split("\n")[:nk.value], ms, ln):
        out[name] = {"ms_per_step": float(t) / steps, "launches_per_step": int(k) / steps, "avg_us": 1e3 * float(t) / max(int(k), 1)}
    for name, evs in calls.items():
        t = sum(a.elapsed_time(b) for a, b in evs)
        out[name] = {"ms_per_step": t / steps, "launches_per_step": len(evs) / steps, "avg_us": 1e3 * t / len(evs),
                     "note": "one library call of several kernels (torch events around the call)"}
    return {k: {kk: (round(vv, 3) if isinstance(vv, float) else vv) for kk, vv in v.items()} for k, v in out.items()}


def kc_pipeline(steps, warmup, dev, extras=True):
    """KCPipeline (keras_cnn_with_compression, BASELINE config 3: k-means k=6
    + GZIPTransformer, kc_pipeline.py:36-63, :128-156, :160-181) on the 1 GiB
    set, gzip INCLUDED.  encode: batched device k-means -> device gzip of the
    float32 ranks, labelled inside the encoder (member-indexed stream, D2H of
    the compressed bytes); decode:
    H2D of the compressed bytes -> device inflate straight into y with the
    tensors' LUTs fused into its stores (phase "lut": building the tables on
    the host and their H2D).  Also: the device part alone, the host
    inflate (16 native threads + H2D of the ranks) and the host gzip -9
    compressor (the reference's GZIPTransformer.forward) timed on a sample.
    extras=False: the pipeline steps only (tools/kc_bench.py, the PMC passes:
    every step launches the same kernels, so dispatches per step are exact)."""
    import torch
    from oracle import eden as O  # host_cores only
    from openfl_amd import lossy
    from openfl_amd.workloads import WORKLOADS, numel
    cores = O.host_cores()
    shapes = WORKLOADS["uniform_1gib"]()
    numels = [numel(s) for _, s in shapes]
    offs = list(np.cumsum([0] + [(n + 63) // 64 * 64 for n in numels[:-1]]))
    tot = offs[-1] + numels[-1]
    x = torch.empty(tot, dtype=torch.float32, device=dev)
    g = torch.Generator(device=dev)
    for j, (o, n) in enumerate(zip(offs, numels)):
        g.manual_seed(j)
        x[o:o + n].normal_(0.0, 0.01, generator=g)
    ranks = torch.empty_like(x)
    y = torch.empty_like(x)
    stage = torch.empty(4 * tot, dtype=torch.uint8).pin_memory()
    stage_np = stage.numpy()
    rng = np.random.RandomState(7)
    ph = {"kmeans": 0.0, "gzip": 0.0, "inflate": 0.0, "lut": 0.0}
    y_bytes = y.view(torch.uint8)

    def plain(name, fn, *a, **kw):
        return fn(*a, **kw)

    tab = lossy.LabelTable(len(numels), dev)

    def encode(call=plain):
        # k-means -> each tensor's labelling rule (LabelTable); the device
        # gzip labels the values as it loads them, so the rank array of the
        # reference's KmeansTransformer output is never written to HBM
        t0 = time.perf_counter()
        _, _, _, uniq = call("lossy::kmeans_batch", lossy.kmeans_batch, x, offs, numels, 6, n_init=6,
                             seed=int(rng.randint(0, 2 ** 31 - 1)), label_out=tab)
        t1 = time.perf_counter()
        z = lossy.gzip_ranks(x, label=tab)
        t2 = time.perf_counter()
        ph["kmeans"] += t1 - t0
        ph["gzip"] += t2 - t1
        return z, [{i: u for i, u in enumerate(uq)} for uq in uniq]

    def decode(z, maps, call=plain):
        # H2D of the stream, device inflate with the tensors' LUTs fused into
        # its stores (lossy.lut_tables: each map applied to every rank), y
        t0 = time.perf_counter()
        lut = call("lossy::lut_tables", lossy.lut_tables, offs, numels, maps, dev)
        t1 = time.perf_counter()
        lossy.gunzip_device(z, y_bytes, lut=lut)
        torch.cuda.synchronize()
        ph["lut"] += t1 - t0
        ph["inflate"] += time.perf_counter() - t1

    for _ in range(warmup):
        decode(*encode())
    for k in ph:
        ph[k] = 0.0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        z, maps = encode()
        decode(z, maps)
    wall = (time.perf_counter() - t0) / steps
    # quality of the timed path itself: y of the last timed step (label-fused
    # encode -> pipelined LUT-fused inflate), before anything below rewrites y
    rel = float(torch.linalg.vector_norm((y - x).double()) / torch.linalg.vector_norm(x.double()))
    phases = {k: round(1e3 * v / steps, 3) for k, v in ph.items()}
    nbytes = 4 * sum(numels)
    # roofline of the pipeline step: its minimum I/O, the Eden line's
    # definition carried over -- read x (4n), write the gzip
    # stream, read it back, write y (4n); k-means passes, the rank arrays and
    # the inflate's output are intermediates and not counted
    alg = 2 * nbytes + 2 * len(z)
    roof = {"bound": "hbm", "achieved": round(alg / wall / 1e9, 1), "peak": PEAK_HBM_GBPS, "unit": "GB/s",
            "frac": round(alg / wall / 1e9 / PEAK_HBM_GBPS, 5), "alg_bytes_per_step": alg, "traffic": None,
            "scope": "KC step = forward + backward of the set (wall time, gzip and inflate included); "
                     "algorithmic bytes = 4n x read + stream write + stream read + 4n y write"}
    name = None
    if extras:  # (the PMC passes of tools/kc_bench.py count the timed steps' dispatches only)
        kern = _kc_kernel_profile(encode, decode, dev)
        name = max(kern, key=lambda k: kern[k]["ms_per_step"])
        roof["dominant_kernel"] = dict(kern[name], name=name,
                                       source="HIP events in a serialized profile pass after the timed region")
        roof["kernels"] = kern
    if os.path.exists(KC_TRAFFIC_JSON):
        with open(KC_TRAFFIC_JSON) as f:
            tj = json.load(f)
        roof["traffic"] = tj.get("hbm_bytes_per_step")
        roof["traffic_unit"] = "HBM bytes per step (2 x FETCH_SIZE + WRITE_SIZE, gfx950 correction)"
        roof["traffic_source"] = (os.path.relpath(KC_TRAFFIC_JSON, ROOT)
                                  + " (rocprofv3 --pmc passes of tools/kc_bench.py, KC kernels only, not this run)")
        # PMC bytes per dispatch of the dominant kernel (the traffic file's names
        # carry the namespace, e.g. gz::tlz::k_tlz_encode for tlz::k_tlz_encode)
        kern_pmc = tj.get("kernels") or {}
        pk = next((v for k, v in kern_pmc.items() if name and (k == name or k.endswith("::" + name))), None)
        if pk:
            roof["dominant_kernel"]["traffic_per_launch"] = pk["read_bytes_per_dispatch"] + pk["write_bytes_per_dispatch"]
    if name and os.path.exists(KC_SQ_JSON):
        # the dominant kernel is compute-bound, not HBM-bound: its VALU issue
        # share from the committed SQ counter passes (tools/r05_evidence.sh b)
        with open(KC_SQ_JSON) as f:
            sq_all = json.load(f)
        sq = next((v for k, v in sq_all.items() if k.split("(")[0].endswith(name.split("(")[0])), None)
        vb = _valu_busy(sq)
        if vb is not None:
            roof["dominant_kernel"]["valu_busy"] = vb
            roof["dominant_kernel"]["limiter"] = ("VALU issue (rocprofv3 SQ_INSTS_VALU / SQ_BUSY_CYCLES, "
                                                  + os.path.relpath(KC_SQ_JSON, ROOT) + ", not this run)")
    if not extras:
        return {"value": round(nbytes / wall / 2 ** 30, 3), "unit": "GiB/s", "ms_per_step": round(1e3 * wall, 3),
                "phases_ms": phases, "wire_ratio": round(len(z) / nbytes, 4), "roofline": roof,
                "check_rel_l2": round(rel, 5), "tensors": len(numels), "bytes": nbytes, "steps": steps,
                "warmup": warmup}
    # device part alone (k-means + ranks, LUT decode; the previous KC line)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        _, _, _, uniq = lossy.kmeans_batch(x, offs, numels, 6, n_init=6, seed=int(rng.randint(0, 2 ** 31 - 1)),
                                           ranks_out=ranks)
        lossy.lut_decode_batch(ranks, offs, numels, [{i: u for i, u in enumerate(uq)} for uq in uniq], y)
    torch.cuda.synchronize()
    dev_only = (time.perf_counter() - t0) / steps
    rel_dev = float(torch.linalg.vector_norm((y - x).double()) / torch.linalg.vector_norm(x.double()))
    # host gzip -9 (the reference compressor) on a 4-tensor sample of the ranks, all host cores
    sample = ranks[:4 * numels[0]].cpu().numpy().tobytes()
    t0 = time.perf_counter()
    zh = lossy.gzip_compress(sample, 9, cores)
    t_h = time.perf_counter() - t0
    host_gz_gibs = len(sample) / t_h / 2 ** 30
    t_host_pipe = wall - ph["gzip"] / steps + nbytes / (host_gz_gibs * 2 ** 30)
    # (the opt-in host-memory policy, openfl_amd.hostmem.keep_large_blocks,
    # is process-wide, so it is not applied here: tools/kc_bench.py --hostmem
    # times it in a process of its own)
    # cpu_baseline: the restated CPU pipeline (oracle/kc.py: sklearn KMeans
    # k=6 n_init=6 -> ranks -> gzip -9, then gunzip -> LUT, per tensor as the
    # reference calls it) on a bounded sample -- the first KC_CPU_SAMPLE
    # elements of the first four tensors -- extrapolated linearly to the set
    cpu = kc_cpu_baseline(x, offs, numels, cores)
    # host inflate variant (native threads into pinned staging, then H2D of the ranks)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    lossy.gunzip(z, cores, out=stage_np)
    ranks.copy_(stage.view(torch.float32)[:tot], non_blocking=True)
    torch.cuda.synchronize()
    t_host_inflate = time.perf_counter() - t0
    return {"value": round(nbytes / wall / 2 ** 30, 3), "unit": "GiB/s", "ms_per_step": round(1e3 * wall, 3),
            "phases_ms": phases, "roofline": roof,
            "wire_ratio": round(len(z) / nbytes, 4), "check_rel_l2": round(rel, 5),
            "check_rel_l2_scope": "y of the last timed step (label-fused encode, pipelined LUT-fused inflate)",
            "device_only": {"value": round(nbytes / dev_only / 2 ** 30, 2), "ms_per_step": round(1e3 * dev_only, 3),
                            "check_rel_l2": round(rel_dev, 5),
                            "scope": "batched k-means fit + ranks and LUT decode, no gzip"},
            "host_gzip9_variant": {"value": round(nbytes / t_host_pipe / 2 ** 30, 4),
                                   "gzip9_GiBps": round(host_gz_gibs, 4), "ratio": round(len(zh) / len(sample), 4),
                                   "sample": f"gzip -9 of 4 tensors' ranks (64 MiB) on {cores} threads, "
                                             "extrapolated to the set in place of the device gzip"},
            "host_inflate_variant": {"inflate_h2d_ms": round(1e3 * t_host_inflate, 3),
                                     "scope": f"ofl_gunzip_members on {cores} host threads + H2D of the ranks, "
                                              "in place of the device inflate"},
            "cpu_baseline": cpu,
            "tensors": len(numels), "bytes": nbytes, "steps": steps, "host_threads": cores,
            "scope": "KCPipeline forward+backward of the set, gzip in the timed region (one member-indexed "
                     "stream for the arena; each tensor's payload is its run of members)"}


def kc_numa_variant(steps=10, warmup=2):
    """The KC pipeline steps (tools/kc_bench.py: the same composition as the
    line) in a child process bound to the GPU's NUMA node, for the line's
    numa_bound_variant; this process stays on the OS placement."""
    env = dict(os.environ)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "kc_bench.py"), "--steps", str(steps),
                        "--warmup", str(warmup)], env=env, capture_output=True, text=True, timeout=300)
    try:
        d = json.loads(r.stdout.strip().splitlines()[-1])
    except (ValueError, IndexError):
        return {"error": f"tools/kc_bench.py rc={r.returncode}: {r.stderr[-300:]}"}
    return {"value": d["value"], "unit": "GiB/s", "ms_per_step": d["ms_per_step"], "phases_ms": d["phases_ms"],
            "wire_ratio": d["wire_ratio"], "numa_cpus": d.get("numa_cpus"),
            "scope": "the same KC steps in a child process bound to the GPU's NUMA node (tools/kc_bench.py)"}


KC_CPU_SAMPLE = 1 << 18  # elements per sampled tensor (4 tensors: 4 MiB, ~10-20 s of CPU work)


def kc_cpu_baseline(x, offs, numels, cores, per=KC_CPU_SAMPLE, ntens=4):
    """The restated KC pipeline (oracle/kc.py) timed on the host on a bounded
    sample: the first `per` elements of the first `ntens` tensors of the set,
    each as one tensor through forward + backward, in order.  sklearn's KMeans
    runs on its OpenMP threads (OMP_NUM_THREADS, 16 on the GPU box), gzip -9 on
    one thread, as in the reference.  The rate extrapolates linearly to the
    set (every tensor of the set has the same size and distribution)."""
    from oracle import kc as K
    sample = [x[offs[j]:offs[j] + min(per, numels[j])].cpu().numpy() for j in range(min(ntens, len(numels)))]
    t_f, t_b, zb = K.time_pipeline(sample)
    nb = sum(4 * s.size for s in sample)
    return {"value": round(nb / 2 ** 30 / (t_f + t_b), 6), "unit": "GiB/s", "cores": cores, "kind": "port",
            "sample": f"first {per} elements of tensors 0..{len(sample) - 1} ({nb / 2 ** 20:.1f} MiB) through "
                      f"oracle/kc.py (sklearn KMeans k=6 n_init=6 on {cores} OpenMP threads, ranks, gzip -9 and "
                      f"gunzip single-threaded, LUT) as the reference's per-tensor calls; forward {t_f:.2f} s, "
                      f"backward {t_b:.2f} s, wire ratio {zb / nb:.4f}; extrapolated linearly to the 1 GiB set"}


# ---------------------------------------------------------------- dry run ---
def dry_run(args, rank, world):
    import torch.distributed as dist
    from openfl_amd.sharding import imbalance, lpt_partition, shard_indices, tensor_cost
    from openfl_amd.workloads import WORKLOADS, numel
    if world > 1:
        dist.init_process_group("gloo")
    sizes = [numel(s) for _, s in WORKLOADS[args.workload]()]
    mine = shard_indices(sizes, rank, world, args.scaling)
    gathered = [mine]
    if world > 1:
        gathered = [None] * world
        dist.all_gather_object(gathered, mine)
    out = None
    if rank == 0:
        flat = sorted(i for g in gathered for i in g)
        out = {"dry_run": True, "n_gpus": world, "gpus_arg": args.gpus, "scaling": args.scaling,
               "workload": args.workload, "tensors": len(sizes),
               "covered": flat == list(range(len(sizes))) if args.scaling == "strong" else
               all(sorted(g) == list(range(len(sizes))) for g in gathered),
               "per_rank_tensors": [len(g) for g in gathered],
               "imbalance": round(imbalance(sizes, gathered), 4) if args.scaling == "strong" else 1.0,
               "imbalance_8": round(imbalance(sizes, lpt_partition(sizes, 8, tensor_cost)), 4)}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return out


# ------------------------------------------------------------------- main ---
def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    if args.hw_queues > 0:  # before anything starts the HIP runtime (the first torch.cuda call)
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.hw_queues)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(args.gpus, argv, args.master_port)
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus and rank == 0:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}; measuring {world} ranks", file=sys.stderr)
    if args.dry_run:
        dry_run(args, rank, world)
        return 0

    import torch
    import torch.distributed as dist
    from openfl_amd.codec import EdenPlan
    from openfl_amd.sharding import max_over_ranks, shard_indices, throughput_gib_s
    from openfl_amd.workloads import WORKLOADS, numel

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # Host placement: the OS's by default.  Binding to the GPU's NUMA node
    # (--numa-bind) speeds the host-heavy KC pipeline up (~52 vs ~48 GiB/s)
    # but measured slower on the device-resident Eden step (422-425 vs 425-438
    # GiB/s, profiles/r06_env_ab.txt), so the line runs unbound and the KC
    # entry carries a bound variant measured in a child process.
    numa_cpus = None
    if args.numa_bind and not args.no_numa_bind:
        from openfl_amd import numa
        numa_cpus = numa.bind_to_device(local)
    # the process placement every number of this line was measured under
    host_env = {"GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES"),
                "GPU_MAX_HW_QUEUES_source": ("bench.py --hw-queues" if args.hw_queues > 0 else
                                             "environment" if "GPU_MAX_HW_QUEUES" in os.environ else
                                             "unset (HIP default, 4)"),
                "numa_bind": (f"CPUs {numa_cpus[0]}-{numa_cpus[-1]} ({len(numa_cpus)}) of the GPU's node"
                              if numa_cpus else "none (OS placement)" if not args.numa_bind else
                              "no node found (unbound)")}
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
    seeds = torch.tensor(rs.randint(0, 2 ** 16, size=max(len(numels), 1)), dtype=torch.int32, device=dev)

    def step():
        if numels:
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
    if not args.no_kernel_events and numels:
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
        rel = float(torch.linalg.vector_norm((y - x).double()) / torch.linalg.vector_norm(x.double())) \
            if numels else 0.0

    in_bytes_rank = 4 * sum(numels)
    value = throughput_gib_s(in_bytes_rank, world, args.steps, elapsed, args.scaling, 4 * sum(sizes))

    alg_step = sum(l["bytes_alg"] for e in (True, False) for l in plan.launches(e))
    step_s = gpu_ms / 1e3 / args.steps
    achieved = alg_step / step_s / 1e9 if step_s > 0 else 0.0
    traffic = None
    traffic_src = args.traffic_json
    default_sched = (args.wave_mib is None and args.streams is None
                     and not any(k.startswith("OFL_EDEN_") for k in os.environ))
    if traffic_src is None and args.workload == "llama3_8b_fp32_update" and args.n_bits == 8 \
            and world == 1 and default_sched:
        # PMC counters cannot be read from inside this process: the committed
        # rocprofv3 --pmc passes of this same workload and default schedule
        # (tools/pmc_run.sh), only when this run uses that schedule
        traffic_src = _newest_profile("r06_final_llama3_8b_hbm_traffic.json", "r05_final_llama3_8b_hbm_traffic.json")
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
            "traffic_source": (os.path.relpath(traffic_src, ROOT)
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
            "alg_GBps": round(k["bytes_alg"] / (k["ms"] / 1e3) / 1e9, 1),
            "alg_frac": round(k["bytes_alg"] / (k["ms"] / 1e3) / 1e9 / PEAK_HBM_GBPS, 4),
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
            if name == "kc_uniform_1gib":
                also[name] = kc_pipeline(max(10, args.also_steps // 2), 4, dev)
                if not args.no_kc_numa_variant and not numa_cpus:
                    also[name]["numa_bound_variant"] = kc_numa_variant()
            else:
                # a ResNet-50 step is ~0.35 ms: more steps for a stable rate
                st = max(args.also_steps, 200) if name == "resnet50_fp32" else args.also_steps
                also[name] = secondary(name, args.n_bits, st, 3, dev, args.wave_mib, args.streams,
                                       cpu=(name == "uniform_1gib" and not args.no_cpu_baseline), graph=True)

    out = None
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            def x_host(i):
                j = mine.index(i)
                off = plan.elem_offsets[j]
                return x[off:off + numels[j]].cpu().numpy()
            cpu = cpu_baseline(shapes, x_host, args.n_bits, args.cpu_budget_s, indices=mine)
        out = {
            "metric": METRIC, "value": round(value, 2), "unit": "GiB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: seeded N(0, 0.01^2) fp32 tensors of the workload's shapes, "
                    "resident in HBM; no checkpoint",
            "config": {"workload": args.workload, "tensors": len(sizes), "tensors_rank0": len(numels),
                       "set_bytes": 4 * sum(sizes), "bytes_rank0": in_bytes_rank, "n_bits": args.n_bits,
                       "slices_rank0": plan.n_slices, "planes_bytes_rank0": plan.planes_bytes,
                       "waves": plan.n_waves, "streams": plan.n_streams, "wave_mib": plan.wave_mib,
                       "parallelism": (f"{world} independent replicas, one update set per GPU"
                                       if args.scaling == "weak" else
                                       f"one update set, per-tensor LPT shards over {world} GPU(s)")},
            "gpu_ms_per_step_rank0": round(gpu_ms / args.steps, 3),
            "check_rel_l2": round(rel, 6),
            "roofline": roof,
            "cpu_baseline": cpu,
            "host_env": host_env,
            "also": also or None,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
