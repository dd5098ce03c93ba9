#!/usr/bin/env python3
"""Device-resident KC / SKC / STC throughput (BASELINE.json config 2).

    python tools/lossy_bench.py [--workload uniform_1gib] [--steps K] [--warmup W]

config 2 is openfl-workspace/keras_cnn_with_compression (KCPipeline: k-means
k=6 + gzip, plan.yaml:43-47) on a 1 GiB fp32 tensor set.  One step = every
tensor through the device part of the pipeline's forward (k-means fit +
labels -> float32 ranks, the GZIPTransformer input) and backward (the
sequential key->value LUT, kc_pipeline.py:79-83), inputs resident in HBM.
gzip stays on the host and is not in the timed region.  SKC
and STC (top-k 10 % sparsify, then k-means / ternary) are timed the same way
and reported under "also".

Prints one JSON line: value = input GiB / step time; roofline from the bytes
the device passes move (each pass reads the tensor once; label/LUT passes
also write it) and from the pipeline's minimum I/O (read x + write ranks,
read ranks + write y); cpu_baseline = the reference's algorithm (sklearn
KMeans(n_clusters=6, n_init=6) + np.choose + _float_to_int, kc_pipeline.py:
47-63 restated) on a bounded sample of one tensor, host cores as stated.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PEAK_HBM_GBPS = 8000.0


class Arena:
    """The tensor set in one fp32 arena (tensor t at offsets[t])."""

    def __init__(self, xs):
        import torch
        self.numels = [x.numel() for x in xs]
        self.offsets, acc = [], 0
        for n in self.numels:
            self.offsets.append(acc)
            acc += (n + 63) // 64 * 64
        self.x = torch.zeros(acc, dtype=torch.float32, device=xs[0].device)
        for x, o in zip(xs, self.offsets):
            self.x[o:o + x.numel()] = x
        self.ranks = torch.empty_like(self.x)
        self.y = torch.empty_like(self.x)
        self.sparse = torch.empty_like(self.x)
        self.ks = [int(np.ceil(n * 0.1)) for n in self.numels]   # p_sparsity 0.1

    def view(self, a, t):
        return a[self.offsets[t]:self.offsets[t] + self.numels[t]]


def kc_step(ar, maps_out=None):
    """KCPipeline device part for the whole set: one batched k-means (fit +
    ranks) and one batched LUT decode."""
    from openfl_amd import lossy
    _, _, _, uniq = lossy.kmeans_batch(ar.x, ar.offsets, ar.numels, 6, n_init=6,
                                       seed=int(np.random.randint(0, 2 ** 31 - 1)), ranks_out=ar.ranks)
    maps = [{i: u for i, u in enumerate(uniq[t])} for t in range(len(ar.numels))]
    lossy.lut_decode_batch(ar.ranks, ar.offsets, ar.numels, maps, ar.y)
    if maps_out is not None:
        maps_out.extend(maps)
    return ar.y


def kc_plugin_step(xs):
    """The same through the per-tensor plugin path (KmeansTransformer._ranks, T = 1)."""
    from openfl_amd import lossy
    from openfl_amd.pipelines.lossy_common import kmeans_ranks
    for x in xs:
        ranks, m = kmeans_ranks(x, 6, np.float32)
        lossy.lut_decode(ranks, m)


def stc_step(ar):
    """STCPipeline.forward device part for the whole set (batched top-k, ternary
    ranks) + batched LUT decode; the ternary maps are O(1) host work per tensor."""
    from openfl_amd import lossy
    from openfl_amd.pipelines.stc_pipeline import ternary_map
    st = lossy.sparsify_topk_batch(ar.x, ar.offsets, ar.numels, ar.ks, ar.sparse)
    maps, r3 = [], []
    for t, n in enumerate(ar.numels):
        m, r = ternary_map(n, st["n_pos"][t], st["n_neg"][t], st["abs_sum"][t])
        maps.append(m)
        r3.append(r)
    lossy.ternary_ranks_batch(ar.sparse, ar.offsets, ar.numels, r3, ar.ranks)
    lossy.lut_decode_batch(ar.ranks, ar.offsets, ar.numels, maps, ar.y)
    return ar.y


def skc_step(ar):
    """SKCPipeline.forward device part for the whole set (batched top-k, batched
    k-means of the sparse vectors with float64 centre values) + LUT decode."""
    from openfl_amd import lossy
    lossy.sparsify_topk_batch(ar.x, ar.offsets, ar.numels, ar.ks, ar.sparse)
    _, _, _, uniq = lossy.kmeans_batch(ar.sparse, ar.offsets, ar.numels, 6, n_init=6,
                                       seed=int(np.random.randint(0, 2 ** 31 - 1)), value_f64=True,
                                       ranks_out=ar.ranks)
    maps = [{i: u for i, u in enumerate(uniq[t])} for t in range(len(ar.numels))]
    lossy.lut_decode_batch(ar.ranks, ar.offsets, ar.numels, maps, ar.y)
    return ar.y


def stc_plugin_step(xs):
    """STC per tensor (SparsityTransformer / TernaryTransformer plugin calls)."""
    from openfl_amd import lossy
    from openfl_amd.pipelines.stc_pipeline import ternary_map
    for x in xs:
        n = x.numel()
        sparse, st = lossy.sparsify_topk(x, int(np.ceil(n * 0.1)))
        m, (rn, rz, rp) = ternary_map(n, st["n_pos"], st["n_neg"], st["abs_sum"])
        lossy.lut_decode(lossy.ternary_ranks(sparse, rn, rz, rp), m)


def skc_plugin_step(xs):
    """SKC per tensor (SparsityTransformer / KmeansTransformer plugin calls)."""
    from openfl_amd import lossy
    from openfl_amd.pipelines.lossy_common import kmeans_ranks
    for x in xs:
        n = x.numel()
        sparse, _ = lossy.sparsify_topk(x, int(np.ceil(n * 0.1)))
        ranks, m = kmeans_ranks(sparse, 6, np.float64)
        lossy.lut_decode(ranks, m)


def timed(fn, xs, steps, warmup):
    import torch
    for _ in range(warmup):
        fn(xs)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn(xs)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def cpu_kc_reference(x, k=6):
    """kc_pipeline.KmeansTransformer.forward + backward (kc_pipeline.py:47-86),
    restated with the same libraries (sklearn, numpy)."""
    from sklearn import cluster
    data = x.reshape((-1, 1))
    km = cluster.KMeans(n_clusters=k, n_init=k)
    km.fit(data)
    quant = np.choose(km.labels_, km.cluster_centers_.squeeze())
    flat = quant.reshape(-1)
    uniq = np.unique(flat)
    ints = np.zeros(flat.shape, np.int32)
    for i, u in enumerate(uniq):
        ints[np.where(flat == u)] = i
    y = ints.astype(np.float32)
    for i, u in enumerate(uniq):
        y[y == i] = u
    return y


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="uniform_1gib")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--cpu-sample", type=int, default=1 << 20, help="elements of the CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--only", default="", help="comma list of kc,kc_plugin,stc,stc_plugin,skc,skc_plugin (default all)")
    args = ap.parse_args()

    import torch
    from openfl_amd.workloads import WORKLOADS, numel
    dev = torch.device("cuda", 0)
    shapes = WORKLOADS[args.workload]()
    g = torch.Generator(device=dev)
    xs = []
    for i, (_, s) in enumerate(shapes):
        g.manual_seed(i)
        xs.append(torch.empty(numel(s), dtype=torch.float32, device=dev).normal_(0.0, 0.01, generator=g))
    nbytes = 4 * sum(x.numel() for x in xs)
    np.random.seed(0)
    only = set(a for a in args.only.split(",") if a) or {"kc", "kc_plugin", "stc", "stc_plugin", "skc", "skc_plugin"}

    ar = Arena(xs)
    res = {}
    for name, fn, arg in (("kc", kc_step, ar), ("kc_plugin", kc_plugin_step, xs), ("stc", stc_step, ar),
                          ("stc_plugin", stc_plugin_step, xs), ("skc", skc_step, ar),
                          ("skc_plugin", skc_plugin_step, xs)):
        if name not in only:
            continue
        t = timed(fn, arg, args.steps, args.warmup)
        res[name] = {"value": round(nbytes / t / 2 ** 30, 3), "ms_per_step": round(1e3 * t, 3)}

    # GZIPTransformer on the KC ranks: GPU gzip of the whole set vs host gzip -9
    if "gzip" in only or not args.only:
        from openfl_amd import lossy
        import gzip as _gz
        kc_step(ar)
        torch.cuda.synchronize()
        z = lossy.gzip_ranks(ar.ranks)
        reps = 3
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            z = lossy.gzip_ranks(ar.ranks)
        t_gz = (time.perf_counter() - t0) / reps
        rb = ar.ranks[:1 << 22].cpu().numpy().tobytes()   # 16 MiB sample for the host reference
        t0 = time.perf_counter()
        zh = _gz.compress(rb, compresslevel=9)
        t_h = time.perf_counter() - t0
        res["gzip_device"] = {"value": round(4 * ar.ranks.numel() / t_gz / 2 ** 30, 3), "ms_per_call": round(1e3 * t_gz, 3),
                              "ratio": round(len(z) / (4 * ar.ranks.numel()), 4),
                              "note": "GB of float32 ranks (whole arena incl. alignment gaps) -> host bytes, D2H included"}
        res["gzip_host_level9"] = {"value": round(len(rb) / t_h / 2 ** 30, 4), "ratio": round(len(zh) / len(rb), 4),
                                   "sample": "16 MiB of the same ranks, gzip.compress(level 9), 1 thread"}

    # quality of the KC result (not timed)
    maps = []
    y = kc_step(ar, maps)
    rel = float(torch.linalg.vector_norm((y - ar.x).double()) / torch.linalg.vector_norm(ar.x.double()))

    cpu = None
    if not args.no_cpu_baseline:
        xh = xs[0][:args.cpu_sample].cpu().numpy()
        t0 = time.perf_counter()
        cpu_kc_reference(xh)
        dt = time.perf_counter() - t0
        cores = int(os.environ.get("OMP_NUM_THREADS", len(os.sched_getaffinity(0))))  # sklearn's OpenMP pool
        cpu = {"value": round(4 * xh.size / dt / 2 ** 30, 6), "unit": "GiB/s", "cores": cores, "kind": "port",
               "sample": f"{xh.size} elements of tensor 0 through sklearn KMeans(6, n_init=6) + np.choose + "
                         f"_float_to_int + LUT backward ({dt:.2f} s; sklearn/BLAS threads = host cores)"}

    kc = res.get("kc")
    out = {"metric": "GiB/s device-resident KC (k-means k=6) encode+decode, fp32 tensor set",
           "value": kc["value"] if kc else None, "unit": "GiB/s", "n_gpus": 1, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": kc["ms_per_step"] if kc else None, "higher_is_better": True,
           "dtype": "f32", "data": "synthetic: seeded N(0, 0.01^2) fp32, resident in HBM",
           "config": {"workload": args.workload, "tensors": len(xs), "bytes": nbytes,
                      "pipeline": "KCPipeline device part: one batched k-means (fit + float32 ranks) over the set, "
                                  "one batched LUT decode; gzip excluded"},
           "check_rel_l2_kc": round(rel, 5), "clusters_used": len(maps[0]),
           "roofline": None, "cpu_baseline": cpu,
           "also": {k: v for k, v in res.items() if k != "kc"}}
    if kc:
        t = kc["ms_per_step"] / 1e3
        io = 4 * nbytes  # read x + write ranks, read ranks + write y
        out["roofline"] = {"bound": "hbm", "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                           "achieved": round(io / t / 1e9, 1), "frac": round(io / t / 1e9 / PEAK_HBM_GBPS, 4),
                           "scope": "pipeline minimum I/O per step: 4n read + 4n ranks write (encode) + "
                                    "4n read + 4n write (decode); the k-means passes re-read x (see DESIGN.md)",
                           "traffic": None}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
