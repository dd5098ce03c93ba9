#!/usr/bin/env python3
"""End-to-end loopback round (BASELINE config 5): 2 collaborators each send a
ResNet-50-shaped fp32 update; per tensor: host ndarray -> Eden encode ->
NamedTensor protobuf bytes -> parse -> Eden decode -> host ndarray.

Modes (wall-clock, both collaborators; every mode runs --rounds rounds and
reports the median of the rounds after the first, with every round's time in
round_s):
  plugin   openfl_amd.pipelines.EdenPipeline per tensor (what TensorCodec calls):
           H2D + encode + D2H per tensor, then H2D + decode + D2H per tensor
  plugin_concurrent  the same per-tensor calls with every collaborator on its
           own thread, as the gRPC server runs them
  batched  EdenPipeline.forward_batch / backward_batch over the whole state
           dict: seeds' serial sums on host threads, one pinned H2D, one
           encode launch sequence, one D2H of the planes arena; the receiver
           does one H2D of all payloads, one decode, one D2H (also with
           seed_mode="fast": "batched_fast_seed")
  cpu      the C oracle (oracle/eden_oracle.c, on all host cores) in the same flow
           (the CPU pipeline timed beside it; test infrastructure)
Prints one JSON line (also written to --out).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def state_dict(shapes, seed):
    rng = np.random.default_rng(seed)
    return [(n, (rng.standard_normal(s, dtype=np.float32) * np.float32(0.01))) for n, s in shapes]


def _bucket(n):
    return "<=100" if n <= 100 else "<=2^15" if n <= 1 << 15 else "<=2^18" if n <= 1 << 18 else ">2^18"


def run_plugin(sd, pipe, P, phases=None):
    """phases: dict to accumulate seconds per (phase, size bucket) into."""
    clk = time.perf_counter
    wire = []
    for name, arr in sd:
        t0 = clk()
        data, md = pipe.forward(arr)
        t1 = clk()
        wire.append(P.construct_named_tensor((name, "col", 1, False, ("trained",)), data, md,
                                             False).SerializeToString())
        if phases is not None:
            k = _bucket(arr.size)
            phases["forward " + k] = phases.get("forward " + k, 0.0) + t1 - t0
            phases["protobuf build"] = phases.get("protobuf build", 0.0) + clk() - t1
    out = []
    for b, (_, arr) in zip(wire, sd):
        t0 = clk()
        nt = P.NamedTensor()
        nt.ParseFromString(b)
        md = P.transformer_metadata_of(nt)
        t1 = clk()
        out.append(pipe.backward(nt.data_bytes, md))
        if phases is not None:
            k = _bucket(arr.size)
            phases["protobuf parse"] = phases.get("protobuf parse", 0.0) + t1 - t0
            phases["backward " + k] = phases.get("backward " + k, 0.0) + clk() - t1
    return out, sum(len(b) for b in wire)


def run_batched(sd, pipe, P):
    """EdenPipeline.forward_batch / backward_batch: the whole state dict per
    call (pinned staging, one H2D / launch sequence / D2H each way)."""
    t = [time.perf_counter()]
    enc = pipe.forward_batch([a for _, a in sd])
    t.append(time.perf_counter())
    wire = [P.construct_named_tensor((name, "col", 1, False, ("trained",)), data, md, False).SerializeToString()
            for (name, _), (data, md) in zip(sd, enc)]
    t.append(time.perf_counter())
    items = []
    for b in wire:
        nt = P.NamedTensor()
        nt.ParseFromString(b)
        items.append((nt.data_bytes, P.transformer_metadata_of(nt)))
    t.append(time.perf_counter())
    out = pipe.backward_batch(items)
    t.append(time.perf_counter())
    run_batched.phases = {k: round(1e3 * (b - a), 2) for k, a, b in
                          zip(("forward_batch_ms", "protobuf_build_ms", "protobuf_parse_ms", "backward_batch_ms"),
                              t[:-1], t[1:])}
    return out, sum(len(b) for b in wire)


def run_cpu(sd, P):
    from oracle import eden as O
    from openfl_amd.pipelines.eden_pipeline import eden_seed
    wire = []
    for name, arr in sd:
        seed = eden_seed(arr)
        if arr.size > 100:
            planes, scales, dims, tot = O.compress(arr, seed, 8)
            md = {"int_list": list(arr.shape), "int_to_float": {0: float(seed), 1: float(tot)}}
            for j, (s, d) in enumerate(zip(scales, dims)):
                md["int_to_float"][2 + 2 * j] = s
                md["int_to_float"][3 + 2 * j] = float(d)
            data = planes.tobytes()
        else:
            data, md = arr.astype(np.float32).tobytes(), {"int_list": list(arr.shape)}
        wire.append(P.construct_named_tensor((name, "col", 1, False, ("trained",)), data, [md], False)
                    .SerializeToString())
    out = []
    for b in wire:
        nt = P.NamedTensor()
        nt.ParseFromString(b)
        m = nt.transformer_metadata[0]
        if len(m.int_to_float):
            dims = [int(m.int_to_float[k]) for k in range(3, max(m.int_to_float) + 1, 2)]
            sc = [m.int_to_float[k] for k in range(2, max(m.int_to_float) + 1, 2)]
            y = O.decompress(nt.data_bytes, int(m.int_to_float[1]), sc, dims, int(m.int_to_float[0]), 8)
            out.append(y.reshape(list(m.int_list)))
        else:
            out.append(np.frombuffer(nt.data_bytes, np.float32).reshape(list(m.int_list)))
    return out, sum(len(b) for b in wire)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="resnet50_fp32")
    ap.add_argument("--collaborators", type=int, default=2)
    ap.add_argument("--modes", default="plugin,batched,cpu")
    ap.add_argument("--out", default=None)
    ap.add_argument("--rounds", type=int, default=7, help="rounds per mode (the first is a warm-up)")
    ap.add_argument("--numa-bind", action="store_true",
                    help="bind the process to the GPU's NUMA node first (openfl_amd.numa, as bench.py does)")
    ap.add_argument("--heap-policy", action="store_true",
                    help="hostmem.keep_large_blocks() first (the opt-in deployment setting: large host "
                         "blocks stay in the heap, so protobuf copies and fresh arrays do not page-fault)")
    args = ap.parse_args()
    if args.heap_policy:
        from openfl_amd import hostmem
        hostmem.keep_large_blocks()
    import torch
    from openfl_amd import protocols as P
    from openfl_amd.pipelines import EdenPipeline
    from openfl_amd.workloads import WORKLOADS
    dev = torch.device("cuda", 0)
    if args.numa_bind:
        from openfl_amd import numa
        numa.bind_to_device(0)
    shapes = WORKLOADS[args.workload]()
    sds = [state_dict(shapes, 100 + c) for c in range(args.collaborators)]
    in_bytes = sum(a.nbytes for sd in sds for _, a in sd)
    res = {"workload": args.workload, "collaborators": args.collaborators, "input_bytes": in_bytes,
           "tensors_per_collaborator": len(shapes), "hostmem_policy": bool(args.heap_policy)}

    def rel_err(sd, out):
        num = sum(float(np.sum((o.astype(np.float64) - a) ** 2)) for (_, a), o in zip(sd, out))
        den = sum(float(np.sum(a.astype(np.float64) ** 2)) for _, a in sd)
        return (num / den) ** 0.5

    def rounds_of(fn, n=args.rounds):
        """fn() per round -> (median seconds of the rounds after the first,
        every round's seconds, the last round's result)."""
        times, out = [], None
        for _ in range(max(n, 2)):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = fn()
            times.append(round(time.perf_counter() - t0, 4))
        return float(np.median(times[1:])), times, out

    modes = args.modes.split(",")
    if "plugin" in modes:
        pipe = EdenPipeline(n_bits=8, dim_threshold=100, device="cuda:0")
        dt, rounds, outs = rounds_of(lambda: [run_plugin(sd, pipe, P) for sd in sds])
        res["plugin"] = {"s": round(dt, 4), "GiB_s": round(in_bytes / dt / 2 ** 30, 3), "round_s": rounds,
                         "wire_bytes": sum(o[1] for o in outs), "rel_err": round(rel_err(sds[0], outs[0][0]), 6)}
        # where a round's time goes (a third, instrumented round)
        ph = {}
        torch.cuda.synchronize()
        for sd in sds:
            run_plugin(sd, pipe, P, ph)
        res["plugin"]["phases_ms"] = {k: round(1e3 * v, 2) for k, v in sorted(ph.items())}
        cnt = {}
        for _, a in sds[0]:
            cnt[_bucket(a.size)] = cnt.get(_bucket(a.size), 0) + len(sds)
        res["plugin"]["tensors_per_bucket"] = cnt
    if "plugin_concurrent" in modes:
        # the gRPC pattern: each collaborator's tensors on its own handler
        # thread (aggregator_server.py:305), per-tensor calls, concurrently
        from concurrent.futures import ThreadPoolExecutor
        pipe = EdenPipeline(n_bits=8, dim_threshold=100, device="cuda:0")
        # (single rounds vary by up to 2x with the host's scheduling of the
        # two caller threads: the median of the rounds after the first)
        with ThreadPoolExecutor(max_workers=len(sds)) as ex:
            dt, rounds, outs = rounds_of(lambda: list(ex.map(lambda sd: run_plugin(sd, pipe, P), sds)))
        res["plugin_concurrent"] = {"s": round(dt, 4), "GiB_s": round(in_bytes / dt / 2 ** 30, 3), "threads": len(sds),
                                    "wire_bytes": sum(o[1] for o in outs),
                                    "rel_err": round(rel_err(sds[0], outs[0][0]), 6), "round_s": rounds}
    if "batched" in modes:
        for mode in ("reference", "fast"):
            pipe = EdenPipeline(n_bits=8, dim_threshold=100, device="cuda:0", seed_mode=mode)
            phs = []

            def one():
                o = []
                for sd in sds:
                    o.append(run_batched(sd, pipe, P))
                    phs.append(dict(run_batched.phases))
                return o
            dt, rounds, outs = rounds_of(one)
            key = "batched" if mode == "reference" else "batched_fast_seed"
            phs = phs[len(sds):]   # the rounds after the first
            nc = len(sds)
            res[key] = {"s": round(dt, 4), "GiB_s": round(in_bytes / dt / 2 ** 30, 3), "round_s": rounds,
                        "wire_bytes": sum(o[1] for o in outs), "rel_err": round(rel_err(sds[-1], outs[-1][0]), 6),
                        # median over the rounds after the first, per collaborator (in call order)
                        "phases_ms_median": [{k: round(float(np.median([p[k] for p in phs[c::nc]])), 2)
                                              for k in phs[0]} for c in range(nc)]}
    if "cpu" in modes:
        from oracle import eden as O
        cores = O.host_cores()
        O.set_threads(cores)
        t0 = time.perf_counter()
        outs = [run_cpu(sd, P) for sd in sds]
        dt = time.perf_counter() - t0
        res["cpu"] = {"s": round(dt, 3), "GiB_s": round(in_bytes / dt / 2 ** 30, 4), "cores": cores, "kind": "port",
                      "wire_bytes": sum(o[1] for o in outs), "rel_err": round(rel_err(sds[0], outs[0][0]), 6)}
    line = json.dumps(res)
    print(line)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
