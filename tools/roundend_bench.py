#!/usr/bin/env python3
"""Aggregator end of round on the device (openfl_amd.aggregation.RoundEnd).

    python tools/roundend_bench.py [--workload resnet50_fp32] [--collaborators 4] [--steps K]

One step = Aggregator._prepare_trained (aggregator.py:780-865) for every
tensor of the model: np.average over the collaborators' updates, delta to the
previous model, Eden encode + decode of the delta (EdenPipeline, 8 bits, fast
seeds), new model = base + decoded delta.  Collaborator updates and the base
model are resident in HBM; the new model is written to HBM.

Prints one JSON line: value = model GiB per second of round-end work
(fused, device-resident, no payload D2H); also: the unfused sequence
(average kernel writes the delta, the encode reads it), the same with the wire
payloads copied to the host, and the reference's call pattern (per tensor:
host np.average, TensorCodec.generate_delta / compress / decompress /
apply_delta with the openfl_amd EdenPipeline) on the same data.
Roofline: the minimal I/O of the step (read C + 1 fp32 arenas, write one)
against the step time.
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="resnet50_fp32")
    ap.add_argument("--collaborators", type=int, default=4)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--seed-mode", default="fast")
    ap.add_argument("--host-steps", type=int, default=1, help="steps of the per-tensor host call pattern (0: skip)")
    args = ap.parse_args()

    import torch
    from openfl_amd.aggregation import RoundEnd
    from openfl_amd.pipelines import EdenPipeline
    from openfl_amd.workloads import WORKLOADS
    dev = torch.device("cuda", 0)
    shapes = [tuple(s) for _, s in WORKLOADS[args.workload]()]
    pipe = EdenPipeline(n_bits=8, device=dev, seed_mode=args.seed_mode)
    re = RoundEnd(pipe, shapes, dev)
    C = args.collaborators
    g = torch.Generator(device=dev)
    arenas = []
    for c in range(C + 1):
        g.manual_seed(1000 + c)
        arenas.append(torch.empty(re.arena_numel, dtype=torch.float32, device=dev).normal_(0.0, 0.01, generator=g))
    base, collabs = arenas[0], arenas[1:]
    w = list(np.random.default_rng(0).random(C) + 0.5)
    out = torch.empty_like(base)
    nbytes = 4 * sum(re.numels)
    np.random.seed(0)

    def timed(fn, steps, warmup):
        for _ in range(warmup):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps

    t_dev = timed(lambda: re.run(collabs, w, base, payloads=False, out=out), args.steps, args.warmup)
    t_pay = timed(lambda: re.run(collabs, w, base, payloads=True, out=out), max(1, args.steps // 2), 1)

    also = {"fused_with_payload_d2h": {"value": round(nbytes / t_pay / 2 ** 30, 3), "ms_per_step": round(1e3 * t_pay, 3)}}
    # A/B: the delta arena written by the averaging kernel and read by the
    # encode (RoundEnd(fused=False)), interleaved with the fused run
    re_u = RoundEnd(pipe, shapes, dev, fused=False)
    t_u, t_f = [], []
    for _ in range(3):
        t_u.append(timed(lambda: re_u.run(collabs, w, base, payloads=False, out=out), args.steps, 1))
        t_f.append(timed(lambda: re.run(collabs, w, base, payloads=False, out=out), args.steps, 1))
    also["unfused_average_then_encode"] = {"value": round(nbytes / min(t_u) / 2 ** 30, 3),
                                           "ms_per_step": round(1e3 * min(t_u), 3),
                                           "fused_same_interleave_ms": round(1e3 * min(t_f), 3)}
    if args.host_steps > 0:
        from openfl_amd.tensor_codec import TensorCodec, TensorKey
        tc = TensorCodec(pipe)
        ch = [[re.view(a, i).cpu().numpy() for i in range(len(shapes))] for a in collabs]
        bh = [re.view(base, i).cpu().numpy() for i in range(len(shapes))]

        def host_round():
            for i in range(len(shapes)):
                agg = np.average([c[i] for c in ch], weights=w, axis=0)
                key = TensorKey(f"t{i}", "aggregator", 0, False, ("aggregated",))
                dk, delta = tc.generate_delta(key, agg, bh[i])
                ck, payload, md = tc.compress(dk, delta)
                _, dec = tc.decompress(ck, payload, md)
                tc.apply_delta(dk, dec, bh[i])
        t0 = time.perf_counter()
        for _ in range(args.host_steps):
            host_round()
        t_host = (time.perf_counter() - t0) / args.host_steps
        also["per_tensor_reference_call_pattern"] = {
            "value": round(nbytes / t_host / 2 ** 30, 4), "ms_per_step": round(1e3 * t_host, 1),
            "note": "host np.average + TensorCodec per tensor, openfl_amd EdenPipeline (GPU codec, one H2D/D2H "
                    "per tensor)"}

    io = 4 * sum(re.numels) * (C + 2)
    line = {"metric": "GiB/s aggregator round end (average + delta + Eden encode/decode + apply), device-resident",
            "value": round(nbytes / t_dev / 2 ** 30, 3), "unit": "GiB/s", "n_gpus": 1, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1e3 * t_dev, 3), "higher_is_better": True,
            "dtype": "f32/f64", "data": "synthetic N(0, 0.01^2) updates and base, resident in HBM",
            "config": {"workload": args.workload, "tensors": len(shapes), "bytes": nbytes, "collaborators": C,
                       "n_bits": 8, "seed_mode": args.seed_mode},
            "roofline": {"bound": "hbm", "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                         "achieved": round(io / t_dev / 1e9, 1), "frac": round(io / t_dev / 1e9 / PEAK_HBM_GBPS, 4),
                         "scope": "minimal step I/O: read C updates + base, write the new model (4 B each per "
                                  "element); the codec's own passes come on top", "traffic": None},
            "also": also}
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
