#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the REFERENCE codecs.

This script is test infrastructure. It runs only in the build container, where
the read-only reference checkout is mounted at /root/reference; it refuses to
run anywhere else. It imports the reference's codec modules (which need only
numpy / torch / scikit-learn) by pre-registering empty ``openfl`` and
``openfl.pipelines`` package objects whose ``__path__`` points into the
reference tree, so the reference's heavy package ``__init__`` (dynaconf, grpc,
...) is never executed. Nothing from the reference is copied: the fixtures are
inputs and outputs only (arrays + JSON), consumed by tests/test_golden_*.py.

Reference functions exercised (citations are /root/reference-relative):
  openfl/pipelines/eden_pipeline.py:76-380   centroid / boundary tables
  openfl/pipelines/eden_pipeline.py:403-449  Eden.rand_diag
  openfl/pipelines/eden_pipeline.py:555-611  Eden.compress
  openfl/pipelines/eden_pipeline.py:632-659  Eden.decompress
  openfl/pipelines/eden_pipeline.py:661-720  Eden.to_bits / from_bits
  openfl/pipelines/eden_pipeline.py:761-818  EdenTransformer.forward/backward
  openfl/pipelines/kc_pipeline.py:36-114     KmeansTransformer
  openfl/pipelines/stc_pipeline.py:30-143    SparsityTransformer / TernaryTransformer
  openfl/pipelines/skc_pipeline.py:33-187    SKC transformers
  openfl/pipelines/random_shift_pipeline.py:12-77  RandomShiftTransformer / Pipeline
  openfl/pipelines/no_compression_pipeline.py:10-15 NoCompressionPipeline

Usage:  python tests/golden/make_golden.py [--only plain]
        (writes tests/golden/*.npz, *.json; --only plain rewrites plain_golden.json only)
"""
import hashlib
import importlib
import json
import os
import sys
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def _load_reference():
    if not os.path.isdir(os.path.join(REF, "openfl", "pipelines")):
        sys.exit("make_golden.py: /root/reference is not present; fixtures are generated "
                 "only in the build container")
    for name, sub in (("openfl", "openfl"), ("openfl.pipelines", "openfl/pipelines")):
        mod = types.ModuleType(name)
        mod.__path__ = [os.path.join(REF, sub)]
        sys.modules[name] = mod
    mods = {}
    for m in ("pipeline", "eden_pipeline", "kc_pipeline", "skc_pipeline", "stc_pipeline",
              "random_shift_pipeline", "no_compression_pipeline"):
        mods[m] = importlib.import_module("openfl.pipelines." + m)
    return mods


def sha(b):
    return hashlib.sha256(bytes(b)).hexdigest()


def gen_input(n, seed, scale=0.01):
    return (np.random.default_rng(seed).standard_normal(n).astype(np.float32)
            * np.float32(scale))


EDEN_NS = [1, 7, 8, 99, 100, 101, 500, 1000, 4096, 37000, 65537]
BIG_N = 300000
FULL_PLANES_MAX = 512 * 1024


def eden_fixtures(ref):
    import torch
    torch.set_num_threads(1)
    eden_mod = ref["eden_pipeline"]
    arrays = {}
    index = {"eden_cases": [], "rand_diag": [], "tables": {}, "forward": []}

    # ---- tables (eden_pipeline.py:76-380) ----
    e8 = eden_mod.Eden(nbits=8)
    for b in range(1, 9):
        arrays[f"centroids_b{b}"] = e8.centroids[b].numpy().astype(np.float32)
        arrays[f"boundaries_b{b}"] = e8.boundaries[b].numpy().astype(np.float32)
    index["tables"] = {"bits": list(range(1, 9))}

    # ---- rand_diag (eden_pipeline.py:403-449): packed sign bits (1 = +1) ----
    for P in (8, 64, 1024, 1 << 20):
        for s in (0, 1, 7, 12345, 40000, 65535, 65536):
            d = e8.rand_diag(P, s).numpy()
            bits = np.packbits((d > 0).astype(np.uint8), bitorder="little")
            key = f"rd_P{P}_s{s}"
            rec = {"P": P, "seed": s, "key": key, "sha256": sha(bits)}
            if P <= 1024:
                arrays[key] = bits
            index["rand_diag"].append(rec)

    # ---- to_bits layout probe (eden_pipeline.py:661-690) ----
    e4 = eden_mod.Eden(nbits=4)
    probe = torch.arange(16) % 16
    arrays["tobits_probe_b4"] = e4.to_bits(probe).numpy()

    # ---- Eden.compress / decompress cases ----
    inputs = {}
    for n in EDEN_NS + [BIG_N]:
        inputs[n] = gen_input(n, 1000 + n)
        arrays[f"x_n{n}"] = inputs[n]

    def run_case(tag, x, b, seed, keep_y=True):
        e = eden_mod.Eden(nbits=b)
        planes, scales, dims, total = e.compress(x, seed)
        planes = np.asarray(planes, dtype=np.uint8)
        md = {0: float(seed), 1: float(total)}
        k = 2
        for sc, dm in zip(scales, dims):
            md[k] = sc
            md[k + 1] = float(dm)
            k += 2
        y = e.decompress(planes.copy(), md).astype(np.float32)
        rec = {"tag": tag, "bits": b, "n": int(x.size), "seed": int(seed),
               "scales": [float(s) for s in scales], "dims": [int(d) for d in dims],
               "total_dim": int(total), "planes_len": int(planes.size),
               "planes_sha256": sha(planes), "y_sha256": sha(y.tobytes()),
               "y_norm": float(np.linalg.norm(y.astype(np.float64))),
               "err_norm": float(np.linalg.norm(y.astype(np.float64) - x.astype(np.float64)))}
        if planes.size <= FULL_PLANES_MAX:
            arrays[f"planes_{tag}"] = planes
            rec["planes_key"] = f"planes_{tag}"
        if keep_y:
            arrays[f"y_{tag}"] = y
            rec["y_key"] = f"y_{tag}"
        else:
            idx = np.arange(0, y.size, max(1, y.size // 4096))
            arrays[f"ysample_{tag}"] = y[idx]
            rec["ysample_key"] = f"ysample_{tag}"
            rec["ysample_stride"] = int(max(1, y.size // 4096))
        index["eden_cases"].append(rec)

    for b in range(1, 9):
        for n in EDEN_NS:
            tag = f"b{b}_n{n}"
            run_case(tag, inputs[n], b, seed=(4242 + 97 * n + b) % 65536)
            index["eden_cases"][-1]["x_key"] = f"x_n{n}"
    for b in (1, 4, 8):
        tag = f"b{b}_n{BIG_N}"
        run_case(tag, inputs[BIG_N], b, seed=4242, keep_y=False)
        index["eden_cases"][-1]["x_key"] = f"x_n{BIG_N}"

    # edge cases (b = 8 and b = 2)
    edge = {
        "zeros": np.zeros(1000, np.float32),
        "const": np.full(1000, 0.5, np.float32),
        "withinf": gen_input(1000, 7).copy(),
        "huge": gen_input(4096, 8) * np.float32(1e30),
        "tiny": gen_input(4096, 9) * np.float32(1e-30),
        "spike": np.zeros(2048, np.float32),
    }
    edge["withinf"][17] = np.inf
    edge["spike"][5] = 3.0
    for name, x in edge.items():
        arrays[f"x_edge_{name}"] = x
        for b in (2, 8):
            tag = f"b{b}_edge_{name}"
            run_case(tag, x, b, seed=321)
            index["eden_cases"][-1]["x_key"] = f"x_edge_{name}"

    # ---- EdenTransformer.forward: seed formula, fp64 input, fallback path ----
    fwd_cases = [
        ("fw_f32_n1000", gen_input(1000, 11)),
        ("fw_f64_n1000", gen_input(1000, 12).astype(np.float64)),
        ("fw_f32_2d", gen_input(64 * 9, 13).reshape(64, 9)),
        ("fw_f32_n100", gen_input(100, 14)),     # == threshold: forward does not compress
        ("fw_f32_n50", gen_input(50, 15)),
        ("fw_f32_n101", gen_input(101, 16)),
    ]
    for i, (tag, x) in enumerate(fwd_cases):
        t = eden_mod.EdenTransformer(n_bits=8, dim_threshold=100, device="cpu")
        np.random.seed(1234 + i)
        state_draw = np.random.RandomState(1234 + i).randint(1, 2 ** 16)
        serial = sum(x.flatten())
        data, md = t.forward(x)
        rec = {"tag": tag, "dtype": str(x.dtype), "shape": list(x.shape),
               "np_seed": 1234 + i, "randint": int(state_draw),
               "serial_sum": float(serial), "serial_sum_type": type(serial).__name__,
               "hash_term": int(hash(serial * 13 + 7)),
               "int_list": [int(v) for v in md["int_list"]],
               "int_to_float": ([[int(k), float(v)] for k, v in md["int_to_float"].items()]
                                if "int_to_float" in md else None),
               "bytes_len": len(data), "bytes_sha256": sha(data)}
        arrays[f"fwx_{tag}"] = np.asarray(x)
        arrays[f"fwb_{tag}"] = np.frombuffer(data, np.uint8).copy()
        if "int_to_float" in md:
            y = t.backward(data, md)
            arrays[f"fwy_{tag}"] = np.asarray(y, np.float32)
        else:
            try:
                y = t.backward(data, md)
                arrays[f"fwy_{tag}"] = np.asarray(y, np.float32)
                rec["backward"] = "ok"
            except Exception as exc:  # the reference's >/>= threshold mismatch
                rec["backward"] = f"raises {type(exc).__name__}"
        index["forward"].append(rec)
    return arrays, index


def kc_fixtures(ref):
    kc = ref["kc_pipeline"]
    stc = ref["stc_pipeline"]
    skc = ref["skc_pipeline"]
    arrays, index = {}, {"kc": [], "stc": [], "skc": []}
    for n in (5, 1000, 65536):
        x = gen_input(n, 5000 + n)
        arrays[f"kcx_n{n}"] = x
        np.random.seed(77)
        t = kc.KmeansTransformer(n_cluster=6)
        ints, md = t.forward(x.copy())
        from sklearn.cluster import KMeans  # inertia of the reference's own fit
        np.random.seed(77)
        km = KMeans(n_clusters=6, n_init=6)
        km.fit(x.reshape(-1, 1)) if n >= 6 else None
        y = t.backward(ints.astype(np.float32), md)
        arrays[f"kcint_n{n}"] = np.asarray(ints, np.int32)
        arrays[f"kcy_n{n}"] = np.asarray(y, np.float32)
        index["kc"].append({"n": n, "int_to_float": [[int(k), float(v)] for k, v in
                                                      md["int_to_float"].items()],
                            "int_list": [int(v) for v in md["int_list"]],
                            "inertia": float(km.inertia_) if n >= 6 else None})
    for n in (5, 1000, 65536):
        x = gen_input(n, 6000 + n)
        arrays[f"stcx_n{n}"] = x
        sp = stc.SparsityTransformer(p=0.1)
        sd, md1 = sp.forward(x.copy())
        tt = stc.TernaryTransformer()
        ti, md2 = tt.forward(sd.copy())
        back = sp.backward(tt.backward(ti.astype(np.float32), md2), md1)
        arrays[f"stcsparse_n{n}"] = np.asarray(sd)
        arrays[f"stcint_n{n}"] = np.asarray(ti, np.int32)
        arrays[f"stcy_n{n}"] = np.asarray(back, np.float32)
        index["stc"].append({"n": n, "k": int(np.ceil(n * 0.1)),
                             "int_to_float": [[int(k), float(v)] for k, v in
                                              md2["int_to_float"].items()]})
    for n in (1000, 65536):
        x = gen_input(n, 7000 + n)
        arrays[f"skcx_n{n}"] = x
        sp = skc.SparsityTransformer(p=0.1)
        sd, md1 = sp.forward(x.copy())
        arrays[f"skcsparse_n{n}"] = np.asarray(sd)
        index["skc"].append({"n": n, "k": int(np.ceil(n * 0.1))})
    return arrays, index


def plain_fixtures(ref):
    """Lossless pipelines: RandomShift (one np.random.uniform draw per call,
    every shift in int_to_float) and NoCompression, in-process and with the
    float32 wire values a receiver sees (MetadataProto.int_to_float)."""
    out = {"random_shift": [], "no_compression": []}
    for shape, seed in (((2, 3), 7), ((5,), 11), ((3, 4, 2), 2024)):
        x = gen_input(int(np.prod(shape)), seed).reshape(shape)
        np.random.seed(seed)
        pipe = ref["random_shift_pipeline"].RandomShiftPipeline()
        data, md = pipe.forward(x)
        rec = {"shape": list(shape), "seed": seed, "x": x.reshape(-1).tolist(),
               "data_hex": bytes(data).hex(),
               "metadata": [{"int_list": list(m.get("int_list", [])),
                             "int_to_float": [[int(k), float(v)] for k, v in m.get("int_to_float", {}).items()]}
                            for m in md]}
        y_mem = pipe.backward(data, [dict(m) for m in md])
        rec["backward_inproc_hex"] = np.ascontiguousarray(y_mem).tobytes().hex()
        rec["backward_inproc_dtype"] = str(y_mem.dtype)
        wire = [{"int_list": list(m.get("int_list", [])),
                 "int_to_float": {int(k): float(np.float32(v)) for k, v in m.get("int_to_float", {}).items()}}
                for m in md]
        y_wire = pipe.backward(data, wire)
        rec["backward_wire_hex"] = np.ascontiguousarray(y_wire).tobytes().hex()
        rec["backward_wire_dtype"] = str(y_wire.dtype)
        out["random_shift"].append(rec)
    for shape, dt in (((4, 3), "float32"), ((7,), "float64")):
        x = gen_input(int(np.prod(shape)), 5).reshape(shape).astype(dt)
        pipe = ref["no_compression_pipeline"].NoCompressionPipeline()
        data, md = pipe.forward(x)
        y = pipe.backward(data, [dict(m) for m in md])
        out["no_compression"].append({"shape": list(shape), "dtype": dt, "x": x.reshape(-1).tolist(),
                                      "data_hex": bytes(data).hex(),
                                      "metadata": [{"int_list": list(m.get("int_list", []))} for m in md],
                                      "backward_hex": y.tobytes().hex(), "backward_dtype": str(y.dtype)})
    return out


def main():
    ref = _load_reference()
    with open(os.path.join(OUT, "plain_golden.json"), "w") as f:
        json.dump(plain_fixtures(ref), f, indent=1)
    if "--only" in sys.argv and sys.argv[sys.argv.index("--only") + 1] == "plain":
        print("wrote plain_golden.json")
        return
    arrays, index = eden_fixtures(ref)
    np.savez_compressed(os.path.join(OUT, "eden_golden.npz"), **arrays)
    with open(os.path.join(OUT, "eden_golden.json"), "w") as f:
        json.dump(index, f, indent=1)
    karrays, kindex = kc_fixtures(ref)
    np.savez_compressed(os.path.join(OUT, "lossy_golden.npz"), **karrays)
    with open(os.path.join(OUT, "lossy_golden.json"), "w") as f:
        json.dump(kindex, f, indent=1)
    meta = {"numpy": np.__version__}
    import torch
    import sklearn
    meta.update(torch=torch.__version__, sklearn=sklearn.__version__,
                python=sys.version.split()[0], reference="/root/reference (openfl 1.6)")
    with open(os.path.join(OUT, "GENERATED_WITH.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("wrote", sorted(os.listdir(OUT)))


if __name__ == "__main__":
    main()
