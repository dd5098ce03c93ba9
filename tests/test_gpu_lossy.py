"""GPU parity of the KC / SKC / STC pipelines against the reference goldens
(tests/golden/lossy_golden.*, generated from the reference by make_golden.py).

Tolerances:
  * top-k sparsify, ternary ranks, +1e-7 rule, decode (sequential key->value
    replacement): exact (no ties in the fixtures);
  * ternary mean: relative 1e-12 (fp64 sums in a different order);
  * k-means: sklearn's RNG cannot be reproduced; our inertia
    <= 1.01 x the reference fit's inertia, labels = nearest of our centres,
    centres carried in the input dtype.
"""
import gzip
import zlib

import numpy as np
import pytest
import torch

from tests import golden_io

pytestmark = pytest.mark.gpu
ARR, IDX = golden_io.lossy()
DEV = "cuda:0"


def _inertia(x, centres):
    x = np.asarray(x, np.float64).reshape(-1)
    c = np.asarray(centres, np.float64)
    return float(np.sum(np.min((x[:, None] - c[None, :]) ** 2, axis=1)))


@pytest.mark.parametrize("rec", IDX["kc"], ids=lambda r: f"n{r['n']}")
def test_kc_kmeans_vs_reference(rec):
    from openfl_amd.pipelines.kc_pipeline import KmeansTransformer
    n = rec["n"]
    x = ARR[f"kcx_n{n}"]
    t = KmeansTransformer(6, DEV)
    np.random.seed(1)
    ints, md = t.forward(x.copy())
    assert md["int_list"] == rec["int_list"]
    ref_map = {int(k): v for k, v in rec["int_to_float"]}
    if n < 6:  # passthrough quantisation: exact
        np.testing.assert_array_equal(ints, ARR[f"kcint_n{n}"])
        assert {k: float(v) for k, v in md["int_to_float"].items()} == ref_map
    else:
        centres = np.array([md["int_to_float"][k] for k in sorted(md["int_to_float"])])
        assert centres.dtype == np.float32 and np.all(np.diff(centres) > 0)
        ours = _inertia(x, centres)
        assert ours <= 1.01 * rec["inertia"] + 1e-12, (ours, rec["inertia"])
        # labels are the nearest (float32) centre
        near = np.argmin(np.abs(x.astype(np.float64)[:, None] - centres[None, :]), axis=1)
        assert np.mean(ints == near) >= 0.9999
        assert ints.shape == (n,) and ints.dtype == np.int32
    # decode the REFERENCE's payload with our backward: exact
    y = t.backward(ARR[f"kcint_n{n}"].astype(np.float32), {"int_list": rec["int_list"],
                                                            "int_to_float": ref_map})
    np.testing.assert_array_equal(y, ARR[f"kcy_n{n}"])


@pytest.mark.parametrize("rec", IDX["stc"], ids=lambda r: f"n{r['n']}")
def test_stc_vs_reference(rec):
    from openfl_amd.pipelines.stc_pipeline import SparsityTransformer, STCPipeline, TernaryTransformer
    n = rec["n"]
    x = ARR[f"stcx_n{n}"]
    sp = SparsityTransformer(0.1, DEV)
    sparse, md1 = sp.forward(x.copy())
    np.testing.assert_array_equal(sparse, ARR[f"stcsparse_n{n}"])     # top-k + 1e-7 rule, exact
    tt = TernaryTransformer(DEV)
    ints, md2 = tt.forward(sparse)
    np.testing.assert_array_equal(ints, ARR[f"stcint_n{n}"])
    ref_map = {int(k): v for k, v in rec["int_to_float"]}
    assert sorted(md2["int_to_float"]) == sorted(ref_map)
    for k in ref_map:
        np.testing.assert_allclose(md2["int_to_float"][k], ref_map[k], rtol=1e-12)
    # fused pipeline: same metadata, payload decodes to the same ranks
    pipe = STCPipeline(p_sparsity=0.1, device=DEV)
    payload, mds = pipe.forward(x.copy())
    assert mds[0]["int_list"] == [n] and mds[2] == {}
    np.testing.assert_array_equal(np.frombuffer(gzip.decompress(payload), np.float32),
                                  ARR[f"stcint_n{n}"].astype(np.float32))
    y = pipe.backward(payload, mds)
    np.testing.assert_array_equal(y, ARR[f"stcy_n{n}"])


@pytest.mark.parametrize("rec", IDX["skc"], ids=lambda r: f"n{r['n']}")
def test_skc_vs_reference(rec):
    from openfl_amd.pipelines.skc_pipeline import SKCPipeline
    from openfl_amd.pipelines.stc_pipeline import SparsityTransformer
    n = rec["n"]
    x = ARR[f"skcx_n{n}"]
    sparse, _ = SparsityTransformer(0.1, DEV).forward(x.copy())
    np.testing.assert_array_equal(sparse, ARR[f"skcsparse_n{n}"])
    pipe = SKCPipeline(p_sparsity=0.1, n_clusters=6, device=DEV)
    np.random.seed(3)
    payload, mds = pipe.forward(x.copy())
    centres = np.array([mds[1]["int_to_float"][k] for k in sorted(mds[1]["int_to_float"])])
    assert centres.dtype == np.float64
    from sklearn.cluster import KMeans
    np.random.seed(77)
    ref = KMeans(n_clusters=6, n_init=6).fit(sparse.reshape(-1, 1))
    assert _inertia(sparse, centres) <= 1.01 * ref.inertia_ + 1e-15
    y = pipe.backward(payload, mds)
    assert y.shape == (n,) and y.dtype == np.float32
    ranks = np.frombuffer(gzip.decompress(payload), np.float32).astype(np.int64)
    np.testing.assert_array_equal(y, centres[ranks].astype(np.float32))


def test_topk_ties_lowest_index():
    from openfl_amd import lossy
    x = np.zeros(10_000, np.float32)
    x[::7] = 1.0                       # 1429 ties at |x| = 1
    x[5] = -3.0
    sp, st = lossy.sparsify_topk(torch.from_numpy(x).to(DEV), 100)
    sp = sp.cpu().numpy()
    kept = np.nonzero(sp)[0]
    assert kept.size == 100 and kept[0] == 0 and 5 in kept
    ties = [i for i in kept if i != 5]
    assert ties == list(range(0, 7 * 99, 7))   # lowest-index ties
    assert st["shifted"]                         # min kept value -3 < 1e-7 -> +1e-7
    assert sp[5] == np.float32(-3.0) + np.float32(1e-7)


@pytest.mark.parametrize("n,k", [(1000, 1), (1000, 1000), (4097, 37), (1 << 20, 104858), (3_000_001, 3)])
def test_topk_exact_vs_numpy(n, k):
    """Distinct magnitudes: the kept set is unique; compare with a full sort."""
    from openfl_amd import lossy
    x = np.random.default_rng(n + k).standard_normal(n).astype(np.float32)
    a = np.abs(x)
    order = np.argsort(-a, kind="stable")
    T = a[order[k - 1]]
    if np.sum(a == T) > 1:
        pytest.skip("tie at the threshold")
    sp, st = lossy.sparsify_topk(torch.from_numpy(x).to(DEV), k)
    kept = np.nonzero(sp.cpu().numpy())[0]
    np.testing.assert_array_equal(kept, np.sort(order[:k]))
    assert st["n_pos"] + st["n_neg"] + st["n_zero"] == k


def test_lut_sequential_semantics():
    """data[data == key] = value applied in sequence: a value equal to a later
    key is replaced again (the reference's in-place loop)."""
    from openfl_amd import lossy
    ranks = torch.tensor([0.0, 1.0, 2.0, 3.0], device=DEV)
    out = lossy.lut_decode(ranks, {0: 2.0, 1: 0.5, 2: 7.0, 3: -1.0}).cpu().numpy()
    ref = ranks.cpu().numpy().copy()
    for k, v in {0: 2.0, 1: 0.5, 2: 7.0, 3: -1.0}.items():
        ref[ref == k] = v
    np.testing.assert_array_equal(out, ref)   # element 0: 0 -> 2 -> 7


def test_kmeans_batch_vs_sklearn_and_deterministic():
    """Batched device k-means (ofl_kmeans1d_batch): every tensor's inertia
    within 1 % of sklearn KMeans(6, n_init=6) on the same tensor, ranks = rank
    of the nearest centre among np.unique(used centres), counts sum to n,
    bit-identical across two runs; ragged sizes, a constant tensor and a
    tensor with fewer distinct values than clusters included."""
    from sklearn.cluster import KMeans
    from openfl_amd import lossy
    rng = np.random.default_rng(17)
    xs = [rng.standard_normal(50_000).astype(np.float32) * np.float32(0.02),
          (rng.standard_normal(70_001) ** 3).astype(np.float32),
          np.full(1000, 0.25, np.float32),
          np.repeat(np.float32([1.0, 2.0, 3.0]), 400),
          rng.uniform(-1, 1, 6).astype(np.float32),
          np.concatenate([rng.standard_normal(30_000) - 4, rng.standard_normal(30_000) + 4]).astype(np.float32)]
    offs, acc = [], 0
    for x in xs:
        offs.append(acc)
        acc += (x.size + 63) // 64 * 64 + 3          # ragged offsets: not 16-B aligned
    arena = torch.zeros(acc, dtype=torch.float32, device=DEV)
    for x, o in zip(xs, offs):
        arena[o:o + x.size] = torch.from_numpy(x).to(DEV)
    outs = []
    for _ in range(2):
        ranks = torch.full_like(arena, -1.0)
        c, cnt, inertia, uniq = lossy.kmeans_batch(arena, offs, [x.size for x in xs], 6, n_init=6, seed=5,
                                                   ranks_out=ranks)
        outs.append((c, cnt, inertia, [u.copy() for u in uniq], ranks.cpu().numpy()))
    for a, b in zip(outs[0][:3], outs[1][:3]):
        np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(outs[0][4], outs[1][4])
    c, cnt, inertia, uniq, rk = outs[0]
    for t, (x, o) in enumerate(zip(xs, offs)):
        assert cnt[t].sum() == x.size and np.all(np.diff(c[t]) >= 0)
        cen32 = c[t].astype(np.float32)
        assert np.array_equal(uniq[t], np.unique(cen32[cnt[t] > 0]))
        r = rk[o:o + x.size].astype(np.int64)
        used = cen32[cnt[t] > 0]
        near = np.argmin(np.abs(x.astype(np.float64)[:, None] - used.astype(np.float64)[None, :]), axis=1)
        assert np.mean(uniq[t][r] == used[near]) >= 0.9999
        ours = _inertia(x, uniq[t])
        if np.unique(x).size > 6:
            np.random.seed(t)
            ref = KMeans(n_clusters=6, n_init=6).fit(x.reshape(-1, 1)).inertia_
            assert ours <= 1.01 * ref + 1e-9, (t, ours, ref)
        else:
            assert ours <= 1e-9


def test_lut_decode_batch_equals_single():
    from openfl_amd import lossy
    rng = np.random.default_rng(4)
    numels = [100_003, 7, 65_536, 200_000]
    offs, acc = [], 0
    for n in numels:
        offs.append(acc)
        acc += n + 5
    ranks = torch.from_numpy(rng.integers(0, 6, acc).astype(np.float32)).to(DEV)
    maps = [{0: 2.0, 1: 0.5, 2: 7.0, 3: -1.0}, {0: 1.5}, {i: float(i) * 0.1 - 0.2 for i in range(6)}, {}]
    out = torch.full_like(ranks, -9.0)
    lossy.lut_decode_batch(ranks, offs, numels, maps, out)
    for o, n, m in zip(offs, numels, maps):
        ref = lossy.lut_decode(ranks[o:o + n].contiguous(), m) if m else ranks[o:o + n]
        assert torch.equal(out[o:o + n], ref)


def test_kc_large_vs_sklearn():
    from sklearn.cluster import KMeans
    from openfl_amd.pipelines import KCPipeline
    x = np.random.default_rng(5).standard_normal((512, 512)).astype(np.float32) * np.float32(0.02)
    pipe = KCPipeline(n_clusters=6, device=DEV)
    payload, mds = pipe.forward(x)
    centres = np.array([mds[0]["int_to_float"][k] for k in sorted(mds[0]["int_to_float"])])
    np.random.seed(0)
    ref = KMeans(n_clusters=6, n_init=6).fit(x.reshape(-1, 1))
    assert _inertia(x, centres) <= 1.01 * ref.inertia_
    y = pipe.backward(payload, mds)
    assert y.shape == x.shape
    assert np.linalg.norm(y - x) / np.linalg.norm(x) < 0.3


def _topk_ref(x, k):
    """numpy restatement of SparsityTransformer._topk_func (skc_pipeline.py:
    72-94) with ties at the k-th magnitude kept lowest index first."""
    order = np.argsort(-np.abs(x), kind="stable")[:k]
    kept = np.zeros(x.size, bool)
    kept[order] = True
    shift = np.float32(1e-7) if np.min(x[kept]) < 1e-7 else np.float32(0)
    sp = np.where(kept, x + shift, np.float32(0)).astype(np.float32)
    v = sp[kept]
    return sp, {"n_pos": int(np.sum(v > 0)), "n_neg": int(np.sum(v < 0)), "n_zero": int(np.sum(v == 0)),
                "abs_sum": float(np.sum(np.abs(v.astype(np.float64)))), "shifted": bool(shift),
                "kept_min": np.min(x[kept])}


def test_sparsify_topk_batch_vs_numpy():
    """Batched device top-k (ofl_sparsify_topk_batch) against the numpy
    restatement: ragged / unaligned offsets, ties straddling 64 Ki-element
    blocks (partial keep inside one block), negative and positive ties at the
    threshold, an all-zero tensor, k = 1 and k = n.  Bit-exact sparse arrays,
    exact counts; fp64 |sum| to 1e-12; deterministic across runs."""
    from openfl_amd import lossy
    rng = np.random.default_rng(23)
    xs, ks = [], []
    a = rng.standard_normal(300_000).astype(np.float32)
    a[rng.choice(a.size, 5000, replace=False)] = np.float32(2.5) * rng.choice([-1, 1], 5000).astype(np.float32)
    xs.append(a); ks.append(int(np.sum(np.abs(a) > 2.5)) + 2600)       # partial keep of the 5000 ties
    b = np.zeros(200_000, np.float32)
    b[1::3] = -0.5                                                       # negative ties only
    b[70_000] = 9.0
    xs.append(b); ks.append(30_000)
    c = np.zeros(1000, np.float32)
    xs.append(c); ks.append(10)                                          # all zeros: T = 0
    d = rng.standard_normal(4097).astype(np.float32)
    xs.append(d); ks.append(1)
    e = np.abs(rng.standard_normal(5000)).astype(np.float32) + np.float32(1.0)
    xs.append(e); ks.append(5000)                                        # k = n, no shift
    f = rng.standard_normal(1 << 20).astype(np.float32)
    xs.append(f); ks.append(int(np.ceil(f.size * 0.1)))
    offs, acc = [], 0
    for x in xs:
        offs.append(acc)
        acc += x.size + 3                                                # unaligned
    arena = torch.zeros(acc, dtype=torch.float32, device=DEV)
    for x, o in zip(xs, offs):
        arena[o:o + x.size] = torch.from_numpy(x).to(DEV)
    res = []
    for _ in range(2):
        out = torch.full_like(arena, 7.0)
        st = lossy.sparsify_topk_batch(arena, offs, [x.size for x in xs], ks, out)
        res.append((out.cpu().numpy(), st))
    np.testing.assert_array_equal(res[0][0], res[1][0])
    out, st = res[0]
    for t, (x, o, k) in enumerate(zip(xs, offs, ks)):
        sp, ref = _topk_ref(x, k)
        np.testing.assert_array_equal(out[o:o + x.size], sp, err_msg=str(t))
        for key in ("n_pos", "n_neg", "n_zero", "shifted"):
            assert st[key][t] == ref[key], (t, key)
        assert st["kept_min"][t] == ref["kept_min"], t
        assert abs(st["abs_sum"][t] - ref["abs_sum"]) <= 1e-12 * max(ref["abs_sum"], 1e-30), t
        assert res[1][1]["abs_sum"][t] == st["abs_sum"][t]
    # per-tensor entry point = batch of one
    sp1, st1 = lossy.sparsify_topk(torch.from_numpy(xs[0]).to(DEV), ks[0])
    np.testing.assert_array_equal(sp1.cpu().numpy(), out[offs[0]:offs[0] + xs[0].size])


def test_ternary_ranks_batch_equals_single():
    from openfl_amd import lossy
    rng = np.random.default_rng(8)
    numels = [70_001, 5, 131_072]
    offs, acc = [], 0
    for n in numels:
        offs.append(acc)
        acc += n + 1
    x = rng.standard_normal(acc).astype(np.float32)
    x[rng.random(acc) < 0.5] = 0
    xd = torch.from_numpy(x).to(DEV)
    r3 = [(0.0, 1.0, 2.0), (0.0, 0.0, 1.0), (1.0, 0.0, 2.0)]
    out = torch.full_like(xd, -1.0)
    lossy.ternary_ranks_batch(xd, offs, numels, r3, out)
    for o, n, r in zip(offs, numels, r3):
        assert torch.equal(out[o:o + n], lossy.ternary_ranks(xd[o:o + n].contiguous(), *r))


@pytest.mark.parametrize("case", ["kc6", "ternary", "constant", "one", "ragged", "all32", "runs"])
def test_gzip_ranks_roundtrip(case):
    """GPU gzip (ofl_gzip_ranks): gzip.decompress returns the exact bytes."""
    from openfl_amd import lossy
    rng = np.random.default_rng(sum(map(ord, case)))
    n = {"one": 1, "ragged": 4096 * 3 + 17}.get(case, 200_000)
    if case == "kc6":
        x = rng.choice(6, n, p=[0.07, 0.2, 0.23, 0.23, 0.2, 0.07]).astype(np.float32)
    elif case == "ternary":
        x = rng.choice(3, n, p=[0.05, 0.9, 0.05]).astype(np.float32)
    elif case == "constant":
        x = np.full(n, 2.0, np.float32)
    elif case == "one":
        x = np.float32([5.0])
    elif case == "all32":
        x = rng.integers(0, 32, n).astype(np.float32)
    elif case == "runs":
        x = np.repeat(rng.integers(0, 6, n // 100 + 1), 100)[:n].astype(np.float32)
    else:
        x = rng.integers(0, 4, n).astype(np.float32)
    z = lossy.gzip_ranks(torch.from_numpy(x).to(DEV))
    assert gzip.decompress(z) == x.tobytes()
    assert z == lossy.gzip_ranks(torch.from_numpy(x).to(DEV))      # deterministic
    # every member carries its 'OZ' subfield (size, segment table): the native
    # parallel inflate reads it
    import ctypes
    from openfl_amd import _lib
    src = np.frombuffer(z, np.uint8)
    need = ctypes.c_size_t()
    assert _lib.lib().ofl_gunzip_members(src.ctypes.data, src.size, None, 0, ctypes.byref(need), 4) == 0
    assert need.value == x.nbytes
    assert lossy.gunzip(z, 4).tobytes() == x.tobytes()
    # pageable output (one D2H per batch) gives the same stream as the pinned one
    # (the kernels write into mapped pinned memory directly)
    from openfl_amd import _lib as LB
    xd = torch.from_numpy(x).to(DEV)
    L = LB.lib()
    cap = int(L.ofl_gzip_ranks_bound(x.size))
    pageable = np.zeros(cap, np.uint8)
    wsb = torch.empty(int(L.ofl_gzip_ranks_workspace_bytes(x.size)), dtype=torch.uint8, device=DEV)
    ln = ctypes.c_size_t()
    LB.check_gzip(L.ofl_gzip_ranks(xd.data_ptr(), x.size, pageable.ctypes.data, cap, ctypes.byref(ln), wsb.data_ptr(),
                                   wsb.numel(), torch.cuda.current_stream().cuda_stream))
    assert pageable[:ln.value].tobytes() == z
    # and the device inflate (TLZ: one lane per segment, copies resolved in
    # LDS) straight into HBM
    out = torch.full((x.nbytes + 64,), 7, dtype=torch.uint8, device=DEV)
    got = lossy.gunzip_device(z, out)
    assert got.numel() == x.nbytes and got.cpu().numpy().tobytes() == x.tobytes()
    assert int(out[x.nbytes:].eq(7).all())                            # nothing written past the data
    # the generic member inflate reads the same stream (plain deflate)
    assert _inflate_generic(z, x.nbytes) == x.tobytes()
    if case == "kc6":  # the optimal parse beats gzip -9 on k-means ranks
        ref = len(gzip.compress(x.tobytes(), compresslevel=9))
        assert len(z) < ref, (len(z), ref)


def _nseg(z):
    return int.from_bytes(z[18:20], "little")


def _inflate_generic(z, nbytes):
    """ofl_inflate_members (one wavefront per member, any deflate data) on a
    stream: the TLZ members are plain deflate to it."""
    import ctypes
    from openfl_amd import _lib
    L = _lib.lib()
    src = np.frombuffer(z, np.uint8)
    cap = src.size // 26 + 1
    idx = np.empty((cap, 4), np.int64)
    nm, tot, mx, tl = ctypes.c_int64(), ctypes.c_size_t(), ctypes.c_uint32(), ctypes.c_int()
    _lib.check_gzip(L.ofl_gzip_member_index(src.ctypes.data, src.size, idx.ctypes.data, cap, ctypes.byref(nm),
                                            ctypes.byref(tot), ctypes.byref(mx), ctypes.byref(tl)))
    assert tl.value == 1 and tot.value == nbytes
    d_in = torch.zeros(src.size + 64, dtype=torch.uint8, device=DEV)
    d_in[:src.size] = torch.from_numpy(src.copy())
    d_idx = torch.from_numpy(idx[:nm.value].copy()).to(DEV)
    out = torch.zeros(nbytes + 64, dtype=torch.uint8, device=DEV)
    ws = torch.empty(256, dtype=torch.uint8, device=DEV)
    _lib.check_gzip(L.ofl_inflate_members(d_in.data_ptr(), d_idx.data_ptr(), nm.value, mx.value, out.data_ptr(),
                                          out.numel(), ws.data_ptr(), ws.numel(), torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    return out[:nbytes].cpu().numpy().tobytes()


def test_tlz_rejects_corrupt_streams():
    """A corrupted TLZ stream fails loudly on the device path where
    gzip.decompress fails (the TLZ decoder hands what it does not expect to
    the generic inflate, which decides); a flipped CRC-32 is reported as such;
    the untouched stream decodes."""
    from openfl_amd import _lib, lossy
    x = np.random.default_rng(5).choice(6, 300_000, p=[0.07, 0.2, 0.23, 0.23, 0.2, 0.07]).astype(np.float32)
    z = lossy.gzip_ranks(torch.from_numpy(x).to(DEV))
    out = torch.zeros(x.nbytes + 64, dtype=torch.uint8, device=DEV)
    assert lossy.gunzip_device(z, out).cpu().numpy().tobytes() == x.tobytes()
    first = int.from_bytes(z[20:24], "little")                # the first member's size ('OZ' field)
    bad_crc = bytearray(z)
    bad_crc[first - 8] ^= 0x5A
    with pytest.raises(_lib.CodecError, match="CRC"):
        lossy.gunzip_device(bytes(bad_crc), out)
    hdr = 28 + 4 * _nseg(z)
    for off in (hdr + 40, hdr + first // 3, first // 2, first - 12):
        bad = bytearray(z)
        bad[off] ^= 0xFF
        with pytest.raises((_lib.CodecError, EOFError, OSError, zlib.error)):
            gzip.decompress(bytes(bad))
        with pytest.raises(_lib.CodecError):
            lossy.gunzip_device(bytes(bad), out)
    # a segment entry point moved: gzip.decompress ignores the table, and so
    # does the device path's fallback (the TLZ decoder refuses the member, the
    # generic inflate reads it as the plain deflate it is)
    bad = bytearray(z)
    bad[28 + 4] ^= 0x01
    assert gzip.decompress(bytes(bad)) == x.tobytes()
    assert lossy.gunzip_device(bytes(bad), out).cpu().numpy().tobytes() == x.tobytes()
    # the segment table is untrusted: entries far past the member (high byte
    # flipped), non-increasing entries, every entry misaligned by 3 bits, and
    # the last member's last entry on its final bit must neither fault nor
    # decode wrongly (the TLZ decoder refuses them, the generic inflate reads
    # the plain deflate data, which is intact)
    starts = [0]
    while starts[-1] < len(z):
        starts.append(starts[-1] + int.from_bytes(z[starts[-1] + 20:starts[-1] + 24], "little"))
    assert starts[-1] == len(z) and len(starts) >= 3
    ns = _nseg(z)
    cases = []
    b = bytearray(z); b[28 + 4 + 3] ^= 0xFF; cases.append(b)                      # noqa: E702
    b = bytearray(z); b[28 + 8:28 + 12] = b[28 + 4:28 + 8]; cases.append(b)       # noqa: E702
    b = bytearray(z)
    for s in range(1, ns):   # entry 0 is checked against the header's end
        e = 28 + 4 * s
        b[e:e + 4] = (int.from_bytes(b[e:e + 4], "little") + 3).to_bytes(4, "little")
    cases.append(b)
    last = starts[-2]
    nl = int.from_bytes(z[last + 18:last + 20], "little")
    in_len = (starts[-1] - last) - (28 + 4 * nl) - 8
    b = bytearray(z)
    e = last + 28 + 4 * (nl - 1)
    b[e:e + 4] = (8 * in_len - 1).to_bytes(4, "little")
    cases.append(b)
    for b in cases:
        assert gzip.decompress(bytes(b)) == x.tobytes()
        assert lossy.gunzip_device(bytes(b), out).cpu().numpy().tobytes() == x.tobytes()
    # a truncated stream (the last member cut inside its data, or just its
    # trailer) raises on both paths and never faults
    for cut in (len(z) - 8 - in_len // 2, len(z) - 3):
        with pytest.raises((_lib.CodecError, EOFError, OSError, zlib.error)):
            gzip.decompress(z[:cut])
        with pytest.raises((_lib.CodecError, EOFError, OSError, zlib.error)):
            lossy.gunzip_device(z[:cut], out)


def test_gzip_ranks_rejects_non_ranks():
    from openfl_amd import _lib, lossy
    for bad in (np.float32([0.5, 1.0]), np.float32([32.0]), np.float32([-1.0]), np.float32([-0.0]),
                np.float32([np.nan])):
        with pytest.raises(_lib.CodecError, match="values must be"):
            lossy.gzip_ranks(torch.from_numpy(bad).to(DEV))


@pytest.mark.parametrize("name", ["KCPipeline", "STCPipeline", "SKCPipeline"])
@pytest.mark.parametrize("shape", [(300, 200), (4,)])
def test_lossy_pipeline_device_gzip_backend(name, shape):
    """gzip_backend="device": device gzip on forward, fused device inflate +
    LUT on backward -- same payload bytes (after gzip.decompress), same
    decoded array and the metadata list consumed exactly like the host
    backend's (the reference's pop semantics); host-gzip payloads (the tiny
    path) decode through the same fused backward."""
    import openfl_amd.pipelines as P
    x = np.random.default_rng(2).standard_normal(shape).astype(np.float32)
    outs = []
    for backend in ("host", "device"):
        pipe = getattr(P, name)(n_clusters=6, device=DEV, gzip_backend=backend)
        np.random.seed(1)
        payload, mds = pipe.forward(x)
        raw = gzip.decompress(payload)
        y = pipe.backward(payload, mds)
        assert mds == []
        outs.append((raw, y))
        # the other backend's payload decodes the same way
        if backend == "device":
            np.random.seed(1)
            p2, m2 = getattr(P, name)(n_clusters=6, device=DEV, gzip_backend="host").forward(x)
            np.testing.assert_array_equal(pipe.backward(p2, m2), y)
    assert outs[0][0] == outs[1][0]
    np.testing.assert_array_equal(outs[0][1], outs[1][1])
    assert outs[1][1].dtype == np.float32 and outs[1][1].shape == shape


@pytest.mark.timeout(900)
def test_kc_2p22_tensor_vs_sklearn():
    """BASELINE config 3 at its own tensor size: one 4096 x 1024 tensor of the
    1 GiB set (N(0, 0.01^2)) through KmeansTransformer: inertia <= 1.01 x
    sklearn KMeans(6, n_init=6) on the same data, labels = nearest of our
    centres; then the whole KCPipeline with the device gzip: the payload
    decodes (native member-parallel inflate) to centres[ranks] exactly."""
    from sklearn.cluster import KMeans
    from openfl_amd.pipelines import KCPipeline
    from openfl_amd.pipelines.kc_pipeline import KmeansTransformer
    g = torch.Generator(device=DEV).manual_seed(0)
    x = torch.empty(4096 * 1024, device=DEV).normal_(0.0, 0.01, generator=g).cpu().numpy().reshape(4096, 1024)
    t = KmeansTransformer(6, DEV)
    np.random.seed(11)
    ints, md = t.forward(x)
    centres = np.array([md["int_to_float"][k] for k in sorted(md["int_to_float"])])
    assert len(centres) == 6 and centres.dtype == np.float32
    ref = KMeans(n_clusters=6, n_init=6, random_state=0).fit(x.reshape(-1, 1).astype(np.float64))
    ours = _inertia(x, centres)
    assert ours <= 1.01 * ref.inertia_, (ours, ref.inertia_)
    xf = x.reshape(-1).astype(np.float64)
    near = np.argmin(np.abs(xf[:, None] - centres[None, :].astype(np.float64)), axis=1)
    assert np.mean(ints.reshape(-1) == near) >= 0.9999
    pipe = KCPipeline(n_clusters=6, device=DEV, gzip_backend="device")
    np.random.seed(11)
    payload, mds = pipe.forward(x)
    ranks = np.frombuffer(gzip.decompress(payload), np.float32).astype(np.int64)
    cen = np.array([mds[0]["int_to_float"][k] for k in sorted(mds[0]["int_to_float"])], np.float32)
    y = pipe.backward(payload, mds)
    assert y.shape == x.shape and y.dtype == np.float32
    np.testing.assert_array_equal(y.reshape(-1), cen[ranks])
    assert len(payload) < 0.16 * x.nbytes


def test_ternary_stats_deterministic():
    """TernaryTransformer.forward's mean (stc_pipeline.py:120-123) is the same
    on every run: per-wave fp64 partials summed in a fixed order."""
    from openfl_amd import lossy
    x = np.random.default_rng(4).standard_normal(3_000_001).astype(np.float32)
    xd = torch.from_numpy(x).to(DEV)
    runs = {lossy.ternary_stats(xd) for _ in range(5)}
    assert len(runs) == 1
    npos, nneg, asum = runs.pop()
    assert npos == int(np.sum(x > 0)) and nneg == int(np.sum(x < 0))
    np.testing.assert_allclose(asum, np.sum(np.abs(x.astype(np.float64))), rtol=1e-12)


@pytest.mark.parametrize("kind", ["stored", "fixed", "dynamic", "flushes", "member64k", "empty", "text"])
def test_inflate_members_foreign_streams(kind):
    """ofl_inflate_members decodes any member-indexed deflate data, not only
    the device gzip's: stored, fixed and dynamic blocks, several blocks per
    member (full flushes emit empty stored blocks), 64 KiB members, empty
    members; the result equals gzip.decompress's."""
    from openfl_amd import lossy
    from tests.bgzf import member_indexed
    rng = np.random.default_rng(sum(map(ord, kind)))
    words = [bytes(rng.integers(97, 123, rng.integers(2, 9)).astype(np.uint8)) for _ in range(300)]
    text = b" ".join(words[i] for i in rng.integers(0, 300, 60_000))
    noise = rng.integers(0, 256, 50_000).astype(np.uint8).tobytes()
    data = (text[:150_000] + noise + text[150_000:])
    args = {"stored": dict(level=0), "fixed": dict(strategy="fixed"), "dynamic": dict(level=9),
            "flushes": dict(level=6, flush_every=3000), "member64k": dict(level=6, chunk=65536),
            "empty": dict(level=6, empty_members=True), "text": dict(level=1, chunk=20_000)}[kind]
    z = member_indexed(data, **args)
    assert gzip.decompress(z) == data
    out = torch.zeros(len(data) + 64, dtype=torch.uint8, device=DEV)
    got = lossy.gunzip_device(z, out)
    assert got.cpu().numpy().tobytes() == data


def test_gzip_roundtrip_concurrent_threads():
    """Device gzip + device inflate from several threads at once (gRPC worker
    threads call the plugin concurrently): each thread's payload decodes to its
    own ranks; payloads of different lengths exercise the scratch regrowth and
    the shared H2D pool."""
    from concurrent.futures import ThreadPoolExecutor
    from openfl_amd import lossy

    def one(k):
        g = torch.Generator(device=DEV).manual_seed(100 + k)
        n = (1 << 20) + 4096 * k + 123 * k
        p = torch.tensor([0.1, 0.2, 0.4, 0.2, 0.1], device=DEV)
        x = torch.multinomial(p, n, replacement=True, generator=g).to(torch.float32)
        z = lossy.gzip_ranks(x)
        assert np.array_equal(np.frombuffer(gzip.decompress(z), np.float32), x.cpu().numpy())
        out = torch.empty(4 * n + 64, dtype=torch.uint8, device=DEV)
        got = lossy.gunzip_device(z, out)
        torch.cuda.current_stream().synchronize()
        return torch.equal(got.view(torch.float32), x)

    with ThreadPoolExecutor(max_workers=4) as ex:
        assert all(ex.map(one, range(8)))


def test_inflate_members_rejects_corrupt_streams():
    """Corrupt data fails loudly (gzip.decompress raises on the same bytes),
    a stream without the 'BC' field decodes on the host, output too small is
    refused."""
    from openfl_amd import _lib, lossy
    from tests.bgzf import member_indexed
    data = bytes(np.random.default_rng(4).integers(0, 6, 100_000).astype(np.uint8))
    z = member_indexed(data, level=6)
    out = torch.zeros(len(data), dtype=torch.uint8, device=DEV)
    assert lossy.gunzip_device(z, out).cpu().numpy().tobytes() == data
    bad_crc = bytearray(z)
    first = int.from_bytes(z[16:18], "little") + 1          # the first member's size
    bad_crc[first - 8] ^= 0x5A                               # its CRC-32
    with pytest.raises(_lib.CodecError, match="CRC"):
        lossy.gunzip_device(bytes(bad_crc), out)
    for off in (30, 200, first // 2):
        bad = bytearray(z)
        bad[off] ^= 0xFF
        with pytest.raises((_lib.CodecError, EOFError, OSError, zlib_error())):
            gzip.decompress(bytes(bad))
        with pytest.raises(_lib.CodecError):
            lossy.gunzip_device(bytes(bad), out)
    plain = gzip.compress(data)                              # no member index: host inflate
    assert lossy.gunzip_device(plain, out).cpu().numpy().tobytes() == data
    with pytest.raises(_lib.CodecError, match="too small"):
        lossy.gunzip_device(z, out[:len(data) - 1])


def zlib_error():
    import zlib
    return zlib.error


@pytest.mark.parametrize("name", ["KCPipeline", "STCPipeline", "SKCPipeline"])
def test_default_gzip_backend_is_device_and_reference_readable(name):
    """The pipelines' default gzip backend is the GPU one (TLZ), and its payload
    is what the reference's GZIPTransformer.backward reads: plain
    gzip.decompress (kc_pipeline.py:152-156) gives the float32 ranks, which
    the reference's LUT backward (sequential key -> value replacement,
    kc_pipeline.py:79-83) turns into the array our backward returns."""
    import openfl_amd.pipelines as P
    x = np.random.default_rng(9).standard_normal((700, 300)).astype(np.float32)
    pipe = getattr(P, name)(n_clusters=6, device=DEV)
    assert pipe.transformers[-1].backend == "device"
    np.random.seed(3)
    payload, mds = pipe.forward(x)
    assert int.from_bytes(payload[12:14], "little") == int.from_bytes(b"OZ", "little")  # a TLZ member
    ranks = np.frombuffer(gzip.decompress(payload), np.float32)
    assert ranks.size == x.size
    m = next(d["int_to_float"] for d in mds if "int_to_float" in d)
    ref = ranks.copy()
    for k in m:                                   # the reference's in-place LUT, in the mapping's order
        ref[ref == k] = m[k]
    y = pipe.backward(payload, [dict(d) for d in mds])
    np.testing.assert_array_equal(y.reshape(-1), ref)


@pytest.mark.parametrize("n,threads", [(5, 2), ((8 << 20) - 1, 2), ((8 << 20) + 4097, 2), ((37 << 20) + 3, 4),
                                       ((21 << 20) + 1, 8)])
def test_copy_h2d_staged(n, threads):
    """ofl_copy_h2d_staged (the pinned-ring H2D of a received payload): the
    device bytes equal the source, the bytes past the copy are untouched, and
    back-to-back calls reusing the ring (other sizes, other thread counts)
    stay correct."""
    from openfl_amd import _lib, hostmem
    L = _lib.lib()
    rng = np.random.default_rng(n)
    d = torch.full((n + 64,), 7, dtype=torch.uint8, device=DEV)
    st = torch.cuda.current_stream().cuda_stream
    for rep in range(3):
        arr = rng.integers(0, 256, n, dtype=np.uint8)
        src = hostmem.bytes_from(arr.ctypes.data, n)
        with hostmem.quiet():
            _lib.check(L.ofl_copy_h2d_staged(d.data_ptr(), np.frombuffer(src, np.uint8).ctypes.data, n,
                                             threads + rep, st))
        del src  # the source may go as soon as the call returns
        torch.cuda.synchronize()
        assert d[:n].cpu().numpy().tobytes() == arr.tobytes()
        assert bool(d[n:].eq(7).all())


def test_copy_h2d_staged_concurrent_threads():
    """Four threads copying at once, each on its own stream and buffer (the
    staging rings are lent per call from a per-device pool, so no call waits
    for another's copy or rebuilds another's events): every copy byte-exact,
    the bytes past each copy untouched, over several rounds of mixed sizes
    and thread counts."""
    from concurrent.futures import ThreadPoolExecutor
    from openfl_amd import _lib
    L = _lib.lib()
    sizes = [(9 << 20) + 5, (17 << 20) + 4093, 12 << 20, (33 << 20) + 1]

    def job(i):
        rng = np.random.default_rng(100 + i)
        st = torch.cuda.Stream(DEV)
        ok = True
        with torch.cuda.stream(st):
            d = torch.full((max(sizes) + 64,), 7, dtype=torch.uint8, device=DEV)
            for rep in range(4):
                n = sizes[(i + rep) % len(sizes)]
                arr = rng.integers(0, 256, n, dtype=np.uint8)
                d.fill_(7)
                _lib.check(L.ofl_copy_h2d_staged(d.data_ptr(), arr.ctypes.data, n, 1 + (i + rep) % 4,
                                                 st.cuda_stream))
                st.synchronize()
                ok &= d[:n].cpu().numpy().tobytes() == arr.tobytes()
                ok &= bool(d[n:].eq(7).all())
        return ok
    with ThreadPoolExecutor(4) as ex:
        assert all(ex.map(job, range(4)))


@pytest.mark.parametrize("case", ["ternary", "kc6", "runs"])
def test_gzip_ranks_deterministic_repeats(case):
    """The device gzip's bytes do not depend on wave timing: several encodes
    of one input (many members, blocks racing each other on the CUs) give
    one stream.  (A missing barrier between the chain links' last writes and
    the match search once made ternary ranks encode differently run to run.)"""
    from openfl_amd import lossy
    rng = np.random.default_rng(7)
    n = (1 << 21) + 333
    if case == "ternary":
        x = rng.choice(3, n, p=[0.05, 0.9, 0.05]).astype(np.float32)
    elif case == "kc6":
        x = rng.choice(6, n, p=[0.07, 0.2, 0.23, 0.23, 0.2, 0.07]).astype(np.float32)
    else:
        x = np.repeat(rng.integers(0, 6, n // 37 + 1), 37)[:n].astype(np.float32)
    xd = torch.from_numpy(x).to(DEV)
    z = lossy.gzip_ranks(xd)
    assert gzip.decompress(z) == x.tobytes()
    for _ in range(5):
        assert lossy.gzip_ranks(xd) == z


def test_gzip_ranks_to_matches_pinned_path():
    """The payload filled batch by batch while the GPU encodes
    (ofl_gzip_ranks_to, lossy.gzip_ranks' path above 8 MiB) is byte for byte
    the stream ofl_gzip_ranks leaves in pinned memory, over three full batches
    of 512 members and a ragged fourth; it decodes with gzip.decompress."""
    import ctypes
    from openfl_amd import _lib, lossy
    n = 3 * (1 << 26) + 12345
    g = torch.Generator(device=DEV).manual_seed(5)
    p = torch.tensor([0.1, 0.2, 0.4, 0.2, 0.1], device=DEV)
    x = torch.empty(n, dtype=torch.float32, device=DEV)
    for o in range(0, n, 1 << 24):
        m = min(1 << 24, n - o)
        x[o:o + m] = torch.multinomial(p, m, replacement=True, generator=g).to(torch.float32)
    z = lossy.gzip_ranks(x)
    L = _lib.lib()
    cap = int(L.ofl_gzip_ranks_bound(n))
    out = torch.empty(cap, dtype=torch.uint8).pin_memory()
    ws = torch.empty(int(L.ofl_gzip_ranks_workspace_bytes(n)), dtype=torch.uint8, device=DEV)
    ln = ctypes.c_size_t()
    _lib.check_gzip(L.ofl_gzip_ranks(x.data_ptr(), n, out.data_ptr(), cap, ctypes.byref(ln), ws.data_ptr(),
                                     ws.numel(), torch.cuda.current_stream().cuda_stream))
    assert type(z) is bytes and len(z) == ln.value
    assert z == out[:ln.value].numpy().tobytes()
    assert hash(z) == hash(bytes(memoryview(z)))
    assert gzip.decompress(z) == x.cpu().numpy().tobytes()


def test_gzip_ranks_full_size_kc_set():
    """BASELINE config 3 at its full size (2^28 ranks = the 1 GiB set): the
    device gzip's stream is a valid gzip stream whose gzip.decompress is the
    ranks' bytes (the reference's GZIPTransformer.backward), the device
    inflate returns the same bytes, the stream is smaller than gzip -9's
    ratio bound for this distribution, and it is deterministic."""
    from openfl_amd import lossy
    n = 1 << 28
    g = torch.Generator(device=DEV).manual_seed(11)
    p = torch.tensor([0.074, 0.1816, 0.2444, 0.2444, 0.1816, 0.074], device=DEV)
    x = torch.empty(n, dtype=torch.float32, device=DEV)
    for o in range(0, n, 1 << 24):
        x[o:o + (1 << 24)] = torch.multinomial(p, 1 << 24, replacement=True, generator=g).to(torch.float32)
    z = lossy.gzip_ranks(x)
    assert len(z) / (4 * n) < 0.1174          # gzip -9 on this distribution: 0.1173-0.1174
    host = x.cpu().numpy().tobytes()
    assert gzip.decompress(z) == host
    out = torch.empty(4 * n + 64, dtype=torch.uint8, device=DEV)
    got = lossy.gunzip_device(z, out)
    assert got.numel() == 4 * n and torch.equal(got.view(torch.float32), x)
    assert lossy.gzip_ranks(x) == z


def _lut_case(seed, sizes, gap=64):
    """A rank arena (tensors 64-aligned with gaps) and per-tensor maps with
    sequential-replacement chains (a value equal to a later key)."""
    rng = np.random.default_rng(seed)
    offs, acc = [], 0
    for n in sizes:
        offs.append(acc)
        acc = (acc + n + gap - 1) // gap * gap
    x = np.zeros(acc, np.float32)
    maps = []
    for t, (o, n) in enumerate(zip(offs, sizes)):
        k = int(rng.integers(2, 7))
        x[o:o + n] = rng.choice(k, n, p=np.full(k, 1.0 / k)).astype(np.float32)
        m = {i: float(rng.standard_normal() * 0.01) for i in range(k)}
        if t % 3 == 0:
            m[0] = 2.0          # 0 -> 2 -> m[2]: the reference's in-place chain
        maps.append(m)
    gaps = np.ones(acc, bool)
    for o, n in zip(offs, sizes):
        gaps[o:o + n] = False
    x[gaps] = rng.integers(0, 6, int(gaps.sum())).astype(np.float32)
    return x, offs, list(sizes), maps


@pytest.mark.parametrize("case", ["few_large", "many_small", "pipelined"])
def test_gunzip_fused_lut_matches_unfused(case, monkeypatch):
    """gunzip_device(lut=lut_tables(...)): the TLZ decoder's stores go through
    each tensor's LUT -- every tensor element equals the unfused inflate +
    lut_decode_batch (the reference's sequential replacement), including
    segments spanning more tensors than the LDS tables hold and a payload
    large enough for the pipelined (piecewise H2D) inflate."""
    from openfl_amd import lossy
    sizes = {"few_large": [300_000, 131_072 * 2 + 17, 5],
             "many_small": [int(n) for n in np.random.default_rng(3).integers(1, 900, 700)],
             "pipelined": [1 << 22] * 5}[case]
    x, offs, nums, maps = _lut_case(11, sizes)
    z = lossy.gzip_ranks(torch.from_numpy(x).to(DEV))
    if case == "pipelined":   # several H2D pieces, each inflated as it lands
        monkeypatch.setattr(lossy, "_INFLATE_PIECE_MIN", 1)
        assert len(z) >= 4 << 20
    ref = torch.empty(x.size, dtype=torch.float32, device=DEV)
    lossy.gunzip_device(z, ref.view(torch.uint8))
    lossy.lut_decode_batch(ref, offs, nums, maps, ref)
    got = torch.full((x.size,), -7.0, dtype=torch.float32, device=DEV)
    lossy.gunzip_device(z, got.view(torch.uint8), lut=lossy.lut_tables(offs, nums, maps, DEV))
    torch.cuda.synchronize()
    r, g = ref.cpu().numpy(), got.cpu().numpy()
    for o, n in zip(offs, nums):
        np.testing.assert_array_equal(g[o:o + n], r[o:o + n])


def test_gunzip_fused_lut_refused_stream_falls_back():
    """A TLZ stream the fused decoder refuses (a moved segment entry) goes
    through the generic inflate and the unfused LUT: same values."""
    from openfl_amd import lossy
    x, offs, nums, maps = _lut_case(12, [200_000, 70_001])
    z = bytearray(lossy.gzip_ranks(torch.from_numpy(x).to(DEV)))
    z[28 + 4] ^= 0x01
    z = bytes(z)
    lut = lossy.lut_tables(offs, nums, maps, DEV)
    got = torch.empty(x.size, dtype=torch.float32, device=DEV)
    lossy.gunzip_device(z, got.view(torch.uint8), lut=lut)
    g = got.cpu().numpy()
    for o, n, m in zip(offs, nums, maps):
        want = x[o:o + n].copy()
        for k, v in m.items():
            want[want == k] = v
        np.testing.assert_array_equal(g[o:o + n], want)


@pytest.mark.parametrize("case", ["few_large", "many_small", "ragged", "kc_like"])
def test_gzip_label_fused_matches_rank_array(case):
    """gzip_ranks(x, label=kmeans_batch(label_out=...)): the k-means labels
    applied inside the TLZ encoder as it loads the values give byte for byte
    the stream of the rank array ranks_out receives (zeros between tensors)
    -- tensors spanning members, segments holding more tensors than the LDS
    window (4), odd offsets and lengths, a leading gap."""
    from openfl_amd import lossy
    rng = np.random.default_rng({"few_large": 1, "many_small": 2, "ragged": 3, "kc_like": 4}[case])
    sizes = {"few_large": [300_000, 131_072 * 2 + 17, 9],
             "many_small": [int(n) for n in rng.integers(6, 900, 700)],
             "ragged": [int(n) for n in rng.integers(6, 40_000, 60)],
             "kc_like": [1 << 20, 3 << 18, 1 << 21, 1000, 1 << 20]}[case]
    offs, acc = [], 37 if case == "ragged" else 0
    for n in sizes:
        offs.append(acc)
        acc += n + (int(rng.integers(0, 9)) if case == "ragged" else (-n) % 64)
    tot = acc + 5
    x = torch.from_numpy((rng.standard_normal(tot) * 0.01).astype(np.float32)).to(DEV)
    ranks = torch.zeros(tot, dtype=torch.float32, device=DEV)
    tab = lossy.LabelTable(len(sizes), DEV)
    lossy.kmeans_batch(x, offs, sizes, 6, n_init=6, seed=9, ranks_out=ranks, label_out=tab)
    z_ref = lossy.gzip_ranks(ranks)
    z = lossy.gzip_ranks(x, label=tab)
    assert z == z_ref
    assert gzip.decompress(z) == ranks.cpu().numpy().tobytes()


def test_kmeans_label_table_checks():
    """Label records need k <= 8 and ascending, non-overlapping tensors."""
    from openfl_amd import lossy
    from openfl_amd._lib import CodecError
    x = torch.randn(4096, device=DEV)
    with pytest.raises(CodecError):
        lossy.kmeans_batch(x, [0], [4096], 12, n_init=2, label_out=lossy.LabelTable(1, DEV))
    with pytest.raises(CodecError):
        lossy.kmeans_batch(x, [2000, 0], [1000, 1000], 6, n_init=2, label_out=lossy.LabelTable(2, DEV))
    with pytest.raises(ValueError):
        lossy.kmeans_batch(x, [0], [4096], 6, n_init=2, label_out=lossy.LabelTable(2, DEV))


def test_side_streams_shared_per_device():
    """ofl_side_stream: three streams per device, the same objects on every
    call (the Eden plans' side streams and the pipelined inflate's), distinct
    from each other and from the caller's stream."""
    import ctypes
    from openfl_amd import _lib, lossy
    L = _lib.lib()
    got = []
    for _ in range(2):
        row = []
        for i in range(3):
            p = ctypes.c_void_p()
            _lib.check(L.ofl_side_stream(i, ctypes.byref(p)))
            row.append(p.value)
        got.append(row)
    assert got[0] == got[1] and len(set(got[0])) == 3 and all(got[0])
    assert torch.cuda.current_stream().cuda_stream not in got[0]
    p = ctypes.c_void_p()
    assert L.ofl_side_stream(3, ctypes.byref(p)) == _lib.OFL_EINVAL
    sides = lossy._side_streams(torch.device(DEV))
    assert [s.cuda_stream for s in sides] == got[0][1:]


def test_gunzip_wrong_length_payloads():
    """A payload that does not decode to the caller's 4n bytes raises the
    pipelines' CodecError before any LUT runs, on every inflate path: a
    foreign gzip stream (host gzip.decompress) whose length is not whole
    float32s or is short, and a device-gzip TLZ stream one value short or
    long; gunzip_device(lut=...) without an expected length still refuses a
    length that is not whole float32s."""
    from openfl_amd import _lib, lossy
    from openfl_amd.pipelines.lossy_common import gzip_lut_backward_device
    m = {0: 0.5, 1: -0.25, 2: 1.0}
    for payload, n in ((gzip.compress(bytes(10)), 3), (gzip.compress(bytes(8)), 3), (gzip.compress(bytes(16)), 3)):
        with pytest.raises(_lib.CodecError, match="payload decodes to"):
            gzip_lut_backward_device(payload, m, n, torch.device(DEV))
    x = torch.from_numpy(np.random.default_rng(8).integers(0, 3, 100_001).astype(np.float32)).to(DEV)
    z = lossy.gzip_ranks(x)
    for n in (100_000, 100_002):
        with pytest.raises(_lib.CodecError, match="payload decodes to"):
            gzip_lut_backward_device(z, m, n, torch.device(DEV))
    y = gzip_lut_backward_device(z, m, 100_001, torch.device(DEV)).cpu().numpy()
    want = x.cpu().numpy().copy()
    for k, v in m.items():
        want[want == k] = v
    np.testing.assert_array_equal(y, want)
    out = torch.empty(64, dtype=torch.uint8, device=DEV)
    with pytest.raises(_lib.CodecError, match="whole float32"):
        lossy.gunzip_device(gzip.compress(bytes(10)), out, lut=lossy.lut_tables([0], [3], [m], DEV))


def test_kc_bench_composition_full_size():
    """bench.py's KC line, exactly as it times it, on its own 64 x 2^22 set
    (BASELINE config 3): kmeans_batch(label_out=...) -> gzip_ranks(x,
    label=...) (the label-fused encoder, several encode batches) ->
    gunzip_device(lut=lut_tables(...)) (the pipelined inflate: 4 H2D pieces,
    each inflated as it lands, LUT fused into the stores).  gzip.decompress of
    the stream (the reference's GZIPTransformer.backward) equals the device
    k-means ranks (the same seed through ranks_out), and y equals the
    reference's sequential replacement (oracle/kc.py:lut_sequential,
    kc_pipeline.py:79-83) of those ranks, element for element."""
    from oracle import kc as K
    from openfl_amd import lossy
    from openfl_amd.workloads import WORKLOADS, numel
    numels = [numel(s) for _, s in WORKLOADS["uniform_1gib"]()]
    offs = list(np.cumsum([0] + [(n + 63) // 64 * 64 for n in numels[:-1]]))
    tot = int(offs[-1] + numels[-1])
    x = torch.empty(tot, dtype=torch.float32, device=DEV)
    g = torch.Generator(device=DEV)
    for j, (o, n) in enumerate(zip(offs, numels)):
        g.manual_seed(j)
        x[o:o + n].normal_(0.0, 0.01, generator=g)
    tab = lossy.LabelTable(len(numels), DEV)
    _, _, _, uniq = lossy.kmeans_batch(x, offs, numels, 6, n_init=6, seed=1234, label_out=tab)
    z = lossy.gzip_ranks(x, label=tab)
    assert len(z) >= lossy._INFLATE_PIECE_MIN << 20          # the pipelined (4-piece) inflate
    maps = [{i: u for i, u in enumerate(uq)} for uq in uniq]
    y = torch.full((tot,), -7.0, dtype=torch.float32, device=DEV)
    lossy.gunzip_device(z, y.view(torch.uint8), lut=lossy.lut_tables(offs, numels, maps, DEV))
    ranks = torch.zeros(tot, dtype=torch.float32, device=DEV)
    _, _, _, uniq2 = lossy.kmeans_batch(x, offs, numels, 6, n_init=6, seed=1234, ranks_out=ranks)
    assert all(np.array_equal(a, b) for a, b in zip(uniq, uniq2))
    r = ranks.cpu().numpy()
    assert np.frombuffer(gzip.decompress(z), np.float32).tobytes() == r.tobytes()
    yh = y.cpu().numpy()
    for o, n, m in zip(offs, numels, maps):
        want = K.lut_sequential(r[o:o + n].copy(), m)
        np.testing.assert_array_equal(yh[o:o + n], want)


def test_gunzip_pipelined_rejects_corrupt_members(monkeypatch):
    """The pipelined inflate (several H2D pieces, members launched as their
    bytes land) refuses corrupt members next to every piece boundary as
    gzip.decompress does, and decodes the intact stream: the members at a
    boundary are launched only once the look-ahead bytes past their trailer
    have landed too."""
    from openfl_amd import _lib, lossy
    monkeypatch.setattr(lossy, "_INFLATE_PIECE_MIN", 1)
    x, offs, nums, maps = _lut_case(21, [1 << 22] * 5)
    z = lossy.gzip_ranks(torch.from_numpy(x).to(DEV))
    assert len(z) >= 4 << 20
    out = torch.empty(x.nbytes + 64, dtype=torch.uint8, device=DEV)
    assert lossy.gunzip_device(z, out).cpu().numpy().tobytes() == x.tobytes()
    starts = [0]
    while starts[-1] < len(z):
        starts.append(starts[-1] + int.from_bytes(z[starts[-1] + 20:starts[-1] + 24], "little"))
    n = lossy._INFLATE_PIECES
    bounds = [min(len(z), (len(z) * k // n + (4 << 20) - 1) // (4 << 20) * (4 << 20)) for k in range(1, n)]
    for b in bounds:
        j = int(np.searchsorted(starts, b, "right")) - 1       # the member holding the boundary
        for m in (j - 1, j):
            bad = bytearray(z)
            bad[starts[m + 1] - 12] ^= 0xFF                       # last data bytes before the trailer
            with pytest.raises((_lib.CodecError, EOFError, OSError, zlib.error)):
                gzip.decompress(bytes(bad))
            with pytest.raises(_lib.CodecError):
                lossy.gunzip_device(bytes(bad), out, lut=lossy.lut_tables(offs, nums, maps, DEV))
