"""Host-side logic that needs no GPU: seed formula, C-ABI exports, plans."""
import re

import numpy as np
import pytest

from tests import golden_io

ARR, IDX = golden_io.eden()


def test_library_exports_every_declared_symbol():
    from openfl_amd import _lib
    L = _lib.lib()
    with open(f"{golden_io.GOLDEN}/../../include/ofl_codec.h") as f:
        hdr = f.read()
    declared = set(re.findall(r"\b(ofl_[a-z0-9_]+)\s*\(", hdr))
    assert declared == set(_lib.EXPORTS)
    for name in declared:
        assert hasattr(L, name), name
    assert b"gfx950" in L.ofl_version()


@pytest.mark.parametrize("rec", IDX["forward"], ids=lambda r: r["tag"])
def test_seed_formula_matches_reference(rec):
    """EdenTransformer.forward seed (eden_pipeline.py:771-772), reproduced exactly."""
    from openfl_amd.pipelines.eden_pipeline import eden_seed
    x = ARR["fwx_" + rec["tag"]]
    np.random.seed(rec["np_seed"])
    seed = eden_seed(x, "reference")
    if rec["int_to_float"] is not None:
        assert seed == int(dict(rec["int_to_float"])[0])
    assert seed == (rec["hash_term"] + rec["randint"]) % 2 ** 16
    # exactly one global RNG draw per call
    np.random.seed(rec["np_seed"])
    np.random.randint(1, 2 ** 16)
    after_ref = np.random.randint(0, 2 ** 31)
    np.random.seed(rec["np_seed"])
    eden_seed(x, "fast")
    assert np.random.randint(0, 2 ** 31) == after_ref


def test_serial_sums_are_left_to_right():
    from openfl_amd.pipelines.eden_pipeline import _serial_sum
    rng = np.random.default_rng(3)
    for dt in (np.float32, np.float64):
        x = (rng.standard_normal(5000) * 1e3).astype(dt)
        s = dt(0)
        for v in x:
            s = s + v
        assert _serial_sum(x) == s and type(_serial_sum(x)) is dt


@pytest.mark.parametrize("n", [0, 1, 7, 8, 9, 5003])
def test_serial_sum_copy_is_left_to_right_and_copies(n):
    """ofl_serial_sum_copy_f32 (the one-tensor encode's staging fill): the
    reference seed's float32 sum(data.flatten()) (:771) and an exact copy."""
    from openfl_amd import _lib
    x = (np.random.default_rng(n).standard_normal(n) * 1e3).astype(np.float32)
    s = np.float32(0)
    for v in x:
        s = s + v
    dst = np.full(n + 1, 7.0, np.float32)
    got = _lib.lib().ofl_serial_sum_copy_f32(x.ctypes.data, dst.ctypes.data, n)
    assert np.float32(got) == s
    assert np.array_equal(dst[:n], x) and dst[n] == 7.0


def test_host_plan_layout():
    from openfl_amd.codec import EdenPlan, slice_plan
    numels = [1000, 300000, 5, 4096 * 1024]
    p = EdenPlan(numels, n_bits=8)
    assert p.n_slices == sum(len(slice_plan(n)[0]) for n in numels)
    for t, n in enumerate(numels):
        assert p.dims[t] == slice_plan(n)[0]
        assert p.planes_nbytes[t] == 8 * sum(p.dims[t]) // 8
        assert p.planes_offsets[t] % 256 == 0
        assert p.elem_offsets[t] % 64 == 0
    ends = [o + b for o, b in zip(p.planes_offsets, p.planes_nbytes)]
    assert all(ends[i] <= p.planes_offsets[i + 1] for i in range(len(numels) - 1))
    assert p.planes_bytes == ends[-1]
    assert p.ws_bytes >= 4 * 4096 * 1024  # large slice intermediates


def test_wave_schedule_layout():
    """Large slices in waves (ofl_eden_plan_set_schedule): wave count, launch
    lists and the workspace (nstreams wave buffers instead of one slot per
    slice).  Outputs are schedule-independent (tests/test_gpu_parity.py)."""
    from openfl_amd import _lib
    from openfl_amd.codec import EdenPlan
    numels = [1 << 22] * 6 + [1000, 1 << 20]        # six 16 MiB slices, a small one, a 4 MiB slice
    one = EdenPlan(numels, 8, wave_mib=0, streams=1)
    assert one.n_waves == 1
    assert one.ws_bytes >= 4 * (6 * (1 << 22) + (1 << 20))
    w2 = EdenPlan(numels, 8, wave_mib=32, streams=2)
    assert w2.n_waves == 4                            # [a b] [c d] [e f] [g]
    assert 4 * 2 * (1 << 23) <= w2.ws_bytes < one.ws_bytes
    for enc in (True, False):
        names = [l["name"] for l in w2.launches(enc)]
        d = "enc" if enc else "dec"
        # small waves (< 4 tiles per CU) take the two-blocks-per-CU row kernels
        assert sum(n in (f"ofl::k_{d}_rowA", f"ofl::k_{d}_rowA2") for n in names) == 4
        assert sum(n.startswith(f"ofl::k_{d}_rowC") for n in names) == 4
        # one k_finalize per wave stream (no mid-call join)
        assert names.count("ofl::k_finalize") == (2 if enc else 0)
        # same algorithmic bytes whatever the schedule
        assert sum(l["bytes_alg"] for l in w2.launches(enc)) == sum(l["bytes_alg"] for l in one.launches(enc))
    w1 = EdenPlan(numels, 8, wave_mib=32, streams=1)
    assert w1.n_waves == 4 and w1.ws_bytes < w2.ws_bytes
    assert [l["name"] for l in w1.launches(True)].count("ofl::k_finalize") == 1
    # kernel choice for the row passes: auto / forced (outputs identical, GPU test)
    names0 = [l["name"] for l in EdenPlan(numels, 8, wave_mib=32, streams=1, row2=0).launches(False)]
    names1 = [l["name"] for l in EdenPlan(numels, 8, wave_mib=32, streams=1, row2=1).launches(False)]
    assert "ofl::k_dec_rowA2" not in names0 and names0.count("ofl::k_dec_rowC") == 4
    assert names1.count("ofl::k_dec_rowA2") == 4 and names1.count("ofl::k_dec_rowC2") == 4
    with pytest.raises(_lib.CodecError, match="row2"):
        EdenPlan(numels, 8, row2=2)
    for pair in (-1, 0, 1):
        assert EdenPlan(numels, 8, row2=1, pair=pair).n_waves == EdenPlan(numels, 8, row2=1).n_waves
    with pytest.raises(_lib.CodecError, match="pair"):
        EdenPlan(numels, 8, pair=2)
    big = EdenPlan([1 << 25, 1 << 22], 8, wave_mib=16, streams=1)   # a slice above the wave size
    assert big.n_waves == 2
    with pytest.raises(_lib.CodecError, match="streams"):
        EdenPlan(numels, 8, streams=3)


def test_two_stream_split_rules():
    """Two-stream plans whose large slices fit one wave: with small-slice
    launches beside them, exactly two waves cut at the closest halves (in-order
    packing against half the total would leave a third wave behind the
    first); large slices only, one wave on the caller's stream."""
    from openfl_amd.codec import EdenPlan
    from openfl_amd.workloads import WORKLOADS, numel
    sizes = [numel(s) for _, s in WORKLOADS["resnet50_fp32"]()]
    rn = EdenPlan(sizes, 8, streams=2, sset=0)
    assert rn.n_waves == 2
    rows = [l["blocks"] for l in rn.launches(True) if l["name"] in ("ofl::k_enc_rowA", "ofl::k_enc_rowA2")]
    assert len(rows) == 2 and abs(rows[0] - rows[1]) <= max(rows) // 4
    # with the small-set launch beside it, a plan that fits one wave keeps it whole
    assert EdenPlan(sizes, 8, streams=2, sset=1).n_waves == 1
    # large slices only, all in one wave: one wave on the caller's stream
    uni = EdenPlan([numel(s) for _, s in WORKLOADS["uniform_1gib"]()], 8, wave_mib=2048, streams=2)
    assert uni.n_waves == 1
    assert [l["name"] for l in uni.launches(True)].count("ofl::k_finalize") == 1
    # the default schedule: 128 MiB waves (the 1 GiB set: eight, alternating
    # streams), one finalize per wave stream
    uni = EdenPlan([numel(s) for _, s in WORKLOADS["uniform_1gib"]()], 8, streams=2)
    assert uni.n_waves == 8
    assert [l["name"] for l in uni.launches(True)].count("ofl::k_finalize") == 2
    # more than one wave of large slices: waves by the wave size, as before
    many = EdenPlan([1 << 22] * 6, 8, wave_mib=32, streams=2)
    assert many.n_waves == 3
    # ... packed largest first, so every wave holds one slice size (batch
    # order would give [2^22] [2^23] [2^22] [2^23] [2^22 2^22]): one column
    # launch per wave
    mixed = EdenPlan([1 << 22, 1 << 23, 1 << 22, 1 << 23, 1 << 22, 1 << 22], 8, wave_mib=32, streams=1)
    assert mixed.n_waves == 4
    cols = [l["name"] for l in mixed.launches(True) if "col" in l["name"]]
    assert len(cols) == 4 and cols.count("ofl::k_col6<8, true, 15>") == 2


def test_small_set_launch():
    """Tiny and small slices go out as ONE small-set launch per direction
    (k_enc_sset / k_dec_sset: groups of one size per 1024-thread workgroup),
    or with sset=0 as one launch per size class.  Same algorithmic bytes."""
    from openfl_amd import _lib
    from openfl_amd.codec import EdenPlan
    from openfl_amd.workloads import WORKLOADS, numel
    sizes = [numel(s) for _, s in WORKLOADS["resnet50_fp32"]()]
    on, off = EdenPlan(sizes, 8, sset=1), EdenPlan(sizes, 8, sset=0)
    for enc in (True, False):
        d = "enc" if enc else "dec"
        n1 = [l["name"] for l in on.launches(enc)]
        n0 = [l["name"] for l in off.launches(enc)]
        # ResNet-50's large slices fit one wave with a k_col_multi launch, so
        # the small-set groups ride in that launch (k_*_colm_set, on the
        # caller's stream) unless OFL_EDEN_FUSESET=0 keeps them apart
        fused = f"ofl::k_{d}_colm_set" in n1
        assert n1.count(f"ofl::k_{d}_sset") + n1.count(f"ofl::k_{d}_colm_set") == 1
        assert fused != ("ofl::k_col_multi" in n1)
        assert not any(n.startswith(f"ofl::k_{d}_small") or n == f"ofl::k_{d}_tiny" for n in n1)
        assert "ofl::k_enc_sset" not in n0 and f"ofl::k_{d}_tiny" in n0
        assert sum(n.startswith(f"ofl::k_{d}_small") for n in n0) == 5
        assert sum(l["bytes_alg"] for l in on.launches(enc)) == sum(l["bytes_alg"] for l in off.launches(enc))
        if not fused:
            # one 1024-thread group per 2^15 elements of one size, tiny ones 4 of one p per group
            sset = [l for l in on.launches(enc) if l["name"].endswith("_sset")][0]
            assert sset["blocks"] < sum(1 for n in sizes if 100 < n <= 1 << 15)
    with pytest.raises(_lib.CodecError, match="sset"):
        EdenPlan(sizes, 8, sset=3)


def test_plan_errors():
    from openfl_amd import _lib
    from openfl_amd.codec import EdenPlan
    with pytest.raises(_lib.CodecError, match="nbits"):
        EdenPlan([1000], n_bits=9)
    with pytest.raises(_lib.CodecError, match="power of two"):
        EdenPlan([1000], n_bits=8, dims=[[1000]])


def test_plan_from_metadata_dims():
    from openfl_amd.codec import EdenPlan
    p = EdenPlan([7], n_bits=3, dims=[[8, 8, 8]])
    assert p.dims == [[8, 8, 8]] and p.planes_bytes == 3 * 24 // 8


def test_batched_seed_draws_match_single_calls():
    """eden_seeds: one vectorised np.random draw = T single draws (values and
    the generator's state afterwards)."""
    from openfl_amd.pipelines.eden_pipeline import eden_seed, eden_seeds
    rng = np.random.default_rng(9)
    totals = [np.float32(v) for v in rng.standard_normal(500)] + [np.float64(0.0), np.float64(-3.25)]
    for s in (0, 1, 12345):
        np.random.seed(s)
        one = [eden_seed(None, "reference", t) for t in totals]
        after = np.random.randint(0, 2 ** 31)
        np.random.seed(s)
        assert eden_seeds(totals) == one
        assert np.random.randint(0, 2 ** 31) == after


def test_host_copy_many_and_serial_sums_many():
    """Host helpers of the batched pipeline path (no GPU): parallel memcpy's
    land where they should; batched serial sums equal the one-array sums."""
    from openfl_amd import _lib
    from openfl_amd.pipelines.eden_pipeline import _copy_many, _serial_sum, _serial_sums
    rng = np.random.default_rng(5)
    srcs = [rng.standard_normal(n).astype(np.float32) for n in (0, 1, 1000, 300_000, 77)]
    dst = np.full(sum(s.size for s in srcs) + 40, -1.0, np.float32)
    offs, acc = [], 0
    for s_ in srcs:
        offs.append(acc)
        acc += s_.size + 8
    _copy_many([dst.ctypes.data + 4 * o for o in offs], [s_.ctypes.data for s_ in srcs], [4 * s_.size for s_ in srcs])
    for o, s_ in zip(offs, srcs):
        np.testing.assert_array_equal(dst[o:o + s_.size], s_)
    flats = srcs + [rng.standard_normal(5000), np.float32([1e8, 1.0, -1e8])]
    got = _serial_sums(flats)
    for g, f in zip(got, flats):
        ref = _serial_sum(f)
        assert g == ref and type(g) is type(ref)
    assert _lib.lib().ofl_host_copy_many(0, None, None, None, 4) == 0


def test_one_call_host_entry_points_check_their_block_layout():
    """ofl_eden_encode_host / _decode_host validate the caller's pinned / device
    block layout against the plan before touching the GPU (OFL_EINVAL)."""
    import ctypes
    from openfl_amd import _lib
    from openfl_amd.codec import EdenPlan
    L = _lib.lib()
    p = EdenPlan([1000], n_bits=8)
    buf = ctypes.create_string_buffer(1 << 16)
    a = ctypes.addressof(buf)
    pb, ns = p.planes_bytes, p.n_slices
    # encode: seeds must sit after the x arena, scales after the planes
    assert L.ofl_eden_encode_host(p.handle, a, a, 8192, 4 * 1000 - 4, a, a, 8192, 1024, None, 0, None) == _lib.OFL_EINVAL
    assert L.ofl_eden_encode_host(p.handle, a, a, 8192, 4096, a, a, pb + 4 * ns, pb - 1, None, 0, None) == _lib.OFL_EINVAL
    assert L.ofl_eden_encode_host(p.handle, a, a, 4096, 4096, a, a, 8192, 1024, None, 0, None) == _lib.OFL_EINVAL
    # decode: scales after the planes, seeds after the scales, y no longer than the arena
    assert L.ofl_eden_decode_host(p.handle, a, a, 8192, pb - 1, 4096, a, a, 4000, None, 0, None) == _lib.OFL_EINVAL
    assert L.ofl_eden_decode_host(p.handle, a, a, 8192, 256, 256, a, a, 4000, None, 0, None) == _lib.OFL_EINVAL
    assert L.ofl_eden_decode_host(p.handle, a, a, 8192, 256, 1024, a, a, 4004, None, 0, None) == _lib.OFL_EINVAL
    assert L.ofl_eden_encode_host(None, a, a, 8192, 4096, a, a, 8192, 1024, None, 0, None) == _lib.OFL_EINVAL


def test_gzip_ranks_to_checks_its_host_buffer():
    """ofl_gzip_ranks_to refuses a missing or too small host destination
    before touching the GPU (OFL_EINVAL, with a message)."""
    import ctypes
    from openfl_amd import _lib
    L = _lib.lib()
    buf = ctypes.create_string_buffer(1 << 12)
    a = ctypes.addressof(buf)
    ln = ctypes.c_size_t()
    assert L.ofl_gzip_ranks_to(a, 1000, a, 4096, None, 4096, 8, ctypes.byref(ln), a, 4096, None) == _lib.OFL_EINVAL
    assert b"host_dst" in L.ofl_gzip_last_error()
    assert L.ofl_gzip_ranks_to(a, 1000, a, 4096, a, 4095, 8, ctypes.byref(ln), a, 4096, None) == _lib.OFL_EINVAL
    assert b"host_cap" in L.ofl_gzip_last_error()


def test_big_slice_sub_waves():
    """A 5-pass slice bigger than the wave size runs passes 1-2 and 4-5 in
    sub-waves (explicit tile lists) around one whole-slice middle pass; the
    sub-waves cover the slice's tiles once per pass.  Plans whose wave holds
    the slice keep whole-slice passes."""
    from openfl_amd.codec import EdenPlan
    split = [(l["name"], l["blocks"]) for l in EdenPlan([1 << 26], 8, wave_mib=64, streams=1).launches(True)]
    rows_a = [b for n, b in split if n == "ofl::k_enc_rowA2"]
    rows_c = [b for n, b in split if n.startswith("ofl::k_enc_rowC2")]
    outer = [b for n, b in split if n == "ofl::k_col<5, false>"]
    assert len(rows_a) == 4 and sum(rows_a) == 2048 and sum(rows_c) == 2048 and sum(outer) == 2 * 2048
    mid = [i for i, (n, _) in enumerate(split) if n == "ofl::k_col<6, true>"]
    assert len(mid) == 1 and split[mid[0]][1] == 2048
    # every row-A sub-wave (and its level-1 pass) before the middle pass, every row-C one after
    assert max(i for i, (n, _) in enumerate(split) if n == "ofl::k_enc_rowA2") < mid[0]
    assert min(i for i, (n, _) in enumerate(split) if n.startswith("ofl::k_enc_rowC2")) > mid[0]
    whole = [n for n, _ in [(l["name"], l["blocks"]) for l in EdenPlan([1 << 26], 8, wave_mib=4096, streams=1).launches(True)]]
    assert whole.count("ofl::k_col<5, false>") == 2 and "ofl::k_enc_rowA2" not in whole
