"""TensorCodec surface (reference tests/openfl/pipelines/test_tensor_codec.py)
and the host parts of openfl_amd.aggregation; no GPU needed."""
from unittest import mock

import numpy as np
import pytest

from openfl_amd.pipelines.no_compression_pipeline import NoCompressionPipeline
from openfl_amd.tensor_codec import TensorCodec, TensorKey, change_tags


@pytest.fixture
def key():
    return TensorKey("tensor_name", "agg", 0, False, ("model",))


def _lossy():
    p = mock.Mock()
    p.is_lossy.return_value = True
    p.forward.return_value = (b"x", [{}])
    p.backward.return_value = np.zeros(3, np.float32)
    return p


def test_change_tags():
    assert change_tags(("b", "a"), add_field="c") == ("a", "b", "c")
    assert change_tags(("a", "a", "b"), remove_field="a") == ("b",)
    assert change_tags(("a",), add_field="a") == ("a",)
    with pytest.raises(Exception, match="not in tags"):
        change_tags(("a",), remove_field="z")


def test_compress_tags(key):
    data = np.arange(4, dtype=np.float32)
    tc = TensorCodec(NoCompressionPipeline())
    k, payload, md = tc.compress(key, data)
    assert "compressed" in k.tags and k[:4] == key[:4]
    k, _, _ = tc.compress(key, data, require_lossless=True)
    assert "compressed" in k.tags
    tc = TensorCodec(_lossy())
    assert isinstance(tc.lossless_pipeline, NoCompressionPipeline)
    k, _, _ = tc.compress(key, data)
    assert "lossy_compressed" in k.tags
    k, _, _ = tc.compress(key, data, require_lossless=True)
    assert "compressed" in k.tags and "lossy_compressed" not in k.tags


def test_decompress_paths(key):
    tc = TensorCodec(_lossy())
    with pytest.raises(AssertionError):
        tc.decompress(key, b"x", [])
    with pytest.raises(AssertionError):
        tc.decompress(key, b"x", [{}])                       # no compression tag
    lk = TensorKey("t", "o", 0, False, ("lossy_compressed",))
    with pytest.raises(AssertionError):
        tc.decompress(lk, b"x", [{}], require_lossless=True)
    k, _ = tc.decompress(lk, b"x", [{}])
    assert "lossy_decompressed" in k.tags and "lossy_compressed" not in k.tags
    tc.compression_pipeline.backward.assert_called_with(b"x", [{}])
    tc.lossless_pipeline = mock.Mock()
    ck = TensorKey("t", "o", 0, False, ("compressed",))
    k, _ = tc.decompress(ck, b"y", [{}], require_lossless=True)
    tc.lossless_pipeline.backward.assert_called_with(b"y", [{}])
    assert "compressed" not in k.tags


def test_deltas(key):
    a = np.arange(6, dtype=np.float32).reshape(2, 3)
    tk = TensorKey("t", "aggregator_x", 1, False, ("trained",))
    dk, d = TensorCodec.generate_delta(tk, a, a)
    assert "delta" in dk.tags and np.array_equal(d, a - a)
    with pytest.raises(AssertionError):
        TensorCodec.generate_delta(key, a, a)                 # 'model' in tags
    nk, m = TensorCodec.apply_delta(dk, a, a)
    assert "delta" not in nk.tags and np.array_equal(m, a + a)
    ck = TensorKey("t", "collab", 1, False, ("trained", "delta"))
    nk, _ = TensorCodec.apply_delta(ck, a, a)
    assert nk.tags == ("model",)


def test_find_dependencies():
    tc = TensorCodec(NoCompressionPipeline())
    k = TensorKey("t", "o", 2, False, ("model",))
    assert tc.find_dependencies(k, False) == []
    assert tc.find_dependencies(TensorKey("t", "o", 2, False, ("trained",)), True) == []
    assert tc.find_dependencies(TensorKey("t", "o", 0, False, ("model",)), True) == []
    d = tc.find_dependencies(k, True)
    assert d[0].round_number == 1 and d[0].tags == k.tags and d[1].tags == ("aggregated", "delta", "compressed")
    assert TensorCodec(_lossy()).find_dependencies(k, True)[1].tags == ("aggregated", "delta", "lossy_compressed")


def test_weight_sum_is_numpys():
    from openfl_amd.aggregation import weight_sum
    rng = np.random.default_rng(1)
    for C in (1, 3, 9, 130):
        w = rng.random(C)
        sums = {weight_sum(w, d) for d in range(5)}
        assert len(sums) == 1
        xs = [rng.standard_normal(5).astype(np.float32) for _ in range(C)]
        _, scl = np.average(xs, weights=w, axis=0, returned=True)
        assert scl[0] == sums.pop()


def test_weights_dtype_rules():
    from openfl_amd import _lib
    from openfl_amd.aggregation import _f64_weights
    assert _f64_weights([1, 2], 2).dtype == np.float64
    with pytest.raises(_lib.CodecError):
        _f64_weights(np.float32([0.5, 0.5]), 2)               # np.average would compute in float32
    with pytest.raises(_lib.CodecError):
        _f64_weights([1.0], 2)
