"""Plugin base classes: mirror of the reference's tests/openfl/pipelines/test_pipeline.py."""
import numpy as np
import pytest

from openfl_amd.pipelines import (Float32NumpyArrayToBytes, NoCompressionPipeline,
                                  TransformationPipeline, Transformer)


@pytest.fixture
def named_tensor():
    """Stand-in for the reference fixture: 32 bytes of b'1', int_list [1, 8]."""
    return {"data_bytes": 32 * b"1", "metadata": {"int_to_float": {1: 1.0}, "int_list": [1, 8],
                                                   "bool_list": [True]}}


def test_transformer_forward():
    with pytest.raises(NotImplementedError):
        Transformer().forward(None)


def test_transformer_backward():
    with pytest.raises(NotImplementedError):
        Transformer().backward(None, None)


def test_f32natb_is_lossy():
    assert Float32NumpyArrayToBytes().lossy is False


def test_f32natb_forward(named_tensor):
    t = Float32NumpyArrayToBytes()
    md = named_tensor["metadata"]
    arr = np.frombuffer(named_tensor["data_bytes"], np.float32).reshape(tuple(md["int_list"]))
    data_bytes, t_md = t.forward(arr)
    assert t_md["int_list"] == md["int_list"]
    assert data_bytes == named_tensor["data_bytes"]


def test_f32natb_backward(named_tensor):
    t = Float32NumpyArrayToBytes()
    md = named_tensor["metadata"]
    out = t.backward(named_tensor["data_bytes"], md)
    assert out.shape == tuple(md["int_list"]) and out.dtype == np.float32


def test_f32natb_casts_float64():
    data_bytes, md = Float32NumpyArrayToBytes().forward(np.arange(6, dtype=np.float64).reshape(2, 3))
    assert np.array_equal(np.frombuffer(data_bytes, np.float32), np.arange(6, dtype=np.float32))
    assert md["int_list"] == [2, 3]


def test_transformation_pipeline_forward(named_tensor):
    tp = TransformationPipeline([Float32NumpyArrayToBytes()])
    arr = np.frombuffer(named_tensor["data_bytes"], np.float32).reshape(1, 8)
    data, md = tp.forward(arr)
    assert isinstance(data, bytes) and len(md) == 1 and md[0]["int_list"] == [1, 8]


def test_transformation_pipeline_backward_pops_metadata(named_tensor):
    tp = TransformationPipeline([Float32NumpyArrayToBytes()])
    md = [named_tensor["metadata"]]
    out = tp.backward(named_tensor["data_bytes"], md)
    assert out.shape == (1, 8)
    assert md == []  # list.pop() semantics (pipeline.py:161-163)


def test_transformation_pipeline_is_lossy():
    class L(Transformer):
        lossy = True
    class N(Transformer):
        lossy = False
    assert TransformationPipeline([N(), L()]).is_lossy()
    assert not TransformationPipeline([N(), N()]).is_lossy()


def test_no_compression_roundtrip():
    x = np.random.default_rng(0).standard_normal((3, 5)).astype(np.float32)
    p = NoCompressionPipeline()
    data, md = p.forward(x)
    assert not p.is_lossy()
    np.testing.assert_array_equal(p.backward(data, md), x)
