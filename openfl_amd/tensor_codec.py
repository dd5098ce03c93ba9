"""TensorCodec with the reference's method surface (openfl/pipelines/tensor_codec.py).

The reference TensorCodec (tensor_codec.py:13-244) wraps a compression
pipeline with TensorKey bookkeeping: compress/decompress pick the lossy or the
lossless pipeline and rename the key's tags; generate_delta / apply_delta are
the NumPy `new - base` / `base + delta` around them; find_dependencies lists
the keys a model tensor is rebuilt from.  This module keeps that surface for
host ndarrays (so callers such as Aggregator / Collaborator run unchanged with
an openfl_amd pipeline plugged in).  The device path for a whole model update
-- average, delta, compress, decompress and apply fused over one arena -- is
openfl_amd.aggregation.RoundEnd.
"""
from collections import namedtuple

import numpy as np

from openfl_amd.pipelines.no_compression_pipeline import NoCompressionPipeline

# openfl/utilities/types.py:10,14
TensorKey = namedtuple("TensorKey", ["tensor_name", "origin", "round_number", "report", "tags"])
LocalTensor = namedtuple("LocalTensor", ["col_name", "tensor", "weight"])


def change_tags(tags, *, add_field=None, remove_field=None):
    """Tags as a sorted tuple with add_field added / remove_field removed
    (openfl/utilities/utils.py:212-241); removing an absent tag raises."""
    out = set(tags)
    if add_field is not None:
        out.add(add_field)
    if remove_field is not None:
        if remove_field not in out:
            raise Exception(f"{remove_field} not in tags {tuple(sorted(out))}")
        out.discard(remove_field)
    return tuple(sorted(out))


class TensorCodec:
    """Lossy/lossless pipeline selection + TensorKey tags (tensor_codec.py:13-244)."""

    def __init__(self, compression_pipeline):
        self.compression_pipeline = compression_pipeline
        self.lossless_pipeline = NoCompressionPipeline() if compression_pipeline.is_lossy() \
            else compression_pipeline

    def set_lossless_pipeline(self, lossless_pipeline):
        assert lossless_pipeline.is_lossy() is False, "The provided pipeline is not lossless"
        self.lossless_pipeline = lossless_pipeline

    def compress(self, tensor_key, data, require_lossless=False, **kwargs):
        """-> (key tagged 'compressed' or 'lossy_compressed', payload, metadata) (:52-85)."""
        pipe = self.lossless_pipeline if require_lossless else self.compression_pipeline
        payload, metadata = pipe.forward(data, **kwargs)
        name, origin, rnd, report, tags = tensor_key
        lossless = require_lossless or not self.compression_pipeline.is_lossy()
        tags = change_tags(tags, add_field="compressed" if lossless else "lossy_compressed")
        return TensorKey(name, origin, rnd, report, tags), payload, metadata

    def decompress(self, tensor_key, data, transformer_metadata, require_lossless=False, **kwargs):
        """-> (key with the compression tag replaced, ndarray) (:87-147)."""
        name, origin, rnd, report, tags = tensor_key
        assert len(transformer_metadata) > 0, "metadata must be included for decompression"
        assert "compressed" in tags or "lossy_compressed" in tags, "Cannot decompress an uncompressed tensor"
        if require_lossless:
            assert "compressed" in tags, "Cannot losslessly decompress lossy tensor"
        lossless = require_lossless or "compressed" in tags
        pipe = self.lossless_pipeline if lossless else self.compression_pipeline
        out = pipe.backward(data, transformer_metadata, **kwargs)
        if "lossy_compressed" in tags:
            new_tags = change_tags(tags, add_field="lossy_decompressed", remove_field="lossy_compressed")
        elif "compressed" in tags:
            new_tags = change_tags(tags, remove_field="compressed")
        else:
            raise NotImplementedError("Decompression is only supported on compressed data")
        return TensorKey(name, origin, rnd, report, new_tags), out

    @staticmethod
    def generate_delta(tensor_key, nparray, base_model_nparray):
        """-> (key + 'delta', nparray - base) (:149-180)."""
        name, origin, rnd, report, tags = tensor_key
        if not np.isscalar(nparray):
            assert nparray.shape == base_model_nparray.shape, (
                f"Shape of updated layer ({nparray.shape}) is not equal to base "
                f"layer shape of ({base_model_nparray.shape})")
        assert "model" not in tags, ("The tensorkey should be provided from the layer with new weights, "
                                     "not the base model")
        return TensorKey(name, origin, rnd, report, change_tags(tags, add_field="delta")), nparray - base_model_nparray

    @staticmethod
    def apply_delta(tensor_key, delta, base_model_nparray, creates_model=False):
        """-> (model key, base + delta) (:182-211)."""
        name, origin, rnd, report, tags = tensor_key
        if not np.isscalar(base_model_nparray):
            assert delta.shape == base_model_nparray.shape, (
                f"Shape of delta ({delta.shape}) is not equal to shape of model layer "
                f"({base_model_nparray.shape})")
        if "aggregator" in origin and not creates_model:
            key = TensorKey(name, origin, rnd, report, change_tags(tags, remove_field="delta"))
        else:
            key = TensorKey(name, origin, rnd, report, ("model",))
        return key, base_model_nparray + delta

    def find_dependencies(self, tensor_key, send_model_deltas):
        """Keys a model tensor is rebuilt from: the previous round's model and
        this round's compressed aggregated delta (:213-244)."""
        name, origin, rnd, report, tags = tensor_key
        if "model" not in tags or not send_model_deltas or rnd < 1:
            return []
        comp = "lossy_compressed" if self.compression_pipeline.is_lossy() else "compressed"
        return [TensorKey(name, origin, rnd - 1, report, tags),
                TensorKey(name, origin, rnd, report, ("aggregated", "delta", comp))]
