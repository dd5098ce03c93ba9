"""Plugin base classes, mirroring openfl/pipelines/pipeline.py.

Same names, signatures and semantics as the reference (citations are to
/root/reference/openfl/pipelines/pipeline.py) so that openfl/federated and
openfl/component can load an openfl_amd pipeline through
``compression_pipeline.template`` unchanged.
"""
import numpy as np


class Transformer:
    """Base transformer: forward(data) -> (data, metadata); backward inverts (:9-48)."""

    def forward(self, data, **kwargs):
        raise NotImplementedError

    def backward(self, data, metadata, **kwargs):
        raise NotImplementedError


class Float32NumpyArrayToBytes(Transformer):
    """Lossless fp32 <-> bytes with {"int_list": shape} metadata (:51-93)."""

    def __init__(self):
        self.lossy = False

    def forward(self, data, **kwargs):
        if data.dtype != np.float32:
            data = data.astype(np.float32)
        return data.tobytes(order="C"), {"int_list": list(data.shape)}

    def backward(self, data, metadata, **kwargs):
        shape = tuple(metadata["int_list"])
        return np.frombuffer(data, dtype=np.float32).reshape(shape, order="C")


class TransformationPipeline:
    """Sequential transformer chain (:96-172).

    forward copies the input, then applies each transformer, collecting one
    metadata entry per transformer.  backward walks the transformers in
    reverse, consuming metadata with list.pop() -- it empties the caller's
    list, exactly like the reference (:161-163).  is_lossy() is any-of.
    """

    def __init__(self, transformers, **kwargs):
        self.transformers = transformers

    def forward(self, data, **kwargs):
        transformer_metadata = []
        data = data.copy()
        for transformer in self.transformers:
            data, metadata = transformer.forward(data=data, **kwargs)
            transformer_metadata.append(metadata)
        return data, transformer_metadata

    def backward(self, data, transformer_metadata, **kwargs):
        for transformer in self.transformers[::-1]:
            data = transformer.backward(data=data, metadata=transformer_metadata.pop(), **kwargs)
        return data

    def is_lossy(self):
        return any(transformer.lossy for transformer in self.transformers)
