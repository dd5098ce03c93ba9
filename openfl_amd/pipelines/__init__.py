"""OpenFL-compatible compression pipelines backed by gfx950 kernels.

Mirrors the class names of openfl/pipelines/__init__.py for the codec path.
EdenPipeline is imported lazily so that `import openfl_amd.pipelines` works on
hosts without torch/ROCm (the Eden path itself then raises when used).
"""
from openfl_amd.pipelines.no_compression_pipeline import NoCompressionPipeline
from openfl_amd.pipelines.pipeline import (Float32NumpyArrayToBytes, TransformationPipeline,
                                           Transformer)

__all__ = ["EdenPipeline", "EdenTransformer", "Float32NumpyArrayToBytes", "NoCompressionPipeline",
           "TransformationPipeline", "Transformer"]


def __getattr__(name):
    if name in ("EdenPipeline", "EdenTransformer", "Eden"):
        from openfl_amd.pipelines import eden_pipeline
        return getattr(eden_pipeline, name)
    raise AttributeError(name)
