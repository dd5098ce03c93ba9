"""OpenFL-compatible compression pipelines backed by gfx950 kernels.

Mirrors the class names of openfl/pipelines/__init__.py for the codec path.
The GPU pipelines (Eden, KC, SKC, STC) are imported lazily so that
`import openfl_amd.pipelines` works on hosts without torch/ROCm (they raise
when used without a GPU).
"""
from openfl_amd.pipelines.no_compression_pipeline import NoCompressionPipeline
from openfl_amd.pipelines.random_shift_pipeline import RandomShiftPipeline, RandomShiftTransformer
from openfl_amd.pipelines.pipeline import (Float32NumpyArrayToBytes, TransformationPipeline,
                                           Transformer)

__all__ = ["EdenPipeline", "EdenTransformer", "Float32NumpyArrayToBytes", "KCPipeline", "NoCompressionPipeline",
           "RandomShiftPipeline", "RandomShiftTransformer", "SKCPipeline", "STCPipeline", "TransformationPipeline",
           "Transformer"]

_LAZY = {"EdenPipeline": "eden_pipeline", "EdenTransformer": "eden_pipeline", "Eden": "eden_pipeline",
         "KCPipeline": "kc_pipeline", "SKCPipeline": "skc_pipeline", "STCPipeline": "stc_pipeline"}


def __getattr__(name):
    if name in _LAZY:
        import importlib
        return getattr(importlib.import_module("openfl_amd.pipelines." + _LAZY[name]), name)
    raise AttributeError(name)
