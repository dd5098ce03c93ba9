"""NoCompressionPipeline (openfl/pipelines/no_compression_pipeline.py:10-15)."""
from openfl_amd.pipelines.pipeline import Float32NumpyArrayToBytes, TransformationPipeline


class NoCompressionPipeline(TransformationPipeline):
    """The lossless pass-through pipeline: fp32 bytes + shape."""

    def __init__(self, **kwargs):
        super().__init__(transformers=[Float32NumpyArrayToBytes()], **kwargs)
