"""NoCompressionPipeline (openfl/pipelines/no_compression_pipeline.py:10-15).

The lossless pass-through: float32 bytes + {"int_list": shape}.  Host NumPy
arrays go through exactly the reference's path.  Device variant: forward also
accepts a tensor resident on a ROCm GPU (e.g. an aggregator keeping its
model on the device) and hands back the same bytes after one D2H through
pinned memory; ``backward_device`` returns the decoded array as a device
tensor (one H2D) for callers that keep it there.  Nothing here computes.
"""
import numpy as np

from openfl_amd.pipelines.pipeline import Float32NumpyArrayToBytes, TransformationPipeline


def _is_device_tensor(x):
    try:
        import torch
    except ImportError:  # pragma: no cover
        return False
    return isinstance(x, torch.Tensor) and x.is_cuda


class NoCompressionPipeline(TransformationPipeline):
    """The lossless pass-through pipeline: fp32 bytes + shape."""

    def __init__(self, device=None, **kwargs):
        super().__init__(transformers=[Float32NumpyArrayToBytes()], **kwargs)
        self.device = None
        if device is not None and str(device) != "cpu":
            from openfl_amd.codec import resolve_device
            self.device = resolve_device(device)

    def forward(self, data, **kwargs):
        if _is_device_tensor(data):
            import torch
            t = data.detach().to(torch.float32).contiguous()
            host = torch.empty(tuple(t.shape), dtype=torch.float32).pin_memory()
            host.copy_(t)  # synchronous D2H into pinned memory
            return host.numpy().tobytes(order="C"), [{"int_list": list(t.shape)}]
        return super().forward(data, **kwargs)

    def backward_device(self, data, transformer_metadata, **kwargs):
        """backward, returning a float32 tensor on this pipeline's device."""
        import torch
        arr = self.backward(data, transformer_metadata, **kwargs)
        dev = self.device if self.device is not None else torch.device("cuda", torch.cuda.current_device())
        return torch.from_numpy(np.array(arr, dtype=np.float32, copy=True)).to(dev)
