"""RandomShiftPipeline (openfl/pipelines/random_shift_pipeline.py:12-77).

A lossless pipeline ("adjacent, not hot").  Semantics kept
from the reference:
  * forward draws ONE ``np.random.uniform(-20, 20, shape)`` from the global
    NumPy RNG (cast to float32), adds it, and records every shift in
    ``int_to_float`` keyed by C-order flat index (:22-43);
  * backward rebuilds the shift array from ``int_to_float[0..len-1]`` and
    subtracts it (:45-68).  With in-process float32 values the result is
    float32; with wire values (Python floats from MetadataProto) numpy
    promotes to float64 -- reproduced, not "fixed".

``device=None`` (default) does the arithmetic with NumPy on the host, as the
reference.  ``device="cuda:N"`` does the add / subtract on the GPU
(``ofl_apply_delta``: float32 add; ``ofl_sub_f32_f64``: the float64 subtract of
wire metadata) -- bit-identical, since both are single IEEE operations.  The
shift still comes from the global NumPy RNG (the reference's stream, on the
host), and the O(n) metadata map is built on the host either way: that map,
not the arithmetic, is this pipeline's cost.  Inputs other than float32
arrays (e.g. the aggregator's float64 deltas) take the host path.
"""
import numpy as np

from openfl_amd.pipelines.pipeline import Float32NumpyArrayToBytes, TransformationPipeline, Transformer


def _device_or_none(device):
    if device is None or str(device) == "cpu":
        return None
    from openfl_amd.codec import resolve_device
    return resolve_device(device)


def _shift_on_device(data, shift, device):
    """data + shift (float32) on the GPU."""
    import torch
    from openfl_amd import _lib
    x = torch.from_numpy(np.require(data, None, ["C", "W"]).reshape(-1)).to(device)
    s = torch.from_numpy(np.ascontiguousarray(shift).reshape(-1)).to(device)
    out = torch.empty_like(x)
    with torch.cuda.device(device):
        _lib.check_agg(_lib.lib().ofl_apply_delta(x.data_ptr(), s.data_ptr(), x.numel(), out.data_ptr(),
                                                  torch.cuda.current_stream(device).cuda_stream))
    return out.cpu().numpy().reshape(data.shape)


def _unshift_on_device(data, shift, device):
    """data - shift on the GPU: float32 (in-process metadata) or float64 (wire)."""
    import torch
    from openfl_amd import _lib
    x = torch.from_numpy(np.require(data, np.float32, ["C", "W"]).reshape(-1)).to(device)
    with torch.cuda.device(device):
        st = torch.cuda.current_stream(device).cuda_stream
        if shift.dtype == np.float32:  # a - b == a + (-b) exactly in IEEE arithmetic
            s = torch.from_numpy(np.ascontiguousarray(-shift).reshape(-1)).to(device)
            out = torch.empty_like(x)
            _lib.check_agg(_lib.lib().ofl_apply_delta(x.data_ptr(), s.data_ptr(), x.numel(), out.data_ptr(), st))
        else:
            s = torch.from_numpy(np.ascontiguousarray(shift, np.float64).reshape(-1)).to(device)
            out = torch.empty(x.numel(), dtype=torch.float64, device=device)
            _lib.check_agg(_lib.lib().ofl_sub_f32_f64(x.data_ptr(), s.data_ptr(), x.numel(), out.data_ptr(), st))
    return out.cpu().numpy().reshape(shift.shape)


class RandomShiftTransformer(Transformer):
    def __init__(self, device=None):
        self.lossy = False
        self.device = _device_or_none(device)

    def forward(self, data, **kwargs):
        shape = data.shape
        shift = np.random.uniform(low=-20, high=20, size=shape).astype(np.float32)
        flat = shift.reshape(-1)  # C order
        if self.device is not None and isinstance(data, np.ndarray) and data.dtype == np.float32 and data.size:
            out = _shift_on_device(data, shift, self.device)
        else:
            out = data + shift
        return out, {"int_to_float": {i: flat[i] for i in range(flat.size)}, "int_list": list(shape)}

    def backward(self, data, metadata, **kwargs):
        shape = tuple(metadata["int_list"])
        itf = metadata["int_to_float"]
        shift = np.array([itf[i] for i in range(len(itf))]).reshape(shape)
        if (self.device is not None and isinstance(data, np.ndarray) and data.dtype == np.float32 and data.size
                and shift.dtype in (np.float32, np.float64) and data.size == shift.size):
            return _unshift_on_device(data.reshape(shape), shift, self.device)
        return data - shift


class RandomShiftPipeline(TransformationPipeline):
    def __init__(self, device=None, **kwargs):
        super().__init__(transformers=[RandomShiftTransformer(device), Float32NumpyArrayToBytes()], **kwargs)
