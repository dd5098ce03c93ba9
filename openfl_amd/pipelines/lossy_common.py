"""Shared pieces of the KC / SKC / STC pipelines (GZIP, k-means, sparsify).

Mirrors the reference classes (paths relative to /root/reference):
  GZIPTransformer     kc_pipeline.py:117-156 (== skc :190-230 == stc :146-215)
  _float_to_int       kc_pipeline.py:88-114
The k-means / top-k / ternary numerics run on the GPU (openfl_amd.lossy);
gzip and tiny (n < n_clusters) cases run on the host exactly as the
reference does.
"""

import numpy as np
import torch

from openfl_amd import lossy
from openfl_amd.codec import PerThreadDevice, resolve_device
from openfl_amd.pipelines.pipeline import Transformer


def float_to_int(np_array):
    """_float_to_int (kc_pipeline.py:88-114): sorted unique values -> int32 ranks."""
    flat = np_array.reshape(-1)
    uniq, idx = lossy.rank_map(flat)
    int_array = idx.astype(np.int32).reshape(np_array.shape)
    return int_array, {i: u for i, u in enumerate(uniq)}


class GZIPTransformer(Transformer):
    """float32 bytes -> gzip (lossless).  backend="device" (the pipelines'
    default): the GPU gzip of rank arrays (lossy.gzip_ranks, TLZ in
    csrc/deflate_kernels.hip); backend="host": gzip.compress at `level`
    (large payloads as a multi-member stream compressed on host threads).
    Either way gzip.decompress reads the stream back to the same bytes."""

    def __init__(self, level=9, threads=8, backend="device"):
        if backend not in ("host", "device"):
            raise ValueError("gzip backend must be 'host' or 'device'")
        self.lossy = False
        self.level = level
        self.threads = threads
        self.backend = backend

    def forward(self, data, **kwargs):
        return lossy.gzip_compress(data.astype(np.float32).tobytes(), self.level, self.threads), {}

    def forward_device(self, ranks_dev):
        """forward of a float32 device array of ranks: on the GPU with the
        device backend (values outside 0..31 go through the host gzip)."""
        if self.backend == "device":
            try:
                return lossy.gzip_ranks(ranks_dev), {}
            except lossy._lib.CodecError as e:
                if "values must be" not in str(e):
                    raise
        return self.forward(ranks_dev.cpu().numpy())

    def backward(self, data, metadata, **kwargs):
        # member-indexed streams inflate on native threads; others via gzip.decompress
        return lossy.gunzip(data, self.threads).view(np.float32)


def gzip_lut_backward_device(data, int2float_map, n, device):
    """GZIPTransformer.backward followed by the LUT backward of the lossy
    transformer before it (KmeansTransformer / TernaryTransformer:
    kc_pipeline.py:79-83, :152-156; stc_pipeline.py:126-130), fused on the
    GPU: the payload inflates straight into HBM (lossy.gunzip_device), the
    LUT decodes it there.  n: element count the payload must decode to.
    -> float32 device tensor of n elements."""
    buf = torch.empty(4 * max(n, 1), dtype=torch.uint8, device=device)
    # the LUT fused into the inflate's stores (one tensor: elements [0, n))
    # (the length is checked against 4n before anything is inflated or looked up)
    raw = lossy.gunzip_device(data, buf, lut=lossy.lut_tables([0], [n], [int2float_map], buf.device) if n else None,
                              expect_bytes=4 * n)
    if n == 0:
        return torch.empty(0, dtype=torch.float32, device=device)
    return raw.view(torch.float32)


def to_device(data, device):
    flat = np.ascontiguousarray(np.asarray(data).reshape(-1), dtype=np.float32)
    if not flat.flags.writeable:  # torch.from_numpy needs a writable buffer
        flat = flat.copy()
    if flat.size == 0:
        return torch.empty(0, dtype=torch.float32, device=device)
    return torch.from_numpy(flat).to(device)


def kmeans_ranks(x_dev, n_cluster, value_dtype):
    """k-means of a device vector -> (float32 rank tensor on device, int_to_float
    map {rank: centre as value_dtype}) with the reference's rank semantics:
    np.unique over the centres actually used (kc_pipeline.py:55-61)."""
    seed = int(np.random.randint(0, 2 ** 31 - 1))  # sklearn draws from the global RNG too
    ranks = torch.empty_like(x_dev)
    _, _, _, uniq = lossy.kmeans_batch(x_dev, [0], [x_dev.numel()], n_cluster, n_init=n_cluster, seed=seed,
                                       value_f64=np.dtype(value_dtype) == np.float64, ranks_out=ranks)
    return ranks, {i: u for i, u in enumerate(uniq[0])}


def lut_backward(data, int2float_map, device):
    """Reference lossy backward on a float32 array: sequential in-place
    `data[data == key] = value` (kc_pipeline.py:79-83), on the GPU."""
    arr = np.asarray(data)
    if arr.size == 0:
        return arr.astype(np.float32, copy=True)
    out = lossy.lut_decode(to_device(arr, device), int2float_map)
    return out.cpu().numpy().reshape(arr.shape)


__all__ = ["GZIPTransformer", "PerThreadDevice", "float_to_int", "gzip_lut_backward_device", "kmeans_ranks", "lut_backward",
           "resolve_device", "to_device"]
