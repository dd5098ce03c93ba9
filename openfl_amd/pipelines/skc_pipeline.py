"""SKCPipeline on MI355X: drop-in for openfl/pipelines/skc_pipeline.py.

SparsityTransformer (top-k, :16-94) + KmeansTransformer (:97-187, no int_list,
runs on the float64 sparse vector) + GZIPTransformer.  Top-k and k-means run
on the GPU (see stc_pipeline / kc_pipeline for the parity notes).
"""
import numpy as np

from openfl_amd.pipelines.lossy_common import (GZIPTransformer, float_to_int, gzip_lut_backward_device,
                                               kmeans_ranks, lut_backward, PerThreadDevice, to_device)
from openfl_amd.pipelines.pipeline import TransformationPipeline, Transformer
from openfl_amd.pipelines.stc_pipeline import SparsityTransformer


class KmeansTransformer(PerThreadDevice, Transformer):
    """k-means on a flattened (sparse, float64) vector; {"int_to_float"} only."""

    def __init__(self, n_cluster=6, device="cpu", share=None):
        self.n_cluster = n_cluster
        self.lossy = True
        self._init_devices(device, share)

    def forward(self, data, **kwargs):
        data = np.asarray(data)
        if data.size >= self.n_cluster:
            ranks, m = kmeans_ranks(to_device(data, self.device), self.n_cluster, data.dtype)
            int_array = ranks.cpu().numpy().astype(np.int32)
        else:
            int_array, m = float_to_int(data.reshape((-1, 1)))
        return int_array.reshape(-1), {"int_to_float": m}

    def backward(self, data, metadata, **kwargs):
        return lut_backward(np.asarray(data, dtype=np.float32), metadata["int_to_float"], self.device)


class SKCPipeline(TransformationPipeline):
    """plan.yaml: template openfl_amd.pipelines.SKCPipeline, settings
    p_sparsity, n_clusters (:233-262)."""

    def __init__(self, p_sparsity=0.1, n_clusters=6, device="cpu", gzip_level=9, gzip_backend="device", **kwargs):
        self.p = p_sparsity
        self.n_cluster = n_clusters
        sp = SparsityTransformer(self.p, device)
        super().__init__(transformers=[sp, KmeansTransformer(n_clusters, device, share=sp),
                                       GZIPTransformer(gzip_level, backend=gzip_backend)], **kwargs)

    def forward(self, data, **kwargs):
        sp, km, gz = self.transformers
        sparse, _ = sp.sparse_device(data)
        if sparse.numel() >= km.n_cluster:
            # the reference clusters the float64 sparse vector: float64 centres
            ranks, m = kmeans_ranks(sparse, km.n_cluster, np.float64)
            payload, gz_md = gz.forward_device(ranks)
            return payload, [{"int_list": list(data.shape)}, {"int_to_float": m}, gz_md]
        return super().forward(data, **kwargs)

    def backward(self, data, transformer_metadata, **kwargs):
        """With the device gzip backend: inflate + LUT fused on the GPU
        (lossy_common.gzip_lut_backward_device), then the sparsity backward's
        reshape; metadata consumed the same way (pop)."""
        sp, lut_t, gz = self.transformers
        if gz.backend != "device":
            return super().backward(data, transformer_metadata, **kwargs)
        transformer_metadata.pop()  # GZIPTransformer's (empty)
        m = transformer_metadata.pop()["int_to_float"]
        shape = list(transformer_metadata.pop()["int_list"])
        y = gzip_lut_backward_device(data, m, int(np.prod(shape)) if shape else 1, sp.device)
        return y.cpu().numpy().reshape(shape)


__all__ = ["GZIPTransformer", "KmeansTransformer", "SKCPipeline", "SparsityTransformer"]
