"""KCPipeline on MI355X: drop-in for openfl/pipelines/kc_pipeline.py.

KmeansTransformer (k-means quantisation, :16-114) + GZIPTransformer (:117-156).
k-means runs on the GPU (openfl_amd/csrc/lossy_kernels.hip); sklearn's
KMeans RNG cannot be reproduced, so centres match the reference statistically
(inertia within 1 %, tests/test_gpu_lossy.py) while the metadata schema, rank
semantics and wire format are the reference's.  Decoding a reference payload
is exact (sequential key->value replacement emulated per element).
"""
import numpy as np

from openfl_amd.pipelines.lossy_common import (GZIPTransformer, float_to_int, gzip_lut_backward_device,
                                               kmeans_ranks, lut_backward, PerThreadDevice, to_device)
from openfl_amd.pipelines.pipeline import TransformationPipeline, Transformer


class KmeansTransformer(PerThreadDevice, Transformer):
    """Quantise to n_cluster k-means centres; int32 ranks + {rank: centre}."""

    def __init__(self, n_cluster=6, device="cpu"):
        self.lossy = True
        self.n_cluster = n_cluster
        self._init_devices(device)

    def _ranks(self, data):
        """-> (float32 rank device tensor or None, int_to_float); None = tiny path."""
        if data.size >= self.n_cluster:
            return kmeans_ranks(to_device(data, self.device), self.n_cluster, np.asarray(data).dtype)
        return None, None

    def forward(self, data, **kwargs):
        metadata = {"int_list": list(data.shape)}
        ranks, m = self._ranks(data)
        if ranks is None:  # n < n_cluster: quantise to itself (:57-58)
            int_array, m = float_to_int(data.reshape((-1, 1)))
        else:
            int_array = ranks.cpu().numpy().astype(np.int32)
        metadata["int_to_float"] = m
        return int_array, metadata

    def backward(self, data, metadata, **kwargs):
        out = lut_backward(np.asarray(data, dtype=np.float32), metadata["int_to_float"], self.device)
        return out.reshape(list(metadata["int_list"]))


class KCPipeline(TransformationPipeline):
    """plan.yaml: template openfl_amd.pipelines.KCPipeline, settings n_clusters
    (p_sparsity accepted and ignored, like the reference :160-181)."""

    def __init__(self, p_sparsity=0.01, n_clusters=6, device="cpu", gzip_level=9, gzip_backend="device", **kwargs):
        self.p = p_sparsity
        self.n_cluster = n_clusters
        super().__init__(transformers=[KmeansTransformer(n_clusters, device), GZIPTransformer(gzip_level, backend=gzip_backend)],
                         **kwargs)

    def forward(self, data, **kwargs):
        # fused: float32 ranks go from the device straight into gzip (the
        # reference's int32 -> float32 round trip yields the same bytes)
        km, gz = self.transformers
        ranks, m = km._ranks(data)
        if ranks is None:
            return super().forward(data, **kwargs)
        payload, gz_md = gz.forward_device(ranks)
        return payload, [{"int_list": list(data.shape), "int_to_float": m}, gz_md]

    def backward(self, data, transformer_metadata, **kwargs):
        """With the device gzip backend: inflate on the GPU straight into the
        rank array (lossy.gunzip_device), LUT-decode there, one D2H of the
        result -- the same values as GZIPTransformer.backward followed by
        KmeansTransformer.backward, metadata consumed the same way (pop)."""
        km, gz = self.transformers
        if gz.backend != "device":
            return super().backward(data, transformer_metadata, **kwargs)
        transformer_metadata.pop()  # GZIPTransformer's (empty)
        md = transformer_metadata.pop()
        shape = list(md["int_list"])
        y = gzip_lut_backward_device(data, md["int_to_float"], int(np.prod(shape)) if shape else 1, km.device)
        return y.cpu().numpy().reshape(shape)
