"""STCPipeline on MI355X: drop-in for openfl/pipelines/stc_pipeline.py.

SparsityTransformer (top-k by magnitude, :13-91) + TernaryTransformer
(+/-mean, :94-143) + GZIPTransformer.  Top-k (exact radix select), the +1e-7
rule, the ternary mean and ranks run on the GPU; ties at the k-th magnitude
are kept lowest index first (the reference's np.argsort tie order is
introsort's, i.e. unspecified).
"""
import numpy as np

from openfl_amd import lossy
from openfl_amd.pipelines.lossy_common import (GZIPTransformer, float_to_int, gzip_lut_backward_device, lut_backward,
                                               PerThreadDevice, to_device)
from openfl_amd.pipelines.pipeline import TransformationPipeline, Transformer


def _topk_count(n, p):
    return int(np.ceil(n * p))  # :40 / skc :45


class SparsityTransformer(PerThreadDevice, Transformer):
    """Keep the ceil(n*p) largest |x|; dense float64 output (:30-51)."""

    def __init__(self, p=0.01, device="cpu"):
        self.lossy = True
        self.p = p
        self._init_devices(device)

    def sparse_device(self, data):
        x = to_device(data.astype(np.float32), self.device)
        return lossy.sparsify_topk(x, _topk_count(x.numel(), self.p))

    def forward(self, data, **kwargs):
        metadata = {"int_list": list(data.shape)}
        sparse, _ = self.sparse_device(data)
        return sparse.cpu().numpy().astype(np.float64), metadata

    def backward(self, data, metadata, **kwargs):
        return data.astype(np.float32).reshape(metadata["int_list"])


def ternary_map(n, n_pos, n_neg, abs_sum):
    """Values present after ternarisation and their ranks (:117-124 then
    _float_to_int): sorted unique of {-m, 0, +m}, m = mean(|data|) over n."""
    m = abs_sum / n
    vals, ranks = [], {}
    for name, present, v in (("neg", n_neg > 0, -m), ("zero", n - n_pos - n_neg > 0, 0.0), ("pos", n_pos > 0, m)):
        if present:
            ranks[name] = float(len(vals))
            vals.append(np.float64(v))
    return ({i: v for i, v in enumerate(vals)},
            (ranks.get("neg", 0.0), ranks.get("zero", 0.0), ranks.get("pos", 0.0)))


class TernaryTransformer(PerThreadDevice, Transformer):
    """x > 0 -> +mean|x|, x < 0 -> -mean|x|, else 0; int32 ranks (:105-130)."""

    def __init__(self, device="cpu", share=None):
        self.lossy = True
        self._init_devices(device, share)

    def forward(self, data, **kwargs):
        x = to_device(data, self.device)
        n_pos, n_neg, asum = lossy.ternary_stats(x)
        m, (rn, rz, rp) = ternary_map(x.numel(), n_pos, n_neg, asum)
        ranks = lossy.ternary_ranks(x, rn, rz, rp)
        return ranks.cpu().numpy().astype(np.int32).reshape(data.shape), {"int_to_float": m}

    def backward(self, data, metadata, **kwargs):
        return lut_backward(np.asarray(data, dtype=np.float32), metadata["int_to_float"], self.device)


class STCPipeline(TransformationPipeline):
    """plan.yaml: template openfl_amd.pipelines.STCPipeline, settings p_sparsity
    (n_clusters accepted and ignored, like the reference :218-245)."""

    def __init__(self, p_sparsity=0.1, n_clusters=6, device="cpu", gzip_level=9, gzip_backend="device", **kwargs):
        self.p = p_sparsity
        sp = SparsityTransformer(self.p, device)
        super().__init__(transformers=[sp, TernaryTransformer(device, share=sp),
                                       GZIPTransformer(gzip_level, backend=gzip_backend)], **kwargs)

    def forward(self, data, **kwargs):
        sp, _, gz = self.transformers
        sparse, st = sp.sparse_device(data)
        n = sparse.numel()
        m, (rn, rz, rp) = ternary_map(n, st["n_pos"], st["n_neg"], st["abs_sum"])
        ranks = lossy.ternary_ranks(sparse, rn, rz, rp)
        payload, gz_md = gz.forward_device(ranks)
        return payload, [{"int_list": list(data.shape)}, {"int_to_float": m}, gz_md]

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


__all__ = ["GZIPTransformer", "STCPipeline", "SparsityTransformer", "TernaryTransformer", "float_to_int"]
