"""CPU restatement of the KC pipeline (KmeansTransformer + GZIPTransformer).

TEST INFRASTRUCTURE ONLY -- see oracle/__init__.py.  Only tests/, smoke() and
bench.py's cpu_baseline leg use it; the product path (openfl_amd/) never does.

Restates /root/reference/openfl/pipelines/kc_pipeline.py with the reference's
own library calls (sklearn KMeans, numpy, the gzip module), per tensor:
  forward  = KmeansTransformer.forward (:36-63: KMeans(n_clusters, n_init =
             n_clusters) on data.reshape(-1, 1) when there are at least
             n_clusters values, np.choose(labels, centres), _float_to_int
             :88-114: ranks of np.unique) -> GZIPTransformer.forward (:128-141:
             gzip.compress of the ranks as float32 bytes, level 9, the
             module's default)
  backward = GZIPTransformer.backward (:152-156: gzip.decompress ->
             float32) -> KmeansTransformer.backward (:65-86: the sequential
             key -> value replacement, then the shape)
Parity of the device path against this restatement is pinned through the
reference-generated fixtures in tests/golden/lossy_golden.* (the k-means RNG of
sklearn is not reproducible, so the tests compare inertia).
"""
import gzip
import time

import numpy as np


def kc_forward(x, n_cluster=6):
    """(payload bytes, metadata) of one tensor: kc_pipeline.py:36-63, :128-141."""
    from sklearn import cluster
    metadata = {"int_list": list(x.shape)}
    data = x.reshape((-1, 1))
    if data.shape[0] >= n_cluster:
        km = cluster.KMeans(n_clusters=n_cluster, n_init=n_cluster)
        km.fit(data)
        quant = np.choose(km.labels_, km.cluster_centers_.squeeze())
    else:
        quant = data
    flat = quant.reshape(-1)
    uniq = np.unique(flat)
    ranks = np.zeros(flat.shape, np.int32)
    i2f = {}
    for idx, u in enumerate(uniq):  # kc_pipeline.py:104-112
        i2f[idx] = u
        ranks[np.where(flat == u)] = idx
    metadata["int_to_float"] = i2f
    return gzip.compress(ranks.reshape(quant.shape).astype(np.float32).tobytes()), metadata


def lut_sequential(data, int_to_float):
    """KmeansTransformer.backward's replacement (kc_pipeline.py:79-83), in
    place on a float32 array: `data[data == key] = value` for every key in
    map order, so a value equal to a later key is replaced again."""
    for key in int_to_float:
        data[data == key] = int_to_float[key]
    return data


def kc_backward(payload, metadata):
    """The tensor back: kc_pipeline.py:152-156, then :65-86."""
    data = np.frombuffer(gzip.decompress(payload), dtype=np.float32).copy()
    lut_sequential(data, metadata["int_to_float"])
    return data.reshape(list(metadata["int_list"]))


def time_pipeline(tensors, n_cluster=6):
    """Forward + backward of every tensor in order (the reference's per-tensor
    calls); returns (seconds forward, seconds backward, payload bytes)."""
    t_f = t_b = 0.0
    zb = 0
    for x in tensors:
        t0 = time.perf_counter()
        z, md = kc_forward(x, n_cluster)
        t1 = time.perf_counter()
        kc_backward(z, md)
        t2 = time.perf_counter()
        t_f += t1 - t0
        t_b += t2 - t1
        zb += len(z)
    return t_f, t_b, zb
