"""End-to-end loopback on the GPU (BASELINE configs 1 and 5).

Two collaborators send their update through the wire format and the
aggregator decodes it, in one process -- the in-process loopback pattern of
openfl/native/native.py:331-344 (the Aggregator object itself as the
collaborator's client).  Per tensor: host ndarray -> EdenPipeline.forward
(or forward_batch) -> construct_named_tensor (protocols/utils.py:101-147) ->
SerializeToString -> ParseFromString -> metadata as protobuf containers
(collaborator.py:552-559) -> backward (or backward_batch) -> host ndarray.

Checked against the CPU oracle on the WIRE contents: the Eden bins of every
payload vs oracle.compress with the seed the metadata carries (>= 99.9 %
equal over the update, per tensor >= the survey's 99.8 % or at most 2
boundary flips -- a 512-element tensor with one flipped bin is 99.80 % --
and |dbin| <= 1), the decoded array vs oracle.decompress of the same
bytes and float32 metadata (rel-L2 and max-abs <= 2e-6), raw fp32 payloads
of small tensors exact, and int_to_float values arriving as float32
(base.proto:22).
"""
import numpy as np
import pytest

from oracle import eden as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _state(shapes, seed):
    rng = np.random.default_rng(seed)
    return [(n, rng.standard_normal(s, dtype=np.float32) * np.float32(0.01)) for n, s in shapes]


def _send(pipe, sd, batched, P):
    if batched:
        enc = pipe.forward_batch([a for _, a in sd])
    else:
        enc = [pipe.forward(a) for _, a in sd]
    wire = []
    for (name, _), (data, mds) in zip(sd, enc):
        nt = P.construct_named_tensor((name, "col", 1, False, ("trained",)), data, mds, False)
        wire.append(nt.SerializeToString())
    return wire, enc


def _receive(pipe, wire, batched, P):
    items = []
    for b in wire:
        nt = P.NamedTensor()
        nt.ParseFromString(b)
        items.append((nt.data_bytes, P.transformer_metadata_of(nt)))
    parsed = [(d, [dict(int_to_float=dict(m["int_to_float"]), int_list=list(m["int_list"]))
                   for m in mds]) for d, mds in items]
    if batched:
        outs = pipe.backward_batch(items)
    else:
        outs = [pipe.backward(d, mds) for d, mds in items]
    return outs, parsed


def _check_tensor(x, data, md, y, bits=8):
    """-> (bins compared, bins that differ) of an Eden payload, (0, 0) else."""
    i2f = md["int_to_float"]
    assert list(md["int_list"]) == list(x.shape)
    assert y.dtype == np.float32 and y.shape == x.shape
    if not i2f:                                   # small tensor: raw float32 bytes (pipeline.py:59-77)
        assert data == x.astype(np.float32).tobytes()
        np.testing.assert_array_equal(y, x)
        return 0, 0
    for v in i2f.values():                        # float32 on the wire (base.proto:22)
        assert np.float32(v) == v
    seed, total = int(i2f[0]), int(i2f[1])
    assert total == x.size
    dims = [int(i2f[k]) for k in range(3, max(i2f) + 1, 2)]
    scales = [i2f[k] for k in range(2, max(i2f) + 1, 2)]
    op, osc, odims, _ = O.compress(x, seed, bits)
    assert odims == dims and len(data) == len(op.tobytes())
    a = O.bins_of(data, sum(dims), bits)
    b = O.bins_of(op, sum(dims), bits)
    diff = int(np.sum(a != b))
    assert (diff <= max(0.002 * a.size, 2)) and np.max(np.abs(a - b)) <= 1
    np.testing.assert_allclose(scales, np.float32(osc), rtol=1e-3)
    yo = O.decompress(data, total, scales, dims, seed, bits).reshape(x.shape)
    ref = yo.astype(np.float64)
    err = y.astype(np.float64) - ref
    assert np.max(np.abs(err)) <= 2e-6 * max(np.max(np.abs(ref)), 1e-30)
    assert np.linalg.norm(err) <= 2e-6 * np.linalg.norm(ref)
    return a.size, diff


@pytest.mark.timeout(600)
@pytest.mark.parametrize("workload,limit", [("mnist_cnn", None), ("resnet50_fp32", None)])
@pytest.mark.parametrize("batched", [False, True], ids=["per_tensor", "batched"])
def test_loopback_two_collaborators(workload, limit, batched):
    from openfl_amd import protocols as P
    from openfl_amd.pipelines import EdenPipeline
    from openfl_amd.workloads import WORKLOADS
    shapes = WORKLOADS[workload]()[:limit]
    agg_pipe = EdenPipeline(n_bits=8, dim_threshold=100, device=DEV)       # aggregator side
    for c in range(2):                                                      # 2 collaborators
        col_pipe = EdenPipeline(n_bits=8, dim_threshold=100, device=DEV)
        sd = _state(shapes, 100 + c)
        np.random.seed(40 + c)
        wire, _ = _send(col_pipe, sd, batched, P)
        outs, parsed = _receive(agg_pipe, wire, batched, P)
        assert len(outs) == len(sd)
        seen = flips = 0
        for (name, x), (data, mds), y in zip(sd, parsed, outs):
            n, d = _check_tensor(x, data, mds[0], y)
            seen, flips = seen + n, flips + d
        assert flips <= 1e-3 * seen
        # Eden error band of the whole update (8-bit, Gaussian): ~6.4e-3
        num = sum(float(np.sum((o.astype(np.float64) - a) ** 2)) for (_, a), o in zip(sd, outs))
        den = sum(float(np.sum(a.astype(np.float64) ** 2)) for _, a in sd)
        assert (num / den) ** 0.5 < 7.5e-3


def test_loopback_batched_equals_per_tensor_wire():
    """The batched path puts the same bytes on the wire as per-tensor calls
    (same np.random draws), for the MNIST CNN update."""
    from openfl_amd import protocols as P
    from openfl_amd.pipelines import EdenPipeline
    from openfl_amd.workloads import WORKLOADS
    sd = _state(WORKLOADS["mnist_cnn"](), 7)
    pipe = EdenPipeline(n_bits=8, device=DEV)
    np.random.seed(5)
    w1, _ = _send(pipe, sd, False, P)
    np.random.seed(5)
    w2, _ = _send(pipe, sd, True, P)
    assert w1 == w2
