"""Device ops behind the KC / SKC / STC pipelines (libofl_codec.so lossy ABI).

Each function takes/returns PyTorch-ROCm device tensors and host scalars; the
heavy O(n) work runs in openfl_amd/csrc/lossy_kernels.hip.  Reference
semantics are cited per function (paths relative to /root/reference).
"""
import ctypes
import gzip
import os
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

from openfl_amd import _lib, hostmem

_tls = threading.local()
GZIP_CHUNK = 8 << 20
_pool = None
_pool_lock = threading.Lock()


def _on_device(fn):
    """Run fn with its first device-tensor argument's GPU current: per-device
    setup inside the library (CRC tables, kernel attributes, CU counts) keys
    on hipGetDevice(), and the launches go to that tensor's stream."""
    import functools

    @functools.wraps(fn)
    def wrap(*args, **kwargs):
        for a in list(args) + list(kwargs.values()):
            if isinstance(a, torch.Tensor) and a.is_cuda:
                with torch.cuda.device(a.device):
                    return fn(*args, **kwargs)
        return fn(*args, **kwargs)
    return wrap


def _ws(device, n):
    need = int(_lib.lib().ofl_lossy_workspace_bytes(int(n)))
    bufs = getattr(_tls, "ws", None)
    if bufs is None:
        bufs = _tls.ws = {}
    b = bufs.get(str(device))
    if b is None or b.numel() < need:
        b = bufs[str(device)] = torch.empty(need, dtype=torch.uint8, device=device)
    return b


def _ws_bytes(device, need):
    bufs = getattr(_tls, "ws", None)
    if bufs is None:
        bufs = _tls.ws = {}
    b = bufs.get(str(device))
    if b is None or b.numel() < need:
        b = bufs[str(device)] = torch.empty(need, dtype=torch.uint8, device=device)
    return b


def _stream(device):
    return torch.cuda.current_stream(device).cuda_stream


def _check_dev(x):
    if not (x.is_cuda and x.dtype == torch.float32 and x.is_contiguous()):
        raise _lib.CodecError("lossy ops take contiguous float32 device tensors")


@_on_device
def kmeans_fit(x, k=6, n_init=6, seed=0, max_exact=8):
    """1-D k-means of a float32 device vector (replaces sklearn KMeans.fit,
    kc_pipeline.py:49-56): -> (sorted centres float64[k], counts int64[k], inertia)."""
    _check_dev(x)
    L = _lib.lib()
    c = np.zeros(k, np.float64)
    cnt = np.zeros(k, np.int64)
    inertia = ctypes.c_double()
    ws = _ws(x.device, x.numel())
    _lib.check_lossy(L.ofl_kmeans1d_fit(x.data_ptr(), x.numel(), k, n_init, seed, max_exact,
                                        c.ctypes.data, cnt.ctypes.data, ctypes.byref(inertia),
                                        ws.data_ptr(), ws.numel(), _stream(x.device)))
    return c, cnt, inertia.value


class LabelTable:
    """The per-tensor labelling rules of one kmeans_batch (ofl_label_rec
    records on the device, include/ofl_codec.h): gzip_ranks(x, label=) labels
    the values as it encodes them, so the rank array is never written."""
    REC_BYTES = 80

    def __init__(self, ntensors, device):
        self.n = int(ntensors)
        self.buf = torch.empty(self.REC_BYTES * self.n, dtype=torch.uint8, device=device)


@_on_device
def kmeans_batch(x_arena, offsets, numels, k=6, n_init=6, seed=0, max_exact=8, value_f64=False, ranks_out=None,
                 label_out=None):
    """Device k-means of many tensors of one float32 arena (ofl_kmeans1d_batch):
    tensor t = x_arena[offsets[t]:offsets[t] + numels[t]].  Writes float32
    ranks (np.unique order of the used centres, value dtype float64 if
    value_f64) into ranks_out (a device arena like x_arena) when given, and
    the labelling rules into label_out (a LabelTable; k <= 8, ascending
    tensors) when given.
    -> (centres [T, k], counts [T, k], inertia [T], uniq: list of arrays)."""
    _check_dev(x_arena)
    L = _lib.lib()
    T = len(numels)
    off = np.ascontiguousarray(offsets, np.int64)
    num = np.ascontiguousarray(numels, np.int64)
    need = int(L.ofl_kmeans1d_batch_workspace_bytes(T, num.ctypes.data))
    ws = _ws_bytes(x_arena.device, need)
    c = np.zeros((T, k), np.float64)
    cnt = np.zeros((T, k), np.int64)
    inertia = np.zeros(T, np.float64)
    nu = np.zeros(T, np.int32)
    uq = np.zeros((T, k), np.float64)
    if ranks_out is not None:
        _check_dev(ranks_out)
    if label_out is not None:
        if not label_out.buf.is_cuda:
            raise _lib.CodecError("label_out must live on the device")
        if label_out.n != T:
            raise ValueError(f"label_out holds {label_out.n} records for {T} tensors")
    _lib.check_lossy(L.ofl_kmeans1d_batch_tab(T, x_arena.data_ptr(), off.ctypes.data, num.ctypes.data, k, n_init,
                                              int(seed), max_exact, 1 if value_f64 else 0,
                                              ranks_out.data_ptr() if ranks_out is not None else None,
                                              label_out.buf.data_ptr() if label_out is not None else None,
                                              c.ctypes.data, cnt.ctypes.data, inertia.ctypes.data, nu.ctypes.data,
                                              uq.ctypes.data, ws.data_ptr(), ws.numel(), _stream(x_arena.device)))
    dt = np.float64 if value_f64 else np.float32
    return c, cnt, inertia, [uq[t, :nu[t]].astype(dt) for t in range(T)]


@_on_device
def kmeans_label(x, centres, rank_of_cluster):
    """out[i] = rank_of_cluster[nearest centre of x[i]] as float32 (device)."""
    _check_dev(x)
    c = np.ascontiguousarray(centres, np.float64)
    r = np.ascontiguousarray(rank_of_cluster, np.float32)
    out = torch.empty_like(x)
    _lib.check_lossy(_lib.lib().ofl_kmeans1d_label(x.data_ptr(), x.numel(), c.ctypes.data, c.size,
                                                   r.ctypes.data, out.data_ptr(), _stream(x.device)))
    return out


@_on_device
def sparsify_topk(x, k):
    """SparsityTransformer top-k (skc_pipeline.py:33-54, 72-94) -> (sparse
    float32 device array, stats dict)."""
    _check_dev(x)
    L = _lib.lib()
    out = torch.empty_like(x)
    kmin = ctypes.c_float()
    npos, nneg, nzero = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    asum = ctypes.c_double()
    shifted = ctypes.c_int()
    ws = _ws(x.device, x.numel())
    _lib.check_lossy(L.ofl_sparsify_topk(x.data_ptr(), x.numel(), int(k), out.data_ptr(), ctypes.byref(kmin),
                                         ctypes.byref(npos), ctypes.byref(nneg), ctypes.byref(nzero),
                                         ctypes.byref(asum), ctypes.byref(shifted), ws.data_ptr(), ws.numel(),
                                         _stream(x.device)))
    return out, {"kept_min": kmin.value, "n_pos": npos.value, "n_neg": nneg.value, "n_zero": nzero.value,
                 "abs_sum": asum.value, "shifted": bool(shifted.value), "k": int(k)}


@_on_device
def sparsify_topk_batch(x_arena, offsets, numels, ks, sparse_out):
    """sparsify_topk for every tensor of a float32 arena in one device pass
    sequence (ofl_sparsify_topk_batch): tensor t = x_arena[offsets[t]:
    offsets[t] + numels[t]], keep ks[t]; sparse_out (device, same layout)
    gets the dense sparse arrays.  -> dict of per-tensor numpy stats."""
    _check_dev(x_arena)
    _check_dev(sparse_out)
    L = _lib.lib()
    T = len(numels)
    off = np.ascontiguousarray(offsets, np.int64)
    num = np.ascontiguousarray(numels, np.int64)
    kk = np.ascontiguousarray(ks, np.int64)
    ws = _ws_bytes(x_arena.device, int(L.ofl_sparsify_topk_batch_workspace_bytes(T, num.ctypes.data)))
    kmin = np.zeros(T, np.float32)
    npos, nneg, nzero = np.zeros(T, np.int64), np.zeros(T, np.int64), np.zeros(T, np.int64)
    asum = np.zeros(T, np.float64)
    shifted = np.zeros(T, np.int32)
    _lib.check_lossy(L.ofl_sparsify_topk_batch(T, x_arena.data_ptr(), off.ctypes.data, num.ctypes.data,
                                               kk.ctypes.data, sparse_out.data_ptr(), kmin.ctypes.data,
                                               npos.ctypes.data, nneg.ctypes.data, nzero.ctypes.data,
                                               asum.ctypes.data, shifted.ctypes.data, ws.data_ptr(), ws.numel(),
                                               _stream(x_arena.device)))
    return {"kept_min": kmin, "n_pos": npos, "n_neg": nneg, "n_zero": nzero, "abs_sum": asum,
            "shifted": shifted.astype(bool), "k": kk}


@_on_device
def ternary_ranks_batch(sparse_arena, offsets, numels, ranks3, out_arena):
    """ternary_ranks for every tensor of an arena (ranks3[t] = (rank_neg,
    rank_zero, rank_pos) of tensor t) in one launch."""
    _check_dev(sparse_arena)
    _check_dev(out_arena)
    L = _lib.lib()
    T = len(numels)
    off = np.ascontiguousarray(offsets, np.int64)
    num = np.ascontiguousarray(numels, np.int64)
    r3 = np.ascontiguousarray(ranks3, np.float32).reshape(T, 3)
    ws = _ws_bytes(sparse_arena.device, int(L.ofl_ternary_ranks_batch_workspace_bytes(T)))
    _lib.check_lossy(L.ofl_ternary_ranks_batch(T, sparse_arena.data_ptr(), off.ctypes.data, num.ctypes.data,
                                               r3.ctypes.data, out_arena.data_ptr(), ws.data_ptr(), ws.numel(),
                                               _stream(sparse_arena.device)))
    return out_arena


@_on_device
def ternary_stats(x):
    """(n_pos, n_neg, fp64 sum |x|) of a float32 device vector."""
    _check_dev(x)
    npos, nneg, asum = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_double()
    ws = _ws(x.device, x.numel())
    _lib.check_lossy(_lib.lib().ofl_ternary_stats(x.data_ptr(), x.numel(), ctypes.byref(npos), ctypes.byref(nneg),
                                                  ctypes.byref(asum), ws.data_ptr(), ws.numel(),
                                                  _stream(x.device)))
    return npos.value, nneg.value, asum.value


@_on_device
def ternary_ranks(sparse, rank_neg, rank_zero, rank_pos):
    _check_dev(sparse)
    out = torch.empty_like(sparse)
    _lib.check_lossy(_lib.lib().ofl_ternary_ranks(sparse.data_ptr(), sparse.numel(), float(rank_neg),
                                                  float(rank_zero), float(rank_pos), out.data_ptr(),
                                                  _stream(sparse.device)))
    return out


@_on_device
def lut_decode(ranks, int_to_float):
    """Reference backward: `for key in map: data[data == key] = map[key]` on a
    float32 array, in the mapping's own iteration order (kc_pipeline.py:81-83)."""
    _check_dev(ranks)
    keys = np.asarray([float(k) for k in int_to_float.keys()], np.float32)
    vals = np.asarray([float(int_to_float[k]) for k in int_to_float.keys()], np.float32)
    out = torch.empty_like(ranks)
    _lib.check_lossy(_lib.lib().ofl_lut_decode(ranks.data_ptr(), ranks.numel(), keys.ctypes.data,
                                               vals.ctypes.data, keys.size, out.data_ptr(),
                                               _stream(ranks.device)))
    return out


@_on_device
def lut_decode_batch(ranks_arena, offsets, numels, maps, out_arena):
    """lut_decode for every tensor of an arena in one launch (maps[t]: the
    tensor's int_to_float mapping, iteration order kept)."""
    _check_dev(ranks_arena)
    _check_dev(out_arena)
    L = _lib.lib()
    T = len(numels)
    mk = max([len(m) for m in maps] + [1])
    keys = np.zeros((T, mk), np.float32)
    vals = np.zeros((T, mk), np.float32)
    nk = np.zeros(T, np.int32)
    for t, m in enumerate(maps):
        nk[t] = len(m)
        for j, (k, v) in enumerate(m.items()):
            keys[t, j], vals[t, j] = float(k), float(v)
    off = np.ascontiguousarray(offsets, np.int64)
    num = np.ascontiguousarray(numels, np.int64)
    ws = _ws_bytes(ranks_arena.device, int(L.ofl_lut_decode_batch_workspace_bytes(T, mk)))
    _lib.check_lossy(L.ofl_lut_decode_batch(T, ranks_arena.data_ptr(), off.ctypes.data, num.ctypes.data,
                                            nk.ctypes.data, keys.ctypes.data, vals.ctypes.data, mk,
                                            out_arena.data_ptr(), ws.data_ptr(), ws.numel(),
                                            _stream(ranks_arena.device)))
    return out_arena


@_on_device
def gzip_ranks(x, label=None):
    """gzip.compress of a float32 device array of ranks (integers 0..31), on
    the GPU (ofl_gzip_ranks, TLZ: optimal-parse token LZ, one deflate block
    per 512 KiB member): a multi-member gzip stream that gzip.decompress reads
    back to x's bytes.  Raises CodecError for other values.  label (a
    LabelTable from kmeans_batch): x holds the VALUES the k-means ran on and
    the stream is that of the ranks ranks_out would hold (0 between tensors),
    labelled inside the encoder (ofl_gzip_label_to)."""
    _check_dev(x)
    if label is not None and not label.buf.is_cuda:
        raise _lib.CodecError("label records must live on the device")
    L = _lib.lib()
    n = x.numel()
    if n == 0:
        return gzip.compress(b"", compresslevel=9)
    ws = _ws_bytes(x.device, int(L.ofl_gzip_ranks_workspace_bytes(n)))
    bound = int(L.ofl_gzip_ranks_bound(n))
    # pinned output sized for a rank stream (a quarter of the input: rank
    # streams compress to 0.05-0.2); the worst-case bound (1.5x the input)
    # only after an OFL_ESPACE
    # the payload `bytes` is filled batch by batch while the GPU encodes the
    # next batch (ofl_gzip_ranks_to); small streams are copied afterwards
    for cap in (min(bound, n + (1 << 20)), bound):
        out = _buf("host", "gz_out", cap, pinned=True)
        ln = ctypes.c_size_t()
        dst = hostmem.new_payload(cap) if _GZ_FILL else None
        if label is not None:
            rc = L.ofl_gzip_label_to(x.data_ptr(), n, label.buf.data_ptr(), label.n, out.data_ptr(), cap,
                                     dst[1] if dst is not None else None, cap if dst is not None else 0,
                                     _GZ_COPY_THREADS, ctypes.byref(ln), ws.data_ptr(), ws.numel(), _stream(x.device))
        elif dst is not None:
            rc = L.ofl_gzip_ranks_to(x.data_ptr(), n, out.data_ptr(), cap, dst[1], cap, _GZ_COPY_THREADS,
                                     ctypes.byref(ln), ws.data_ptr(), ws.numel(), _stream(x.device))
        else:
            rc = L.ofl_gzip_ranks(x.data_ptr(), n, out.data_ptr(), cap, ctypes.byref(ln), ws.data_ptr(), ws.numel(),
                                  _stream(x.device))
        if rc != _lib.OFL_ESPACE or cap == bound:
            break
    _lib.check_gzip(rc)
    payload = hostmem.seal_payload(dst[0], ln.value) if dst is not None else hostmem.bytes_from(out.data_ptr(), ln.value)
    _trim_bufs()
    return payload


def gunzip(data, threads=8, out=None):
    """gzip.decompress (kc_pipeline.py:152-156) of `data` -> uint8 numpy array.
    Member-indexed streams (the device gzip's, every member carrying its size
    in an extra subfield) inflate in parallel on native threads (ofl_gunzip_members),
    into `out` (a uint8 numpy array, e.g. a pinned staging view) when given;
    any other stream goes through gzip.decompress."""
    L = _lib.lib()
    src = np.frombuffer(data, np.uint8)
    need = ctypes.c_size_t()
    rc = L.ofl_gunzip_members(src.ctypes.data if src.size else None, src.size, None, 0, ctypes.byref(need),
                              threads)
    if rc == _lib.OFL_EFORMAT or src.size == 0:
        raw = np.frombuffer(gzip.decompress(bytes(data)), np.uint8)
        if out is None:
            return raw
        out[:raw.size] = raw
        return out[:raw.size]
    _lib.check_gzip(rc)
    dst = out if out is not None else np.empty(need.value, np.uint8)
    if dst.size < need.value:
        raise _lib.CodecError("gunzip: output buffer too small")
    _lib.check_gzip(L.ofl_gunzip_members(src.ctypes.data, src.size, dst.ctypes.data, dst.size,
                                         ctypes.byref(need), threads))
    return dst[:need.value]


def _parallel_copy(dst, src, nbytes, threads=8, piece=4 << 20):
    """memcpy of a large host buffer in pieces on native threads
    (ofl_host_copy_many, no GIL)."""
    if nbytes <= 0:
        return
    offs = np.arange(0, nbytes, piece, dtype=np.int64)
    sizes = np.minimum(piece, nbytes - offs).astype(np.int64)
    d = (np.uint64(dst) + offs.astype(np.uint64))
    s = (np.uint64(src) + offs.astype(np.uint64))
    _lib.check(_lib.lib().ofl_host_copy_many(offs.size, d.ctypes.data, s.ctypes.data, sizes.ctypes.data, threads))


_RETAIN_BYTES = 512 << 20


def _trim_bufs():
    """Release this thread's scratch buffers above _RETAIN_BYTES (after the
    call that needed them): a one-off large call does not keep gigabytes
    pinned per thread."""
    bufs = getattr(_tls, "bufs", None) or {}
    for k in [k for k, b in bufs.items() if b.numel() * b.element_size() > _RETAIN_BYTES]:
        del bufs[k]


def _buf(device, name, nbytes, pinned=False):
    """Thread-local scratch buffers (device, or pinned host) that only grow."""
    bufs = getattr(_tls, "bufs", None)
    if bufs is None:
        bufs = _tls.bufs = {}
    key = (str(device), name)
    b = bufs.get(key)
    if b is None or b.numel() < nbytes:
        # 1/8 headroom: payload sizes wander from call to call (a compressed
        # stream's length), and each regrowth of a pinned buffer costs a
        # fresh pinned allocation
        nbytes = max(nbytes, 1)
        nbytes = (nbytes + (nbytes >> 3) + (2 << 20) - 1) // (2 << 20) * (2 << 20) if nbytes > (1 << 20) else nbytes
        if pinned:
            b = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
        else:
            b = torch.empty(nbytes, dtype=torch.uint8, device=device)
        bufs[key] = b
    return b


def lut_tables(offsets, numels, maps, device):
    """The fused LUT of gunzip_device(lut=...): per tensor t, its int_to_float
    map (the reference's sequential key -> value replacement,
    kc_pipeline.py:79-83) applied to every rank 0..31, in float32 as
    lut_decode_batch compares and assigns; with the tensors' element ranges
    [offsets[t], offsets[t] + numels[t]) of the decoded arena.  One H2D."""
    T = len(numels)
    lens = [len(m) for m in maps]
    mk = max(lens + [1])
    if T and min(lens) == mk:  # every map the same length (the batched k-means': one array each)
        keys = np.array([list(m.keys()) for m in maps], np.float32)
        vals = np.array([list(m.values()) for m in maps], np.float32)
    else:
        keys = np.full((T, mk), np.nan, np.float32)   # NaN never compares equal: a shorter map's padding
        vals = np.zeros((T, mk), np.float32)
        for t, m in enumerate(maps):
            if m:
                keys[t, :len(m)] = np.array(list(m.keys()), np.float32)
                vals[t, :len(m)] = np.array(list(m.values()), np.float32)
    tab = np.broadcast_to(np.arange(32, dtype=np.float32), (T, 32)).copy()
    for j in range(mk):   # in map order: a value equal to a later key is replaced again
        tab = np.where(tab == keys[:, j:j + 1], vals[:, j:j + 1], tab)
    start = np.asarray(offsets, np.int64)
    order = np.argsort(start, kind="stable")
    blob = np.concatenate([tab[order].reshape(-1).view(np.uint8), start[order].view(np.uint8),
                           (start + np.asarray(numels, np.int64))[order].view(np.uint8)])
    d = torch.from_numpy(blob).to(torch.device(device))
    return {"tab": d[:128 * T].view(torch.float32), "start": d[128 * T:136 * T].view(torch.int64),
            "end": d[136 * T:144 * T].view(torch.int64),
            "n": T, "offsets": list(offsets), "numels": list(numels), "maps": list(maps)}


@_on_device
def gunzip_device(data, out, lut=None, expect_bytes=None):
    """gzip.decompress (kc_pipeline.py:152-156) of `data` into `out`, a uint8
    DEVICE tensor (returns the view of the decompressed bytes).  Member-indexed
    streams inflate on the GPU from the compressed bytes (the index is built
    on the host from the member headers, ofl_gzip_member_index): the device
    gzip's TLZ members through ofl_inflate_tlz (one lane per 2048-value
    segment, then the copies resolved in LDS; CRC-32 and ISIZE checked), other
    member-indexed streams through ofl_inflate_members (one wavefront per
    member).  Any other gzip stream (e.g. gzip.compress output) is a
    different format: gzip.decompress on the host, then one H2D.
    lut (lut_tables(...)): the decoded ranks go through the tensors' LUTs
    (the lossy pipelines' backward, kc_pipeline.py:79-83) -- fused into the
    TLZ decoder's stores, or one lut_decode_batch after any other inflate.
    expect_bytes: the decoded length the caller requires; a stream of any
    other length raises CodecError before anything is inflated or looked up
    (with lut, the decoded length must also be whole float32s)."""
    if not (out.is_cuda and out.dtype == torch.uint8 and out.is_contiguous()):
        raise _lib.CodecError("gunzip_device: out must be a contiguous uint8 device tensor")
    tr = _gunzip_trace("start")
    L = _lib.lib()
    src = np.frombuffer(data, np.uint8)
    dev = out.device
    nm, tot, mx, tl = ctypes.c_int64(), ctypes.c_size_t(), ctypes.c_uint32(), ctypes.c_int()
    # the stream goes H2D straight from the payload, on a pool thread while
    # this one indexes the members (both release the GIL); the inflate
    # kernels read up to ~48 bytes past a member's data (its 8-byte trailer
    # included) before they stop on corrupt data, hence the padding
    d_in = _buf(dev, "gz_in", src.size + 128)
    # d_in belongs to the caller's current stream, and the inflate runs there:
    # the pool thread enqueues the copy on that same stream
    caller_stream = torch.cuda.current_stream(dev)

    # the stream crosses PCIe in pieces (large payloads): each piece's TLZ
    # members inflate on a side stream as soon as their bytes have landed,
    # beside the H2D of the next piece
    npieces = _INFLATE_PIECES if src.size >= (_INFLATE_PIECE_MIN << 20) else 1
    bounds = [0] + [min(src.size, (src.size * k // npieces + (4 << 20) - 1) // (4 << 20) * (4 << 20))
                    for k in range(1, npieces)] + [src.size]
    landed = [threading.Event() for _ in range(npieces)]
    piece_ev = [None] * npieces

    def h2d():
        # straight from the immutable payload through the C ABI (no torch
        # wrapper of a read-only buffer); the caller's stream orders it
        # (no page freeing meanwhile: hostmem.quiet)
        try:
            if src.size:
                with torch.cuda.device(dev), hostmem.quiet():
                    for k in range(npieces):
                        lo, hi = bounds[k], bounds[k + 1]
                        if hi > lo:
                            _lib.check(_h2d(L, d_in.data_ptr() + lo, src.ctypes.data + lo, hi - lo,
                                            caller_stream.cuda_stream))
                        ev = torch.cuda.Event()
                        ev.record(caller_stream)
                        piece_ev[k] = ev
                        tr and tr(f"h2d{k}")
                        landed[k].set()
        finally:
            for e in landed:
                e.set()
    # one pass over the headers: a member takes >= 26 bytes, so n // 26 + 1
    # entries always suffice (untouched pages of the array cost nothing)
    cap = src.size // 26 + 1
    idx = np.empty((cap, 4), np.int64)
    copy = _h2d_pool().submit(h2d)
    try:
        rc = L.ofl_gzip_member_index(src.ctypes.data if src.size else None, src.size, idx.ctypes.data, cap,
                                     ctypes.byref(nm), ctypes.byref(tot), ctypes.byref(mx), ctypes.byref(tl)) \
            if src.size else _lib.OFL_EFORMAT
        tr and tr("index")
        if rc != _lib.OFL_OK or not tl.value or npieces == 1:
            copy.result()
    except BaseException:
        copy.result()
        raise
    if rc == _lib.OFL_EFORMAT:
        raw = np.frombuffer(gzip.decompress(bytes(data)), np.uint8)
        _check_len(raw.size, expect_bytes, lut)
        if raw.size > out.numel():
            raise _lib.CodecError("gunzip_device: output buffer too small")
        if raw.size:
            out[:raw.size].copy_(torch.from_numpy(raw.copy()))
        _apply_lut(out, raw.size, lut)
        return out[:raw.size]
    if rc != _lib.OFL_OK:
        copy.result()
    _lib.check_gzip(rc)
    try:
        _check_len(tot.value, expect_bytes, lut)   # the members' ISIZE sum, before any launch
    except _lib.CodecError:
        copy.result()
        raise
    if tot.value > out.numel():
        copy.result()
        raise _lib.CodecError("gunzip_device: output buffer too small")
    idx = idx[:nm.value]
    d_idx = _buf(dev, "gz_idx", max(idx.nbytes, 8))
    d_idx[:idx.nbytes].copy_(torch.from_numpy(idx.view(np.uint8).reshape(-1)))
    if tl.value:
        ws = _buf(dev, "gz_status", int(L.ofl_inflate_tlz_workspace_bytes(nm.value)))
        args = (d_in.data_ptr(), d_idx.data_ptr())
        tail = (out.data_ptr(), out.numel(), ws.data_ptr(), ws.numel())
        if lut is not None:
            lut_args = (lut["tab"].data_ptr(), lut["start"].data_ptr(), lut["end"].data_ptr(), lut["n"])

            def launch(first, count, st):
                return L.ofl_inflate_tlz_launch_lut(*args, first, count, *tail, *lut_args, st)
        else:
            def launch(first, count, st):
                return L.ofl_inflate_tlz_launch(*args, first, count, *tail, st)
        if npieces == 1 and lut is None:
            _lib.check_gzip(L.ofl_inflate_tlz(*args, nm.value, *tail, _stream(dev)))
        elif npieces == 1:
            _lib.check_gzip(L.ofl_inflate_tlz_async(*args, 0, 0, *tail, caller_stream.cuda_stream))
            _lib.check_gzip(launch(0, nm.value, caller_stream.cuda_stream))
            _lut_finish(L, args, tail, nm, mx, out, tot.value, lut, caller_stream)
        else:
            # status reset and the index on the caller's stream, then every
            # piece on a side stream after its bytes and that reset
            _lib.check_gzip(L.ofl_inflate_tlz_async(*args, 0, 0, *tail, caller_stream.cuda_stream))
            ready = torch.cuda.Event()
            ready.record(caller_stream)
            # a member is launched with the piece in which its end lands PLUS
            # the decoder's look-ahead (_INFLATE_LOOKAHEAD bytes past the
            # trailer), so every byte a lane may read -- of a valid or a
            # corrupt member -- has landed before the launch
            ends = idx[:, 0] + (idx[:, 1] & ((1 << 62) - 1)) + 8 + _INFLATE_LOOKAHEAD
            sides = _side_streams(dev)
            first = 0
            try:
                for k in range(npieces):
                    landed[k].wait()
                    if piece_ev[k] is None:   # the copy failed: its error surfaces below
                        break
                    last = nm.value if k == npieces - 1 else int(np.searchsorted(ends, bounds[k + 1], "right"))
                    if last > first:
                        st = sides[k % len(sides)]
                        st.wait_event(ready)
                        st.wait_event(piece_ev[k])
                        _lib.check_gzip(launch(first, last - first, st.cuda_stream))
                        tr and tr(f"launch{k}")
                        first = last
            finally:
                copy.result()
                for st in sides:
                    caller_stream.wait_stream(st)
            if lut is None:
                _lib.check_gzip(L.ofl_inflate_tlz_wait(*args, nm.value, *tail, caller_stream.cuda_stream))
            else:
                _lut_finish(L, args, tail, nm, mx, out, tot.value, lut, caller_stream)
            tr and tr("checked")
    else:
        copy.result()
        ws = _buf(dev, "gz_status", 256)
        _lib.check_gzip(L.ofl_inflate_members(d_in.data_ptr(), d_idx.data_ptr(), nm.value, mx.value, out.data_ptr(),
                                              out.numel(), ws.data_ptr(), ws.numel(), _stream(dev)))
        _apply_lut(out, tot.value, lut)
    _trim_bufs()
    return out[:tot.value]


_GUNZIP_TRACE = os.environ.get("OFL_GUNZIP_TRACE") is not None  # diagnostics: gunzip_device's timeline


def _gunzip_trace(first):
    """OFL_GUNZIP_TRACE: a recorder of (label, perf_counter) marks appended to
    lossy.gunzip_trace_log (one list per call); otherwise None."""
    if not _GUNZIP_TRACE:
        return None
    import time
    marks = [(first, time.perf_counter())]
    gunzip_trace_log.append(marks)
    return lambda label: marks.append((label, time.perf_counter()))


gunzip_trace_log = []
_INFLATE_PIECES = int(os.environ.get("OFL_INFLATE_PIECES", "4"))  # H2D pieces of a large TLZ payload, each inflated as it lands
_INFLATE_PIECE_MIN = 32  # MiB: smaller payloads cross in one piece
_INFLATE_LOOKAHEAD = 64  # bytes the inflate kernels may read past a member's trailer (d_in keeps 128 of padding)
_H2D_THREADS = int(os.environ.get("OFL_H2D_THREADS", "2"))  # host threads staging a large pageable payload (0: one plain hipMemcpyAsync)


def _check_len(nbytes, expect, lut):
    """gunzip_device's length checks: the caller's expected decoded length,
    and whole float32s wherever a LUT will read the bytes as values."""
    if expect is not None and nbytes != expect:
        raise _lib.CodecError(f"payload decodes to {nbytes} bytes, expected {expect}")
    if lut is not None and nbytes % 4:
        raise _lib.CodecError(f"payload decodes to {nbytes} bytes, not whole float32 values")


def _apply_lut(out, nbytes, lut):
    """The LUT after an inflate that did not fuse it (lut_decode_batch in place)."""
    if lut is None or nbytes == 0:
        return
    _check_len(nbytes, None, lut)
    y = out[:nbytes].view(torch.float32)
    lut_decode_batch(y, lut["offsets"], lut["numels"], lut["maps"], y)


def _lut_finish(L, args, tail, nm, mx, out, nbytes, lut, stream):
    """After fused-LUT launches: the TLZ decoder's verdict; where it refused a
    member, the generic inflate of every member, then the LUT unfused."""
    rc = L.ofl_inflate_tlz_check(nm.value, tail[2], tail[3], stream.cuda_stream)
    if rc == _lib.OFL_EFORMAT:
        _lib.check_gzip(L.ofl_inflate_members(*args, nm.value, mx.value, *tail, stream.cuda_stream))
        _apply_lut(out, nbytes, lut)
        return
    _lib.check_gzip(rc)


_GZ_COPY_THREADS = int(os.environ.get("OFL_GZ_COPY_THREADS", "8"))  # host threads filling the gzip payload
_GZ_FILL = os.environ.get("OFL_GZ_FILL", "1") != "0"  # 0: copy the payload after the call (A/B)


def _h2d(L, dst, src, nbytes, stream):
    """H2D of a pageable payload: staged through the library's pinned ring on
    _H2D_THREADS threads (ofl_copy_h2d_staged), or one hipMemcpyAsync."""
    if _H2D_THREADS > 0:
        return L.ofl_copy_h2d_staged(dst, src, nbytes, _H2D_THREADS, stream)
    return L.ofl_copy_h2d_async(dst, src, nbytes, stream)


_h2d_executor = None
_sides = {}


def _side_streams(dev):
    """The side streams of a pipelined inflate's pieces: the library's shared
    side streams 1 and 2 of the device (ofl_side_stream; a new stream per
    caller would push later streams onto HW queues already in use)."""
    with _pool_lock:
        key = str(dev)
        if key not in _sides:
            L = _lib.lib()
            sides = []
            with torch.cuda.device(dev):
                for i in (1, 2):
                    p = ctypes.c_void_p()
                    _lib.check(L.ofl_side_stream(i, ctypes.byref(p)))
                    sides.append(torch.cuda.ExternalStream(p.value, device=dev))
            _sides[key] = sides
        return _sides[key]


def _h2d_pool():
    global _h2d_executor
    with _pool_lock:
        if _h2d_executor is None:
            _h2d_executor = ThreadPoolExecutor(max_workers=4)  # concurrent callers do not queue behind one copy
        return _h2d_executor


def rank_map(values):
    """_float_to_int (kc_pipeline.py:88-114): sorted unique values -> ranks.
    Returns (unique sorted values, rank index per input value)."""
    u = np.unique(np.asarray(values))
    return u, np.searchsorted(u, values)


def gzip_compress(data_bytes, level=9, threads=8):
    """gzip.compress (kc_pipeline.py:138-139) of float32 bytes.  Large payloads
    are split into independent gzip members compressed in parallel; Python's
    gzip.decompress (the reference GZIPTransformer.backward) reads
    multi-member streams, so the bytes stay wire compatible."""
    global _pool
    mv = memoryview(data_bytes)
    if len(mv) <= GZIP_CHUNK or threads <= 1:
        return gzip.compress(bytes(mv), compresslevel=level)
    with _pool_lock:
        if _pool is None:
            _pool = ThreadPoolExecutor(max_workers=threads)
    parts = [mv[i:i + GZIP_CHUNK] for i in range(0, len(mv), GZIP_CHUNK)]
    return b"".join(_pool.map(lambda p: gzip.compress(bytes(p), compresslevel=level), parts))
