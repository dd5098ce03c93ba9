"""EdenPipeline on MI355X: drop-in for openfl/pipelines/eden_pipeline.py.

Same classes, constructor keywords, metadata schema and wire bytes as the
reference (/root/reference/openfl/pipelines/eden_pipeline.py):

  Eden.compress / Eden.decompress    :555-611 / :632-659   -> libofl_codec.so
  EdenTransformer.forward            :761-793
  EdenTransformer.backward           :795-818
  EdenPipeline(n_bits, dim_threshold, device, **kw)  :821-851

The numerics run in the gfx950 kernels of openfl_amd/csrc/eden_kernels.hip;
this module only moves host NumPy buffers to/from the device and builds the
metadata dict.  There is no CPU fallback: without a ROCm GPU and the built
library every Eden call raises openfl_amd._lib.CodecError.

Deliberate differences (DESIGN.md "Reference quirks"):
  * backward() decides "compressed?" with the same `size > dim_threshold`
    test as forward(); the reference uses `>=` there (:808), so a tensor of
    exactly dim_threshold elements crashes it with KeyError.
  * seed_mode="fast" (opt-in) replaces the O(n) serial Python sum in the
    seed hash with a sum over the first 4096 elements; the default
    "reference" reproduces the reference seed exactly.  The seed is carried
    in the metadata either way, so decoding never depends on it.
  * device="cpu" (the reference default) selects the current GPU.
"""
import contextlib
import ctypes
import os
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

from openfl_amd import _lib, hostmem
from openfl_amd.codec import EdenCodec, PerThreadDevice
from openfl_amd.pipelines.pipeline import Float32NumpyArrayToBytes, TransformationPipeline, Transformer

_FAST_SEED_PREFIX = 4096
# host staging / per-thread device buffers above this size are dropped at the
# end of the call instead of being kept for the next one (a Llama-sized batch
# would otherwise pin tens of GB per gRPC worker thread for the process life)
_RETAIN_BYTES = 512 << 20


def _serial_sum(flat):
    """`sum(data.flatten())` of the reference seed (:771): left-to-right, in
    the array's own precision (NumPy scalar arithmetic)."""
    L = _lib.lib()
    if flat.dtype == np.float32:
        a = np.ascontiguousarray(flat)
        return np.float32(L.ofl_serial_sum_f32(a.ctypes.data, a.size))
    if flat.dtype == np.float64:
        a = np.ascontiguousarray(flat)
        return np.float64(L.ofl_serial_sum_f64(a.ctypes.data, a.size))
    return sum(flat)


def _serial_sums(flats):
    """_serial_sum of many arrays: float32 / float64 ones in one native
    multi-threaded call (ofl_serial_sums_many), others one by one."""
    out = [None] * len(flats)
    for dt, f64 in ((np.float32, 0), (np.float64, 1)):
        idx = [i for i, f in enumerate(flats) if f.dtype == dt]
        if not idx:
            continue
        arrs = [np.ascontiguousarray(flats[i]) for i in idx]
        ptrs = np.asarray([a.ctypes.data for a in arrs], np.uint64)
        lens = np.asarray([a.size for a in arrs], np.int64)
        res = np.zeros(len(idx), np.float64)
        _lib.check(_lib.lib().ofl_serial_sums_many(len(idx), ptrs.ctypes.data, lens.ctypes.data, f64,
                                                   res.ctypes.data, 16))
        for i, v in zip(idx, res):
            out[i] = dt(v)
    for i, f in enumerate(flats):
        if out[i] is None:
            out[i] = _serial_sum(f)
    return out


def eden_seed(data, mode="reference", total=None, draw=None):
    """Seed of EdenTransformer.forward (:771-772); draws ONE np.random value
    (unless `draw` is that value, taken earlier).  total: the precomputed
    serial sum (forward_batch computes them in parallel)."""
    if total is None:
        flat = data.reshape(-1)
        if mode == "fast":
            flat = flat[:_FAST_SEED_PREFIX]
        total = _serial_sum(flat)
    seed = (hash(total * 13 + 7) + (np.random.randint(1, 2 ** 16) if draw is None else int(draw))) % (2 ** 16)
    return int(float(seed))


def eden_seeds(totals, draws=None):
    """eden_seed for many tensors in order from their serial sums: one
    np.random.randint(1, 2**16, size=T) call -- the legacy generator yields the
    same values and end state as T single calls (MT19937 32-bit bounded draws
    are unbuffered), without T Python-level calls.  draws: the values, if the
    callers drew them already."""
    if draws is None:
        draws = np.random.randint(1, 2 ** 16, size=len(totals)) if len(totals) else []
    return [int(float((hash(t * 13 + 7) + int(r)) % (2 ** 16))) for t, r in zip(totals, draws)]


_pool = None
_pool_lock = threading.Lock()


def _copy_many(dst, src, nbytes, threads=8):
    """Host memcpy's on native threads (ofl_host_copy_many, no GIL)."""
    n = len(dst)
    if n == 0:
        return
    d = np.asarray(dst, np.uint64)
    s = np.asarray(src, np.uint64)
    b = np.asarray(nbytes, np.int64)
    _lib.check(_lib.lib().ofl_host_copy_many(n, d.ctypes.data, s.ctypes.data, b.ctypes.data, threads))


def _threads():
    global _pool
    with _pool_lock:
        if _pool is None:
            _pool = ThreadPoolExecutor(max_workers=8)
        return _pool


class Eden(PerThreadDevice):
    """Device Eden codec with the reference Eden class's method surface.

    device: one GPU ("cpu" = the current one, "cuda:N"), or several ("cuda" =
    all visible, "cuda:0,cuda:1", a list): each calling thread is bound to one
    of them round-robin on its first call (codec.ThreadDevices), so the gRPC
    server's concurrent compress / decompress calls spread over the GPUs with
    the plugin surface unchanged.  Plans, workspaces, streams and staging are
    per device and per thread."""

    def __init__(self, nbits=8, device="cpu"):
        if nbits not in [1, 2, 3, 4, 5, 6, 7, 8]:
            raise Exception("nbits value is not supported")  # :389-390
        self.nbits = int(nbits)
        self._init_devices(device)
        self.num_hadamard = 2           # :394
        self.max_padding_overhead = 0.1  # :397
        self._codecs = [EdenCodec(self.nbits, d) for d in self.devices]
        self._tls = threading.local()

    @property
    def codec(self):
        """The calling thread's device codec (plan cache + workspaces)."""
        return self._codecs[self._thread_devices.slot()]

    def _stream(self):
        st = getattr(self._tls, "stream", None)
        if st is None:
            st = self._tls.stream = torch.cuda.Stream(device=self.device)
        return st

    def _staging(self):
        sg = getattr(self._tls, "staging", None)
        if sg is None:
            sg = self._tls.staging = _Staging()
        return sg

    def _dev(self, name, n, dtype):
        """Per-thread device buffers of the one-tensor calls (power-of-two
        growth; ones above _RETAIN_BYTES are released by _trim)."""
        bufs = getattr(self._tls, "dev", None)
        if bufs is None:
            bufs = self._tls.dev = {}
        b = bufs.get(name)
        if b is None or b.numel() < n or b.dtype != dtype:
            b = bufs[name] = torch.empty(1 << max(int(n) - 1, 4095).bit_length(), dtype=dtype, device=self.device)
        return b

    def _trim(self):
        """Drop this thread's oversized staging and device buffers (after the
        call's stream has been synchronised)."""
        bufs = getattr(self._tls, "dev", None) or {}
        for k in [k for k, b in bufs.items() if b.numel() * b.element_size() > _RETAIN_BYTES]:
            del bufs[k]
        sg = getattr(self._tls, "staging", None)
        if sg is not None:
            sg.trim(_RETAIN_BYTES)
        self.codec.ws.trim(self.device, _RETAIN_BYTES)

    def _ctx(self, key, make):
        """Per-thread call context of one tensor shape (small calls only)."""
        cache = getattr(self._tls, "ctx", None)
        if cache is None:
            cache = self._tls.ctx = {}
        c = cache.get(key)
        if c is None:
            if len(cache) >= _CTX_MAX:
                cache.clear()
            c = cache[key] = make()
        return c

    def _enc_ctx(self, n):
        plan = self.codec.plan([n], streams=1)
        return _CallCtx(plan, self.device, self._stream(), enc=True)

    def _dec_ctx(self, total_dim, dims):
        plan = self.codec.plan([total_dim], dims=[list(dims)], streams=1)
        return _CallCtx(plan, self.device, self._stream(), enc=False, total_dim=total_dim)

    def compress(self, vec, seed, seed_of_sum=None):
        """(planes uint8 ndarray, scales list[float], dims list[int], total_dim) (:555-611).
        One tensor in one native call (ofl_eden_encode_host): pinned input
        block [x | seed] -> one H2D, the launches, one D2H of [planes |
        scales], one sync.  With seed_of_sum the seed is seed_of_sum(the
        reference's serial sum of vec) -- for float32 input taken while vec is
        copied into the pinned block (ofl_serial_sum_copy_f32) -- the seed
        argument is unused, and the result is (the tuple above, seed)."""
        src = np.asarray(vec).reshape(-1)
        fuse = seed_of_sum is not None and src.dtype == np.float32
        if seed_of_sum is not None and not fuse:
            seed = seed_of_sum(_serial_sum(src))
        flat = np.ascontiguousarray(src, dtype=np.float32)
        n = flat.size
        if 0 < n <= _CTX_NUMEL and _USE_CTX:
            # small tensors: a cached per-shape context (own pinned / device
            # buffers and the native call's arguments prepared once) -- the
            # call is latency-bound and its Python work was most of it
            c = self._ctx(("e", n), lambda: self._enc_ctx(n))
            if fuse:
                seed = seed_of_sum(np.float32(_lib.lib().ofl_serial_sum_copy_f32(flat.ctypes.data, c.in_ptr, n)))
            else:
                c.x_view[:] = flat
            c.seed_view[0] = int(seed) & 0xFFFFFFFF
            c.run()
            out = (np.frombuffer(ctypes.string_at(c.out_ptr, c.pb), np.uint8), c.scales_view.tolist(), list(c.dims), n)
            return out if seed_of_sum is None else (out, int(seed))
        L = _lib.lib()
        plan = self.codec.plan([n], streams=_one_tensor_streams(n))
        pb, ns = plan.planes_bytes, plan.n_slices
        off_seeds = _al256(4 * plan.arena_numel)
        in_bytes = off_seeds + 4
        off_scales = _al256(pb)
        out_bytes = off_scales + 4 * ns
        stg = self._staging()
        oh = stg.get("out1", out_bytes, torch.uint8)
        idev = self._dev("in", in_bytes, torch.uint8)
        odev = self._dev("out", out_bytes, torch.uint8)
        ws = self.codec.ws.get(plan.ws_bytes, self.device)
        st = self._stream().cuda_stream
        with _device_guard(self.device):
            if _PAGEABLE:
                # x H2D from where it lies (ofl_eden_encode_host_x); with the
                # reference seed the DMA runs beside the serial sum.  Faster
                # on one reused array, slower over a model's many fresh ones
                # (profiles/r03_e2e_*), hence opt-in
                x_ptr = flat.ctypes.data if n else None
                if fuse:
                    _lib.check(L.ofl_copy_h2d_async(idev.data_ptr(), x_ptr, 4 * n, st))
                    x_ptr = None
                    seed = seed_of_sum(np.float32(L.ofl_serial_sum_f32(flat.ctypes.data, n)))
                _lib.check(L.ofl_eden_encode_host_x(
                    plan.handle, x_ptr, 4 * n, int(seed) & 0xFFFFFFFF, idev.data_ptr(), off_seeds, odev.data_ptr(),
                    oh.data_ptr(), out_bytes, off_scales, ws.data_ptr(), ws.numel(), st))
            else:
                # x into pinned staging in chunks, each chunk's H2D issued as
                # soon as it is there (ofl_copy_h2d_chunked): the DMA runs
                # beside the copy and the reference seed's serial sum; then the
                # seed, the launches and one D2H (ofl_eden_encode_seeded)
                ih = stg.get("in1", in_bytes, torch.uint8)
                sm = ctypes.c_float(0.0)
                _lib.check(L.ofl_copy_h2d_chunked(flat.ctypes.data if n else None, ih.data_ptr(), idev.data_ptr(), n,
                                                  _H2D_CHUNK, 1 if fuse else 0, ctypes.byref(sm), st))
                if fuse:
                    seed = seed_of_sum(np.float32(sm.value))
                _lib.check(L.ofl_eden_encode_seeded(
                    plan.handle, idev.data_ptr(), off_seeds, int(seed) & 0xFFFFFFFF, odev.data_ptr(),
                    oh.data_ptr(), out_bytes, off_scales, ws.data_ptr(), ws.numel(), st))
        oa = oh.numpy()
        # one host copy, pinned -> bytes; the array is a zero-copy view of it
        out = (np.frombuffer(hostmem.bytes_from(oa.ctypes.data, pb), np.uint8),
               [float(v) for v in oa[off_scales:off_scales + 4 * ns].view(np.float32)], list(plan.dims[0]), n)
        self._trim()
        return out if seed_of_sum is None else (out, int(seed))

    def decompress(self, bins, metadata):
        """bins: uint8 planes; metadata: int_to_float mapping (:632-659).  One
        native call (ofl_eden_decode_host): [planes | scales | seed] -> one H2D,
        the launches, one D2H of y, one sync."""
        seed = int(metadata[0])
        total_dim = int(metadata[1])
        keys = list(metadata.keys())
        scales, dims = [], []
        for k in range(2, max(keys) + 1, 2):
            scales.append(metadata[k])
            dims.append(int(metadata[k + 1]))
        if total_dim > sum(dims):
            raise ValueError(f"Eden metadata: total_dim {total_dim} exceeds the slices ({sum(dims)})")
        planes_h = np.frombuffer(bins, dtype=np.uint8) if isinstance(bins, (bytes, bytearray, memoryview)) \
            else np.asarray(bins, dtype=np.uint8).reshape(-1)
        if 0 < total_dim <= _CTX_NUMEL and sum(dims) <= 2 * _CTX_NUMEL and _USE_CTX:
            c = self._ctx(("d", total_dim, tuple(dims)), lambda: self._dec_ctx(total_dim, dims))
            if planes_h.size < c.pb:
                raise ValueError(f"Eden payload has {planes_h.size} bytes, expected {c.pb}")
            c.planes_view[:] = planes_h[:c.pb]
            c.scales_view[:] = scales
            c.seed_view[0] = seed & 0xFFFFFFFF
            c.run()
            return c.y_view.copy()  # D2H into pinned memory, then a small host copy
        plan = self.codec.plan([total_dim], dims=[dims], streams=_one_tensor_streams(sum(dims)))
        if planes_h.size < plan.planes_bytes:
            raise ValueError(f"Eden payload has {planes_h.size} bytes, expected {plan.planes_bytes}")
        pb, ns = plan.planes_bytes, plan.n_slices
        off_scales = _al256(pb)
        off_seeds = _al256(off_scales + 4 * ns)
        in_bytes = off_seeds + 4
        out_bytes = 4 * total_dim
        sc = np.asarray(scales, np.float32)
        y = np.empty(max(total_dim, 1), np.float32) if _PAGEABLE else None
        idev = self._dev("in", in_bytes, torch.uint8)
        ydev = self._dev("y", max(plan.arena_numel, 1), torch.float32)
        ws = self.codec.ws.get(plan.ws_bytes, self.device)
        L = _lib.lib()
        with _device_guard(self.device):
            if _PAGEABLE:
                # planes H2D from the payload itself (opt-in, see compress)
                _lib.check(L.ofl_eden_decode_host_x(
                    plan.handle, planes_h.ctypes.data, pb, sc.ctypes.data, ns, seed & 0xFFFFFFFF, idev.data_ptr(),
                    off_scales, off_seeds, ydev.data_ptr(), y.ctypes.data, out_bytes, ws.data_ptr(), ws.numel(),
                    self._stream().cuda_stream))
            else:
                # y D2H into pinned staging, then a threaded copy into the
                # fresh array (its first-touch faults taken in parallel, huge
                # pages above 4 MiB): a pageable D2H into fresh memory ran at
                # ~3 GB/s in the end-to-end loop (profiles/r03_e2e_*)
                stg = self._staging()
                ih = stg.get("in1", in_bytes, torch.uint8)
                ia = ih.numpy()
                ia[:pb] = planes_h[:pb]
                ia[off_scales:off_scales + 4 * ns].view(np.float32)[:] = sc
                ia[off_seeds:off_seeds + 4].view(np.uint32)[0] = seed & 0xFFFFFFFF
                yh = stg.get("out1", max(out_bytes, 4), torch.uint8)
                _lib.check(L.ofl_eden_decode_host(
                    plan.handle, ih.data_ptr(), idev.data_ptr(), in_bytes, off_scales, off_seeds, ydev.data_ptr(),
                    yh.data_ptr(), out_bytes, ws.data_ptr(), ws.numel(), self._stream().cuda_stream))
                y = hostmem.array_from(yh.data_ptr(), max(total_dim, 1), np.float32)
        self._trim()
        return y[:total_dim]


# one-tensor calls of at most this many elements use cached per-shape call
# contexts (_CallCtx); OFL_PLUGIN_CTX=0 turns them off (A/B)
_CTX_NUMEL = 1 << 16
_CTX_MAX = 256
_USE_CTX = os.environ.get("OFL_PLUGIN_CTX", "1") != "0"
# larger one-tensor calls: OFL_PLUGIN_PAGEABLE=1 moves x / planes straight
# from the caller's arrays (ofl_eden_*_host_x) instead of via pinned staging
_PAGEABLE = os.environ.get("OFL_PLUGIN_PAGEABLE", "0") == "1"
# larger one-tensor encodes: x goes H2D in chunks of this many elements
_H2D_CHUNK = 1 << 18
# contexts whose slices are all <= 2^15: kernels on mapped pinned memory
# (OFL_PLUGIN_MAPPED=0: H2D / D2H copies around the launch, A/B)
_USE_MAPPED = os.environ.get("OFL_PLUGIN_MAPPED", "1") != "0"


class _CallCtx:
    """One tensor shape's one-call encode or decode, prepared once per thread:
    the plan (single stream), pinned in/out blocks and device buffers of
    exactly its size, numpy views into the pinned blocks, and the native
    call's argument list (ofl_eden_encode_host / ofl_eden_decode_host, or
    the zero-copy ofl_eden_encode_mapped / ofl_eden_decode_mapped)."""

    def __init__(self, plan, device, stream, enc, total_dim=0):
        self.plan = plan
        self.pb, ns = plan.planes_bytes, plan.n_slices
        self.dims = plan.dims[0]
        self.dev_index = device.index
        self.stream = stream
        # slices of <= 2^15 only: one launch that reads / writes the pinned
        # blocks directly (ofl_eden_*_mapped, no DMA copies)
        self.mapped = _USE_MAPPED and all(d <= 1 << 15 for d in self.dims)
        ws = torch.empty(max(plan.ws_bytes, 256), dtype=torch.uint8, device=device)
        L = _lib.lib()
        if enc:
            off_seeds = _al256(4 * plan.arena_numel)
            in_bytes = off_seeds + 4
            off_scales = _al256(self.pb)
            out_bytes = off_scales + 4 * ns
            ih = torch.empty(in_bytes, dtype=torch.uint8).pin_memory()
            oh = torch.empty(out_bytes, dtype=torch.uint8).pin_memory()
            ia, oa = ih.numpy(), oh.numpy()
            self.x_view = ia[:4 * plan.numels[0]].view(np.float32)
            self.seed_view = ia[off_seeds:off_seeds + 4].view(np.uint32)
            self.scales_view = oa[off_scales:off_scales + 4 * ns].view(np.float32)
            idev = odev = None
            if not self.mapped:
                idev = torch.empty(in_bytes, dtype=torch.uint8, device=device)
                odev = torch.empty(out_bytes, dtype=torch.uint8, device=device)
            self.in_ptr, self.out_ptr = ih.data_ptr(), oh.data_ptr()
            if self.mapped:
                self._fn = L.ofl_eden_encode_mapped
                self._args = [plan.handle, ih.data_ptr(), off_seeds, oh.data_ptr(), off_scales, ws.data_ptr(),
                              ws.numel(), stream.cuda_stream]
                self._keep = (ih, oh, ws)
            else:
                self._fn = L.ofl_eden_encode_host
                self._args = [plan.handle, ih.data_ptr(), idev.data_ptr(), in_bytes, off_seeds, odev.data_ptr(),
                              oh.data_ptr(), out_bytes, off_scales, ws.data_ptr(), ws.numel(), stream.cuda_stream]
                self._keep = (ih, oh, idev, odev, ws)
        else:
            off_scales = _al256(self.pb)
            off_seeds = _al256(off_scales + 4 * ns)
            in_bytes = off_seeds + 4
            ih = torch.empty(in_bytes, dtype=torch.uint8).pin_memory()
            ia = ih.numpy()
            self.planes_view = ia[:self.pb]
            self.scales_view = ia[off_scales:off_scales + 4 * ns].view(np.float32)
            self.seed_view = ia[off_seeds:off_seeds + 4].view(np.uint32)
            yh = torch.empty(max(plan.arena_numel, 1), dtype=torch.float32).pin_memory()
            self.y_view = yh.numpy()[:total_dim]
            if self.mapped:
                self._fn = L.ofl_eden_decode_mapped
                self._args = [plan.handle, ih.data_ptr(), off_scales, off_seeds, yh.data_ptr(), ws.data_ptr(),
                              ws.numel(), stream.cuda_stream]
                self._keep = (ih, yh, ws)
            else:
                idev = torch.empty(in_bytes, dtype=torch.uint8, device=device)
                ydev = torch.empty(max(plan.arena_numel, 1), dtype=torch.float32, device=device)
                self._fn = L.ofl_eden_decode_host
                self._args = [plan.handle, ih.data_ptr(), idev.data_ptr(), in_bytes, off_scales, off_seeds,
                              ydev.data_ptr(), yh.data_ptr(), 4 * total_dim, ws.data_ptr(), ws.numel(),
                              stream.cuda_stream]
                self._keep = (ih, idev, ydev, yh, ws)

    def run(self):
        if self.dev_index is not None and self.dev_index != torch.cuda.current_device():
            with torch.cuda.device(self.dev_index):
                _lib.check(self._fn(*self._args))
        else:
            _lib.check(self._fn(*self._args))


def _one_tensor_streams(n):
    """Stream count of a one-tensor plan: up to 2^24 elements one stream (no
    side-stream fork/join per call: the per-tensor path is latency-bound);
    larger tensors keep the two-stream wave schedule."""
    return 1 if n <= (1 << 24) else None


def _al256(b):
    return (int(b) + 255) // 256 * 256


def _device_guard(dev):
    """Make dev current for a library call when it is not (plans and their
    device tables belong to the device current at their first use)."""
    if dev.index is None or dev.index == torch.cuda.current_device():
        return contextlib.nullcontext()
    return torch.cuda.device(dev)


class _Staging:
    """Pinned host buffers of one batch shape (grown on demand; trim() drops
    the oversized ones)."""

    def __init__(self):
        self.bufs = {}

    def trim(self, limit):
        for k in [k for k, b in self.bufs.items() if b.numel() * b.element_size() > limit]:
            del self.bufs[k]

    def get(self, name, n, dtype):
        b = self.bufs.get(name)
        if b is None or b.numel() < n or b.dtype != dtype:
            # power-of-two growth: pinning is slow, tensor sizes vary call to call
            b = torch.empty(1 << max(int(n) - 1, 4095).bit_length(), dtype=dtype).pin_memory()
            self.bufs[name] = b
        return b


_CHUNKS = 4  # host <-> device copies of a batch go in this many pieces, overlapped


def _pieces(offsets, sizes, k):
    """Split tensors [0, n) (arena order) into <= k contiguous runs of about
    equal bytes: [(first, last + 1), ...]."""
    n = len(sizes)
    tot = sum(sizes)
    runs, start, acc = [], 0, 0
    for i, sz in enumerate(sizes):
        acc += sz
        if acc * k >= tot * (len(runs) + 1) and i + 1 < n and len(runs) + 1 < k:
            runs.append((start, i + 1))
            start = i + 1
    runs.append((start, n))
    return [r for r in runs if r[1] > r[0]]


def _batch_stage(eden, arrays):
    """First half of a batch encode: plan, then the fill of the pinned arena
    and its H2D in pieces, so that the copy of piece k+1 (native threads)
    overlaps the DMA of piece k.  Returns the state _batch_encode finishes."""
    codec = eden.codec
    flats = [np.ascontiguousarray(np.asarray(a).reshape(-1), dtype=np.float32) for a in arrays]
    plan = codec.plan([f.size for f in flats])
    st = eden._stream()
    xh = eden._staging().get("x", plan.arena_numel, torch.float32)
    base = xh.data_ptr()
    with torch.cuda.stream(st):  # allocated on the stream that fills and reads it
        x = torch.empty(max(plan.arena_numel, 1), dtype=torch.float32, device=eden.device)
    offs = plan.elem_offsets
    for lo, hi in _pieces(offs, [f.size for f in flats], _CHUNKS):
        _copy_many([base + 4 * offs[i] for i in range(lo, hi)], [flats[i].ctypes.data for i in range(lo, hi)],
                   [4 * flats[i].size for i in range(lo, hi)])
        e0, e1 = offs[lo], offs[hi - 1] + flats[hi - 1].size
        if e1 > e0:
            with torch.cuda.stream(st):
                x[e0:e1].copy_(xh[e0:e1], non_blocking=True)
    return plan, flats, x


def _batch_encode(eden, staged, seeds):
    """Second half: seeds, the launch sequence, one D2H of planes + scales.
    -> [(planes bytes, scales, dims)] per array, the per-tensor Eden.compress
    results."""
    plan, flats, x = staged
    codec = eden.codec
    st = eden._stream()
    stg = eden._staging()
    ph = stg.get("planes", plan.planes_bytes, torch.uint8)
    sh = stg.get("scales", plan.n_slices, torch.float32)
    with torch.cuda.stream(st):
        sd = torch.tensor(seeds, dtype=torch.int32).pin_memory().to(eden.device, non_blocking=True)
        planes, scales = codec.encode_arena(plan, x, sd, stream=st)
        ph[:max(plan.planes_bytes, 1)].copy_(planes[:max(plan.planes_bytes, 1)], non_blocking=True)
        sh[:max(plan.n_slices, 1)].copy_(scales[:max(plan.n_slices, 1)], non_blocking=True)
    st.synchronize()
    pn, sn = ph.numpy(), sh.numpy()
    out = []
    for t in range(len(flats)):
        po, pb, fs = plan.planes_offsets[t], plan.planes_nbytes[t], plan.first_slice[t]
        dims = plan.dims[t]
        # the one host copy a `bytes` payload needs (protobuf's data_bytes
        # takes bytes only), straight from the pinned D2H buffer
        out.append((hostmem.bytes_from(pn.ctypes.data + po, pb), [float(v) for v in sn[fs:fs + len(dims)]], list(dims)))
    del x, planes, scales
    eden._trim()
    return out


def _batch_decode(eden, items):
    """Eden-decode many payloads (planes bytes, int_to_float metadata) with one
    plan.  -> fresh float32 arrays (flat, total_dim elements each).  The D2H of
    the decoded arena goes in pieces; each piece is copied out to its arrays
    (native threads) while the next one is in flight."""
    codec = eden.codec
    totals, dims, scales, seeds = [], [], [], []
    for data, md in items:
        keys = list(md.keys())
        totals.append(int(md[1]))
        dims.append([int(md[k + 1]) for k in range(2, max(keys) + 1, 2)])
        scales.append([md[k] for k in range(2, max(keys) + 1, 2)])
        seeds.append(int(md[0]))
        if totals[-1] > sum(dims[-1]):
            raise ValueError(f"Eden metadata: total_dim {totals[-1]} exceeds the slices ({sum(dims[-1])})")
    plan = codec.plan(totals, dims=dims)
    st = eden._stream()
    stg = eden._staging()
    ph = stg.get("planes_in", plan.planes_bytes, torch.uint8)
    yh = stg.get("y", plan.arena_numel, torch.float32)
    sc = np.asarray([v for s_ in scales for v in s_] or [0.0], np.float32)
    bufs = [np.frombuffer(items[t][0], dtype=np.uint8) for t in range(len(items))]
    for t, b in enumerate(bufs):
        if b.size < plan.planes_nbytes[t]:
            raise ValueError(f"Eden payload has {b.size} bytes, expected {plan.planes_nbytes[t]}")
    pbase = ph.data_ptr()
    _copy_many([pbase + plan.planes_offsets[t] for t in range(len(items))], [b.ctypes.data for b in bufs],
               [plan.planes_nbytes[t] for t in range(len(items))])
    offs = plan.elem_offsets
    pieces = _pieces(offs, totals, _CHUNKS)
    events = []
    with torch.cuda.stream(st):
        planes = torch.empty(max(plan.planes_bytes, 1), dtype=torch.uint8, device=eden.device)
        planes.copy_(ph[:max(plan.planes_bytes, 1)], non_blocking=True)
        scd = torch.from_numpy(sc).pin_memory().to(eden.device, non_blocking=True)
        sdd = torch.tensor(seeds, dtype=torch.int32).pin_memory().to(eden.device, non_blocking=True)
        y = codec.decode_arena(plan, planes, scd, sdd, stream=st)
        for lo, hi in pieces:
            e0, e1 = offs[lo], offs[hi - 1] + totals[hi - 1]
            if e1 > e0:
                yh[e0:e1].copy_(y[e0:e1], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(st)
            events.append(ev)
    outs = [np.empty(totals[t], np.float32) for t in range(len(items))]
    ybase = yh.data_ptr()
    for (lo, hi), ev in zip(pieces, events):
        ev.synchronize()
        _copy_many([outs[t].ctypes.data for t in range(lo, hi)], [ybase + 4 * offs[t] for t in range(lo, hi)],
                   [4 * totals[t] for t in range(lo, hi)])
    st.synchronize()
    del planes, y
    eden._trim()
    return outs


class EdenTransformer(Transformer):
    """Eden quantising transformer (:723-818)."""

    def __init__(self, n_bits=8, dim_threshold=100, device="cpu", seed_mode="reference"):
        self.lossy = True
        self.eden = Eden(nbits=n_bits, device=device)
        self.dim_threshold = dim_threshold
        self.no_comp = Float32NumpyArrayToBytes()
        if seed_mode not in ("reference", "fast"):
            raise ValueError("seed_mode must be 'reference' or 'fast'")
        self.seed_mode = seed_mode

    def _metadata(self, shape, seed, total_dim, scales, dims):
        md = {"int_list": list(shape), "int_to_float": {0: float(seed), 1: float(total_dim)}}
        k = 2
        for scale, dim in zip(scales, dims):
            md["int_to_float"][k] = scale
            md["int_to_float"][k + 1] = float(dim)
            k += 2
        return md

    def _forward_one(self, data, draw=None):
        """forward of one tensor above the threshold (draw: its np.random
        value, if the caller took it already)."""
        if self.seed_mode == "reference":  # the seed's sum taken while the input is staged
            (int_array, scale_list, dim_list, total_dim), seed = self.eden.compress(
                data, None, seed_of_sum=lambda total: eden_seed(None, total=total, draw=draw))
        else:
            seed = eden_seed(data, self.seed_mode, draw=draw)
            int_array, scale_list, dim_list, total_dim = self.eden.compress(data, seed)
        b = int_array.base
        payload = b if isinstance(b, bytes) and len(b) == int_array.nbytes else int_array.tobytes()
        return payload, self._metadata(data.shape, seed, total_dim, scale_list, dim_list)

    def forward(self, data, **kwargs):
        if data.size > self.dim_threshold:
            return self._forward_one(data)
        eden_seed(data, self.seed_mode)  # the reference draws its RNG value for every tensor (:771)
        return self.no_comp.forward(data)

    def backward(self, data, metadata, **kwargs):
        if np.prod(metadata["int_list"]) > self.dim_threshold:  # reference: >= (:808), see module doc
            out = self.eden.decompress(np.frombuffer(data, dtype=np.uint8), metadata["int_to_float"])
            # already a fresh float32 array: astype would only copy it again
            return out.reshape(list(metadata["int_list"]))
        out = self.no_comp.backward(data, metadata)
        return out.astype(np.float32)

    # -- many tensors per call (same results as forward/backward in order) --
    def forward_batch(self, arrays):
        """[forward(a) for a in arrays], with the Eden tensors coded in one
        batch: the seeds' serial sums run in parallel host threads, then the
        np.random draws happen in tensor order exactly as per-tensor calls do."""
        return self._forward_many([np.asarray(a) for a in arrays])

    def _forward_many(self, arrays, draws=None):
        big = [i for i, a in enumerate(arrays) if a.size > self.dim_threshold]
        # the seeds' serial sums (native threads, no GIL) run while this
        # thread stages the Eden tensors and starts their H2D
        sums = _threads().submit(_serial_sums, [a.reshape(-1)[:_FAST_SEED_PREFIX] if self.seed_mode == "fast"
                                                else a.reshape(-1) for a in arrays])
        staged = _batch_stage(self.eden, [arrays[i] for i in big]) if big else None
        seeds = eden_seeds(sums.result(), draws)
        enc = _batch_encode(self.eden, staged, [seeds[i] for i in big]) if big else []
        out = [None] * len(arrays)
        for i, (planes, scales, dims) in zip(big, enc):
            out[i] = (planes, self._metadata(arrays[i].shape, seeds[i], arrays[i].size, scales, dims))
        for i, a in enumerate(arrays):
            if out[i] is None:
                out[i] = self.no_comp.forward(a)
        return out

    def backward_batch(self, items):
        """[backward(data, md) for data, md in items], the Eden ones decoded in one batch."""
        big = [i for i, (_, md) in enumerate(items) if np.prod(md["int_list"]) > self.dim_threshold]
        dec = _batch_decode(self.eden, [(items[i][0], items[i][1]["int_to_float"]) for i in big]) if big else []
        out = [None] * len(items)
        for i, y in zip(big, dec):
            out[i] = y.reshape(list(items[i][1]["int_list"]))
        for i, (data, md) in enumerate(items):
            if out[i] is None:
                out[i] = self.no_comp.backward(data, md).astype(np.float32)
        return out


class EdenPipeline(TransformationPipeline):
    """plan.yaml: template openfl_amd.pipelines.EdenPipeline, settings n_bits /
    dim_threshold / device (:821-851); extra keyword seed_mode."""

    def __init__(self, n_bits=8, dim_threshold=100, device="cpu", seed_mode="reference", **kwargs):
        transformers = [EdenTransformer(n_bits, dim_threshold, device, seed_mode)]
        super().__init__(transformers=transformers, **kwargs)

    def forward(self, data, **kwargs):
        # The reference copies the input first (pipeline.py:144) to protect it
        # from in-place transformers; EdenTransformer never writes its input,
        # so the O(n) host copy is skipped.
        transformer_metadata = []
        for transformer in self.transformers:
            data, metadata = transformer.forward(data=data, **kwargs)
            transformer_metadata.append(metadata)
        return data, transformer_metadata

    def forward_batch(self, arrays):
        """Batch form of forward for a whole model update (the aggregator's
        end-of-round loop, a model snapshot): [(bytes, [metadata]), ...],
        identical to [forward(a) for a in arrays] (same bytes, metadata and
        np.random draws); one H2D / launch sequence / D2H for all tensors."""
        return [(b, [md]) for b, md in self.transformers[0].forward_batch(arrays)]

    def backward_batch(self, items):
        """[backward(data, metadata_list) for ...] in one batch; like backward,
        pops each item's metadata list (pipeline.py:161-163)."""
        return self.transformers[0].backward_batch([(data, mds.pop()) for data, mds in items])
