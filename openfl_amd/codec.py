"""Device-level Eden codec: batch plans over PyTorch-ROCm buffers.

This is the layer the plugin (openfl_amd.pipelines.eden_pipeline) and
bench.py sit on.  A batch of tensors lives in one fp32 arena (tensor t at
element offset ``plan.elem_offsets[t]``); its Eden bit planes live in one byte
arena (tensor t at ``plan.planes_offsets[t]``, ``plan.planes_nbytes[t]``
bytes, the reference's to_bits layout, eden_pipeline.py:661-690) and its
per-slice scales in one float array (tensor t's slices start at
``plan.first_slice[t]``).  Encode/decode are asynchronous on the given HIP
stream; nothing here synchronises.
"""
import ctypes
import threading

import numpy as np
import torch

from openfl_amd import _lib

_ALIGN = 64  # elements: every tensor starts 256-B aligned in the fp32 arena


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if isinstance(a, np.ndarray) else ctypes.c_void_p(a)


def slice_plan(n):
    """Reference slicing rule (eden_pipeline.py:569-606): (padded sizes, valid lengths)."""
    L = _lib.lib()
    ns = L.ofl_eden_slice_plan(int(n), None, None, 0)
    P = np.zeros(max(ns, 1), np.int64)
    ln = np.zeros(max(ns, 1), np.int64)
    L.ofl_eden_slice_plan(int(n), _ptr(P), _ptr(ln), ns)
    return [int(v) for v in P[:ns]], [int(v) for v in ln[:ns]]


class EdenPlan:
    """Layout + launch plan for one batch shape (list of numels, optional dims)."""

    def __init__(self, numels, n_bits=8, dims=None, elem_offsets=None, wave_mib=None, streams=None, row2=None,
                 sset=None, fuse=None, pair=None):
        """wave_mib / streams: large-slice schedule (ofl_eden_plan_set_schedule;
        None keeps the library default); row2: row-pass kernels
        (ofl_eden_plan_set_row2: None/-1 auto, 0 persistent, 1 two blocks per
        CU); pair: tile pairs sharing their D1 sign words in those kernels
        (ofl_eden_plan_set_pair: None/-1 auto, 0 never, 1 always); sset: tiny / small slices in one launch (ofl_eden_plan_set_sset:
        None/-1 default, 0 one launch per size class, 1 one launch); fuse:
        that launch inside a one-wave plan's column launch on the caller's
        stream (ofl_eden_plan_set_fuse: None/-1 default, 0 no, 1 yes).
        Outputs do not depend on any of them."""
        L = _lib.lib()
        self.n_bits = int(n_bits)
        self.numels = [int(n) for n in numels]
        nt = len(self.numels)
        if elem_offsets is None:
            offs, acc = [], 0
            for n in self.numels:
                offs.append(acc)
                acc += (n + _ALIGN - 1) // _ALIGN * _ALIGN
        else:
            offs = [int(o) for o in elem_offsets]
        self.arena_numel = max([o + n for o, n in zip(offs, self.numels)] + [0])
        self.elem_offsets = offs
        numel_a = np.asarray(self.numels, np.int64)
        off_a = np.asarray(offs, np.int64)
        if dims is not None:
            ns_a = np.asarray([len(d) for d in dims], np.int32)
            dims_a = np.asarray([int(v) for d in dims for v in d] or [0], np.int64)
            args = (_ptr(ns_a), _ptr(dims_a))
        else:
            args = (None, None)
        h = ctypes.c_void_p()
        _lib.check(L.ofl_eden_plan_create(nt, _ptr(numel_a), _ptr(off_a), args[0], args[1],
                                          self.n_bits, ctypes.byref(h)))
        self._h = h
        self._L = L
        if wave_mib is not None or streams is not None:
            _lib.check(L.ofl_eden_plan_set_schedule(h, -1 if wave_mib is None else int(float(wave_mib) * 2 ** 20),
                                                    0 if streams is None else int(streams)))
        if row2 is not None:
            _lib.check(L.ofl_eden_plan_set_row2(h, int(row2)))
        if pair is not None:
            _lib.check(L.ofl_eden_plan_set_pair(h, int(pair)))
        if sset is not None:
            _lib.check(L.ofl_eden_plan_set_sset(h, int(sset)))
        if fuse is not None:
            _lib.check(L.ofl_eden_plan_set_fuse(h, int(fuse)))
        self.n_waves = int(L.ofl_eden_plan_num_waves(h))
        wb, ns = ctypes.c_int64(), ctypes.c_int()
        _lib.check(L.ofl_eden_plan_get_schedule(h, ctypes.byref(wb), ctypes.byref(ns)))
        self.wave_mib, self.n_streams = wb.value / 2 ** 20, ns.value
        self.n_slices = int(L.ofl_eden_plan_num_slices(h))
        self.planes_bytes = int(L.ofl_eden_plan_planes_bytes(h))
        self.ws_bytes = int(L.ofl_eden_plan_workspace_bytes(h))
        self.planes_offsets, self.planes_nbytes, self.first_slice, self.dims = [], [], [], []
        for t in range(nt):
            po, pb = ctypes.c_int64(), ctypes.c_int64()
            fs, ns = ctypes.c_int32(), ctypes.c_int32()
            _lib.check(L.ofl_eden_plan_tensor_info(h, t, ctypes.byref(po), ctypes.byref(pb),
                                                   ctypes.byref(fs), ctypes.byref(ns)))
            d = np.zeros(max(ns.value, 1), np.int64)
            _lib.check(L.ofl_eden_plan_tensor_dims(h, t, _ptr(d)))
            self.planes_offsets.append(po.value)
            self.planes_nbytes.append(pb.value)
            self.first_slice.append(fs.value)
            self.dims.append([int(v) for v in d[:ns.value]])

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            self._L.ofl_eden_plan_destroy(h)
            self._h = None

    @property
    def handle(self):
        """The C-ABI plan (ofl_eden_plan_t) for direct library calls."""
        return self._h

    # -- raw launches (all pointers are device tensors) --
    def encode(self, x_arena, seeds, planes, scales, ws, stream=None):
        """x_arena fp32[arena_numel] -> planes u8[planes_bytes], scales f32[n_slices]."""
        self._check(x_arena, torch.float32, self.arena_numel)
        self._check(planes, torch.uint8, self.planes_bytes)
        self._check(scales, torch.float32, self.n_slices)
        self._check(seeds, torch.int32, len(self.numels))
        st = stream if stream is not None else torch.cuda.current_stream(x_arena.device)
        _lib.check(self._L.ofl_eden_encode(self._h, x_arena.data_ptr(), seeds.data_ptr(),
                                           planes.data_ptr(), scales.data_ptr(),
                                           ws.data_ptr() if ws is not None else None,
                                           ws.numel() if ws is not None else 0, st.cuda_stream))

    def decode(self, planes, seeds, scales, y_arena, ws, stream=None, base=None):
        """planes u8 + scales f32 -> y_arena fp32 (numel[t] elements of each
        tensor); with base (an arena of this layout): y = base + decoded
        (TensorCodec.apply_delta fused, ofl_eden_decode_add)."""
        self._check(y_arena, torch.float32, self.arena_numel)
        self._check(planes, torch.uint8, self.planes_bytes)
        self._check(scales, torch.float32, self.n_slices)
        self._check(seeds, torch.int32, len(self.numels))
        if base is not None:
            self._check(base, torch.float32, self.arena_numel)
        st = stream if stream is not None else torch.cuda.current_stream(y_arena.device)
        _lib.check(self._L.ofl_eden_decode_add(self._h, planes.data_ptr(), seeds.data_ptr(),
                                               scales.data_ptr(), base.data_ptr() if base is not None else None,
                                               y_arena.data_ptr(), ws.data_ptr() if ws is not None else None,
                                               ws.numel() if ws is not None else 0, st.cuda_stream))

    # -- profiling (HIP events between launches; see ofl_codec.h) --
    def profile(self, enable=True):
        _lib.check(self._L.ofl_eden_plan_profile(self._h, 1 if enable else 0))

    def launches(self, encode):
        out = []
        for i in range(self._L.ofl_eden_plan_num_launches(self._h, 1 if encode else 0)):
            name = ctypes.create_string_buffer(128)
            blocks, mv, al = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
            _lib.check(self._L.ofl_eden_plan_launch_info(self._h, 1 if encode else 0, i, name, 128,
                                                         ctypes.byref(blocks), ctypes.byref(mv),
                                                         ctypes.byref(al)))
            out.append({"name": name.value.decode(), "blocks": blocks.value,
                        "bytes_moved": mv.value, "bytes_alg": al.value})
        return out

    def profile_collect(self, encode):
        """-> (per-launch summed ms, number of recorded calls)."""
        n = self._L.ofl_eden_plan_num_launches(self._h, 1 if encode else 0)
        ms = np.zeros(max(n, 1), np.float64)
        calls = ctypes.c_int()
        _lib.check(self._L.ofl_eden_plan_profile_collect(self._h, 1 if encode else 0, _ptr(ms), n,
                                                         ctypes.byref(calls)))
        return ms[:n], calls.value

    @staticmethod
    def _check(t, dtype, min_numel):
        if not t.is_cuda:
            raise _lib.CodecError("openfl_amd codec buffers must be device tensors")
        if t.dtype != dtype or not t.is_contiguous() or t.numel() < min_numel:
            raise _lib.CodecError(f"buffer must be contiguous {dtype} with >= {min_numel} elements")


_capture_streams = {}
_capture_locks = {}
_capture_guard = threading.Lock()


def _capture_stream(dev):
    """One capture stream per device for every EdenStepGraph, with the lock
    that serialises captures on it: each new stream takes the next HW queue
    round robin, and a queue shared with a busy stream serialises
    (ofl_side_stream in include/ofl_codec.h); two captures begun on one stream
    at once would both fail, so EdenStepGraph holds the lock while it
    captures.  -> (stream, lock)."""
    key = str(dev)
    with _capture_guard:
        if key not in _capture_streams:
            _capture_streams[key] = torch.cuda.Stream(device=dev)
            _capture_locks[key] = threading.Lock()
        return _capture_streams[key], _capture_locks[key]


class EdenStepGraph:
    """One plan's encode + decode over fixed device buffers, captured once as a
    hipGraph (torch.cuda.CUDAGraph around the C-ABI calls; the plan's
    side-stream fork/join becomes graph edges) and replayed: the launches of a
    step are submitted as one graph instead of one by one.  Outputs are
    bit-identical to the eager calls (tools/graph_ab.py).  The plan runs once
    eagerly first: its descriptor tables go to the device on first use, which
    must not happen inside a capture (ofl_codec.h)."""

    def __init__(self, plan, x, seeds, planes, scales, y, ws):
        dev = x.device
        self._stream, lock = _capture_stream(dev)
        # one construction at a time per device: the captures share the
        # device's capture stream, and the eager run's synchronize must not
        # fall inside another thread's capture; thread_local capture mode so
        # that unrelated threads' calls do not invalidate this capture
        with lock:
            plan.encode(x, seeds, planes, scales, ws)
            plan.decode(planes, seeds, scales, y, ws)
            torch.cuda.synchronize(dev)
            self._stream.wait_stream(torch.cuda.current_stream(dev))
            self._graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self._graph, stream=self._stream, capture_error_mode="thread_local"):
                plan.encode(x, seeds, planes, scales, ws)
                plan.decode(planes, seeds, scales, y, ws)
        self._keep = (plan, x, seeds, planes, scales, y, ws)  # the graph holds their addresses

    def replay(self):
        self._graph.replay()


class Workspace:
    """Per-(thread, device) growable device scratch buffer."""

    def __init__(self):
        self._tls = threading.local()

    def get(self, nbytes, device):
        bufs = getattr(self._tls, "bufs", None)
        if bufs is None:
            bufs = self._tls.bufs = {}
        key = str(device)
        b = bufs.get(key)
        if b is None or b.numel() < nbytes:
            b = torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=device)
            bufs[key] = b
        return b

    def trim(self, device, limit):
        """Drop this thread's buffer for device if it exceeds limit bytes."""
        bufs = getattr(self._tls, "bufs", None) or {}
        b = bufs.get(str(device))
        if b is not None and b.numel() > limit:
            del bufs[str(device)]


def resolve_device(device):
    """Map a reference `device` setting to a ROCm device.

    The reference's Eden defaults to device="cpu" (eden_pipeline.py:738,834).
    This package only has the gfx950 path, so "cpu"/None select the current
    GPU; "cuda:N" selects GPU N.  No GPU -> CodecError (no CPU fallback).
    """
    if not torch.cuda.is_available():
        raise _lib.CodecError("openfl_amd Eden codec needs a ROCm GPU (no CPU fallback)")
    if device is None or str(device) == "cpu":
        return torch.device("cuda", torch.cuda.current_device())
    d = torch.device(device)
    if d.type != "cuda":
        raise _lib.CodecError(f"unsupported device {device!r}")
    return d if d.index is not None else torch.device("cuda", torch.cuda.current_device())


def resolve_devices(device):
    """A plugin `device` setting -> the list of ROCm devices it names.

    One device: "cpu" / None / "cuda" (the current GPU, as torch and the
    reference mean it), "cuda:N".  Several (calls from different threads
    spread over them, ThreadDevices): "cuda:all" (every visible GPU),
    "cuda:0,cuda:2" or a list / tuple of single-device settings -- only ever
    named explicitly, so a process-per-GPU deployment that calls
    torch.cuda.set_device(k) and passes "cuda" stays on GPU k.  The reference
    has one device per pipeline (eden_pipeline.py:738); its callers reach
    several GPUs only through the gRPC server's concurrent worker threads
    (transport/grpc/aggregator_server.py:305, component/aggregator/
    aggregator.py:643-646), which is what the per-thread mapping serves."""
    if isinstance(device, (list, tuple)):
        devs = [resolve_device(d) for d in device]
    elif isinstance(device, str) and "," in device:
        devs = [resolve_device(d.strip()) for d in device.split(",") if d.strip()]
    elif isinstance(device, str) and device.strip() == "cuda:all":
        if not torch.cuda.is_available():
            raise _lib.CodecError("openfl_amd codecs need a ROCm GPU (no CPU fallback)")
        devs = [torch.device("cuda", i) for i in range(torch.cuda.device_count())]
    else:
        devs = [resolve_device(device)]
    if not devs:
        raise _lib.CodecError(f"device setting {device!r} names no GPU")
    return devs


class ThreadDevices:
    """Which of a plugin's devices a calling thread uses: the first call from
    a thread takes the next slot round-robin, and the thread keeps it (its
    streams, staging and device buffers are thread-local too).  Pure Python:
    no device is touched here."""

    def __init__(self, n):
        if n < 1:
            raise ValueError("ThreadDevices needs at least one device")
        self.n = int(n)
        self._tls = threading.local()
        self._next = 0
        self._lock = threading.Lock()

    def slot(self):
        s = getattr(self._tls, "slot", None)
        if s is None:
            with self._lock:
                s = self._next % self.n
                self._next += 1
            self._tls.slot = s
        return s


class PerThreadDevice:
    """Mixin: `self.device` is the calling thread's device among
    `self.devices` (set up by _init_devices from a plugin device setting)."""

    def _init_devices(self, device, share=None):
        """share: another PerThreadDevice whose thread -> device mapping this
        one follows (the transformers of one pipeline stay on one GPU per
        thread)."""
        if share is not None:
            self.devices, self._thread_devices = share.devices, share._thread_devices
            return
        self.devices = resolve_devices(device)
        self._thread_devices = ThreadDevices(len(self.devices))

    @property
    def device(self):
        return self.devices[self._thread_devices.slot()]


class EdenCodec:
    """Batch Eden codec on one device with a plan cache.

    encode(list of fp32 device tensors, seeds) -> (planes u8, scales f32, plan)
    decode(planes, scales, seeds, plan) -> fp32 arena (slice per tensor with plan).
    """

    def __init__(self, n_bits=8, device=None, max_plans=256):
        if n_bits not in (1, 2, 3, 4, 5, 6, 7, 8):
            raise Exception("nbits value is not supported")  # eden_pipeline.py:389-390
        self.n_bits = int(n_bits)
        self.device = resolve_device(device)
        self._plans = {}
        self._order = []
        self._max = max_plans
        self._lock = threading.Lock()
        self.ws = Workspace()

    def plan(self, numels, dims=None, streams=None):
        """Cached plan of a batch shape.  streams: the large-slice schedule's
        stream count (None: the library default, two)."""
        key = (tuple(int(n) for n in numels), None if dims is None else tuple(tuple(d) for d in dims), streams)
        with self._lock:
            p = self._plans.get(key)
            if p is None:
                p = EdenPlan(key[0], self.n_bits, dims=None if dims is None else [list(d) for d in key[1]],
                             streams=streams)
                self._plans[key] = p
                self._order.append(key)
                if len(self._order) > self._max:
                    self._plans.pop(self._order.pop(0), None)
            return p

    def seeds_tensor(self, seeds):
        return torch.tensor([int(s) for s in seeds], dtype=torch.int32).to(self.device, non_blocking=True)

    def encode_arena(self, plan, x_arena, seeds_dev, stream=None):
        planes = torch.empty(max(plan.planes_bytes, 1), dtype=torch.uint8, device=self.device)
        scales = torch.empty(max(plan.n_slices, 1), dtype=torch.float32, device=self.device)
        ws = self.ws.get(plan.ws_bytes, self.device)
        plan.encode(x_arena, seeds_dev, planes, scales, ws, stream)
        return planes, scales

    def decode_arena(self, plan, planes, scales, seeds_dev, stream=None, out=None):
        y = out if out is not None else torch.empty(max(plan.arena_numel, 1), dtype=torch.float32,
                                                    device=self.device)
        ws = self.ws.get(plan.ws_bytes, self.device)
        plan.decode(planes, seeds_dev, scales, y, ws, stream)
        return y
