"""The aggregator's end-of-round tensor work on the device.

Reference (paths relative to /root/reference/openfl):
  interface/aggregation_functions/weighted_average.py:12-58
      WeightedAverage.call -> np.average(tensors, weights=weights, axis=0)
  component/aggregator/aggregator.py:780-865  _prepare_trained, per tensor:
      agg = WeightedAverage(local tensors)            (float64)
      delta = TensorCodec.generate_delta(agg, base)   (agg - base, float64)
      payload, md = TensorCodec.compress(delta)       (the compression pipeline)
      dec = TensorCodec.decompress(payload, md)       (float32)
      model = TensorCodec.apply_delta(dec, base)      (base + dec, float32)
  pipelines/tensor_codec.py:150-211  generate_delta / apply_delta

RoundEnd does that for every tensor of a model update in one device pass
sequence over flat arenas (csrc/agg_kernels.hip + the Eden plan): average +
delta in one kernel (float64 arithmetic in NumPy's order, delta rounded to
float32 as Eden.compress does), the seeds' serial sums from the delta's values
summed on the device (fast mode: a 4096-element prefix per tensor, reference
mode: all of it, one lane per tensor in Python's left-to-right order) and
hashed there with CPython's float hash (no host round trip), one
Eden encode and decode of all the big tensors, and apply_delta in place.  The
payloads, metadata, np.random draws and new model are identical to calling
the reference's functions tensor by tensor with an openfl_amd EdenPipeline
(tests/test_gpu_aggregation.py).  No CPU fallback: without the library or a
GPU every call raises CodecError.
"""
import numpy as np
import torch

from openfl_amd import _lib, hostmem
from openfl_amd.codec import EdenPlan, resolve_device, slice_plan
from openfl_amd.pipelines.eden_pipeline import _FAST_SEED_PREFIX

_ALIGN = 64
_ROW_TILE = 1 << 15  # slices above this go through the row passes (kRowLog)


def _stream(device):
    return torch.cuda.current_stream(device).cuda_stream


def _f64_weights(weights, n):
    w = np.asarray(weights)
    if w.ndim != 1 or w.size != n:
        raise _lib.CodecError("one weight per collaborator tensor")
    if np.result_type(np.float32, w.dtype) != np.float64:
        raise _lib.CodecError("weights must promote float32 tensors to float64 (np.average result dtype)")
    return np.ascontiguousarray(w, np.float64)


def weight_sum(weights, ndim):
    """np.average's denominator for tensors of `ndim` dimensions: NumPy's own
    float64 sum of the broadcast weights (weighted_average.py:14)."""
    w = np.asarray(weights)
    stack = np.zeros((w.size,) + (1,) * ndim, np.float32)
    scl = np.average(stack, weights=w, axis=0, returned=True)[1]
    return float(np.asarray(scl).reshape(-1)[0])


def _wavg_launch(xs, w64, wsum, base, n, agg=None, delta64=None, delta32=None, device=None):
    ptrs = np.asarray([x.data_ptr() for x in xs], np.uint64)
    _lib.check_agg(_lib.lib().ofl_wavg_delta(
        len(xs), ptrs.ctypes.data, w64.ctypes.data, wsum, base.data_ptr() if base is not None else None, int(n),
        agg.data_ptr() if agg is not None else None, delta64.data_ptr() if delta64 is not None else None,
        delta32.data_ptr() if delta32 is not None else None, _stream(device)))


def _points_launch(xs, w64, wsum, base, idx, agg, delta32, device, ws):
    ptrs = np.asarray([x.data_ptr() for x in xs], np.uint64)
    ix = np.ascontiguousarray(idx, np.int64)
    L = _lib.lib()
    need = int(L.ofl_wavg_points_workspace_bytes(len(xs), ix.size))
    buf = ws(need)
    _lib.check_agg(L.ofl_wavg_delta_points(
        len(xs), ptrs.ctypes.data, w64.ctypes.data, wsum, base.data_ptr() if base is not None else None, ix.size,
        ix.ctypes.data, agg.data_ptr() if agg is not None else None, None,
        delta32.data_ptr() if delta32 is not None else None, buf.data_ptr(), buf.numel(), _stream(device)))


class _Scratch:
    def __init__(self, device):
        self.device = device
        self.buf = None

    def __call__(self, nbytes):
        if self.buf is None or self.buf.numel() < nbytes:
            self.buf = torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=self.device)
        return self.buf


def weighted_average(tensors, weights, device=None):
    """np.average(tensors, weights=weights, axis=0) on the GPU
    (weighted_average.py:12-14): float32 tensors, float64 result, bit-exact."""
    dev = resolve_device(device)
    arrs = [np.asarray(t) for t in tensors]
    if not arrs:
        raise _lib.CodecError("weighted_average: no tensors")
    shape = arrs[0].shape
    if any(a.shape != shape or a.dtype != np.float32 for a in arrs):
        raise _lib.CodecError("weighted_average: float32 tensors of one shape")
    w64 = _f64_weights(weights, len(arrs))
    wsum = weight_sum(w64, len(shape))
    if wsum == 0.0:
        raise ZeroDivisionError("Weights sum to zero, can't be normalized")
    n = int(np.prod(shape, dtype=np.int64))
    with torch.cuda.device(dev):
        xs = [torch.from_numpy(np.ascontiguousarray(a).reshape(-1)).to(dev) for a in arrs]
        agg = torch.empty(max(n, 1), dtype=torch.float64, device=dev)
        if n == 1:
            _points_launch(xs, w64, wsum, None, [0], agg, None, dev, _Scratch(dev))
        elif n:
            _wavg_launch(xs, w64, wsum, None, n, agg=agg, device=dev)
        return agg[:n].cpu().numpy().reshape(shape)


class WeightedAverage:
    """AggregationFunction plugin (weighted_average.py:17-58): call(local_tensors, ...)
    -> np.average of the LocalTensor tensors by their weights, on the GPU."""

    def __init__(self, device=None):
        self.device = device

    def call(self, local_tensors, *_):
        tensors, weights = zip(*[(x.tensor, x.weight) for x in local_tensors])
        return weighted_average(tensors, weights, self.device)

    def __call__(self, local_tensors, *args):
        return self.call(local_tensors, *args)


class RoundEnd:
    """Aggregator._prepare_trained for a whole model update (aggregator.py:780-865).

    pipeline: an openfl_amd EdenPipeline (its n_bits, dim_threshold and
    seed_mode apply); shapes: the model's tensor shapes in the aggregator's
    order.  Tensors live in flat float32 arenas, tensor i at offsets[i]
    (64-element aligned); arena() / pack() / view() make and read them.
    fused (default): without agg_out and with at most 16 collaborators the
    large slices' first encode pass computes the delta from the collaborator
    arenas itself (ofl_eden_encode_wavg) instead of reading a delta arena
    the averaging kernel wrote -- same bytes, 8 B/element less HBM traffic.
    """

    def __init__(self, pipeline, shapes, device=None, fused=True):
        tr = pipeline.transformers[0]
        self.transformer = tr
        self.device = resolve_device(device) if device is not None else tr.eden.device
        self.dim_threshold = tr.dim_threshold
        self.seed_mode = tr.seed_mode
        self.n_bits = tr.eden.nbits
        self.shapes = [tuple(int(d) for d in s) for s in shapes]
        self.numels = [int(np.prod(s, dtype=np.int64)) for s in self.shapes]
        self.offsets, acc = [], 0
        for n in self.numels:
            self.offsets.append(acc)
            acc += (n + _ALIGN - 1) // _ALIGN * _ALIGN
        self.arena_numel = max(acc, 1)
        # the alignment padding between tensors (and the arena's tail): zeroed
        # in every output arena, so it is the same whichever path ran
        gaps = [np.arange(o + n, o + (n + _ALIGN - 1) // _ALIGN * _ALIGN) for o, n in zip(self.offsets, self.numels)]
        gaps.append(np.arange(acc, self.arena_numel))
        gap_idx = np.concatenate(gaps).astype(np.int64) if gaps else np.zeros(0, np.int64)
        self._gap_idx = torch.from_numpy(gap_idx).to(self.device) if gap_idx.size else None
        self.big = [i for i, n in enumerate(self.numels) if n > self.dim_threshold]
        self.single = [i for i, n in enumerate(self.numels) if n == 1]
        self.plan = EdenPlan([self.numels[i] for i in self.big], self.n_bits,
                             elem_offsets=[self.offsets[i] for i in self.big]) if self.big else None
        self._ws = _Scratch(self.device)
        self._codec_ws = None
        # tensors the codec does not touch (small, <= dim_threshold): their
        # apply_delta runs on these ranges (device tables)
        rest = [i for i in range(len(self.numels)) if i not in set(self.big) and self.numels[i] > 0]
        self._rest_n = len(rest)
        self._rest_total = sum(self.numels[i] for i in rest)
        dst = np.cumsum([0] + [self.numels[i] for i in rest]).astype(np.int64)
        self._rest_start = torch.tensor([self.offsets[i] for i in rest] or [0], dtype=torch.int64).to(self.device)
        self._rest_dst = torch.from_numpy(dst).to(self.device)
        # seed ranges (a prefix per tensor in fast mode, all of it in reference
        # mode) as device tables: the seeds are computed without a host round trip
        T = len(self.numels)
        counts = [min(n, _FAST_SEED_PREFIX) if self.seed_mode == "fast" else n for n in self.numels]
        self._seed_total = int(sum(counts))
        self._seed_start = torch.tensor(self.offsets or [0], dtype=torch.int64).to(self.device)
        self._seed_dst = torch.from_numpy(np.cumsum([0] + counts).astype(np.int64)).to(self.device)
        self._seed_single = torch.tensor([1 if n == 1 else 0 for n in self.numels] or [0], dtype=torch.int32).to(self.device)
        self._seed_sums = torch.empty(max(T, 1), dtype=torch.float64, device=self.device)
        self._seeds = torch.empty(max(T, 1), dtype=torch.int32, device=self.device)
        self._packed = torch.empty(max(self._seed_total, 1), dtype=torch.float64, device=self.device)
        self._big_idx = torch.tensor(self.big or [0], dtype=torch.int64).to(self.device)
        # fused round-end encode (ofl_eden_encode_wavg): the large slices' row
        # pass computes the delta from the collaborators' arenas itself, so the
        # delta arena is written only where something else reads it -- the
        # tensors the codec does not touch and the slices of <= 2^15 elements
        self.fused = bool(fused) and self.plan is not None
        fz = [(self.offsets[i], self.numels[i]) for i in rest]
        for t, i in enumerate(self.big):
            _, lens = slice_plan(self.numels[i])
            xo = self.offsets[i]
            for P, ln in zip(self.plan.dims[t], lens):
                if P <= _ROW_TILE and ln > 0:
                    fz.append((xo, ln))
                xo += ln
        fz.sort()
        self._fz_n = len(fz)
        self._fz_total = sum(n for _, n in fz)
        self._fz_start = torch.tensor([o for o, _ in fz] or [0], dtype=torch.int64).to(self.device)
        self._fz_dst = torch.from_numpy(np.cumsum([0] + [n for _, n in fz]).astype(np.int64)).to(self.device)
        self._host_args = None   # pinned [collaborator pointers | weights | draws], reused after _args_done
        self._dev_args = None
        self._args_done = None

    # -- arenas --
    def arena(self):
        return torch.zeros(self.arena_numel, dtype=torch.float32, device=self.device)

    def pack(self, arrays):
        a = self.arena()
        for i, x in enumerate(arrays):
            x = np.asarray(x, np.float32).reshape(-1)
            if x.size != self.numels[i]:
                raise _lib.CodecError(f"tensor {i}: {x.size} elements, expected {self.numels[i]}")
            a[self.offsets[i]:self.offsets[i] + x.size] = torch.from_numpy(x).to(self.device)
        return a

    def view(self, arena, i):
        return arena[self.offsets[i]:self.offsets[i] + self.numels[i]].view(self.shapes[i])

    def _wsum(self, w64):
        sums = {weight_sum(w64, d) for d in {len(s) for s in self.shapes}}
        if len(sums) != 1:
            raise _lib.CodecError("weight sums differ between tensor ranks")
        s = sums.pop()
        if s == 0.0:
            raise ZeroDivisionError("Weights sum to zero, can't be normalized")
        return s

    def run(self, collab_arenas, weights, base_arena=None, agg_out=None, payloads=True, out=None):
        """collab_arenas: one float32 device arena per collaborator (this
        layout); weights: per collaborator; base_arena: the previous model
        (None: no base, the delta is the average).  Writes the new model
        into `out` (default: a new arena; may be base_arena) and, if given,
        the float64 average into agg_out (arena_numel elements).
        -> (new model arena, [(payload bytes, [metadata])] per tensor or None,
        seeds: a list with payloads, else the device int32 tensor -- without
        payloads nothing synchronises with the host)."""
        dev = self.device
        xs = list(collab_arenas)
        for x in xs + ([base_arena] if base_arena is not None else []):
            if not (x.is_cuda and x.dtype == torch.float32 and x.is_contiguous() and x.numel() >= self.arena_numel):
                raise _lib.CodecError("arenas must be contiguous float32 device tensors of arena_numel elements")
        if agg_out is not None and not (agg_out.dtype == torch.float64 and agg_out.numel() >= self.arena_numel):
            raise _lib.CodecError("agg_out must be float64 with arena_numel elements")
        w64 = _f64_weights(weights, len(xs))
        wsum = self._wsum(w64)
        L = _lib.lib()
        fused = self.fused and agg_out is None and len(xs) <= 16
        with torch.cuda.device(dev):
            delta = torch.empty(self.arena_numel, dtype=torch.float32, device=dev)
            if agg_out is None and len(xs) > 16:  # running sums between chained launches
                agg_out = torch.empty(self.arena_numel, dtype=torch.float64, device=dev)
            # 1. average + delta (float64), delta rounded to float32 -- fused:
            # only on the ranges the large slices' encode does not compute
            if fused:
                ptrs = np.asarray([x.data_ptr() for x in xs], np.uint64)
                _lib.check_agg(L.ofl_wavg_delta32_ranges(
                    len(xs), ptrs.ctypes.data, w64.ctypes.data, wsum,
                    base_arena.data_ptr() if base_arena is not None else None, self._fz_n,
                    self._fz_start.data_ptr(), self._fz_dst.data_ptr(), self._fz_total, delta.data_ptr(),
                    _stream(dev)))
            else:
                _wavg_launch(xs, w64, wsum, base_arena, self.arena_numel, agg=agg_out, delta32=delta, device=dev)
            if self.single:
                _points_launch(xs, w64, wsum, base_arena, [self.offsets[i] for i in self.single], agg_out, delta,
                               dev, self._ws)
            # 2. seeds on the device: serial sums of the float64 delta, CPython's
            # float hash, one np.random draw per tensor in order (drawn here)
            T = len(self.numels)
            C = len(xs)
            draws = np.random.randint(1, 2 ** 16, size=T).astype(np.int64) if T else np.zeros(0, np.int64)
            need = 2 * C + max(T, 1)
            if self._host_args is None or self._host_args.numel() < need:
                self._host_args = torch.empty(need, dtype=torch.int64).pin_memory()
                self._dev_args = torch.empty(need, dtype=torch.int64, device=dev)
                self._args_done = torch.cuda.Event()
            else:
                self._args_done.synchronize()  # the previous call's copy has left the pinned buffer
            ha = self._host_args.numpy()
            ha[:C] = np.asarray([x.data_ptr() for x in xs], np.uint64).view(np.int64)
            ha[C:2 * C] = w64.view(np.int64)
            ha[2 * C:2 * C + T] = draws
            self._dev_args[:need].copy_(self._host_args[:need], non_blocking=True)
            self._args_done.record()
            dp = self._dev_args.data_ptr()
            _lib.check_agg(L.ofl_wavg_delta_seeds(
                C, dp, dp + 8 * C, wsum, base_arena.data_ptr() if base_arena is not None else None, T,
                self._seed_start.data_ptr(), self._seed_dst.data_ptr(), self._seed_single.data_ptr(), self._seed_total,
                dp + 16 * C, self._seeds.data_ptr(), self._seed_sums.data_ptr(), self._packed.data_ptr(), _stream(dev)))
            seeds = None
            if payloads:
                seeds = [int(v) for v in self._seeds[:T].cpu().numpy()]
            # 3. encode, (payloads), decode in place, apply
            result = [None] * len(self.numels) if payloads else None
            if self.plan is not None:
                p = self.plan
                sd = self._seeds.index_select(0, self._big_idx)
                planes = torch.empty(max(p.planes_bytes, 1), dtype=torch.uint8, device=dev)
                scales = torch.empty(max(p.n_slices, 1), dtype=torch.float32, device=dev)
                if self._codec_ws is None or self._codec_ws.numel() < p.ws_bytes:
                    self._codec_ws = torch.empty(max(p.ws_bytes, 256), dtype=torch.uint8, device=dev)
                if fused:
                    _lib.check(L.ofl_eden_encode_wavg(
                        p.handle, dp, dp + 8 * C, C, wsum, base_arena.data_ptr() if base_arena is not None else None,
                        delta.data_ptr(), sd.data_ptr(), planes.data_ptr(), scales.data_ptr(),
                        self._codec_ws.data_ptr(), self._codec_ws.numel(), _stream(dev)))
                else:
                    p.encode(delta, sd, planes, scales, self._codec_ws)
                if payloads:
                    pn = planes[:p.planes_bytes].cpu().numpy()
                    sn = scales[:p.n_slices].cpu().numpy()
                    for t, i in enumerate(self.big):
                        po, pb, fs = p.planes_offsets[t], p.planes_nbytes[t], p.first_slice[t]
                        md = {0: float(seeds[i]), 1: float(self.numels[i])}
                        for k, (s, d) in enumerate(zip(sn[fs:fs + len(p.dims[t])], p.dims[t])):
                            md[2 + 2 * k] = float(s)
                            md[3 + 2 * k] = float(d)
                        result[i] = (hostmem.bytes_from(pn.ctypes.data + po, pb), [{"int_list": list(self.shapes[i]), "int_to_float": md}])
                if base_arena is not None:  # decode + apply_delta fused: out = base + decoded
                    if out is None:
                        out = torch.empty(self.arena_numel, dtype=torch.float32, device=dev)
                    p.decode(planes, sd, scales, out, self._codec_ws, base=base_arena)
                else:
                    p.decode(planes, sd, scales, delta, self._codec_ws)
            if payloads:
                small = [i for i in range(len(self.numels)) if result[i] is None]
                if small:  # float32 bytes of the delta (Float32NumpyArrayToBytes), one D2H
                    dh = torch.cat([delta[self.offsets[i]:self.offsets[i] + self.numels[i]] for i in small]).cpu().numpy()
                    o = 0
                    for i in small:
                        result[i] = (hostmem.bytes_from(dh.ctypes.data + 4 * o, 4 * self.numels[i]), [{"int_list": list(self.shapes[i])}])
                        o += self.numels[i]
            if out is None:
                out = torch.empty(self.arena_numel, dtype=torch.float32, device=dev)
            if base_arena is not None:
                if self.plan is not None:
                    _lib.check_agg(L.ofl_apply_delta_ranges(
                        base_arena.data_ptr(), delta.data_ptr(), out.data_ptr(), self._rest_n,
                        self._rest_start.data_ptr(), self._rest_dst.data_ptr(), self._rest_total, _stream(dev)))
                else:
                    _lib.check_agg(L.ofl_apply_delta(base_arena.data_ptr(), delta.data_ptr(), self.arena_numel,
                                                     out.data_ptr(), _stream(dev)))
            else:
                out.copy_(delta)
            if self._gap_idx is not None:
                out.index_fill_(0, self._gap_idx, 0.0)
        return out, result, (seeds if payloads else self._seeds[:len(self.numels)])
