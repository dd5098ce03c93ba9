"""ctypes front-end of the C oracle (oracle/eden_oracle.c).

TEST INFRASTRUCTURE ONLY -- see oracle/__init__.py.  Restates
/root/reference/openfl/pipelines/eden_pipeline.py (per-function citations in
eden_oracle.c).  Tables (centroids/boundaries, eden_pipeline.py:76-380) are
taken from the golden fixture that make_golden.py captured from the reference.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libeden_oracle.so")
_GOLDEN = os.path.join(os.path.dirname(_HERE), "tests", "golden", "eden_golden.npz")
_lib = None
_tables = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        i64, i32, vp = ctypes.c_int64, ctypes.c_int, ctypes.c_void_p
        L.oracle_rand_signs.argtypes = [i64, i64, vp]
        L.oracle_fwht.argtypes = [vp, i64]
        L.oracle_slice_plan.argtypes = [i64, vp, vp, i32]
        L.oracle_slice_plan.restype = i32
        L.oracle_eden_compress.argtypes = [vp, i64, i64, i32, vp, vp, vp, vp, vp, i32]
        L.oracle_eden_compress.restype = i32
        L.oracle_eden_decompress.argtypes = [vp, i64, vp, vp, i32, i64, i32, vp, vp]
        L.oracle_serial_sum_f32.argtypes = [vp, i64]
        L.oracle_serial_sum_f32.restype = ctypes.c_float
        L.oracle_serial_sum_f64.argtypes = [vp, i64]
        L.oracle_serial_sum_f64.restype = ctypes.c_double
        L.oracle_set_threads.argtypes = [i32]
        L.oracle_get_threads.restype = i32
        _lib = L
    return _lib


def host_cores():
    """Host cores this process may use: the affinity mask, capped by
    OMP_NUM_THREADS when set (the GPU box exports the job's CPU share there)."""
    n = len(os.sched_getaffinity(0))
    env = os.environ.get("OMP_NUM_THREADS", "")
    if env.isdigit() and int(env) > 0:
        n = min(n, int(env))
    return max(1, n)


def set_threads(n):
    """OpenMP threads of the oracle's loops (results do not depend on it)."""
    lib().oracle_set_threads(int(n))


def get_threads():
    return int(lib().oracle_get_threads())


def tables(nbits):
    """(centroids, boundaries) float32 for nbits (reference data)."""
    global _tables
    if _tables is None:
        g = np.load(_GOLDEN)
        _tables = {b: (g[f"centroids_b{b}"].astype(np.float32), g[f"boundaries_b{b}"].astype(np.float32))
                   for b in range(1, 9)}
    return _tables[nbits]


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def rand_signs(P, seed):
    """Packed sign bits of rand_diag(P, seed): bit i = 1 <=> +1."""
    out = np.zeros((P + 7) // 8, np.uint8)
    lib().oracle_rand_signs(P, seed, _p(out))
    return out


def rand_diag(P, seed):
    bits = np.unpackbits(rand_signs(P, seed), bitorder="little")[:P]
    return np.where(bits == 1, 1.0, -1.0).astype(np.float32)


def fwht(v):
    v = np.ascontiguousarray(v, np.float32).copy()
    lib().oracle_fwht(_p(v), v.size)
    return v


def slice_plan(n):
    Ps = np.zeros(64, np.int64)
    Ls = np.zeros(64, np.int64)
    ns = lib().oracle_slice_plan(n, _p(Ps), _p(Ls), 64)
    return [int(p) for p in Ps[:ns]], [int(l) for l in Ls[:ns]]


def compress(x, seed, nbits):
    """Eden.compress -> (planes uint8, scales list[float], dims list[int], total_dim)."""
    x = np.ascontiguousarray(np.asarray(x).reshape(-1), np.float32)
    C, B = tables(nbits)
    Ps, _ = slice_plan(x.size)
    Ptot = sum(Ps)
    planes = np.zeros(nbits * Ptot // 8, np.uint8)
    scales = np.zeros(len(Ps), np.float32)
    dims = np.zeros(len(Ps), np.int64)
    ns = lib().oracle_eden_compress(_p(x), x.size, seed, nbits, _p(C), _p(B), _p(planes),
                                    _p(scales), _p(dims), len(Ps))
    assert ns == len(Ps)
    return planes, [float(s) for s in scales], [int(d) for d in dims], int(x.size)


def decompress(planes, total_dim, scales, dims, seed, nbits):
    planes = np.ascontiguousarray(np.frombuffer(bytes(planes), np.uint8))
    C, _ = tables(nbits)
    sc = np.asarray(scales, np.float32)
    dm = np.asarray(dims, np.int64)
    y = np.zeros(int(total_dim), np.float32)
    lib().oracle_eden_decompress(_p(planes), int(total_dim), _p(sc), _p(dm), len(dm), seed,
                                 nbits, _p(C), _p(y))
    return y


def bins_of(planes, Ptot, nbits):
    """Unpack bit planes (to_bits layout, eden_pipeline.py:661-690) to bins."""
    planes = np.frombuffer(bytes(planes), np.uint8).reshape(nbits, Ptot // 8)
    bits = np.unpackbits(planes, axis=1, bitorder="little").astype(np.int32)
    return (bits << np.arange(nbits, dtype=np.int32)[:, None]).sum(0)


def serial_sum(x):
    x = np.ascontiguousarray(np.asarray(x).reshape(-1))
    if x.dtype == np.float64:
        return np.float64(lib().oracle_serial_sum_f64(_p(x), x.size))
    x = x.astype(np.float32, copy=False)
    return np.float32(lib().oracle_serial_sum_f32(_p(x), x.size))
