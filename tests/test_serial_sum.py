"""The reference seed's serial float32 sum (eden_pipeline.py:771,
`sum(data.flatten())`) evaluated exactly on several threads
(csrc/serial_sum.cpp): bit-identical to the left-to-right chain on inputs that
stress every branch -- ties at the sum's last bit, binade crossings, zeros,
subnormals, huge ranges, Inf / NaN, ragged tails."""

import numpy as np
import pytest

from openfl_amd import _lib


def _serial(x):
    """The chain itself: NumPy's cumsum is a sequential float32 loop."""
    return np.cumsum(x, dtype=np.float32)[-1] if x.size else np.float32(0)


def _cases():
    rng = np.random.default_rng(5)
    n = 1 << 20
    idx = np.arange(n)
    return {
        "update N(0,.01)": (rng.standard_normal(n) * 0.01).astype(np.float32),
        "biased N(.001,.01)": (rng.standard_normal(n) * 0.01 + 0.001).astype(np.float32),
        "N(0,1)": rng.standard_normal(n).astype(np.float32),
        "ties (k / 1024)": (rng.integers(-512, 512, n) / 1024).astype(np.float32),
        "small ints": rng.integers(-3, 4, n).astype(np.float32),
        "huge range": (rng.standard_normal(n) * 10.0 ** rng.integers(-30, 30, n)).astype(np.float32),
        "zeros": np.zeros(n, np.float32),
        "subnormal": (rng.standard_normal(n) * 1e-42).astype(np.float32),
        "ones (saturates at 2^24)": np.ones(1 << 25, np.float32),
        "two chunks N(.002,.01)": (rng.standard_normal((1 << 24) + 777_777) * 0.01 + 0.002).astype(np.float32),
        "alternating big/small": (np.where(idx % 2 == 0, 1e8, 1e-3) * np.where(idx % 4 < 2, 1, -1)).astype(np.float32),
        "nan": np.where(idx == 500_000, np.nan, rng.standard_normal(n)).astype(np.float32),
        "inf": np.where(idx == 7777, np.inf, rng.standard_normal(n)).astype(np.float32),
        "inf - inf": np.where(idx == 10, np.inf, np.where(idx == 99_999, -np.inf, 1.0)).astype(np.float32),
        "ragged": (rng.standard_normal(1_234_567) * 0.01).astype(np.float32),
        "short": (rng.standard_normal(300) * 0.01).astype(np.float32),
        # the multi-run phase B: partial sums crossing binades inside sub-chunks
        "ramp N(.05,.001) (crossings mid sub-chunk)": (rng.standard_normal(n) * 0.001 + 0.05).astype(np.float32),
        "ramp down through zero": (0.5 - idx * (1.0 / n) + rng.standard_normal(n) * 1e-4).astype(np.float32),
        "ties walk (k / 8)": (rng.integers(-8, 9, n) / 8 + 0.125).astype(np.float32),
    }


def _same(a, b):
    return (np.isnan(a) and np.isnan(b)) or np.float32(a).tobytes() == np.float32(b).tobytes()


@pytest.mark.parametrize("name", list(_cases().keys()))
def test_mt_sum_bit_identical(name):
    x = _cases()[name]
    assert x.dtype == np.float32
    L = _lib.lib()
    want = _serial(x)
    for threads in (1, 2, 8, 16):
        dst = np.empty_like(x)
        got = L.ofl_serial_sum_f32_mt(x.ctypes.data, x.size, dst.ctypes.data, threads)
        assert _same(got, want), (name, threads, got, want)
        assert np.array_equal(dst, x, equal_nan=True)
    assert _same(L.ofl_serial_sum_f32(x.ctypes.data, x.size), want)
    dst = np.empty_like(x)
    assert _same(L.ofl_serial_sum_copy_f32(x.ctypes.data, dst.ctypes.data, x.size), want)
    assert np.array_equal(dst, x, equal_nan=True)


def test_matches_python_sum_of_reference():
    """The reference's own expression on a small array: builtin sum over
    NumPy float32 scalars, starting from int 0."""
    x = (np.random.default_rng(9).standard_normal(70_000) * 0.01).astype(np.float32)
    want = sum(x.flatten())
    assert isinstance(want, np.float32)
    assert _same(_lib.lib().ofl_serial_sum_f32_mt(x.ctypes.data, x.size, None, 8), want)


def test_sums_many_with_a_huge_array():
    """ofl_serial_sums_many sends arrays >= 2^22 through the threaded chain."""
    rng = np.random.default_rng(3)
    arrs = [(rng.standard_normal(n) * 0.01).astype(np.float32) for n in (1 << 22, 5000, 1 << 17, 3)]
    ptrs = np.asarray([a.ctypes.data for a in arrs], np.uint64)
    lens = np.asarray([a.size for a in arrs], np.int64)
    out = np.zeros(len(arrs), np.float64)
    _lib.check(_lib.lib().ofl_serial_sums_many(len(arrs), ptrs.ctypes.data, lens.ctypes.data, 0, out.ctypes.data, 8))
    for a, v in zip(arrs, out):
        assert _same(np.float32(v), _serial(a))


def test_concurrent_callers():
    """A caller that finds the thread pool busy runs the plain chain: results
    do not depend on the interleaving."""
    from concurrent.futures import ThreadPoolExecutor
    rng = np.random.default_rng(4)
    arrs = [(rng.standard_normal(1 << 18) * 0.01 + 0.01 * i).astype(np.float32) for i in range(12)]
    L = _lib.lib()
    with ThreadPoolExecutor(6) as ex:
        got = list(ex.map(lambda a: L.ofl_serial_sum_f32_mt(a.ctypes.data, a.size, None, 4), arrs))
    for a, g in zip(arrs, got):
        assert _same(g, _serial(a))


def test_forked_child_does_not_deadlock():
    """A fork()ed child inherits the pool's state but none of its threads:
    its threaded sums run serially instead of waiting for workers that do
    not exist (csrc/serial_sum.cpp Pool, pid recorded at creation)."""
    import os
    x = (np.random.default_rng(6).standard_normal(1 << 21) * 0.01).astype(np.float32)
    L = _lib.lib()
    want = _serial(x)
    assert _same(L.ofl_serial_sum_f32_mt(x.ctypes.data, x.size, None, 8), want)  # the pool exists now
    pid = os.fork()
    if pid == 0:  # child: exit status says whether the sum was right
        try:
            ok = _same(L.ofl_serial_sum_f32_mt(x.ctypes.data, x.size, None, 8), want)
        finally:
            os._exit(0 if ok else 3)
    import time
    t0 = time.monotonic()
    while time.monotonic() - t0 < 60:
        done, status = os.waitpid(pid, os.WNOHANG)
        if done:
            assert os.WEXITSTATUS(status) == 0
            return
        time.sleep(0.05)
    os.kill(pid, 9)
    os.waitpid(pid, 0)
    raise AssertionError("threaded sum in a forked child hung")
