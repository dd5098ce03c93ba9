"""Cost of pinning a payload `bytes` in place (hipHostRegister) against the
staged copy: for a 125 MB payload (the KC stream of the 1 GiB set), per
variant the median ms over reps.  H2D: staged (ofl_copy_h2d_staged, 2
threads) vs register + hipMemcpyAsync + unregister, on a resident (filled)
payload.  D2H into a FRESH payload (hostmem.new_payload, pages untouched):
pinned staging + host copy on 8 threads vs register + direct DMA +
unregister.  Prints one JSON line."""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from openfl_amd import _lib, hostmem, lossy  # noqa: E402

N = 125 << 20


def med(f, reps=7):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        f()
        torch.cuda.synchronize()
        ts.append(1e3 * (time.perf_counter() - t0))
    return round(float(np.median(ts)), 3), round(min(ts), 3)


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(0)
    from openfl_amd import numa
    numa.bind_to_device(0)
    hip = ctypes.CDLL("libamdhip64.so.7")  # the runtime torch loaded (same SONAME)
    hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    L = _lib.lib()
    d = torch.empty(N, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    res = {}
    b, addr = hostmem.new_payload(N)
    ctypes.memset(addr, 7, N)   # resident
    res["h2d_staged"] = med(lambda: _lib.check(L.ofl_copy_h2d_staged(d.data_ptr(), addr, N, 2, st)))

    def reg_h2d():
        t0 = time.perf_counter()
        e = hip.hipHostRegister(addr, N, 0)
        t1 = time.perf_counter()
        _lib.check(L.ofl_copy_h2d_async(d.data_ptr(), addr, N, st))
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        e2 = hip.hipHostUnregister(addr)
        t3 = time.perf_counter()
        parts.append((1e3 * (t1 - t0), 1e3 * (t2 - t1), 1e3 * (t3 - t2), int(e), int(e2)))
    parts = []
    res["h2d_register"] = med(reg_h2d)
    res["h2d_register_parts_ms(reg,copy,unreg,rc,rc)"] = parts[-1]
    # D2H into fresh payloads
    src = torch.empty(N, dtype=torch.uint8, device=dev).fill_(3)
    pin = torch.empty(N, dtype=torch.uint8).pin_memory()

    def d2h_staged():
        bb, a2 = hostmem.new_payload(N)
        pin.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        lossy._parallel_copy(a2, pin.data_ptr(), N, 8)
        del bb
    res["d2h_staged_fresh"] = med(d2h_staged)
    parts2 = []

    def d2h_register():
        bb, a2 = hostmem.new_payload(N)
        t0 = time.perf_counter()
        e = hip.hipHostRegister(a2, N, 0)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        e3 = hip.hipMemcpyAsync(a2, src.data_ptr(), N, 2, st)  # hipMemcpyDeviceToHost
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        e2 = hip.hipHostUnregister(a2)
        t3 = time.perf_counter()
        parts2.append((1e3 * (t1 - t0), 1e3 * (t2 - t1), 1e3 * (t3 - t2), int(e), int(e2), int(e3)))
        del bb
    try:
        res["d2h_register_fresh"] = med(d2h_register)
        res["d2h_register_parts_ms(reg,copy,unreg,rc,rc,rc)"] = parts2[-1]
    except Exception as ex:  # noqa: BLE001
        res["d2h_register_fresh"] = repr(ex)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
