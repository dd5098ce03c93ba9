"""Timeline of the KC decode (lossy.gunzip_device with the fused LUT) on the
1 GiB set: per call, the marks of OFL_GUNZIP_TRACE (member index, each H2D
piece landed, each piece's launch, verdict checked, then synchronize), and
beside it the parts alone: the staged H2D of the payload, the member index,
and the inflate kernels over a payload already in HBM.  Prints JSON."""
import ctypes
import json
import os
import sys
import time

os.environ["OFL_GUNZIP_TRACE"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from openfl_amd import _lib, hostmem, lossy  # noqa: E402
from openfl_amd.workloads import WORKLOADS, numel  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    shapes = WORKLOADS["uniform_1gib"]()
    numels = [numel(s) for _, s in shapes]
    offs = list(np.cumsum([0] + [(n + 63) // 64 * 64 for n in numels[:-1]]))
    tot = offs[-1] + numels[-1]
    x = torch.empty(tot, dtype=torch.float32, device=dev)
    g = torch.Generator(device=dev)
    for j, (o, n) in enumerate(zip(offs, numels)):
        g.manual_seed(j)
        x[o:o + n].normal_(0.0, 0.01, generator=g)
    tab = lossy.LabelTable(len(numels), dev)
    _, _, _, uniq = lossy.kmeans_batch(x, offs, numels, 6, n_init=6, seed=3, label_out=tab)
    z = lossy.gzip_ranks(x, label=tab)
    maps = [{i: u for i, u in enumerate(uq)} for uq in uniq]
    if os.environ.get("PROBE_DUMP"):  # the stream's head, for offline token statistics
        with open(os.environ["PROBE_DUMP"], "wb") as f:
            f.write(z[:1 << 18])
    y = torch.empty_like(x)
    yb = y.view(torch.uint8)
    res = {"payload_bytes": len(z), "calls": [], "configs": {}}
    for pieces in [4, 2, 3, 6, 8, 4]:
        lossy._INFLATE_PIECES = pieces
        ts, gaps = [], []
        for r in range(7):
            lut = lossy.lut_tables(offs, numels, maps, dev)
            torch.cuda.synchronize()
            lossy.gunzip_trace_log.clear()
            t0 = time.perf_counter()
            lossy.gunzip_device(z, yb, lut=lut)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            m = dict(lossy.gunzip_trace_log[0])
            ts.append(1e3 * (t2 - t0))
            gaps.append(1e3 * (t2 - m[f"h2d{pieces - 1}"]))
        res["configs"][f"p{pieces}"] = {"ms_med": round(float(np.median(ts[1:])), 3),
                                                "last_landed_to_synced_med": round(float(np.median(gaps[1:])), 3)}
    lossy._INFLATE_PIECES = 4
    for r in range(10):
        lut = lossy.lut_tables(offs, numels, maps, dev)
        torch.cuda.synchronize()
        lossy.gunzip_trace_log.clear()
        t0 = time.perf_counter()
        lossy.gunzip_device(z, yb, lut=lut)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        marks = lossy.gunzip_trace_log[0]
        c = {k: round(1e3 * (t - t0), 3) for k, t in marks}
        c["returned"] = round(1e3 * (t1 - t0), 3)
        c["synced"] = round(1e3 * (t2 - t0), 3)
        res["calls"].append(c)
    # the parts alone
    L = _lib.lib()
    src = np.frombuffer(z, np.uint8)
    d_in = torch.empty(src.size + 128, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    h = []
    for _ in range(6):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with hostmem.quiet():
            _lib.check(lossy._h2d(L, d_in.data_ptr(), src.ctypes.data, src.size, st))
        torch.cuda.synchronize()
        h.append(1e3 * (time.perf_counter() - t0))
    res["h2d_staged_ms"] = [round(v, 3) for v in h]
    nm, tb, mx, tl = ctypes.c_int64(), ctypes.c_size_t(), ctypes.c_uint32(), ctypes.c_int()
    cap = src.size // 26 + 1
    idx = np.empty((cap, 4), np.int64)
    ti = []
    for _ in range(5):
        t0 = time.perf_counter()
        _lib.check_gzip(L.ofl_gzip_member_index(src.ctypes.data, src.size, idx.ctypes.data, cap, ctypes.byref(nm),
                                                ctypes.byref(tb), ctypes.byref(mx), ctypes.byref(tl)))
        ti.append(1e3 * (time.perf_counter() - t0))
    res["member_index_ms"] = [round(v, 3) for v in ti]
    idx = idx[:nm.value]
    d_idx = torch.from_numpy(idx.view(np.uint8).reshape(-1).copy()).to(dev)
    ws = torch.empty(int(L.ofl_inflate_tlz_workspace_bytes(nm.value)), dtype=torch.uint8, device=dev)
    lut = lossy.lut_tables(offs, numels, maps, dev)
    args = (d_in.data_ptr(), d_idx.data_ptr())
    tail = (yb.data_ptr(), yb.numel(), ws.data_ptr(), ws.numel())
    la = (lut["tab"].data_ptr(), lut["start"].data_ptr(), lut["end"].data_ptr(), lut["n"])
    tk = []
    for _ in range(6):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        _lib.check_gzip(L.ofl_inflate_tlz_async(*args, 0, 0, *tail, st))
        _lib.check_gzip(L.ofl_inflate_tlz_launch_lut(*args, 0, nm.value, *tail, *la, st))
        _lib.check_gzip(L.ofl_inflate_tlz_check(nm.value, ws.data_ptr(), ws.numel(), st))
        torch.cuda.synchronize()
        tk.append(1e3 * (time.perf_counter() - t0))
    res["kernels_resident_ms"] = [round(v, 3) for v in tk]
    res["members"] = nm.value
    print(json.dumps(res))


if __name__ == "__main__":
    main()
