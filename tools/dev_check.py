"""Dev check: GPU Eden encode/decode vs the CPU oracle over every kernel class."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from oracle import eden as O
from openfl_amd.codec import EdenCodec

def stats(n, b, seed=1234):
    x = (np.random.default_rng(n).standard_normal(n).astype(np.float32) * np.float32(0.01))
    codec = EdenCodec(b, "cuda:0")
    plan = codec.plan([n])
    xd = torch.from_numpy(x).cuda()
    sd = torch.tensor([seed], dtype=torch.int32).cuda()
    planes, scales = codec.encode_arena(plan, xd, sd)
    y = codec.decode_arena(plan, planes, scales, sd)
    torch.cuda.synchronize()
    planes_h = planes[:plan.planes_bytes].cpu().numpy(); sc = scales[:plan.n_slices].cpu().numpy()
    yg = y[:n].cpu().numpy()
    op, osc, odims, _ = O.compress(x, seed, b)
    assert odims == plan.dims[0], (odims, plan.dims[0])
    Ptot = sum(odims)
    gb = O.bins_of(planes_h, Ptot, b); ob = O.bins_of(op, Ptot, b)
    mis = (gb != ob).mean(); maxd = np.abs(gb - ob).max()
    screl = np.max(np.abs(sc - np.array(osc)) / np.maximum(np.abs(osc), 1e-30))
    # decode parity on the SAME bytes: GPU decode of oracle planes vs oracle decode
    yo = O.decompress(op, n, osc, odims, seed, b)
    plan2 = codec.plan([n], dims=[odims])
    y2 = codec.decode_arena(plan2, torch.from_numpy(op).cuda(), torch.tensor(np.array(osc, np.float32)).cuda(), sd)
    y2 = y2[:n].cpu().numpy()
    drel = np.linalg.norm(y2 - yo) / max(np.linalg.norm(yo), 1e-30)
    err = np.linalg.norm(yg - x) / np.linalg.norm(x)
    print(f"n={n:9d} b={b} dims={odims[:4]} binmis={mis:.2e} maxd={maxd} screl={screl:.1e} dec_rel={drel:.1e} e2e_rel={err:.2e}", flush=True)
    return mis, maxd, drel

sizes = [int(a) for a in sys.argv[1:]] or [1, 7, 100, 300, 1000, 2048, 3000, 4096, 8192, 16384, 16385,
         32768, 65536, 1 << 17, 1 << 18, 1 << 19, 1 << 20, 1 << 21, 1 << 22, 1 << 23, (1 << 24) + 12345]
bad = 0
for n in sizes:
    for b in (8, 3):
        mis, maxd, drel = stats(n, b)
        if mis > 2e-3 or maxd > 1 or drel > 2e-6: bad += 1; print("  ^^^ FAIL")
print("FAILURES", bad)
sys.exit(1 if bad else 0)
