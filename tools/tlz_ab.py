"""TLZ encoder A/B: the streams' sha256, sizes and gzip.decompress check on
fixed rank sets, and the KC pipeline's phases, for the library in
OFL_CODEC_LIB (default: the in-tree build).  Two runs (base / new library)
print comparable JSON lines:
    OFL_CODEC_LIB=tools/bin/var/libofl_codec_gzbase.so python tools/tlz_ab.py base
    python tools/tlz_ab.py new
"""
import gzip
import hashlib
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openfl_amd import lossy  # noqa: E402
from tools.tlz_check import cases, kc_like  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "run"
dev = "cuda:0"
out = {"tag": tag, "lib": os.environ.get("OFL_CODEC_LIB", "in-tree"), "streams": {}}
allcases = list(cases()) + [("kc6_2p26", kc_like(1 << 26, 4))]
for name, x in allcases:
    xd = torch.from_numpy(x).to(dev)
    z = lossy.gzip_ranks(xd)
    ok = gzip.decompress(z) == x.tobytes()
    out["streams"][name] = {"bytes": len(z), "ratio": round(len(z) / max(1, x.nbytes), 5),
                            "sha256": hashlib.sha256(z).hexdigest()[:16], "ok": ok}
# time of the encode of the 2^26-value set (16 launches' worth averaged)
xd = torch.from_numpy(allcases[-1][1]).to(dev)
for _ in range(2):
    lossy.gzip_ranks(xd)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(5):
    lossy.gzip_ranks(xd)
out["gzip_2p26_ms"] = round(1e3 * (time.perf_counter() - t0) / 5, 3)
print(json.dumps(out), flush=True)
