"""OFL_GZ_PHASES=1 python tools/tlz_phases.py: the TLZ encoder's phase times
(block 0 of the first launch) on a KC-like rank set of 2^26 values."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from openfl_amd import lossy  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 26
g = torch.Generator(device="cuda:0").manual_seed(0)
p = torch.tensor([0.074, 0.1816, 0.2444, 0.2444, 0.1816, 0.074], device="cuda:0")
x = torch.multinomial(p, n, replacement=True, generator=g).to(torch.float32)
for _ in range(2):
    z = lossy.gzip_ranks(x)
print("ratio", len(z) / (4 * n))
