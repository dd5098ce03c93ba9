import os, sys
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from openfl_amd.codec import EdenPlan, EdenCodec
DEV = torch.device("cuda", 0)
T = int(sys.argv[1]) if len(sys.argv) > 1 else 1100
numels = [65536 + (t % 5) for t in range(T)]
plan = EdenPlan(numels, 8)
g = torch.Generator(device=DEV).manual_seed(3)
arena = torch.empty(plan.arena_numel, device=DEV).normal_(0, 0.01, generator=g)
seeds = [(7 * t + 1) % 65536 for t in range(T)]
c = EdenCodec(8, "cuda:0")
sd = torch.tensor(seeds, dtype=torch.int32, device=DEV)
planes, scales = c.encode_arena(plan, arena, sd)
torch.cuda.synchronize()
planes = planes.cpu().numpy(); scales = scales.cpu().numpy()
bad = []
for t in range(T):
    off, n = plan.elem_offsets[t], numels[t]
    p1 = EdenPlan([n], 8)
    x = arena[off:off + n].contiguous()
    pp, ss = c.encode_arena(p1, x, sd[t:t+1])
    pp = pp[:p1.planes_bytes].cpu().numpy()
    po, pb = plan.planes_offsets[t], plan.planes_nbytes[t]
    if not np.array_equal(planes[po:po + pb], pp):
        bad.append(t)
        if len(bad) <= 3:
            a_, b_ = planes[po:po + pb], pp
            nz = int(np.count_nonzero(a_)), int(np.count_nonzero(b_))
            fs = plan.first_slice[t]
            print("  t", t, "mismatch bytes", int((a_ != b_).sum()), "of", pb, "nonzero batched/single", nz,
                  "scales", scales[fs:fs + len(plan.dims[t])], ss[:len(plan.dims[t])].cpu().numpy())
print("lib", os.environ.get("OFL_CODEC_LIB", "base"), "T", T, "bad", len(bad), bad[:20], bad[-5:])
