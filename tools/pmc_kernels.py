"""Per-kernel mean of every PMC counter per dispatch from rocprofv3
--pmc passes (DIR/pass*/**/*counter_collection.csv), for the kernels whose
name contains one of the given substrings.  Usage:
  python tools/pmc_kernels.py DIR OUT.json substr [substr ...]
SQ_* counters are summed over the shader engines by rocprofv3 already.
Derived (when the inputs are present): valu_busy = SQ_ACTIVE_INST_VALU /
(SQ_BUSY_CYCLES x 4 SIMDs x 32 CUs per SE); waves per SIMD over the
dispatch = SQ_WAVE_CYCLES / SQ_BUSY_CYCLES / 1024 SIMDs x 8 SEs ... is left
to the reader: the raw means are what the JSON records."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root, out = sys.argv[1], sys.argv[2]
subs = sys.argv[3:]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(root, "pass*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if subs and not any(s in k for s in subs):
            continue
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {}
for k, cs in acc.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    m["dispatches"] = max(len(v) for v in cs.values())
    res[k] = m
json.dump(res, open(out, "w"), indent=1, sort_keys=True)
for k, m in sorted(res.items()):
    print(k[:60], " ".join(f"{c}={v:.4g}" for c, v in sorted(m.items())))
