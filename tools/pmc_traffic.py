"""HBM traffic of the codec from rocprofv3 counter passes (tools/pmc_run.sh).

Per kernel: mean bytes per dispatch from FETCH_SIZE and WRITE_SIZE (both KiB).
gfx950 correction (/opt/skills/guides/MI355X_MICROARCH.md, HBM section):
FETCH_SIZE counts half the bytes of wide coalesced reads, so read bytes =
2 x FETCH_SIZE x 1024; WRITE_SIZE is exact for 16-B-per-lane streaming stores.
Both count L2->fabric traffic, Infinity-Cache hits included, so this is an
upper bound on DRAM bytes.  Dispatches per codec step = dispatches / (steps +
warmup) of the profiled bench run.

Usage: python tools/pmc_traffic.py PMC_DIR STEPS_PLUS_WARMUP [out.json]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    root, nsteps = sys.argv[1], int(sys.argv[2])
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(root, "pass*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if not any(ns in k for ns in ("ofl::", "lossy::", "gz::")):
                continue
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    kernels = {}
    step = 0.0
    for k, cs in vals.items():
        if "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs:
            continue
        rd = 2.0 * 1024.0 * sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"])
        wr = 1024.0 * sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"])
        per_step = len(cs["FETCH_SIZE"]) / nsteps
        name = k.split("(")[0].replace("void ", "").strip()
        kernels[name] = {"read_bytes_per_dispatch": round(rd), "write_bytes_per_dispatch": round(wr),
                         "dispatches_per_step": round(per_step, 3)}
        step += (rd + wr) * per_step
    out = {"hbm_bytes_per_step": round(step), "kernels": kernels,
           "note": "2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes), gfx950 correction; Infinity-Cache hits included"}
    s = json.dumps(out, indent=1)
    print(s)
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
