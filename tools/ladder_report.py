"""Round-6 ladder report from the GPU runs of
tools/r06_ladder.sh, tools/r06_ladder2.sh and tools/r06_mall2.sh:
    python tools/ladder_report.py > profiles/r06_ladder_mall_waves.txt"""
import csv
import glob
import json
import os

G = "gpurun_out"
R = ("lad1", "lad2", "lad3", "full")
NAME = {"lad1": "1 loads+stores", "lad2": "2 +butterflies", "lad3": "3 +signs", "full": "4 full"}


def j(p):
    with open(p) as f:
        return json.load(f)


print("# r06 ladder: the real large-slice kernels at MALL-sized waves, one rung of work at a time")
print("# (-DOFL_LADDER, openfl_amd/csrc/eden_kernels.hip; rungs 1-3 give wrong results and exist only for this):")
print("#   1 = tile loads and stores only (same addresses, layouts, bytes), 2 = + butterflies and LDS exchanges,")
print("#   3 = + sign generation (D1 per-element hashes, the D2 byte table), 4 = the product (+ quantiser / plane")
print("#   pack, centroid unpack, block reductions).  The 1 GiB set (64 x 2^22 slices), bench.py --workload uniform_1gib.")
print()
print("## A. Step time, no per-launch events in the timed region (tools/r06_ladder2.sh), ms per encode+decode step")
print("rung            streams  64 MiB   128 MiB  2 GiB (one wave)")
for l in ("lad1", "full"):
    for s in (1, 2):
        v = [j(f"{G}/r06_ladder2/{l}_s{s}_w{w}.json")["gpu_ms_per_step_rank0"] for w in (64, 128, 2048)]
        print(f"{NAME[l]:15s} {s:7d}  {v[0]:7.3f}  {v[1]:7.3f}  {v[2]:7.3f}")
print("memory-only microbenchmark (tools/dataflow_bench.hip, per-pass launches, p=22): ", end="")
for line in open(f"{G}/r06_ladder2/dataflow_bench.txt"):
    if line.startswith("p=22 base"):
        ms = float(line.split(")")[1].split()[0])
        print(f"{line.split('(')[1].split(')')[0]} {ms / 4 * 2:.3f} ms/step; ", end="")
print("(2 directions x 2^28 of its 2^30 elements)")
print()
print("## B. Kernel durations at 64 MiB waves, one stream (rocprofv3 --kernel-trace --stats, us per launch)")
rows = {}
for l in ("lad1", "full"):
    f = glob.glob(f"{G}/r06_ladder2/prof_{l}_w64/**/*kernel_stats.csv", recursive=True)[0]
    for r in csv.DictReader(open(f)):
        if "ofl::" in r["Name"] and "finalize" not in r["Name"]:
            rows.setdefault(r["Name"].split("(")[0].replace("void ", ""), {})[l] = float(r["AverageNs"]) / 1e3
mv = {"k_enc_rowA2": 8, "k_col6": 8, "k_dec_rowC2": 8, "k_dec_rowA2": 5, "k_enc_rowC2": 5}
print(f"{'kernel':30s} {'rung 1':>8s} {'full':>8s} {'work':>8s}   moved TB/s (rung 1 / full)")
for k, v in rows.items():
    b = next(b for n, b in mv.items() if n in k) * (1 << 24)
    print(f"{k:30s} {v['lad1']:8.2f} {v['full']:8.2f} {v['full'] - v['lad1']:8.2f}   {b / v['lad1'] / 1e6:5.2f} / {b / v['full'] / 1e6:5.2f}")
print()
print("## C. Per-rung kernel times from HIP events around every launch (tools/r06_ladder.sh; the events add")
print("##    ~2-4 us per launch, so compare rungs within a column, not with B), us per launch")
for w in (64, 128, 2048):
    print(f"-- {w} MiB waves" + (" (one wave: the persistent row kernels)" if w == 2048 else " (two-blocks-per-CU row kernels)"))
    tab = {}
    for l in R:
        for k, v in j(f"{G}/r06_ladder/{l}_w{w}.json")["roofline"]["kernels"].items():
            if "finalize" not in k:
                tab.setdefault(k.replace("ofl::", ""), {})[l] = v["avg_us"]
    print(f"   {'kernel':26s}" + "".join(f"{NAME[l]:>16s}" for l in R))
    for k, v in tab.items():
        print(f"   {k:26s}" + "".join(f"{v.get(l, 0):16.1f}" for l in R))
print()
print("## D. SQ counters per rung, 64 MiB waves, one stream (rocprofv3 --pmc, 2 passes per rung; means per dispatch;")
print("##    profiles/r06_ladder/sq_<rung>_w64.json).  waves/SIMD = SQ_WAVE_CYCLES x 4 / (SQ_BUSY_CYCLES / 32) / 1024")
print(f"   {'kernel':26s} {'rung':>5s} {'VALU inst':>10s} {'LDS inst':>9s} {'LDS confl':>10s} {'SALU':>9s} {'waves/SIMD':>10s} {'wait any / wave cyc':>20s}")
for k0 in ("k_enc_rowA2", "k_col6", "k_enc_rowC2", "k_dec_rowA2", "k_dec_rowC2"):
    for l in R:
        d = j(f"profiles/r06_ladder/sq_{l}_w64.json")
        k = next(n for n in d if k0 in n)
        m = d[k]
        wps = m["SQ_WAVE_CYCLES"] * 4 / (m["SQ_BUSY_CYCLES"] / 32) / 1024
        print(f"   {k0:26s} {l:>5s} {m['SQ_INSTS_VALU']:10.3g} {m['SQ_INSTS_LDS']:9.3g} {m['SQ_LDS_BANK_CONFLICT']:10.3g} "
              f"{m['SQ_INSTS_SALU']:9.3g} {wps:10.2f} {m['SQ_WAIT_ANY'] / m['SQ_WAVE_CYCLES']:20.2f}")
print()
print("## E. Reorderings at MALL waves, product kernels, no events (tools/r06_mall2.sh, ms per step, two runs)")
for line in open(f"{G}/r06_mall2.txt"):
    if line.startswith("u_"):
        t = line.split()
        print(f"   {t[0]:22s} {t[3]} ms  ({t[1]} GiB/s)")
print("   (r20 = persistent one-block-per-CU row kernels with register prefetch, r21 = two-blocks-per-CU row kernels;")
print("    default = one 1 GiB wave on the caller's stream)")
print()
print("## F. The sign work's share at MALL waves (tools/r06_signs_bound.sh: the product with the D1/D2 sign")
print("##    generation compiled out, -DOFL_LADDER=5, wrong results) and one way to cut it (tools/r06_sgn_ab.sh:")
print("##    D1 sign bitmaps from a k_signs launch per wave, one hash per 8 elements, read by the two-blocks-per-CU")
print("##    row kernels; patch tools/ab/r06_sign_bitmaps.patch, bit-exact: tests/test_gpu_parity.py 290 passed)")
for f in ("r06_signs.txt", "r06_sgn.txt"):
    for line in open(f"{G}/{f}"):
        if line.startswith(("u ", "rn ")):
            print("   " + line.rstrip())
print("   (u = 1 GiB set, two streams, ms per step last; rn = ResNet-50; full = product, lad5 = no sign work;")
print("    sgn=1 bitmaps, sgn=0 per-element hashes = the product.  The bitmaps lose: their extra launch per wave")
print("    and direction costs more than the hashes they save; reverted.  Written instead by blocks appended to an")
print("    earlier row launch of the same stream, they lose too: profiles/r06_sign_bitmaps_fused_ab.txt.)")
print()
print("## G. Narrower intermediates, memory-pattern stubs on the Llama step (VERDICT r05 item 3; tools/r06_ladder2.sh:")
print("##    -DOFL_WS_FMT=16 the high 16 bits of each fp32, =24 split planes hi-16 + lo-8; wrong results)")
for line in open(f"{G}/r06_ladder2.txt"):
    if line.startswith("llama"):
        t = line.split()
        print(f"   {t[1]:5s} run {t[2]}: {t[3]} GiB/s, {t[4]} ms/step; " + " ".join(line.split("[")[1].split("), ")[:4]))
