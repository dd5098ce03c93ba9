"""Token statistics of a TLZ gzip stream's first members (offline, no GPU):
per segment of 2048 values the literal / copy counts, the symbols a lane of
k_tlz_ops decodes, and the pointer-jumping rounds k_tlz_resolve needs
(synchronous rounds: an upper bound of the kernel's in-place rounds).
Usage: python tools/tlz_token_stats.py HEAD.gz [members]"""
import struct
import sys

import numpy as np


class Bits:
    def __init__(self, data, pos_bits):
        self.d = data
        self.p = pos_bits

    def get(self, n):
        v = 0
        for i in range(n):
            b = (self.d[(self.p + i) >> 3] >> ((self.p + i) & 7)) & 1
            v |= b << i
        self.p += n
        return v


def huff_table(lens):
    """canonical code -> {(len, code): sym} with codes read bit by bit (MSB first)"""
    maxl = max(lens) if lens else 0
    cnt = [0] * (maxl + 1)
    for L in lens:
        if L:
            cnt[L] += 1
    code, nxt = 0, [0] * (maxl + 2)
    for b in range(1, maxl + 1):
        code = (code + cnt[b - 1]) << 1 if b > 1 else 0
        nxt[b] = code
    tab = {}
    for s, L in enumerate(lens):
        if L:
            tab[(L, nxt[L])] = s
            nxt[L] += 1
    return tab, maxl


def dec(bits, tab):
    code = 0
    for L in range(1, 16):
        code = (code << 1) | bits.get(1)
        if (L, code) in tab:
            return tab[(L, code)]
    raise ValueError("bad code")


LBASE = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258]
LEXT = [0] * 8 + [1] * 4 + [2] * 4 + [3] * 4 + [4] * 4 + [5] * 4 + [0]
DBASE = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073,
         4097, 6145, 8193, 12289, 16385, 24577]
DEXT = [0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13]
CLORD = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]


def member(data, off):
    """-> (tokens, next offset); tokens: ('L', byte) / ('C', length, distance) in bytes"""
    assert data[off] == 0x1F and data[off + 1] == 0x8B
    flg = data[off + 3]
    p = off + 10
    if flg & 4:
        xlen = struct.unpack_from("<H", data, p)[0]
        p += 2 + xlen
    bits = Bits(data, 8 * p)
    assert bits.get(1) == 1 and bits.get(2) == 2
    nlit, ndist, ncl = bits.get(5) + 257, bits.get(5) + 1, bits.get(4) + 4
    cl = [0] * 19
    for i in range(ncl):
        cl[CLORD[i]] = bits.get(3)
    ct, _ = huff_table(cl)
    lens = []
    while len(lens) < nlit + ndist:
        s = dec(bits, ct)
        if s < 16:
            lens.append(s)
        elif s == 16:
            lens += [lens[-1]] * (3 + bits.get(2))
        elif s == 17:
            lens += [0] * (3 + bits.get(3))
        else:
            lens += [0] * (11 + bits.get(7))
    lt, _ = huff_table(lens[:nlit])
    dt, _ = huff_table(lens[nlit:])
    toks = []
    while True:
        s = dec(bits, lt)
        if s < 256:
            toks.append(("L", s))
        elif s == 256:
            break
        else:
            c = s - 257
            ln = LBASE[c] + bits.get(LEXT[c])
            d = dec(bits, dt)
            dist = DBASE[d] + bits.get(DEXT[d])
            toks.append(("C", ln, dist))
    end = (bits.p + 7) >> 3
    return toks, end + 8


def main():
    data = open(sys.argv[1], "rb").read()
    nmem = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    off = 0
    seg_rows = []
    for _ in range(nmem):
        toks, off = member(data, off)
        # values: literal values (4 byte symbols) and copies (in values)
        ops, nbytes = [], 0
        pend = 0
        for t in toks:
            if t[0] == "L":
                pend += 1
                if pend == 4:
                    ops.append(("L",))
                    pend = 0
            else:
                ops.append(("C", t[1] // 4, t[2] // 4))
        # per segment
        pos = 0
        seg = []
        for o in ops:
            if pos % 2048 == 0 and (not seg or seg[-1]):
                pass
            seg.append(o)
            pos += 1 if o[0] == "L" else o[1]
            if pos % 2048 == 0:
                seg_rows.append(seg)
                seg = []
        if seg:
            seg_rows.append(seg)
    lits = [sum(1 for o in s if o[0] == "L") for s in seg_rows]
    cps = [sum(1 for o in s if o[0] == "C") for s in seg_rows]
    syms = [4 * a + 2 * b for a, b in zip(lits, cps)]
    # pointer jumping rounds, synchronous
    rounds = []
    unres = {}
    for s in seg_rows:
        e = []
        for o in s:
            if o[0] == "L":
                e.append(-1)
            else:
                e += [o[2]] * o[1]
        e = np.array(e[:2048])
        k = np.arange(e.size)
        res = e < 0
        dist = np.where(res, 0, e)
        r = 0
        while True:
            r += 1
            src = k - dist
            nres = res.copy()
            ndist = dist.copy()
            un = ~res
            outside = un & (src < 0)
            nres[outside] = True
            inside = un & (src >= 0)
            si = src[inside]
            rs = res[si]
            idx = np.nonzero(inside)[0]
            nres[idx[rs]] = True
            ndist[idx[~rs]] = dist[idx[~rs]] + dist[si[~rs]]
            res, dist = nres, ndist
            unres.setdefault(r, []).append(float((~res).mean()))
            if res.all():
                break
        rounds.append(r)
    cl = [o[1] for s in seg_rows for o in s if o[0] == "C"]
    cd = [o[2] for s in seg_rows for o in s if o[0] == "C"]
    print(f"segments {len(seg_rows)}: literals/seg mean {np.mean(lits):.0f} max {max(lits)}; copies/seg mean "
          f"{np.mean(cps):.0f} max {max(cps)}; symbols/seg mean {np.mean(syms):.0f} max {max(syms)}; ops/seg mean "
          f"{np.mean([a + b for a, b in zip(lits, cps)]):.0f}")
    print(f"copy length mean {np.mean(cl):.1f} median {np.median(cl):.0f}; distance median {np.median(cd):.0f}, "
          f"share < 2048: {np.mean(np.array(cd) < 2048):.2f}")
    print("unresolved after round:", {r: round(float(np.mean(v)), 3) for r, v in sorted(unres.items())})
    print(f"jump rounds/seg mean {np.mean(rounds):.1f} max {max(rounds)} hist {np.bincount(rounds).tolist()}")


if __name__ == "__main__":
    main()
