"""Static checks of the register-layout tables in eden_kernels.hip: every FWHT
covers every index bit exactly once, active bits live in registers, and each
layout's half-wave lanes hit 32 distinct LDS banks under the pad() map."""
import os
import re

import pytest

SRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "openfl_amd", "csrc", "eden_kernels.hip")


def _parse(body):
    lays = {k: [int(x) for x in v.split(",")][1:] for k, v in
            re.findall(r"(L\d)\{(\d+(?:, *\d+){5,6})\}", body)}
    masks = {k: {int(x) for x in v.split(",")} for k, v in
             re.findall(r"(F\d[a-e]) = bits_mask\(\{([\d, ]+)\}\)", body)}
    return lays, masks


def _sets():
    src = open(SRC).read()
    out = {}
    for m in re.finditer(r"template <> struct SmallSet<(\d+)> \{(.*?)\n\};", src, re.S):
        out[("small", int(m.group(1)))] = _parse(m.group(2))
    m = re.search(r"struct RowSet6 \{(.*?)\n\};", src, re.S)
    assert m, "RowSet6 not found"
    out[("row", 15)] = _parse(m.group(1))
    return out


SETS = _sets()


def pad(e):
    return e + (e >> 5) + (e >> 10)


def lane_bits(regs, nb):
    return [b for b in range(nb) if b not in regs][:5]


@pytest.mark.parametrize("key", sorted(SETS))
def test_each_fwht_covers_every_bit_once(key):
    kind, p = key
    lays, m = SETS[key]
    nr = len(lays["L1"])
    assert all(len(v) == nr for v in lays.values())
    assert sorted(m["F1a"] | m["F1b"] | m["F1c"]) == list(range(p))
    assert len(m["F1a"]) + len(m["F1b"]) + len(m["F1c"]) == p
    assert sorted(m["F2c"] | m["F2d"] | m["F2e"]) == list(range(p))
    assert len(m["F2c"]) + len(m["F2d"]) + len(m["F2e"]) == p
    for lay, act in (("L1", "F1a"), ("L2", "F1b"), ("L3", "F1c"), ("L3", "F2c"), ("L4", "F2d"),
                     ("L5", "F2e")):
        assert m[act] <= set(lays[lay]), (lay, act)
    assert lays["L5"] == list(range(nr))          # contiguous bins for plane packing
    assert lays["L1"][:2] == [0, 1]               # float4 loads / stores


@pytest.mark.parametrize("key", sorted(SETS))
def test_exchanges_bank_conflict_free(key):
    kind, p = key
    lays, _ = SETS[key]
    for name, regs in lays.items():
        lb = lane_bits(regs, p)
        banks = set()
        for lane in range(32):
            e = sum(((lane >> i) & 1) << b for i, b in enumerate(lb))
            banks.add(pad(e) % 32)
        assert len(banks) == 32, (p, name, lb)
