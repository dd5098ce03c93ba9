"""Member-indexed gzip streams written with zlib, for the inflate tests: every
member carries the RFC 1952 extra subfield 'BC' (member size - 1), as the
device gzip's members do (csrc/deflate_kernels.hip), but the deflate data is
zlib's (stored / fixed / dynamic blocks, optional full flushes).  Test data
generator only."""
import struct
import zlib


def member_indexed(data, chunk=16384, level=6, strategy="default", flush_every=None, empty_members=False):
    strat = {"default": zlib.Z_DEFAULT_STRATEGY, "fixed": zlib.Z_FIXED}[strategy]
    parts = [data[i:i + chunk] for i in range(0, len(data), chunk)] or [b""]
    if empty_members:
        parts = [p for q in parts for p in (q, b"")]
    out = bytearray()
    for part in parts:
        c = zlib.compressobj(level, zlib.DEFLATED, -15, 8, strat)
        if flush_every:
            body = b"".join(c.compress(part[j:j + flush_every]) + c.flush(zlib.Z_FULL_FLUSH)
                            for j in range(0, len(part), flush_every)) + c.flush()
        else:
            body = c.compress(part) + c.flush()
        size = 18 + len(body) + 8
        assert size <= 65536
        out += bytes([0x1F, 0x8B, 8, 4, 0, 0, 0, 0, 0, 0xFF, 6, 0]) + b"BC" + struct.pack("<HH", 2, size - 1)
        out += body + struct.pack("<II", zlib.crc32(part), len(part))
    return bytes(out)
