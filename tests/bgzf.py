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


def oz_members(data, values_per_member=131072, level=6):
    """Members with the TLZ header ('OZ' subfield: version 1, log2 segment 11,
    segment count, member size, value count, a segment table) around zlib's
    deflate data: the host index and the host inflate must read them; the
    table is zeros (zlib's symbols do not start there), so the TLZ decoder
    refuses them and the generic inflate decodes them."""
    nb = 4 * values_per_member
    parts = [data[i:i + nb] for i in range(0, len(data), nb)]
    out = bytearray()
    for part in parts:
        assert len(part) % 4 == 0
        nval = len(part) // 4
        nseg = (nval + 2047) // 2048
        c = zlib.compressobj(level, zlib.DEFLATED, -15)
        body = c.compress(part) + c.flush()
        ln = 12 + 4 * nseg
        size = 12 + 4 + ln + len(body) + 8
        out += bytes([0x1F, 0x8B, 8, 4, 0, 0, 0, 0, 0, 0xFF]) + struct.pack("<H", 4 + ln) + b"OZ"
        out += struct.pack("<HBBHII", ln, 1, 11, nseg, size, nval) + bytes(4 * nseg)
        out += body + struct.pack("<II", zlib.crc32(part), len(part))
    return bytes(out)
