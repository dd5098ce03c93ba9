"""Host inflate of member-indexed gzip streams (ofl_gunzip_members, the
GZIPTransformer.backward fast path; kc_pipeline.py:152-156 gzip.decompress).
CPU only: streams are built here with zlib in the device gzip's member format
(RFC 1952 header with the 'BC' extra field = member size - 1)."""
import gzip
import struct

import numpy as np
import pytest

from openfl_amd import _lib, lossy
from tests.bgzf import member_indexed


def stream(raw, chunk=16384):
    return member_indexed(raw, chunk=chunk)


@pytest.mark.parametrize("n", [0, 1, 5000, 16384, 16385, 300_000])
def test_member_stream_roundtrip(n):
    rng = np.random.default_rng(n)
    raw = rng.integers(0, 6, n).astype(np.float32).tobytes()
    z = stream(raw)
    assert gzip.decompress(z) == raw            # a valid gzip stream for the reference reader
    for threads in (1, 4):
        assert lossy.gunzip(z, threads).tobytes() == raw
    out = np.zeros(len(raw) + 64, np.uint8)       # into a caller buffer
    assert lossy.gunzip(z, 3, out=out).tobytes() == raw


def test_plain_gzip_falls_back():
    raw = np.arange(100_000, dtype=np.float32).tobytes()
    z = gzip.compress(raw, compresslevel=9)
    L = _lib.lib()
    import ctypes
    need = ctypes.c_size_t()
    src = np.frombuffer(z, np.uint8)
    assert L.ofl_gunzip_members(src.ctypes.data, src.size, None, 0, ctypes.byref(need), 2) == _lib.OFL_EFORMAT
    assert lossy.gunzip(z).tobytes() == raw


def test_corrupt_member_raises():
    raw = np.ones(50_000, np.float32).tobytes()
    z = bytearray(stream(raw))
    z[-8] ^= 0xFF                                  # last member's CRC-32
    with pytest.raises(_lib.CodecError):
        lossy.gunzip(bytes(z))


def test_member_index_for_the_device_inflate():
    """ofl_gzip_member_index (host half of ofl_inflate_members): data range,
    output offset, ISIZE and CRC-32 of every member."""
    import ctypes
    import zlib
    raw = np.random.default_rng(3).integers(0, 6, 50_000).astype(np.float32).tobytes()
    z = member_indexed(raw, chunk=16384)
    L = _lib.lib()
    src = np.frombuffer(z, np.uint8)
    nm, tot, mx = ctypes.c_int64(), ctypes.c_size_t(), ctypes.c_uint32()
    assert L.ofl_gzip_member_index(src.ctypes.data, src.size, None, 0, ctypes.byref(nm), ctypes.byref(tot),
                                   ctypes.byref(mx), None) == 0
    assert (nm.value, tot.value, mx.value) == (13, len(raw), 16384)
    idx = np.zeros((nm.value, 4), np.int64)
    assert L.ofl_gzip_member_index(src.ctypes.data, src.size, idx.ctypes.data, nm.value - 1, ctypes.byref(nm),
                                   ctypes.byref(tot), ctypes.byref(mx), None) == _lib.OFL_ESPACE
    tl = ctypes.c_int(7)
    assert L.ofl_gzip_member_index(src.ctypes.data, src.size, idx.ctypes.data, nm.value, ctypes.byref(nm),
                                   ctypes.byref(tot), ctypes.byref(mx), ctypes.byref(tl)) == 0
    assert tl.value == 0  # 'BC' members are not TLZ
    for k, (off, ln, out, meta) in enumerate(idx.tolist()):
        meta &= (1 << 64) - 1
        part = raw[16384 * k:16384 * (k + 1)]
        assert out == 16384 * k and (meta & 0xFFFFFFFF) == len(part) and (meta >> 32) == zlib.crc32(part)
        assert zlib.decompress(z[off:off + ln], -15) == part
    plain = np.frombuffer(gzip.compress(raw), np.uint8)
    assert L.ofl_gzip_member_index(plain.ctypes.data, plain.size, None, 0, ctypes.byref(nm), ctypes.byref(tot),
                                   ctypes.byref(mx), None) == _lib.OFL_EFORMAT


def test_oz_members_index_and_host_inflate():
    """Members carrying the TLZ 'OZ' subfield (size, value count, segment
    table): the index flags them (bit 62 of the data length, all_tlz), the
    host parallel inflate and gzip.decompress read them, and a value count
    that contradicts ISIZE clears the flag."""
    import ctypes
    import zlib
    from tests.bgzf import oz_members
    raw = np.random.default_rng(4).integers(0, 6, 131072 * 2 + 5000).astype(np.float32).tobytes()
    z = oz_members(raw)
    assert gzip.decompress(z) == raw
    L = _lib.lib()
    src = np.frombuffer(z, np.uint8)
    nm, tot, mx, tl = ctypes.c_int64(), ctypes.c_size_t(), ctypes.c_uint32(), ctypes.c_int()
    idx = np.zeros((8, 4), np.int64)
    assert L.ofl_gzip_member_index(src.ctypes.data, src.size, idx.ctypes.data, 8, ctypes.byref(nm), ctypes.byref(tot),
                                   ctypes.byref(mx), ctypes.byref(tl)) == 0
    assert (nm.value, tot.value, tl.value) == (3, len(raw), 1)
    for k in range(3):
        off, ln = int(idx[k, 0]), int(idx[k, 1])
        assert ln >> 62 == 1
        ln &= (1 << 62) - 1
        assert zlib.decompress(z[off:off + ln], -15) == raw[4 * 131072 * k:4 * 131072 * (k + 1)]
    assert lossy.gunzip(z, 4).tobytes() == raw
    bad = bytearray(z)
    bad[24] ^= 1                                  # the first member's value count
    src = np.frombuffer(bytes(bad), np.uint8)
    assert L.ofl_gzip_member_index(src.ctypes.data, src.size, idx.ctypes.data, 8, ctypes.byref(nm), ctypes.byref(tot),
                                   ctypes.byref(mx), ctypes.byref(tl)) == 0
    assert tl.value == 0 and idx[0, 1] >> 62 == 0 and idx[1, 1] >> 62 == 1


@pytest.mark.parametrize("fake", [False, True])
def test_large_stream_parallel_index(fake):
    """Streams above 8 MiB are indexed by several threads that each look for
    the first member signature in their piece, then must link up exactly; a
    signature planted in stored (level 0) data makes a piece start on a fake
    header, which the linkage check rejects (serial walk, same index)."""
    rng = np.random.default_rng(11)
    raw = bytearray(rng.integers(0, 256, 24 << 20, dtype=np.uint8).tobytes())
    if fake:  # a fake 'BC' member header every 700 KB (verbatim in stored blocks)
        sig = bytes([0x1F, 0x8B, 8, 4, 0, 0, 0, 0, 0, 0xFF, 6, 0]) + b"BC" + struct.pack("<HH", 2, 99)
        for off in range(1000, len(raw) - 64, 700_000):
            raw[off:off + len(sig)] = sig
    raw = bytes(raw)
    z = member_indexed(raw, chunk=60_000, level=0)
    assert lossy.gunzip(z, 8).tobytes() == raw
    import ctypes
    L = _lib.lib()
    src = np.frombuffer(z, np.uint8)
    nm, tot, mx = ctypes.c_int64(), ctypes.c_size_t(), ctypes.c_uint32()
    assert L.ofl_gzip_member_index(src.ctypes.data, src.size, None, 0, ctypes.byref(nm), ctypes.byref(tot),
                                   ctypes.byref(mx), None) == 0
    assert nm.value == -(-len(raw) // 60_000) and tot.value == len(raw)
