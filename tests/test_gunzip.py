"""Host inflate of member-indexed gzip streams (ofl_gunzip_members, the
GZIPTransformer.backward fast path; kc_pipeline.py:152-156 gzip.decompress).
CPU only: streams are built here with zlib in the device gzip's member format
(RFC 1952 header with the 'BC' extra field = member size - 1)."""
import gzip
import struct
import zlib

import numpy as np
import pytest

from openfl_amd import _lib, lossy


def member(raw, level=6):
    c = zlib.compressobj(level, zlib.DEFLATED, -15)
    body = c.compress(raw) + c.flush()
    size = 18 + len(body) + 8
    hdr = bytes([0x1F, 0x8B, 8, 4, 0, 0, 0, 0, 0, 0xFF]) + struct.pack("<HBBHH", 6, ord("B"), ord("C"), 2, size - 1)
    return hdr + body + struct.pack("<II", zlib.crc32(raw) & 0xFFFFFFFF, len(raw))


def stream(raw, chunk=16384):
    return b"".join(member(raw[i:i + chunk]) for i in range(0, len(raw), chunk)) if raw else member(b"")


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
