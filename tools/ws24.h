// ws24.h -- 24-bit block-floating-point storage of fp32 FWHT intermediates.
//
// The large-slice passes of the Eden codec hand their fp32 intermediates to
// each other through HBM.  Stored as 24 bits per
// element instead of 32 they move 3/4 of the bytes.  Format: groups of 8
// consecutive elements share one 8-bit exponent Eq (the group's largest
// |value|, clamped to [22, 254]); each element keeps a sign and a 22-bit
// magnitude m = round(|v| * 2^(148 - Eq)) < 2^22, i.e. an absolute error
// <= 2^-23 of the group's power-of-two range -- about 1e-7 of the group's
// largest value.  A group holding Inf or NaN stores Eq = 255 and decodes to
// NaN throughout (non-finite data stays non-finite, so the codec's NaN-scale
// zero fallback, eden_pipeline.py:522-525, still triggers).
//
// Element code (24 bits): [21:0] m, [22] bit (g) of Eq where g = element
// index mod 8, [23] sign.  Group k occupies bytes [24k, 24k + 24): codes of
// elements 8k+4h .. 8k+4h+3 (h = 0, 1) form 3 little-endian dwords.  The byte
// offset of element e's dword is 3e + (e & 3) (elements with e & 3 == 3 own
// no dword).
//
// In every layout of the codec the 8 elements of a group sit on 8 adjacent
// lanes (lane bits 0..2 = element bits 0..2), so the exponent reduction and
// the dword assembly are cross-lane DPP moves within a quad / half-row; no
// LDS traffic, no layout change.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace ws24 {

#define WS24_DEVI __device__ __forceinline__

// DPP controls (gfx9): quad_perm(s0,s1,s2,s3) = s0 | s1 << 2 | s2 << 4 | s3 << 6
constexpr int kQuadXor1 = 1 | 0 << 2 | 3 << 4 | 2 << 6;   // [1,0,3,2]
constexpr int kQuadXor2 = 2 | 3 << 2 | 0 << 4 | 1 << 6;   // [2,3,0,1]
constexpr int kHalfMirror = 0x141;                          // row_half_mirror: lane i <-> 7 - i within 8
constexpr int kQuadNext = 1 | 2 << 2 | 3 << 4 | 3 << 6;    // [1,2,3,3]: code of lane q+1
constexpr int kQuadPrev = 0 | 0 << 2 | 1 << 4 | 2 << 6;    // [0,0,1,2]: dword q-1
constexpr int kQuadSelf = 0 | 1 << 2 | 2 << 4 | 2 << 6;    // [0,1,2,2]: dword min(q,2)

template <int CTRL>
WS24_DEVI uint32_t dpp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}

// largest of the 8 lanes' values (unsigned)
WS24_DEVI uint32_t max8(uint32_t x) {
    x = max(x, dpp<kQuadXor1>(x));
    x = max(x, dpp<kQuadXor2>(x));
    return max(x, dpp<kHalfMirror>(x));
}
WS24_DEVI uint32_t or8(uint32_t x) {
    x |= dpp<kQuadXor1>(x);
    x |= dpp<kQuadXor2>(x);
    return x | dpp<kHalfMirror>(x);
}

#ifdef WS24_TRIVIAL
// A/B instrumentation only (wrong numerics): the memory pattern of the format
// without its arithmetic -- top 24 bits of each value, no cross-lane work
WS24_DEVI uint32_t pack(float v, uint32_t g) {
    (void)g;
    return __float_as_uint(v) >> 8;
}
WS24_DEVI float unpack(uint32_t d, uint32_t g) {
    (void)g;
    return __uint_as_float(d << 8);
}
#else
// fp32 value of this lane -> the dword this lane stores (valid for lanes with
// (lane & 3) < 3).  g = lane & 7 (= element index & 7).
WS24_DEVI uint32_t pack(float v, uint32_t g) {
    const uint32_t b = __float_as_uint(v);
    const uint32_t a = b & 0x7fffffffu;                 // |v|: integer order = float order, NaN > Inf
    const uint32_t E = max8(a) >> 23;
    const uint32_t Eq = E >= 255u ? 255u : max(E, 22u);
    const float s = __uint_as_float((275u - min(Eq, 254u)) << 23);  // 2^(148 - Eq)
    const float af = Eq == 255u ? 0.0f : __uint_as_float(a);       // no NaN into the conversion
    const uint32_t m = min((uint32_t)fmaf(af, s, 0.5f), 0x3fffffu);
    const uint32_t code = ((b >> 31) << 23) | (((Eq >> g) & 1u) << 22) | m;
    const uint32_t nxt = dpp<kQuadNext>(code);
    const uint32_t q = g & 3u;
    return (code >> (8u * q)) | (nxt << (24u - 8u * q));
}

// the dword this lane loaded (lanes with (lane & 3) == 3: anything) -> fp32
WS24_DEVI float unpack(uint32_t d, uint32_t g) {
    const uint32_t lo = dpp<kQuadPrev>(d), hi = dpp<kQuadSelf>(d);
    const uint32_t code = __builtin_amdgcn_alignbit(hi, lo, (32u - 8u * (g & 3u)) & 31u) & 0xffffffu;
    const uint32_t Eq = or8(((code >> 22) & 1u) << g);
    const float mag = (float)(code & 0x3fffffu) * __uint_as_float((Eq - 21u) << 23);
    const float v = __uint_as_float(__float_as_uint(mag) | ((code << 8) & 0x80000000u));
    return Eq == 255u ? __uint_as_float(0x7fc00000u) : v;
}
#endif

// byte offset of element e's dword in a ws24 buffer
WS24_DEVI constexpr uint32_t boff(uint32_t e) { return 3u * e + (e & 3u); }

}  // namespace ws24
