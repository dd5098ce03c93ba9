// deflate_kernels.hip -- gzip on the GPU for the lossy pipelines' rank arrays
// (SURVEY §8(f) row 3).  Reference: GZIPTransformer.forward / backward
// (kc_pipeline.py:128-156, skc_pipeline.py:201-230, stc_pipeline.py:185-215):
// gzip.compress(float32 ranks bytes), decoded by gzip.decompress.  Any valid
// gzip stream decodes to the same bytes, so the wire stays compatible.
//
// Two parts:
//  * TLZ (namespace gz::tlz, below the generic inflate): the encoder of the
//    rank arrays -- an optimal-parse token LZ over the whole 32 KiB window,
//    one dynamic-Huffman block per 512 KiB member, with per-segment entry
//    points in an RFC 1952 extra subfield -- and its lane-parallel two-kernel
//    inflate;
//  * a generic member inflate (k_inflate_members: stored, fixed and dynamic
//    blocks, any deflate data of a member-indexed stream), used for streams
//    that are not TLZ (e.g. BGZF-style members written by zlib) and as the
//    fallback of the TLZ inflate.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include <thread>
#include <zlib.h>

#include "ofl_codec.h"
#include "ofl_util.h"

#define DEVI __device__ __forceinline__

namespace gz {

constexpr int kLit = 286, kDist = 30, kCL = 19;

__constant__ uint16_t c_dbase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129,
                                     193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t c_dext[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t c_clord[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
__constant__ uint16_t c_lbase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59,
                                     67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t c_lext[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint32_t c_adv[32][32];       // raw CRC advance by 2^k zero bytes: GF(2) matrix columns

// Huffman scratch (the serial fallback of huff_lengths_wave, the RLE)
struct HScratch {
    uint32_t w[2 * kLit];
    int16_t parent[2 * kLit];
    int16_t sym[kLit];
    uint8_t dead[2 * kLit];
    uint16_t rle_sym[kLit + kDist];
    uint16_t rle_ext[kLit + kDist];
};
constexpr int kHdrW = 160;                 // deflate block header words (<= 4642 bits)

DEVI void put_bits(uint32_t* out, uint32_t pos, uint32_t val, int nb) {
    if (nb == 0) return;
    const uint32_t w = pos >> 5, sh = pos & 31u;
    atomicOr(&out[w], val << sh);
    if (sh + (uint32_t)nb > 32u) atomicOr(&out[w + 1], val >> (32u - sh));
}
DEVI uint32_t rev_bits(uint32_t c, int n) { return __brev(c) >> (32 - n); }
// distance code of a distance d in 1..32768 (RFC 1951 3.2.5): codes 0..3 are
// d - 1, then two codes per power of two
DEVI int dist_code(uint32_t d) {
    if (d <= 4u) return (int)d - 1;
    const uint32_t m = d - 1u;
    const int b = 31 - __builtin_clz(m);
    return 2 * b + (int)((m >> (b - 1)) & 1u);
}
// index into c_lbase (symbol 257 + index) of a length of l bytes, 3..258
DEVI int len_code(uint32_t l) {
    if (l == 258u) return 28;
    const uint32_t m = l - 3u;
    if (m < 8u) return (int)m;
    const int b = 31 - __builtin_clz(m);
    return 4 * (b - 1) + (int)((m >> (b - 2)) & 3u);
}
// a length's / distance's code with its extra bits computed (no table
// loads: the tables are in constant memory, and a per-lane index into them is
// a vector memory load per lookup): l, d in bytes, l in 11..258, d >= 1
DEVI void len_sym(uint32_t l, int& lc, int& ne, uint32_t& ev) {
    const uint32_t m = l - 3u;
    if (m < 8u) { lc = (int)m; ne = 0; ev = 0; return; }
    const int b = 31 - __builtin_clz(m);
    lc = 4 * (b - 1) + (int)((m >> (b - 2)) & 3u);
    ne = b - 2;
    ev = m & ((1u << ne) - 1u);
}
DEVI void dist_sym(uint32_t d, int& dc, int& ne, uint32_t& ev) {
    const uint32_t m = d - 1u;
    if (d <= 4u) { dc = (int)m; ne = 0; ev = 0; return; }
    const int b = 31 - __builtin_clz(m);
    dc = 2 * b + (int)((m >> (b - 1)) & 1u);
    ne = b - 1;
    ev = m & ((1u << ne) - 1u);
}
// advance by 2^k zero bytes (k uniform: the matrix columns are scalar loads)
DEVI uint32_t crc_adv_pow2(uint32_t v, int k) {
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i) r ^= ((v >> i) & 1u) ? c_adv[k][i] : 0u;
    return r;
}
// raw (zero-initialised, reflected) CRC-32 steps, bitwise: a byte, a
// little-endian word
DEVI uint32_t crc_byte(uint32_t r, uint32_t b) {
    r ^= b;
#pragma unroll
    for (int k = 0; k < 8; ++k) r = (r >> 1) ^ (0xEDB88320u & (0u - (r & 1u)));
    return r;
}
DEVI uint32_t crc_word(uint32_t r, uint32_t w) {
    r ^= w;
#pragma unroll
    for (int k = 0; k < 32; ++k) r = (r >> 1) ^ (0xEDB88320u & (0u - (r & 1u)));
    return r;
}
DEVI uint32_t crc_adv(uint32_t v, uint32_t len) {
    for (int k = 0; k < 32; ++k)
        if ((len >> k) & 1u) {
            uint32_t r = 0;
            for (int i = 0; i < 32; ++i) r ^= ((v >> i) & 1u) ? c_adv[k][i] : 0u;
            v = r;
        }
    return v;
}

// Huffman code lengths of freq[0..n) limited to maxlen (thread 0): two
// smallest live nodes merged until one is left; if too deep, halve the
// frequencies (keeping them >= 1) and rebuild
// complete: a lone symbol gets a partner (zlib accepts an incomplete code only
// for distances)
DEVI void huff_lengths(const uint32_t* freq, int n, int maxlen, uint8_t* len, HScratch& h, bool complete) {
    int m = 0;
    for (int s = 0; s < n; ++s) { len[s] = 0; if (freq[s]) { h.sym[m] = (int16_t)s; h.w[m] = freq[s]; ++m; } }
    if (m == 0) return;
    if (m == 1) {
        len[h.sym[0]] = 1;
        if (complete) len[h.sym[0] == 0 ? 1 : 0] = 1;
        return;
    }
    for (;;) {
        for (int i = 0; i < 2 * m; ++i) { h.dead[i] = 0; h.parent[i] = -1; }
        int nodes = m;
        for (int it = 0; it < m - 1; ++it) {
            int a = -1, b = -1;
            for (int i = 0; i < nodes; ++i) {
                if (h.dead[i]) continue;
                if (a < 0 || h.w[i] < h.w[a]) { b = a; a = i; }
                else if (b < 0 || h.w[i] < h.w[b]) b = i;
            }
            h.w[nodes] = h.w[a] + h.w[b];
            h.dead[a] = h.dead[b] = 1;
            h.parent[a] = h.parent[b] = (int16_t)nodes;
            ++nodes;
        }
        int deepest = 0;
        for (int i = 0; i < m; ++i) {
            int d = 0;
            for (int j = i; h.parent[j] >= 0; j = h.parent[j]) ++d;
            len[h.sym[i]] = (uint8_t)d;
            deepest = d > deepest ? d : deepest;
        }
        if (deepest <= maxlen) return;
        for (int i = 0; i < m; ++i) h.w[i] = (h.w[i] >> 1) | 1u;
    }
}
// canonical codes (RFC 1951 3.2.2), stored bit-reversed for LSB-first output
DEVI void huff_codes(const uint8_t* len, int n, uint16_t* code) {
    uint32_t cnt[16] = {0}, next[16];
    for (int s = 0; s < n; ++s) cnt[len[s]]++;
    cnt[0] = 0;
    uint32_t c = 0;
    for (int b = 1; b < 16; ++b) { c = (c + cnt[b - 1]) << 1; next[b] = c; }
    for (int s = 0; s < n; ++s) code[s] = len[s] ? (uint16_t)rev_bits(next[len[s]]++, len[s]) : 0;
}

// ---- the same on one wave (lanes 0..63 of the block) ----------------------
// The serial versions above are latency-bound on one lane (~60 % of a
// member's time).  The rank alphabets use a few dozen literal bytes and
// length / distance codes, so one symbol per lane fits: the used symbols are
// compacted in symbol order, bitonic-sorted by (weight, symbol) across the
// lanes (shfl_xor), and the two-queue merge (leaves in sorted order, internal
// nodes in creation order, both nondecreasing) runs on wave-uniform values
// through readlane / writelane; depths are assigned top-down.  Returns false
// (lengths zeroed) when more than 64 symbols occur: the caller then runs the
// serial huff_lengths on lane 0.  scratch: 64 LDS words.
DEVI uint32_t rdl(uint32_t v, int i) { return (uint32_t)__builtin_amdgcn_readlane((int)v, i); }
DEVI uint32_t wrl(uint32_t v, int i, uint32_t old) { return (int)(threadIdx.x & 63u) == i ? v : old; }

DEVI bool huff_lengths_wave(const uint32_t* freq, int n, int maxlen, uint8_t* len, uint32_t* scratch, bool complete) {
    const int lane = (int)(threadIdx.x & 63u);
    int m = 0;
    for (int b = 0; b < n; b += 64) {
        const int s = b + lane;
        const uint32_t f = s < n ? freq[s] : 0u;
        const uint64_t mask = __ballot(f != 0u);
        const int rank = __popcll(mask & ((1ull << lane) - 1ull));
        if (f != 0u && m + rank < 64) scratch[m + rank] = (f << 9) | (uint32_t)s;
        if (s < n) len[s] = 0;
        m += __popcll(mask);
    }
    if (m > 64) return false;
    if (m == 0) return true;
    if (m == 1) {
        const int s = (int)(scratch[0] & 511u);
        if (lane == 0) {
            len[s] = 1;
            if (complete) len[s == 0 ? 1 : 0] = 1;
        }
        return true;
    }
    uint32_t key0 = lane < m ? scratch[lane] : 0xffffffffu;
    for (;;) {
        uint32_t key = key0;
        for (int k = 2; k <= 64; k <<= 1)
            for (int j = k >> 1; j > 0; j >>= 1) {
                const uint32_t o = (uint32_t)__shfl_xor((int)key, j, 64);
                const bool up = (lane & k) == 0, lower = (lane & j) == 0;
                key = (lower == up) ? min(key, o) : max(key, o);
            }
        const uint32_t w = key >> 9;  // lane i: the i-th smallest leaf weight
        uint32_t iw = 0, ca = 0, cb = 0;  // lane k: internal node k's weight and children
        int li = 0, ij = 0, ni = 0;
        for (int step = 0; step < m - 1; ++step) {
            uint32_t cw0, cw1;
            int c0, c1;
            {
                const uint32_t lw = li < m ? rdl(w, li) : 0xffffffffu, nw = ij < ni ? rdl(iw, ij) : 0xffffffffu;
                if (li < m && (ij >= ni || lw <= nw)) { c0 = li; cw0 = lw; ++li; } else { c0 = 64 + ij; cw0 = nw; ++ij; }
            }
            {
                const uint32_t lw = li < m ? rdl(w, li) : 0xffffffffu, nw = ij < ni ? rdl(iw, ij) : 0xffffffffu;
                if (li < m && (ij >= ni || lw <= nw)) { c1 = li; cw1 = lw; ++li; } else { c1 = 64 + ij; cw1 = nw; ++ij; }
            }
            iw = wrl(cw0 + cw1, ni, iw);
            ca = wrl((uint32_t)c0, ni, ca);
            cb = wrl((uint32_t)c1, ni, cb);
            ++ni;
        }
        uint32_t di = 0, dl = 0;  // depth of internal node k (lane k) / of the i-th leaf (lane i)
        int deepest = 0;
        for (int k = ni - 1; k >= 0; --k) {
            const uint32_t d = rdl(di, k) + 1u;
            const int a = (int)rdl(ca, k), b = (int)rdl(cb, k);
            if (a >= 64) di = wrl(d, a - 64, di); else { dl = wrl(d, a, dl); deepest = max(deepest, (int)d); }
            if (b >= 64) di = wrl(d, b - 64, di); else { dl = wrl(d, b, dl); deepest = max(deepest, (int)d); }
        }
        if (deepest <= maxlen) {
            if (lane < m) len[key & 511u] = (uint8_t)dl;
            return true;
        }
        // too deep: flatten the weights (>= 1) and rebuild, as huff_lengths
        key0 = lane < m ? (((((key0 >> 9) >> 1) | 1u)) << 9) | (key0 & 511u) : 0xffffffffu;
    }
}

// canonical codes on one wave: counts per length and ranks by ballots
DEVI void huff_codes_wave(const uint8_t* len, int n, uint16_t* code) {
    const int lane = (int)(threadIdx.x & 63u);
    const uint64_t below = (1ull << lane) - 1ull;
    uint32_t cnt[16];
#pragma unroll
    for (int b = 0; b < 16; ++b) cnt[b] = 0;
    for (int base = 0; base < n; base += 64) {
        const int s = base + lane;
        const int L = s < n ? len[s] : 0;
#pragma unroll
        for (int b = 1; b < 16; ++b) cnt[b] += (uint32_t)__popcll(__ballot(L == b));
    }
    uint32_t run[16];
    uint32_t c = 0;
    run[0] = 0;
#pragma unroll
    for (int b = 1; b < 16; ++b) { c = (c + (b > 1 ? cnt[b - 1] : 0u)) << 1; run[b] = c; }
    for (int base = 0; base < n; base += 64) {
        const int s = base + lane;
        const int L = s < n ? len[s] : 0;
        uint32_t mine = 0;
#pragma unroll
        for (int b = 1; b < 16; ++b) {
            const uint64_t mk = __ballot(L == b);
            if (L == b) mine = run[b] + (uint32_t)__popcll(mk & below);
            run[b] += (uint32_t)__popcll(mk);
        }
        if (s < n) code[s] = L ? (uint16_t)rev_bits(mine, L) : 0;
    }
}

// exclusive scan of the member sizes (one block) -> offsets, total at [n]
// running (nullable): the stream bytes of earlier batches, added to every
// offset and advanced by this batch's total; cap: the output's size (a batch
// that would not fit sets *bad = 2 and advances nothing)
__global__ __launch_bounds__(1024) void k_gzip_scan(const uint32_t* sizes, int n, uint64_t* off, uint64_t* running,
                                                    uint64_t cap, int* bad) {
    __shared__ uint64_t part[1024 / 64];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int per = (n + 1023) / 1024;
    const int b0 = tid * per, b1 = std::min(n, b0 + per);
    uint64_t s = 0;
    for (int i = b0; i < b1; ++i) s += sizes[i];
    uint64_t inc = s;
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t t = __shfl_up(inc, o, 64);
        if (lane >= o) inc += t;
    }
    if (lane == 63) part[w] = inc;
    __syncthreads();
    const uint64_t run0 = running ? *running : 0;
    uint64_t tot = 0;
    for (int j = 0; j < 1024 / 64; ++j) tot += part[j];
    const bool fits = run0 + tot <= cap;
    uint64_t base = inc - s + run0;
    for (int j = 0; j < w; ++j) base += part[j];
    for (int i = b0; i < b1; ++i) { off[i] = fits ? base : ~0ull; base += sizes[i]; }
    if (tid == 1023) off[n] = base;
    __syncthreads();
    if (tid == 0 && running) {
        if (fits) *running = run0 + tot;
        else atomicOr(bad, 2);
    }
}

// ============================================================================
// Device inflate of member-indexed streams (GZIPTransformer.backward,
// kc_pipeline.py:152-156: gzip.decompress).  One wavefront per member; the
// Huffman decode is inherently serial, so every lane runs it on the same
// (wave-uniform) values and the lanes split the work that is parallel: table
// construction, each copy's bytes (an overlapping copy d < L is the periodic
// extension out[p + i] = out[p - d + i % d]) and the store.  Default (RING):
// only the last WIN = 1 KiB of a member's output stays in LDS, every byte is
// also stored to global memory as it is produced, and the rare copy reaching
// further back than the ring reads those global bytes back (stored earlier by
// the same wavefront; a wavefront-scope acquire/release fence orders them);
// the window decoder (RING = false, OFL_GZ_INFLATE=window) keeps the whole
// output in a 16 / 64 KiB LDS window instead.  The compressed bytes stream
// through a small LDS ring.
// Any valid deflate data decodes (stored, fixed and dynamic blocks, RFC 1951).
// ISIZE and the CRC-32 (over the member's output, wave-parallel) are checked here.
constexpr int kRing = 512;                 // compressed-input ring per wave (bytes)
#ifndef OFL_INF_FASTBITS
#define OFL_INF_FASTBITS 9
#endif
#ifndef OFL_INF_WAVES
#define OFL_INF_WAVES 1
#endif
constexpr int kFastBits = OFL_INF_FASTBITS; // first-level decode table: codes of <= 9 bits

// A first-level table entry says what the symbol means, so the serial decode
// (scalar-unit bound: one SALU pipe per CU serves all its waves) needs no
// per-symbol branching on the symbol value:
//   bits 0..3   code length (0: the code is longer than kFastBits, or unused)
//   bits 4..7   extra bits that follow the code (length / distance codes)
//   bits 8..9   kind: 0 literal (or plain symbol), 1 length / distance, 2 end
//               of block, 3 not a valid symbol here
//   bits 16..31 value: literal byte / symbol, length base, distance base
enum { kKindLit = 0, kKindCopy = 1, kKindEnd = 2, kKindBad = 3 };
enum { kAlphaLit = 0, kAlphaDist = 1, kAlphaPlain = 2 };
template <int FB, int NS>
struct InfCodeT {                          // one canonical Huffman code
    static constexpr int kFB = FB, kSize = 1 << FB;
    uint32_t fast[kSize];                  // entries as above (code length in bits 0..3)
    uint16_t cnt[16];                      // codes per length
    uint16_t sorted[NS];                   // symbols ordered by (length, symbol)
};
// literal / length (and code-length) codes: 9-bit first level, 288 symbols;
// distance codes: 8-bit first level, 30 symbols -- 1.5 KiB less LDS per
// member (more members resident per CU for the scalar-bound decode; a
// distance code longer than 8 bits takes the canonical walk)
using InfCode = InfCodeT<kFastBits, 288>;
using InfDistCode = InfCodeT<8, 32>;
// (length, distance) pair table: the next kPairBits bits of the stream ->
// one whole copy when its length code, length extra bits, distance code and
// distance extra bits all fit in them: bits 0..4 bits consumed, 5..13
// length, 14..29 distance, bit 30 valid.  The device gzip's rank streams are
// mostly 4-byte copies (a token's previous occurrence) with short distance
// codes, so most copies decode with one table read instead of two decodes
// and two extra-bit reads on the scalar unit.
constexpr int kPairBits = 10;
constexpr int kPair = 1 << kPairBits;
template <int WIN, bool PAIR>
struct InfSmem {
    alignas(16) uint8_t win[WIN];          // the member's output
    alignas(4) uint8_t ring[kRing];
    InfCode lit;
    InfDistCode dist;
    uint8_t lens[320];                     // code lengths (literal/length | distance)
    uint32_t pair[PAIR ? kPair : 1];
};

struct InfArgs {
    const uint8_t* src;                    // device copy of the stream
    const int64_t* idx;                    // per member: data offset, data length, output offset, isize | crc << 32
    int64_t nmem;
    uint8_t* out;
    uint64_t out_cap;
    int* status;                           // OR of kInf* flags over the members
};
constexpr int kInfCorrupt = 1, kInfSize = 2, kInfCrc = 4, kInfRange = 8;

// base value and extra-bit count of a length code c (0..28) / a distance code
// c (0..29), RFC 1951 3.2.5, in closed form
DEVI uint32_t len_base(int c, int& ext) {
    if (c < 8) { ext = 0; return 3u + (uint32_t)c; }
    if (c == 28) { ext = 0; return 258u; }
    ext = (c >> 2) - 1;
    return ((4u + (uint32_t)(c & 3)) << ext) + 3u;
}
DEVI uint32_t dist_base(int c, int& ext) {
    if (c < 4) { ext = 0; return 1u + (uint32_t)c; }
    ext = (c >> 1) - 1;
    return ((2u + (uint32_t)(c & 1)) << ext) + 1u;
}
// the table entry of symbol s of an alphabet (code length not included)
DEVI uint32_t inf_entry(int s, int alpha) {
    int ext = 0;
    if (alpha == kAlphaPlain) return (uint32_t)s << 16;
    if (alpha == kAlphaDist) {
        if (s > 29) return (uint32_t)kKindBad << 8;
        const uint32_t b = dist_base(s, ext);
        return (b << 16) | ((uint32_t)kKindCopy << 8) | ((uint32_t)ext << 4);
    }
    if (s < 256) return (uint32_t)s << 16;
    if (s == 256) return (uint32_t)kKindEnd << 8;
    if (s > 285) return (uint32_t)kKindBad << 8;
    const uint32_t b = len_base(s - 257, ext);
    return (b << 16) | ((uint32_t)kKindCopy << 8) | ((uint32_t)ext << 4);
}

// canonical code from lengths (wave-parallel): counts and ranks by ballots,
// the fast table filled by the symbols' lanes.  false: over-subscribed.
template <typename C>
DEVI bool inf_build(C& c, const uint8_t* lens, int n, int alpha) {
    const int lane = (int)(threadIdx.x & 63u);
    const uint64_t below = (1ull << lane) - 1ull;
    for (int k = lane; k < C::kSize; k += 64) c.fast[k] = 0;
    uint32_t cnt[16];
#pragma unroll
    for (int b = 0; b < 16; ++b) cnt[b] = 0;
    for (int base = 0; base < n; base += 64) {
        const int s = base + lane;
        const int L = s < n ? lens[s] : 0;
#pragma unroll
        for (int b = 1; b < 16; ++b) cnt[b] += (uint32_t)__popcll(__ballot(L == b));
    }
    int left = 1;
#pragma unroll
    for (int b = 1; b < 16; ++b) { left = (left << 1) - (int)cnt[b]; if (left < 0) return false; }
    if (lane < 16) c.cnt[lane] = (uint16_t)(lane ? cnt[lane] : 0u);
    uint32_t off[16], next[16];
    uint32_t o = 0, code = 0;
#pragma unroll
    for (int b = 1; b < 16; ++b) {
        off[b] = o;
        o += cnt[b];
        code = (code + (b > 1 ? cnt[b - 1] : 0u)) << 1;
        next[b] = code;
    }
    for (int base = 0; base < n; base += 64) {
        const int s = base + lane;
        const int L = s < n ? lens[s] : 0;
        uint32_t my_off = 0, my_code = 0;
#pragma unroll
        for (int b = 1; b < 16; ++b) {
            const uint64_t mk = __ballot(L == b);
            if (L == b) {
                const uint32_t r = (uint32_t)__popcll(mk & below);
                my_off = off[b] + r;
                my_code = next[b] + r;
            }
            off[b] += (uint32_t)__popcll(mk);
            next[b] += (uint32_t)__popcll(mk);
        }
        if (L) {
            c.sorted[my_off] = (uint16_t)s;
            if (L <= C::kFB) {
                const uint32_t e = inf_entry(s, alpha) | (uint32_t)L;
                for (uint32_t k = rev_bits(my_code, L); k < (uint32_t)C::kSize; k += 1u << L) c.fast[k] = e;
            }
        }
    }
    __builtin_amdgcn_wave_barrier();
    return true;
}

// the pair table of a block's codes (wave-parallel, after both builds)
template <int WIN, bool PAIR>
DEVI void inf_build_pairs(InfSmem<WIN, PAIR>& S) {
    if constexpr (PAIR) {
        const int lane = (int)(threadIdx.x & 63u);
        for (int k = lane; k < kPair; k += 64) {
            uint32_t out = 0;
            const uint32_t e = S.lit.fast[k & (InfCode::kSize - 1)];
            const uint32_t l = e & 15u, x = (e >> 4) & 15u;
            if (l && ((e >> 8) & 3u) == (uint32_t)kKindCopy && l + x <= (uint32_t)kPairBits) {
                const uint32_t len = (e >> 16) + (((uint32_t)k >> l) & ((1u << x) - 1u));
                const uint32_t r = (uint32_t)k >> (l + x);
                const uint32_t f = S.dist.fast[r & (InfDistCode::kSize - 1)];
                const uint32_t l2 = f & 15u, x2 = (f >> 4) & 15u;
                const uint32_t nb = l + x + l2 + x2;
                if (l2 && ((f >> 8) & 3u) == (uint32_t)kKindCopy && nb <= (uint32_t)kPairBits) {
                    const uint32_t d = (f >> 16) + ((r >> l2) & ((1u << x2) - 1u));
                    out = nb | (len << 5) | (d << 14) | (1u << 30);
                }
            }
            S.pair[k] = out;
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// wave-uniform value from LDS into a scalar register: the decode state then
// lives in SGPRs and its arithmetic runs on the scalar unit (one wave-wide
// VALU op per step of the serial decode would cost 4+ cycles each)
DEVI uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }

// codes longer than the first-level table: canonical walk, most significant
// bit first (rare: the slow path of inf_decode)
template <typename C>
DEVI uint32_t inf_decode_long(const C& c, uint64_t& bb, int& bc, int alpha) {
    int code = 0, first = 0, index = 0;
#pragma unroll 1
    for (int len = 1; len <= 15; ++len) {
        code |= (int)(bb & 1u);
        bb >>= 1;
        --bc;
        const int n = (int)uni(c.cnt[len]);
        if (code - first < n) return inf_entry((int)uni(c.sorted[index + code - first]), alpha);
        index += n;
        first = (first + n) << 1;
        code <<= 1;
    }
    return (uint32_t)kKindBad << 8;
}

// one symbol's table entry (needs >= 15 bits in bb), its code consumed;
// kKindBad if the bits are no code
template <typename C>
DEVI uint32_t inf_decode(const C& c, uint64_t& bb, int& bc, int alpha) {
    const uint32_t e = uni(c.fast[bb & (uint64_t)(C::kSize - 1)]);
    const int l = (int)(e & 15u);
    if (l) {
        bb >>= l;
        bc -= l;
        return e;
    }
    return inf_decode_long(c, bb, bc, alpha);
}

// RING = false: the member's whole output stays in the WIN-byte LDS window
// until it is complete, then one coalesced store.  RING = true: the LDS holds
// only the last WIN output bytes (a ring) and every byte also goes to global
// memory as it is produced; a copy reaching further back than the ring reads
// global memory (bytes this wavefront stored earlier: same-address order
// within a wavefront).  Less LDS per member -> more members per CU.
template <int WIN, bool RING, bool PAIR>
__global__ __launch_bounds__(64, OFL_INF_WAVES) void k_inflate_members(InfArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    InfSmem<WIN, PAIR>& S = *reinterpret_cast<InfSmem<WIN, PAIR>*>(smem_raw);
    const int lane = threadIdx.x;
    const int64_t m = blockIdx.x;
    if (m >= a.nmem) return;
    const int64_t* ix = a.idx + 4 * m;
    const uint8_t* src = a.src + ix[0];
    const uint32_t in_len = (uint32_t)ix[1];
    const int64_t out_off = ix[2];
    const uint32_t isize = (uint32_t)((uint64_t)ix[3] & 0xffffffffu), want_crc = (uint32_t)((uint64_t)ix[3] >> 32);
    if ((!RING && isize > (uint32_t)WIN) || out_off < 0 || (uint64_t)out_off + isize > a.out_cap) {
        if (lane == 0) atomicOr(a.status, kInfRange);
        return;
    }
    uint8_t* const dst = a.out + out_off;
    constexpr uint32_t M = RING ? (uint32_t)WIN - 1u : 0xffffffffu;  // window index mask
    // bit reader: bb holds bc bits; pos = next ring byte; the ring holds [fill - kRing, fill)
    uint64_t bb = 0;
    int bc = 0;
    uint32_t pos = 0, fill = 0;
    auto refill = [&]() {  // the next kRing / 2 bytes (zeros past the end)
        for (int k = lane; k < kRing / 2; k += 64) {
            const uint32_t g = fill + (uint32_t)k;
            S.ring[g & (kRing - 1)] = g < in_len ? src[g] : 0;
        }
        fill += kRing / 2;
        __builtin_amdgcn_wave_barrier();
    };
    auto topup = [&]() {  // >= 33 bits in bb
        while (bc <= 32) {
            if (pos + 8u > fill) refill();
            const uint32_t* w = reinterpret_cast<const uint32_t*>(S.ring);
            const uint32_t q = (pos & (kRing - 1)) >> 2;
            const uint32_t v = uni(__builtin_amdgcn_alignbyte(w[(q + 1) & (kRing / 4 - 1)], w[q], pos & 3u));
            bb |= (uint64_t)v << bc;
            bc += 32;
            pos += 4;
        }
    };
    auto bits = [&](int n) -> uint32_t {  // n <= 32, bb holds >= n bits
        const uint32_t v = (uint32_t)(bb & ((1ull << n) - 1ull));
        bb >>= n;
        bc -= n;
        return v;
    };
    int err = 0;
    uint32_t p = 0;  // output bytes so far
    bool last = false;
    while (!last && !err) {
        if (pos > in_len + 16u) { err = kInfCorrupt; break; }  // past the data (zeros)
        topup();
        last = bits(1) != 0;
        const int type = (int)bits(2);
        if (type == 0) {  // stored: byte-align, LEN, NLEN, raw bytes
            bits(bc & 7);
            topup();
            const uint32_t len = bits(16), nlen = bits(16);
            if ((len ^ 0xffffu) != nlen || p + len > isize) { err = kInfCorrupt; break; }
            pos -= (uint32_t)(bc >> 3);  // hand the buffered whole bytes back to the ring
            bb = 0;
            bc = 0;
            uint32_t left = len;
            while (left) {
                if (pos + 64u > fill) refill();
                const uint32_t ch = min(left, 64u);
                if ((uint32_t)lane < ch) {
                    const uint8_t v = S.ring[(pos + lane) & (kRing - 1)];
                    S.win[(p + lane) & M] = v;
                    if (RING) dst[p + lane] = v;
                }
                __builtin_amdgcn_wave_barrier();
                p += ch;
                pos += ch;
                left -= ch;
            }
            continue;
        }
        if (type == 3) { err = kInfCorrupt; break; }
        if (type == 1) {  // fixed codes (RFC 1951 3.2.6)
            for (int i = lane; i < 320; i += 64)
                S.lens[i] = i < 144 ? 8 : i < 256 ? 9 : i < 280 ? 7 : i < 288 ? 8 : 5;
            __builtin_amdgcn_wave_barrier();
            inf_build(S.lit, S.lens, 288, kAlphaLit);
            inf_build(S.dist, S.lens + 288, 30, kAlphaDist);
            inf_build_pairs(S);
        } else {  // dynamic: code-length code, then the literal/length and distance lengths
            topup();
            const int nlit = (int)bits(5) + 257, ndist = (int)bits(5) + 1, ncl = (int)bits(4) + 4;
            if (nlit > 286 || ndist > 30) { err = kInfCorrupt; break; }
            for (int i = lane; i < 19; i += 64) S.lens[i] = 0;
            __builtin_amdgcn_wave_barrier();
            for (int i = 0; i < ncl; ++i) {
                topup();
                const uint32_t v = bits(3);
                if (lane == 0) S.lens[c_clord[i]] = (uint8_t)v;
            }
            __builtin_amdgcn_wave_barrier();
            if (!inf_build(S.lit, S.lens, 19, kAlphaPlain)) { err = kInfCorrupt; break; }
            const int total = nlit + ndist;
            int i = 0;
            while (i < total) {
                topup();
                const uint32_t ce = inf_decode(S.lit, bb, bc, kAlphaPlain);
                if (ce & 0x300u) { err = kInfCorrupt; break; }
                const int sy = (int)(ce >> 16);
                if (sy < 16) {
                    if (lane == 0) S.lens[i] = (uint8_t)sy;
                    ++i;
                    continue;
                }
                int rep, val = 0;
                if (sy == 16) {
                    if (i == 0) { err = kInfCorrupt; break; }
                    val = (int)uni(S.lens[i - 1]);
                    rep = 3 + (int)bits(2);
                } else if (sy == 17) {
                    rep = 3 + (int)bits(3);
                } else {
                    rep = 11 + (int)bits(7);
                }
                if (i + rep > total) { err = kInfCorrupt; break; }
                __builtin_amdgcn_wave_barrier();
                for (int k = lane; k < rep; k += 64) S.lens[i + k] = (uint8_t)val;
                __builtin_amdgcn_wave_barrier();
                i += rep;
            }
            if (err) break;
            __builtin_amdgcn_wave_barrier();
            if (uni(S.lens[256]) == 0) { err = kInfCorrupt; break; }
            // the distance lengths move out of the literal range before the builds
            const uint8_t dl = lane < ndist ? S.lens[nlit + lane] : 0;
            __builtin_amdgcn_wave_barrier();
            for (int k = nlit + lane; k < 288; k += 64) S.lens[k] = 0;
            __builtin_amdgcn_wave_barrier();
            if (lane < 32) S.lens[288 + lane] = lane < ndist ? dl : 0;
            __builtin_amdgcn_wave_barrier();
            if (!inf_build(S.lit, S.lens, nlit, kAlphaLit) || !inf_build(S.dist, S.lens + 288, ndist, kAlphaDist)) {
                err = kInfCorrupt;
                break;
            }
            inf_build_pairs(S);
        }
        // symbols of the block
        for (;;) {
            topup();
            if constexpr (PAIR) {
                const uint32_t pe = uni(S.pair[bb & (uint64_t)(kPair - 1)]);
                if (pe >> 30) {  // a whole copy from one lookup
                    const uint32_t nb = pe & 31u, len = (pe >> 5) & 511u, d = (pe >> 14) & 0xffffu;
                    bb >>= nb;
                    bc -= (int)nb;
                    if (d > p) { err = kInfCorrupt; break; }
                    if (p + len > isize) { err = kInfSize; break; }
                    __builtin_amdgcn_wave_barrier();
                    if ((!RING || d + len <= (uint32_t)WIN) && len <= 64u) {
                        if ((uint32_t)lane < len) {
                            const uint32_t k = (uint32_t)lane;
                            const uint8_t v = S.win[(p - d + (d >= len ? k : k % d)) & M];
                            S.win[(p + k) & M] = v;
                            if (RING) dst[p + k] = v;
                        }
                    } else if (!RING || d + len <= (uint32_t)WIN) {
                        for (uint32_t k = lane; k < len; k += 64) {
                            const uint8_t v = S.win[(p - d + (d >= len ? k : k % d)) & M];
                            S.win[(p + k) & M] = v;
                            if (RING) dst[p + k] = v;
                        }
                    } else {
                        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
                        for (uint32_t k = lane; k < len; k += 64) {
                            const uint8_t v = dst[p - d + k];
                            S.win[(p + k) & M] = v;
                            dst[p + k] = v;
                        }
                    }
                    __builtin_amdgcn_wave_barrier();
                    p += len;
                    continue;
                }
            }
            const uint32_t e = inf_decode(S.lit, bb, bc, kAlphaLit);
            const uint32_t kind = (e >> 8) & 3u;
            if (kind == kKindLit) {
                if (p >= isize) { err = kInfSize; break; }
                if (lane == 0) {
                    S.win[p & M] = (uint8_t)(e >> 16);
                    if (RING) dst[p] = (uint8_t)(e >> 16);
                }
                ++p;
            } else if (kind == kKindEnd) {
                break;
            } else {
                if (kind == kKindBad) { err = kInfCorrupt; break; }
                const uint32_t len = (e >> 16) + bits((int)((e >> 4) & 15u));
                topup();
                const uint32_t f = inf_decode(S.dist, bb, bc, kAlphaDist);
                if (((f >> 8) & 3u) != kKindCopy) { err = kInfCorrupt; break; }
                const uint32_t d = (f >> 16) + bits((int)((f >> 4) & 15u));
                if (d > p) { err = kInfCorrupt; break; }
                if (p + len > isize) { err = kInfSize; break; }
                __builtin_amdgcn_wave_barrier();
                if ((!RING || d + len <= (uint32_t)WIN) && len <= 64u) {  // one lane per byte, no loop
                    if ((uint32_t)lane < len) {
                        const uint32_t k = (uint32_t)lane;
                        const uint8_t v = S.win[(p - d + (d >= len ? k : k % d)) & M];
                        S.win[(p + k) & M] = v;
                        if (RING) dst[p + k] = v;
                    }
                } else if (!RING || d + len <= (uint32_t)WIN) {  // the source is in the window
                    if (d >= len) {
                        for (uint32_t k = lane; k < len; k += 64) {
                            const uint8_t v = S.win[(p - d + k) & M];
                            S.win[(p + k) & M] = v;
                            if (RING) dst[p + k] = v;
                        }
                    } else {
                        for (uint32_t k = lane; k < len; k += 64) {
                            const uint8_t v = S.win[(p - d + k % d) & M];
                            S.win[(p + k) & M] = v;
                            if (RING) dst[p + k] = v;
                        }
                    }
                } else {  // ring only: further back than the ring (d > WIN - len >= len)
                    // the source bytes are this wavefront's earlier global stores
                    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
                    for (uint32_t k = lane; k < len; k += 64) {
                        const uint8_t v = dst[p - d + k];
                        S.win[(p + k) & M] = v;
                        dst[p + k] = v;
                    }
                }
                __builtin_amdgcn_wave_barrier();
                p += len;
            }
        }
    }
    // every byte of the deflate data used, none past it; the whole ISIZE produced
    if (!err && (pos - (uint32_t)(bc >> 3) != in_len)) err = kInfCorrupt;
    if (!err && p != isize) err = kInfSize;
    if (err) {
        if (lane == 0) atomicOr(a.status, err);
        return;
    }
    __builtin_amdgcn_wave_barrier();
    if (RING) __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");  // the CRC reads the stores back
    // CRC-32 of the output, checked here: lane l takes bytes [l sg, (l+1) sg)
    // of the output seen as the tail of 64 sg bytes (leading zeros leave a
    // zero-initialised CRC unchanged), bitwise (vector work beside the other
    // waves' scalar-bound decode), then a tree over the lanes whose level-l
    // shift (sg 2^l bytes) is the same for every lane.  The ring decoder
    // reads its own stores back (same-address order within a wavefront).
    {
        int lg = 0;
        while ((64ull << lg) < (uint64_t)isize) ++lg;
        const int64_t sg = 1ll << lg;
        const int64_t b0 = (int64_t)lane * sg - (int64_t)((64ull << lg) - isize);
        uint32_t r = 0;
        const bool vec = RING && sg >= 16 && ((reinterpret_cast<uintptr_t>(dst) | isize) & 15u) == 0;
        if (vec) {  // b0 is a multiple of 16 here
            for (int64_t i = b0 < 0 ? 0 : b0; i < b0 + sg; i += 64) {
                uint4 w[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) w[k] = i + 16 * k < b0 + sg ? reinterpret_cast<const uint4*>(dst + i)[k] : make_uint4(0, 0, 0, 0);
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (i + 16 * k < b0 + sg) {
                        r = crc_word(r, w[k].x); r = crc_word(r, w[k].y);
                        r = crc_word(r, w[k].z); r = crc_word(r, w[k].w);
                    }
            }
        } else {
            for (int64_t i = b0 < 0 ? 0 : b0; i < b0 + sg; ++i) r = crc_byte(r, RING ? dst[i] : S.win[i]);
        }
#pragma unroll
        for (int l = 0; l < 6; ++l) {
            const uint32_t x = (uint32_t)__shfl_xor((int)r, 1 << l, 64);
            const uint32_t sh = crc_adv_pow2(r, lg + l);
            r = (lane & (1 << l)) ? r : (sh ^ x);
        }
        if (lane == 0 && (crc_adv(0xffffffffu, isize) ^ r ^ 0xffffffffu) != want_crc) atomicOr(a.status, kInfCrc);
    }
    if (RING) return;  // already stored as produced
    __builtin_amdgcn_wave_barrier();
    if (((reinterpret_cast<uintptr_t>(dst) | isize) & 15u) == 0) {
        const uint4* w = reinterpret_cast<const uint4*>(S.win);
        for (uint32_t i = lane; i < isize / 16u; i += 64) reinterpret_cast<uint4*>(dst)[i] = w[i];
    } else {
        for (uint32_t i = lane; i < isize; i += 64) dst[i] = S.win[i];
    }
}


// ============================================================================
// TLZ: token-LZ gzip of rank arrays (GZIPTransformer.forward,
// kc_pipeline.py:128-141, skc_pipeline.py:201-215, stc_pipeline.py:185-199)
// and its lane-parallel inflate (GZIPTransformer.backward,
// kc_pipeline.py:152-156: gzip.decompress).
//
// Format: a multi-member gzip stream (RFC 1952).  A member covers up to
// kMemTok float32 ranks (512 KiB of input) as ONE dynamic-Huffman deflate
// block (RFC 1951) over the whole 32 KiB window, whose copies are whole
// tokens: 12..256 bytes (3..64 float32 values) at distances that are
// multiples of 4 bytes; a value without a copy is its 4 literal bytes.  The
// member's values are cut into segments of kSeg; no copy crosses a segment
// end, so a decoder can start at any segment: an RFC 1952 extra subfield
// 'OZ' in the member header holds the bit offset (from the first bit of the
// deflate data) of every segment's first symbol.  gzip.decompress, zlib and
// any gzip reader skip the subfield and read the member as plain deflate.
//   header (28 + 4 nseg bytes): 1f 8b 08 04 | mtime 0 | xfl 0 | os ff | XLEN |
//     'O' 'Z' | LEN | version 1 | log2(kSeg) | nseg (u16) | member bytes (u32)
//     | values (u32) | nseg x u32 segment bit offsets
//   deflate data (one block, BFINAL = 1, BTYPE = 2) | CRC-32 | ISIZE
//
// Encoder (k_tlz_encode, one 512-thread block per member, a segment at a
// time): 3-gram chains (per-wave ballot matching, then the waves' and the
// earlier segments' last occurrences), the longest-match frontier of every
// position over kCand (12) chain candidates (1 <= 3 (length, distance)
// pairs), an optimal parse by a segmented backward DP (each thread its 4
// positions, the other threads' costs from the previous sweep, 4 sweeps)
// under a cost model re-estimated from the member's symbol counts after every
// segment, the DP's path followed by Jacobi rounds (every thread walks its 4
// positions from its left neighbour's exit until no entry changes), then one
// Huffman code per member and the bits.  The parse is what gzip -9 lacks: 0.115 of the input
// on KC ranks against gzip -9's 0.117 (tools/tlz_proto.c simulates it).
// Decoder: k_tlz_ops (one wavefront per member, one lane per segment:
// Huffman decode from the segment's bit offset with the member's tables in
// LDS; each lane writes its segment's ops into that segment's own output
// bytes) and k_tlz_resolve (one block per member, a segment at a time: op
// positions by a block scan, every value's source by pointer jumping in LDS
// against the window of earlier values, then the values, CRC-32, ISIZE).
namespace tlz {
constexpr int kNT = 512;                           // encoder threads per member block
constexpr int kSegLog = 11, kSeg = 1 << kSegLog;   // values per segment
constexpr int kMemSeg = 64;
constexpr int kMemTok = kSeg * kMemSeg;            // values per member
constexpr int kPer = kSeg / kNT;                   // positions per thread
constexpr int kWin = 8192;                         // window, values (32 KiB)
constexpr int kMaxL = 64, kMinL = 3;               // copy length, values
#ifndef OFL_TLZ_CAND
// 11 chain candidates (round 5, after the DP rework made the frontier the
// largest phase): KC gzip phase 12.5 -> 12.1 ms per GiB for ratio 0.1165 ->
// 0.1167 (10: 11.9 ms, 0.1170; gzip -9: 0.1171-0.1174;
// profiles/r05_tlz_cand_sweep_ab.txt).  Round 4: 12 instead of 16, encode
// 14.0 -> 12.8 ms (profiles/r04_tlz_cand_ab2.txt)
#define OFL_TLZ_CAND 11
#endif
#ifndef OFL_TLZ_SWEEPS
#define OFL_TLZ_SWEEPS 4
#endif
constexpr int kCand = OFL_TLZ_CAND;                // chain candidates per position (A/B: -DOFL_TLZ_CAND)
constexpr int kBuckets = 512;                      // 3-gram buckets: exact for values < 8, hashed (into the same) above
constexpr int kBucketBits = 9;
static_assert(kBuckets == 1 << kBucketBits, "bucket ids are kBucketBits wide");
constexpr int kSweeps = OFL_TLZ_SWEEPS;            // DP sweeps (segments of kPer = 4 positions; tools/tlz_proto.c)
constexpr int kRing = 16384;                       // value ring (ids), + 8 mirrored bytes
constexpr int kLitMax = 11, kDistMax = 10;         // code length limits = the inflate's table bits
constexpr int kHdrFixed = 28;                      // member header bytes before the segment table
constexpr uint16_t kPending = 0xffffu;
constexpr int kSlotPerTok = 6;                     // worst-case member bytes per value (4 literals x 11 bits)
constexpr int kSlotPad = 8192;                     // + headers
constexpr int kBatch = 512;                        // members per launch

struct EncSmem {
    alignas(16) uint8_t tok[kRing + 32];      // + the first 32 bytes again (a candidate's 20-byte read)
    union {
        struct {
            uint16_t prev[kRing];                  // distance to the previous same-bucket position (0: none), by position mod kRing
            union {
                uint16_t lastw[kNT / 64][kBuckets];  // chains: per wave, this segment: position - range start + 1
                uint32_t cost[2][kSeg + 8];        // then the DP's costs to the segment end, 1/8 bit
                uint32_t hw[kNT / 64][(kLit + kDist + 1) / 2];  // then per-wave symbol counts of the segment, two u16 per word
            };
        } m;
        struct {
            HScratch h;
            uint32_t hdrw[kHdrW];
            uint8_t hb[kHdrFixed + 4 * kMemSeg];
            // the bit emission's tables (code | extra bits) << 0 | n << 24:
            // a literal value's first two and last two bytes, a copy length
            uint32_t litlo[32], lithi[32], lenw[kMaxL + 1];
        } f;
    } u;
    uint32_t head[2][kBuckets];                    // last position + 1 per bucket (earlier segments); segment c reads [c & 1], writes [~c & 1]
    uint16_t dec[kSeg];                            // chosen op: length (0: literal) | frontier entry << 8
    uint16_t entry[kNT + 1];                       // parse: each thread's first position
    uint32_t hl[kLit], hd[kDist], hc[kCL];
    uint32_t totl, totd;
    uint16_t symc[kLit + kDist];
    uint16_t litc[32], lenc[kMaxL + 1], dcst[kDist];
    uint8_t ll[kLit], ld[kDist], lc[kCL];
    uint16_t kl[kLit], kd[kDist], kc[kCL];
    uint32_t crct[1][256];                         // CRC-32 byte table (the word tables went to the DP's 32-bit costs)
    uint32_t adv13[8][16];                         // CRC advance by a segment's 8 KiB, per input nibble
    uint32_t cid4[kPer][32];                       // raw CRC of a thread's 16 bytes with only value q = id (from 0)
    uint32_t segop[kMemSeg + 1], segbit[kMemSeg];
    uint32_t scan[kNT / 64];
    uint32_t crc_w[kNT / 64];
    uint32_t ops_n, crc_raw, hdr_bits, total_bits, nrle, nlit_ndist;
    int bad;
    // fused k-means labelling (EncArgs::lab): the records of tensors lab_t0 ..
    // lab_t0 + 3 (start = end = INT64_MAX past the last); positions below
    // lab_hi lie in one of them or in no tensor
    int32_t lab_t0;
    int64_t lab_s[4], lab_e[4], lab_hi;
    float lab_m[4][8], lab_r[4][8];
};
static_assert(sizeof(EncSmem) <= 80 * 1024, "two member blocks per CU");

struct EncArgs {
    const float* x;
    int64_t n;
    int64_t mem0;            // first member of this launch
    uint8_t* slots;          // [members][slot_bytes]
    uint32_t* ops;           // [members][ops_stride]
    uint32_t* sizes;         // [members]
    int* bad;
    uint32_t slot_bytes, ops_stride;
    int aligned;             // x is 16-byte aligned
    uint64_t* phases;        // diagnostics (OFL_GZ_PHASES): block 0's time per phase (10 ns ticks), else null
    const ofl_label_rec* lab;  // non-null: x holds values, labelled through these records as they load
    int32_t lab_n;
};
constexpr int kEncPhases = 16;

// k-means label of one value (k_bkm_label's rule, lossy_kernels.hip)
DEVI float lab_rank(float v, const float* m, const float* r) {
    float o = r[0];
#pragma unroll
    for (int j = 0; j < 7; ++j) o = v > m[j] ? r[j + 1] : o;
    return o;
}
// wave 0: the label window for a segment starting at s0 -- the first tensor
// ending after s0 (64-way search from the previous window, ends ascending)
// and the three after it
DEVI void lab_fill(const EncArgs& a, EncSmem& S, int64_t s0, int lane) {
    int lo = S.lab_t0, hi = a.lab_n;
    while (lo < hi) {
        const int stride = (hi - lo + 63) >> 6;
        const int i = lo + lane * stride;
        const int cnt = __popcll(__ballot(i < hi && a.lab[i].end <= s0));
        if (cnt == 0) break;
        const int nlo = lo + (cnt - 1) * stride + 1;
        hi = min(lo + cnt * stride, hi);
        lo = nlo;
    }
    if (lane < 4) {
        const int t = lo + lane;
        if (t < a.lab_n) {
            const ofl_label_rec r = a.lab[t];
            S.lab_s[lane] = r.start;
            S.lab_e[lane] = r.end;
#pragma unroll
            for (int j = 0; j < 8; ++j) { S.lab_m[lane][j] = r.mid[j]; S.lab_r[lane][j] = r.rank[j]; }
        } else {
            S.lab_s[lane] = S.lab_e[lane] = INT64_MAX;
        }
    }
    if (lane == 0) {
        S.lab_t0 = lo;
        S.lab_hi = lo + 4 < a.lab_n ? a.lab[lo + 4].start : INT64_MAX;
    }
}
// the label of the value v at arena position g (any position of the segment)
DEVI float lab_one(const EncArgs& a, const EncSmem& S, int64_t g, float v) {
    const int sl = (g >= S.lab_s[1]) + (g >= S.lab_s[2]) + (g >= S.lab_s[3]);
    if (g >= S.lab_s[sl] && g < S.lab_e[sl]) return lab_rank(v, S.lab_m[sl], S.lab_r[sl]);
    if (g < S.lab_hi) return 0.f;  // between tensors
    int lo = S.lab_t0 + 4, hi = a.lab_n - 1;  // past the window (> 4 tensors in this segment): last start <= g
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (a.lab[mid].start <= g) lo = mid; else hi = mid - 1;
    }
    const ofl_label_rec& r = a.lab[lo];
    return g >= r.start && g < r.end ? lab_rank(v, r.mid, r.rank) : 0.f;
}

DEVI int pslot(int p) { return p & (kRing - 1); }
// the DP's costs live modulo 2^16: all candidates of one position lie within
// 64 values of each other, < 64 x 4 literals x 15 bits x 8 < 2^15 apart
DEVI bool lt16(uint32_t a, uint32_t b) { return (int16_t)(uint16_t)(a - b) < 0; }
DEVI uint32_t tk4r(const uint8_t* tok, int p) {
    const int r = p & (kRing - 1);
    const uint32_t* w = reinterpret_cast<const uint32_t*>(tok);
    return __builtin_amdgcn_alignbyte(w[(r >> 2) + 1], w[r >> 2], (uint32_t)(r & 3));
}
// 3-gram bucket: exact for values < 8 (512 buckets), hashed into the same
// 512 above (a collision only adds chain entries the comparison rejects)
DEVI int bucket(const uint8_t* tok, int p) {
    const uint32_t v = tk4r(tok, p) & 0xffffffu;
    const uint32_t a = v & 0xffu, b = (v >> 8) & 0xffu, c = v >> 16;
    if ((a | b | c) < 8u) return (int)(a | (b << 3) | (c << 6));
    return (int)(((a | (b << 5) | (c << 10)) * 0x9E3779B1u) >> (32 - kBucketBits));
}
DEVI int match_len(const uint8_t* tok, int i, int j, int lim) {
    int L = 0;
    while (L < lim) {
        const uint32_t x = tk4r(tok, i + L) ^ tk4r(tok, j + L);
        if (x) { L += __builtin_ctz(x) >> 3; break; }
        L += 4;
    }
    return min(L, lim);
}
// raw CRC-32 of one little-endian word, a byte at a time (T: the byte table);
// used only at set-up and for a member's partial last piece
DEVI uint32_t crc4(const uint32_t (*T)[256], uint32_t c, uint32_t w) {
    c ^= w;
#pragma unroll
    for (int i = 0; i < 4; ++i) c = (c >> 8) ^ T[0][c & 0xffu];
    return c;
}
// 1/8 bit: -log2(count / total) >= 1 bit, an unseen symbol log2(total + 1) + 2
// bits, at most 15 bits
DEVI uint32_t sym_cost(uint32_t cnt, uint32_t tot) {
    const float v = cnt ? 8.f * (__log2f((float)tot) - __log2f((float)cnt))
                        : 8.f * (__log2f((float)tot + 1.f) + 2.f);
    return (uint32_t)fminf(120.f, fmaxf(8.f, rintf(v)));
}
// per-symbol costs -> the DP's tables: a literal value (its 4 bytes), a copy
// length (code + extra bits), a distance code (+ extra bits)
DEVI void tlz_model(EncSmem& S, int tid, bool prior) {
    for (int s = tid; s < kLit + kDist; s += kNT) {
        uint32_t c;
        if (prior) c = s < 256 ? 48u : s < kLit ? 32u : 40u;
        else c = s < kLit ? sym_cost(S.hl[s], S.totl) : sym_cost(S.hd[s - kLit], S.totd);
        S.symc[s] = (uint16_t)c;
    }
    __syncthreads();
    if (tid < 32) {
        const uint32_t b = __float_as_uint((float)tid);
        S.litc[tid] = (uint16_t)(S.symc[b & 0xffu] + S.symc[(b >> 8) & 0xffu] + S.symc[(b >> 16) & 0xffu] + S.symc[b >> 24]);
    } else if (tid < 32 + kMaxL + 1) {
        const int l = tid - 32;
        if (l >= kMinL) {
            const int lc = len_code(4u * (uint32_t)l);
            S.lenc[l] = (uint16_t)(S.symc[257 + lc] + 8u * c_lext[lc]);
        } else {
            S.lenc[l] = 0;
        }
    } else if (tid < 32 + kMaxL + 1 + kDist) {
        const int c = tid - 32 - kMaxL - 1;
        S.dcst[c] = (uint16_t)(S.symc[kLit + c] + 8u * c_dext[c]);
    }
    __syncthreads();
}
// block-wide exclusive scan of v over NT threads (returns the exclusive prefix; *total)
template <int NT>
DEVI uint32_t block_scan(uint32_t v, uint32_t* scan, uint32_t* total) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    uint32_t inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = (uint32_t)__shfl_up((int)inc, o, 64);
        if (lane >= o) inc += t;
    }
    if (lane == 63) scan[w] = inc;
    __syncthreads();
    uint32_t base = 0, tot = 0;
#pragma unroll
    for (int j = 0; j < NT / 64; ++j) {
        base += j < w ? scan[j] : 0u;
        tot += scan[j];
    }
    __syncthreads();
    *total = tot;
    return base + inc - v;
}

__global__ __launch_bounds__(kNT) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_tlz_encode(EncArgs a) {  // 2 blocks per CU: 4 waves per SIMD
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    EncSmem& S = *reinterpret_cast<EncSmem*>(smem_raw);
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    uint64_t ph_t = 0, ph_acc[kEncPhases] = {};
    const bool ph_on = a.phases && blockIdx.x == 0 && tid == 0;
    // (diagnostics: a barrier before every mark, so a phase's time is its
    // slowest wave's, not wave 0's; launch-uniform condition)
    auto PH = [&](int k) {
        if (a.phases) __syncthreads();
        if (ph_on) { const uint64_t t = wall_clock64(); if (k > 0) ph_acc[k] += t - ph_t; ph_t = t; }
    };
    PH(0);
    const int64_t g0 = (a.mem0 + blockIdx.x) * (int64_t)kMemTok;
    const int ntok = (int)min<int64_t>(kMemTok, a.n - g0);
    const int nseg = (ntok + kSeg - 1) >> kSegLog;
    uint32_t* const ops = a.ops + (int64_t)blockIdx.x * a.ops_stride;
    if (tid < 256) {
        uint32_t r = (uint32_t)tid;
        for (int k = 0; k < 8; ++k) r = (r & 1u) ? (r >> 1) ^ 0xEDB88320u : r >> 1;
        S.crct[0][tid] = r;
    } else if (tid < 256 + 128) {  // the per-segment CRC advance as nibble tables
        const int e = tid - 256, j = e >> 4, v = e & 15;
        uint32_t r = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) r ^= ((v >> b) & 1) ? c_adv[kSegLog + 2][4 * j + b] : 0u;
        S.adv13[j][v] = r;
    }
    for (int i = tid; i < kBuckets; i += kNT) {
        S.head[0][i] = S.head[1][i] = 0;
#pragma unroll
        for (int w = 0; w < kNT / 64; ++w) S.u.m.lastw[w][i] = 0;
    }
    for (int i = tid; i < kLit; i += kNT) S.hl[i] = 0;
    if (tid < kDist) S.hd[tid] = 0;
    if (tid < kCL) S.hc[tid] = 0;
    if (tid == 0) { S.totl = S.totd = 0; S.ops_n = 0; S.crc_raw = 0; S.bad = 0; S.lab_t0 = 0; S.lab_hi = INT64_MIN; }
    __syncthreads();
    // the raw CRC is linear: a thread's 16 bytes (4 values, ids < 32) hash to
    // the XOR of one table entry per value, 4 independent reads instead of
    // 16 dependent ones
    if (tid < kPer * 32) {
        const int q = tid >> 5;
        const uint32_t bits = __float_as_uint((float)(tid & 31));
        uint32_t cr = 0;
#pragma unroll
        for (int k = 0; k < kPer; ++k) cr = crc4(S.crct, cr, k == q ? bits : 0u);
        S.cid4[q][tid & 31] = cr;
    }
    __syncthreads();
    tlz_model(S, tid, true);

    uint32_t crc_acc = 0, crc_last = 0;
    int nv_last = 0;
    for (int c = 0; c < nseg; ++c) {
        // thread-derived values recomputed every segment from an opaque tid
        // (hoisted out of the loop, they were spilled and reloaded instead)
        uint32_t tid_o = threadIdx.x;
        asm volatile("" : "+v"(tid_o));
        const int tid = (int)tid_o, lane = tid & 63, wv = tid >> 6;
        const int c0 = c << kSegLog;
        const int send = min(c0 + kSeg, ntok);
        const int lo = c0 + kPer * tid;                 // this thread's positions [lo, lo + kPer)
        if (a.lab) {  // a new label window when this segment reaches past the current one
            const int64_t lab_hi = S.lab_hi;
            if (g0 + send > lab_hi) {
                __syncthreads();
                if (wv == 0) lab_fill(a, S, g0 + c0, lane);
                __syncthreads();
            }
        }
        // ---- A: values -> ids in the ring, validity, raw CRC-32 ----
        uint32_t idw[kPer / 4] = {};                    // this thread's ids, packed 4 per word
        {
            const int nv = max(0, min(kPer, send - lo));
            float v[kPer];
            if (nv == kPer && a.aligned) {
                const float4* p = reinterpret_cast<const float4*>(a.x + g0 + lo);
#pragma unroll
                for (int u = 0; u < kPer / 4; ++u) {
                    const float4 v0 = p[u];
                    v[4 * u] = v0.x; v[4 * u + 1] = v0.y; v[4 * u + 2] = v0.z; v[4 * u + 3] = v0.w;
                }
            } else {
#pragma unroll
                for (int q = 0; q < kPer; ++q) v[q] = q < nv ? a.x[g0 + lo + q] : 0.f;
            }
            if (a.lab) {  // values -> ranks (the k-means labels the rank array would hold)
                const int64_t gp = g0 + lo;
                const int sl = (gp >= S.lab_s[1]) + (gp >= S.lab_s[2]) + (gp >= S.lab_s[3]);
                if (nv == kPer && gp >= S.lab_s[sl] && gp + kPer <= S.lab_e[sl]) {  // one tensor (the common case)
                    float m[7], r[8];
#pragma unroll
                    for (int j = 0; j < 7; ++j) m[j] = S.lab_m[sl][j];
#pragma unroll
                    for (int j = 0; j < 8; ++j) r[j] = S.lab_r[sl][j];
#pragma unroll
                    for (int q = 0; q < kPer; ++q) v[q] = lab_rank(v[q], m, r);
                } else {
#pragma unroll
                    for (int q = 0; q < kPer; ++q)
                        if (q < nv) v[q] = lab_one(a, S, gp + q, v[q]);
                }
            }
            uint32_t crc = 0;
            bool bad = false;
#pragma unroll
            for (int q = 0; q < kPer; ++q) {
                if (q < nv) {
                    const int t = (int)v[q];
                    const uint32_t bits = __float_as_uint(v[q]);
                    if (!(t >= 0 && t < 32 && bits == __float_as_uint((float)t))) bad = true;
                    const uint32_t id = (t >= 0 && t < 32) ? (uint32_t)t : 0u;
                    idw[q >> 2] |= id << (8 * (q & 3));
                    crc ^= S.cid4[q][id];  // (a bad value fails the member: its CRC is never used)
                }
            }
            if (nv < kPer) {  // a partial last piece: the values' own chain
                crc = 0;
#pragma unroll
                for (int q = 0; q < kPer; ++q)
                    if (q < nv) crc = crc4(S.crct, crc, __float_as_uint(v[q]));
            }
            if (bad) atomicOr(&S.bad, 1);
            for (int b = tid; b < kBuckets; b += kNT)  // the chains' wave tables (they share memory with the DP's costs)
#pragma unroll
                for (int w2 = 0; w2 < kNT / 64; ++w2) S.u.m.lastw[w2][b] = 0;
            const int r = lo & (kRing - 1);
#pragma unroll
            for (int u = 0; u < kPer / 4; ++u) {
                reinterpret_cast<uint32_t*>(S.tok)[(r >> 2) + u] = idw[u];
                if (r + 4 * u < 32) reinterpret_cast<uint32_t*>(S.tok)[((kRing + r) >> 2) + u] = idw[u];
            }
            // raw CRC-32 by Horner per thread: acc covers this thread's pieces
            // of the full segments so far (each advanced by the 8 KiB of every
            // later segment); the last segment's piece and the combination
            // over the threads follow the loop
            if (c + 1 < nseg) {
                uint32_t adv = 0;
#pragma unroll
                for (int j = 0; j < 8; ++j) adv ^= S.adv13[j][(crc_acc >> (4 * j)) & 15u];
                crc_acc = adv ^ crc;
            }
            else crc_last = crc, nv_last = nv;
        }
        __syncthreads();
        if (S.bad) {  // block-uniform
            if (tid == 0) { atomicOr(a.bad, 1); a.sizes[blockIdx.x] = 0; }
            return;
        }
        PH(1);
        // ---- B: 3-gram chains of [c0 - 2, send - 2) (the last two of a
        // segment wait for the next segment's values) ----
        const int s_ins = c == 0 ? 0 : c0 - 2;
        const int e_ins = send - 2;
        const int m_ins = max(0, e_ins - s_ins);
        const int part = (m_ins + kNT - 1) / kNT * 64;
        const int w_lo = s_ins + wv * part, w_hi = min(e_ins, w_lo + part);
        for (int p0 = w_lo; p0 < w_hi; p0 += 64) {
            const int p = p0 + lane;
            const bool act = p < w_hi;
            const int bk = act ? bucket(S.tok, p) : 0;
            uint64_t m = __ballot(act);
#pragma unroll
            for (int b = 0; b < kBucketBits; ++b) {  // buckets < 2^kBucketBits
                const bool on = ((bk >> b) & 1) != 0;
                const uint64_t bb = __ballot(act && on);
                m &= on ? bb : ~bb;
            }
            const uint64_t below = m & ((1ull << lane) - 1ull);
            uint32_t d;
            if (below) {
                d = (uint32_t)(lane - (63 - __builtin_clzll(below)));
            } else {
                const uint32_t lw = act ? S.u.m.lastw[wv][bk] : 0u;
                d = lw ? (uint32_t)(p - (s_ins + (int)lw - 1)) : kPending;
            }
            if (act) {
                S.u.m.prev[pslot(p)] = (uint16_t)d;
                if ((m >> lane) == 1ull) S.u.m.lastw[wv][bk] = (uint16_t)(p - s_ins + 1);
            }
        }
        PH(12);
        __syncthreads();
        // per bucket, in place: an exclusive prefix max of the waves' last
        // occurrences (the nearest one in an earlier wave's part: parts are
        // in wave order), and the next segment's heads; then every pending
        // position takes its link with one read
        const uint32_t* head = S.head[c & 1];
        for (int b = tid; b < kBuckets; b += kNT) {
            uint32_t run = 0;
#pragma unroll
            for (int w2 = 0; w2 < kNT / 64; ++w2) {
                const uint32_t t = S.u.m.lastw[w2][b];
                S.u.m.lastw[w2][b] = (uint16_t)run;
                run = max(run, t);
            }
            S.head[(c + 1) & 1][b] = run ? (uint32_t)s_ins + run : head[b];
        }
        __syncthreads();
        for (int p0 = w_lo; p0 < w_hi; p0 += 64) {
            const int p = p0 + lane;
            if (p < w_hi && S.u.m.prev[pslot(p)] == kPending) {
                const int bk = bucket(S.tok, p);
                const uint32_t lw = S.u.m.lastw[wv][bk];
                const uint32_t h = head[bk];
                uint32_t d = 0;
                if (lw) d = (uint32_t)(p - (s_ins + (int)lw - 1));
                else if (h && p - (int)(h - 1u) <= kWin) d = (uint32_t)(p - (int)(h - 1u));
                S.u.m.prev[pslot(p)] = (uint16_t)d;
            }
        }
        // the frontier reads the chain links of every position, pending ones
        // resolved just above by other waves (without this barrier a wave
        // could read a link before its writer: valid output, but not
        // deterministic -- tools/tlz_check.py "det")
        __syncthreads();
        PH(2);
        // ---- C: each position's frontier of (length, distance) pairs ----
        uint32_t fa[kPer], fb[kPer], fc[kPer];  // entries: length | distance << 7 (lengths increasing)
        int nf[kPer];
        {
            // chain candidates in increasing distance, branch-free: a
            // candidate's first 8 values are compared at once (3 aligned LDS
            // dwords, the 4 positions' loads issued together); a match of 8
            // or more values walks further behind one wave-uniform test (12
            // values at once cost 4 % more encode time for the same stream)
            const uint32_t* tw = reinterpret_cast<const uint32_t*>(S.tok);
            constexpr int kCW = 2;  // values compared at once: 4 kCW
            uint32_t ti[kPer][kCW];  // values i .. i + 4 kCW - 1 of each position
            {
                const int rb = (lo & (kRing - 1)) >> 2;  // lo is a multiple of 8
                uint32_t w[kCW + 3];
#pragma unroll
                for (int k = 0; k < kCW + 3; ++k) w[k] = tw[rb + k];
#pragma unroll
                for (int q = 0; q < kPer; ++q)
#pragma unroll
                    for (int k = 0; k < kCW; ++k) ti[q][k] = __builtin_amdgcn_alignbyte(w[(q >> 2) + k + 1], w[(q >> 2) + k], (uint32_t)(q & 3));
            }
            int j[kPer], bl[kPer], lim[kPer];
            bool act[kPer];
#pragma unroll
            for (int q = 0; q < kPer; ++q) {
                const int i = lo + q;
                fa[q] = fb[q] = fc[q] = 0;
                bl[q] = kMinL - 1;  // an improvement is then also a copy of >= kMinL values
                lim[q] = min(kMaxL, send - i);
                const uint32_t pd = lim[q] >= kMinL ? S.u.m.prev[pslot(i)] : 0u;
                act[q] = pd != 0;
                j[q] = i - (int)pd;
            }
#pragma unroll 1
            for (int step = 0; step < kCand; ++step) {
                bool any = false;
#pragma unroll
                for (int h = 0; h < kPer; h += 4) {  // two halves: fewer loads in flight, fewer registers
                    uint32_t cw[4][kCW + 1], pd[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int q = h + u;
                        const int jj = act[q] ? j[q] : lo;
                        const int jb = (jj & (kRing - 1)) >> 2;
#pragma unroll
                        for (int k = 0; k <= kCW; ++k) cw[u][k] = tw[jb + k];
                        pd[u] = S.u.m.prev[pslot(jj)];
                    }
                    int Lq[4];
                    bool okq[4], longq[4];
                    bool anylong = false;
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int q = h + u;
                        const int i = lo + q;
                        const uint32_t sh = (uint32_t)(j[q] & 3);
                        int L = 4 * kCW;
#pragma unroll
                        for (int k = kCW - 1; k >= 0; --k) {
                            const uint32_t x = __builtin_amdgcn_alignbyte(cw[u][k + 1], cw[u][k], sh) ^ ti[q][k];
                            L = x ? 4 * k + (__builtin_ctz(x) >> 3) : L;
                        }
                        okq[u] = act[q] && i - j[q] <= kWin;
                        longq[u] = okq[u] && L == 4 * kCW && lim[q] > 4 * kCW;
                        anylong |= longq[u];
                        Lq[u] = L;
                    }
                    // rare: a long match walks on.  One wave-uniform test for
                    // the four positions (per-position divergent branches cost
                    // ~50 scalar instructions per step even when no lane took them)
                    if (__builtin_expect(__ballot(anylong) != 0ull, 0)) {
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            const int q = h + u;
                            if (longq[u])
                                Lq[u] = 4 * kCW + match_len(S.tok, lo + q + 4 * kCW, j[q] + 4 * kCW, lim[q] - 4 * kCW);
                        }
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int q = h + u;
                        const int i = lo + q;
                        const bool ok = okq[u];
                        const int L = min(Lq[u], lim[q]);
                        // branch-free (selects, no exec-mask juggling): the
                        // first two improvements go to fa and fb, and fc
                        // always takes the latest (the frontier's count is
                        // read off the three words after the walk)
                        const bool imp = ok && L > bl[q];
                        const uint32_t e = (uint32_t)L | ((uint32_t)(i - j[q]) << 7);
                        fb[q] = imp && fa[q] != 0u && fb[q] == 0u ? e : fb[q];
                        fa[q] = imp && fa[q] == 0u ? e : fa[q];
                        fc[q] = imp ? e : fc[q];
                        bl[q] = imp ? L : bl[q];
                        act[q] = ok && bl[q] < lim[q] && pd[u] != 0;
                        j[q] -= (int)pd[u];
                        any |= act[q];
                    }
                }
                if (!any) break;
            }
#pragma unroll
            for (int q = 0; q < kPer; ++q)  // 0..3 entries; fc repeats fa or fb below three
                nf[q] = fa[q] == 0u ? 0 : fb[q] == 0u ? 1 : fc[q] == fb[q] ? 2 : 3;
        }
        PH(3);
        // ---- D: segmented backward DP (kSweeps sweeps) ----
        // Costs are absolute (1/8 bit to the segment end, < 2^20: 2048 values
        // x 4 literals x 15 bits x 8), so a candidate is one 32-bit key
        // (cost << 3 | candidate index) and the best of a position is a plain
        // min: the index orders the candidates as the old strict-less scan
        // did (literal, lengths kMinL..kU, the three frontier entries), so
        // ties keep the earlier one and the parse is unchanged.  The sweep-
        // invariant part of every candidate is precomputed per position, 16
        // bits each (0xffff: no such candidate; a candidate's cost differs
        // from the literal's by < 3100, so it then never wins):
        //   cA[q] = literal | length 3 << 16, cB[q] = 4 | 5 << 16,
        //   cC[q] = 6 | entry a << 16, cD[q] = entry b | entry c << 16;
        //   a length l: its length + distance cost; an entry (its own length
        //   > kU): l | cost << 7, 0 = none
        uint32_t dc3[kPer];
#pragma unroll
        for (int q = 0; q < kPer; ++q) {
            const uint32_t da = nf[q] > 0 ? min(255u, (uint32_t)S.dcst[dist_code(4u * (fa[q] >> 7))]) : 0u;
            const uint32_t db = nf[q] > 1 ? min(255u, (uint32_t)S.dcst[dist_code(4u * (fb[q] >> 7))]) : 0u;
            const uint32_t dc = nf[q] > 2 ? min(255u, (uint32_t)S.dcst[dist_code(4u * (fc[q] >> 7))]) : 0u;
            dc3[q] = da | (db << 8) | (dc << 16);
        }
        __syncthreads();  // the wave tables are dead: the DP's costs take their memory
        for (int k = tid; k <= kSeg; k += kNT) {
            const int rem = max(0, send - c0 - k);
            S.u.m.cost[1][k] = 32u * (uint32_t)rem;  // sweep 0's estimate beyond a thread's positions: 4 bits per value
            if (k >= send - c0) S.u.m.cost[0][k] = 0;
        }
        __syncthreads();
        const int klo = kPer * tid;  // segment-relative
        {
            // own positions' costs in registers (indices are compile-time
            // after unrolling); lengths kMinL..kU branch-free, longer ones
            // only as the frontier entries' own lengths, whose costs beyond
            // this thread's positions come from the previous sweep
            constexpr int kU = 6;              // lengths unrolled: kMinL .. kU (longer: only the entries' own lengths; the same ratio, tools/tlz_proto.c)
            constexpr int kW = kU;             // costs beyond this thread's positions within reach
            static_assert(kU == 6 && kMinL == 3, "the packed candidate table holds lengths 3..6");
            constexpr uint32_t kNone = 0xffffu;
            uint32_t lenr[kU + 1];
#pragma unroll
            for (int l = kMinL; l <= kU; ++l) lenr[l] = S.lenc[l];
            uint32_t cA[kPer], cB[kPer], cC[kPer], cD[kPer];
            bool live[kPer];
#pragma unroll
            for (int q = 0; q < kPer; ++q) {
                const uint32_t lit = min(511u, (uint32_t)S.litc[(idw[q >> 2] >> (8 * (q & 3))) & 0xffu]);
                const int La = (int)(fa[q] & 127u), Lb = (int)(fb[q] & 127u);
                const int Lm = nf[q] == 0 ? 0 : (int)((nf[q] == 1 ? fa[q] : nf[q] == 2 ? fb[q] : fc[q]) & 127u);
                live[q] = c0 + klo + q < send;
                uint32_t lc[kU + 1];
#pragma unroll
                for (int l = kMinL; l <= kU; ++l) {
                    const uint32_t e = l <= La ? 0u : l <= Lb ? 1u : 2u;
                    lc[l] = l <= Lm ? lenr[l] + ((dc3[q] >> (8 * e)) & 255u) : kNone;
                }
                uint32_t E[3];
#pragma unroll
                for (int e = 0; e < 3; ++e) {
                    const int l = e == 0 ? La : e == 1 ? Lb : Lm;
                    const bool use = l > kU && l <= Lm && nf[q] > e;
                    const uint32_t dcost = (dc3[q] >> (8 * e)) & 255u;
                    E[e] = use ? (uint32_t)l | (min(511u, (uint32_t)S.lenc[l] + dcost) << 7) : 0u;
                }
                cA[q] = lit | (lc[3] << 16);
                cB[q] = lc[4] | (lc[5] << 16);
                cC[q] = lc[6] | (E[0] << 16);
                cD[q] = E[1] | (E[2] << 16);
            }
#pragma unroll 1
            for (int sw = 0; sw < kSweeps; ++sw) {
                uint32_t* cur = S.u.m.cost[sw & 1];
                const uint32_t* prv = S.u.m.cost[(sw + 1) & 1];
                uint32_t pw[kW + 1];
#pragma unroll
                for (int u = 0; u <= kW; ++u) pw[u] = prv[min(klo + kPer + u, kSeg)];
                // the frontier entries read costs of the previous sweep only:
                // their reads are issued here, before the chain, unconditionally
                // (el = 0 reads the position's own cost, then discarded:
                // behind a branch each cost ~5 scalar instructions of exec
                // juggling), and each position's best entry key is formed
                uint32_t me[kPer];
#pragma unroll
                for (int h = 0; h < kPer; h += 2) {  // two positions' six reads at a time (registers)
                    uint32_t pe[2][3];
#pragma unroll
                    for (int u = 0; u < 2; ++u)
#pragma unroll
                        for (int e = 0; e < 3; ++e) {
                            const int q = h + u;
                            const uint32_t En = e == 0 ? (cC[q] >> 16) : e == 1 ? (cD[q] & 0xffffu) : (cD[q] >> 16);
                            pe[u][e] = prv[min(klo + q + (int)(En & 127u), kSeg)];
                        }
                    asm volatile("" : "+v"(pe[0][0]), "+v"(pe[0][1]), "+v"(pe[0][2]), "+v"(pe[1][0]), "+v"(pe[1][1]),
                                 "+v"(pe[1][2]));
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        const int q = h + u;
                        me[q] = 0xffffffffu;
#pragma unroll
                        for (int e = 0; e < 3; ++e) {
                            const uint32_t En = e == 0 ? (cC[q] >> 16) : e == 1 ? (cD[q] & 0xffffu) : (cD[q] >> 16);
                            const uint32_t cc = (((En >> 7) + pe[u][e]) << 3) | (uint32_t)(5 + e);
                            me[q] = min(me[q], (En & 127u) != 0u ? cc : 0xffffffffu);
                        }
                    }
                }
                uint32_t cr[kPer], key[kPer];
#pragma unroll
                for (int q = kPer - 1; q >= 0; --q) {
                    auto CV = [&](int kk) -> uint32_t { return kk < kPer ? cr[kk] : pw[kk - kPer]; };  // kk = q + l
                    uint32_t best = min((((cA[q] & 0xffffu) + CV(q + 1)) << 3), me[q]);
                    best = min(best, (((cA[q] >> 16) + CV(q + 3)) << 3) | 1u);
                    best = min(best, (((cB[q] & 0xffffu) + CV(q + 4)) << 3) | 2u);
                    best = min(best, (((cB[q] >> 16) + CV(q + 5)) << 3) | 3u);
                    best = min(best, (((cC[q] & 0xffffu) + CV(q + 6)) << 3) | 4u);
                    cr[q] = live[q] ? best >> 3 : 0u;
                    key[q] = best;
                }
                // (a position past the segment's values stores 0: its cost already)
#pragma unroll
                for (int q = 0; q < kPer; ++q) cur[klo + q] = cr[q];
                if (sw == kSweeps - 1) {  // the choices: length | frontier entry << 8 (0: literal)
#pragma unroll
                    for (int q = 0; q < kPer; ++q) {
                        if (!live[q]) continue;
                        const uint32_t k = key[q] & 7u;
                        uint32_t ch = 0;
                        if (k >= 5u) {
                            const uint32_t ent = k == 5u ? fa[q] : k == 6u ? fb[q] : fc[q];
                            ch = (ent & 127u) | ((k - 5u) << 8);
                        } else if (k >= 1u) {
                            const uint32_t l = k + 2u, La = fa[q] & 127u, Lb = fb[q] & 127u;
                            ch = l | ((l <= La ? 0u : l <= Lb ? 1u : 2u) << 8);
                        }
                        S.dec[klo + q] = (uint16_t)ch;
                    }
                }
                __syncthreads();
            }
        }
        PH(4);
        // ---- E: the DP's path from the segment start: Jacobi rounds ----
        auto nxt = [&](int p) -> int { const int l = S.dec[p - c0] & 0xff; return p + (l ? l : 1); };
        for (int i = tid; i < (kNT / 64) * ((kLit + kDist + 1) / 2); i += kNT) (&S.u.m.hw[0][0])[i] = 0;  // F's tables (the DP's costs are dead)
        {
            int p = tid == 0 ? c0 : max(c0, lo - kMaxL);
            while (p < lo && p < send) p = nxt(p);
            S.entry[tid] = (uint16_t)(p - c0);
        }
        __syncthreads();
#pragma unroll 1
        for (;;) {
            int p = c0 + S.entry[tid];
            while (p < lo + kPer && p < send) p = nxt(p);
            __syncthreads();
            int changed = 0;
            if (tid + 1 < kNT && (int)S.entry[tid + 1] != p - c0) { S.entry[tid + 1] = (uint16_t)(p - c0); changed = 1; }
            if (ph_on) ++ph_acc[11];
            if (!__syncthreads_or(changed)) break;
        }
        PH(5);
        // ---- F: this segment's ops, in order; symbol counts ----
        {
            uint32_t opm = 0;
            for (int p = c0 + S.entry[tid]; p < lo + kPer && p < send; p = nxt(p)) opm |= 1u << (p - lo);
            PH(13);
            uint32_t tot;
            const uint32_t off = block_scan<kNT>((uint32_t)__popc(opm), S.scan, &tot);
            PH(14);
            const uint32_t base = S.ops_n;
            uint32_t k = base + off;
            uint32_t nl = 0, nd = 0;
            // symbol counts into this wave's own table (same-wave atomics only)
            uint32_t* const hw = S.u.m.hw[wv];
            auto cnt = [&](int sym) { atomicAdd(&hw[sym >> 1], (sym & 1) ? 0x10000u : 1u); };
#pragma unroll
            for (int q = 0; q < kPer; ++q) {
                if (!((opm >> q) & 1u)) continue;
                const uint32_t dq = S.dec[klo + q];
                const uint32_t l = dq & 0xffu;
                uint32_t rec;
                if (l == 0) {
                    const uint32_t id = (idw[q >> 2] >> (8 * (q & 3))) & 0xffu;
                    rec = 0x80000000u | id;
                    const uint32_t b = __float_as_uint((float)id);
#pragma unroll
                    for (int y = 0; y < 4; ++y) cnt((int)((b >> (8 * y)) & 0xffu));
                    nl += 4;
                } else {
                    const uint32_t e = dq >> 8;
                    const uint32_t ent = e == 0 ? fa[q] : e == 1 ? fb[q] : fc[q];
                    const uint32_t d = ent >> 7;
                    rec = l | (d << 7);
                    cnt(257 + len_code(4u * l));
                    cnt(kLit + dist_code(4u * d));
                    nl += 1;
                    nd += 1;
                }
                ops[k++] = rec;
            }
            for (int o = 32; o > 0; o >>= 1) {
                nl += (uint32_t)__shfl_xor((int)nl, o, 64);
                nd += (uint32_t)__shfl_xor((int)nd, o, 64);
            }
            if (lane == 0) { atomicAdd(&S.totl, nl); atomicAdd(&S.totd, nd); }
            if (tid == 0) S.segop[c] = base;
            __syncthreads();
            if (tid == 0) S.ops_n = base + tot;
            for (int sym = tid; sym < kLit + kDist; sym += kNT) {  // merge the waves' counts
                uint32_t v = 0;
#pragma unroll
                for (int w = 0; w < kNT / 64; ++w) v += (S.u.m.hw[w][sym >> 1] >> (16 * (sym & 1))) & 0xffffu;
                if (sym < kLit) S.hl[sym] += v; else S.hd[sym - kLit] += v;
            }
        }
        PH(6);
        __syncthreads();  // the merged counts
        if (c + 1 < nseg) tlz_model(S, tid, false);
        PH(7);
    }

    {  // the member's raw CRC-32: every thread's pieces advanced to the member's end, XOR-ed
        const uint32_t bl = 4u * (uint32_t)(ntok - ((nseg - 1) << kSegLog));  // bytes of the last segment
        uint32_t r = nv_last ? crc_adv(crc_last, bl - 4u * kPer * (uint32_t)tid - 4u * (uint32_t)nv_last) : 0u;
        if (nseg > 1) r ^= crc_adv(crc_acc, (uint32_t)(kSeg * 4) + bl - 4u * kPer * (uint32_t)(tid + 1));
        for (int o = 32; o > 0; o >>= 1) r ^= (uint32_t)__shfl_xor((int)r, o, 64);
        if (lane == 0) S.crc_w[wv] = r;
        __syncthreads();
        if (tid == 0) {
            uint32_t x = 0;
            for (int w = 0; w < kNT / 64; ++w) x ^= S.crc_w[w];
            S.crc_raw = x;
        }
    }
    // ---- G: the member's Huffman code (lengths limited to the inflate's table bits) ----
    const int ln = lane;
    if (wv == 0) {
        HScratch& h = S.u.f.h;
        if (ln == 0) S.hl[256] = 1;  // end of block
        __builtin_amdgcn_wave_barrier();
        if (!huff_lengths_wave(S.hl, kLit, kLitMax, S.ll, h.w, true) && ln == 0) huff_lengths(S.hl, kLit, kLitMax, S.ll, h, true);
    } else if (wv == 1) {
        HScratch& h = S.u.f.h;
        const bool anyd = __ballot(ln < kDist && S.hd[ln] != 0u) != 0ull;
        if (!anyd && ln == 0) S.hd[0] = 1;  // one (unused) distance code
        __builtin_amdgcn_wave_barrier();
        huff_lengths_wave(S.hd, kDist, kDistMax, S.ld, reinterpret_cast<uint32_t*>(h.rle_ext), false);
    }
    __syncthreads();
    if (wv == 1) huff_codes_wave(S.ll, kLit, S.kl);
    if (wv == 2) huff_codes_wave(S.ld, kDist, S.kd);
    if (wv == 0) {  // run-length code of the code lengths (as RFC 1951 3.2.7)
        HScratch& h = S.u.f.h;
        int nlit = 257, ndist = 1;
        for (int cc = 0; cc < (kLit + 63) / 64; ++cc) {
            const int i = 64 * cc + ln;
            const uint64_t m = __ballot(i < kLit && S.ll[i] != 0);
            if (m) nlit = max(nlit, 64 * cc + 64 - __builtin_clzll(m));
        }
        {
            const uint64_t m = __ballot(ln < kDist && S.ld[ln] != 0);
            if (m) ndist = max(ndist, 64 - __builtin_clzll(m));
        }
        const int N = nlit + ndist;
        auto val = [&](int i) -> int { return i < nlit ? S.ll[i] : S.ld[i - nlit]; };
        uint64_t starts[(kLit + kDist + 63) / 64];
#pragma unroll
        for (int cc = 0; cc < (kLit + kDist + 63) / 64; ++cc) {
            const int i = 64 * cc + ln;
            starts[cc] = __ballot(i < N && (i == 0 || val(i) != val(i - 1)));
        }
        if (ln == 0) {
            int nr = 0, cc = 0, s0 = 0;
            uint64_t m = starts[0];
            m &= m - 1;
            for (;;) {
                while (!m && cc + 1 < (kLit + kDist + 63) / 64) m = starts[++cc];
                const int s1 = m ? 64 * cc + __builtin_ctzll(m) : N;
                if (m) m &= m - 1;
                const int cur = val(s0);
                int left = s1 - s0;
                if (cur == 0) {
                    while (left >= 11) { const int r = left < 138 ? left : 138; h.rle_sym[nr] = 18; h.rle_ext[nr++] = (uint16_t)(r - 11); left -= r; }
                    if (left >= 3) { h.rle_sym[nr] = 17; h.rle_ext[nr++] = (uint16_t)(left - 3); left = 0; }
                    while (left > 0) { h.rle_sym[nr] = 0; h.rle_ext[nr++] = 0; --left; }
                } else {
                    h.rle_sym[nr] = (uint16_t)cur; h.rle_ext[nr++] = 0; --left;
                    while (left >= 3) { const int r = left < 6 ? left : 6; h.rle_sym[nr] = 16; h.rle_ext[nr++] = (uint16_t)(r - 3); left -= r; }
                    while (left > 0) { h.rle_sym[nr] = (uint16_t)cur; h.rle_ext[nr++] = 0; --left; }
                }
                if (s1 >= N) break;
                s0 = s1;
            }
            for (int i = 0; i < nr; ++i) S.hc[h.rle_sym[i]]++;
            S.nrle = (uint32_t)nr;
            S.nlit_ndist = (uint32_t)(nlit | (ndist << 16));
        }
    }
    __syncthreads();
    if (wv == 0) {
        HScratch& h = S.u.f.h;
        huff_lengths_wave(S.hc, kCL, 7, S.lc, h.w, true);
        huff_codes_wave(S.lc, kCL, S.kc);
    }
    if (tid == 0) {  // the deflate block header's bits (words of the member's data start)
        HScratch& h = S.u.f.h;
        const int nr = (int)S.nrle, nlit = (int)(S.nlit_ndist & 0xffffu), ndist = (int)(S.nlit_ndist >> 16);
        int ncl = kCL;
        while (ncl > 4 && S.lc[c_clord[ncl - 1]] == 0) --ncl;
        uint64_t acc = 0;
        int nb = 0;
        uint32_t wi = 0, pos = 0;
        auto put = [&](uint32_t v, int n) {
            acc |= (uint64_t)v << nb;
            nb += n;
            pos += (uint32_t)n;
            if (nb >= 32) { S.u.f.hdrw[wi++] = (uint32_t)acc; acc >>= 32; nb -= 32; }
        };
        put(1u, 1);  // BFINAL
        put(2u, 2);  // BTYPE = dynamic
        put((uint32_t)(nlit - 257), 5);
        put((uint32_t)(ndist - 1), 5);
        put((uint32_t)(ncl - 4), 4);
        for (int i = 0; i < ncl; ++i) put(S.lc[c_clord[i]], 3);
        for (int i = 0; i < nr; ++i) {
            const int sy = h.rle_sym[i];
            put(S.kc[sy], S.lc[sy]);
            const int eb = sy == 16 ? 2 : (sy == 17 ? 3 : (sy == 18 ? 7 : 0));
            put(h.rle_ext[i], eb);
        }
        if (nb > 0) S.u.f.hdrw[wi] = (uint32_t)acc;
        S.hdr_bits = pos;
    }
    __syncthreads();

    PH(8);
    // ---- H: bits of the ops (a block scan of their costs), segment offsets ----
    // every op's code and extra bits come from small LDS tables (a literal
    // value: its four codes in two words; a length: code | extra bits) and
    // the distance's code index and extra bits by arithmetic
    if (tid < 32) {
        const uint32_t bb = __float_as_uint((float)tid);
        uint32_t v[2] = {0, 0}, n[2] = {0, 0};
#pragma unroll
        for (int y = 0; y < 4; ++y) {
            const uint32_t by = (bb >> (8 * y)) & 0xffu;
            v[y >> 1] |= (uint32_t)S.kl[by] << n[y >> 1];
            n[y >> 1] += S.ll[by];
        }
        S.u.f.litlo[tid] = v[0] | (n[0] << 24);
        S.u.f.lithi[tid] = v[1] | (n[1] << 24);
    } else if (tid >= 64 && tid < 64 + kMaxL + 1) {
        const int l = tid - 64;
        uint32_t w = 0;
        if (l >= kMinL) {
            int lc, ne;
            uint32_t ev;
            len_sym(4u * (uint32_t)l, lc, ne, ev);
            const uint32_t cl = S.ll[257 + lc];
            w = ((uint32_t)S.kl[257 + lc] | (ev << cl)) | ((cl + (uint32_t)ne) << 24);
        }
        S.u.f.lenw[l] = w;
    }
    __syncthreads();
    const uint32_t nops = S.ops_n, H = S.hdr_bits;
    const uint32_t o_lo = (uint32_t)((uint64_t)nops * tid / kNT), o_hi = (uint32_t)((uint64_t)nops * (tid + 1) / kNT);
    auto dist_w = [&](uint32_t dv) -> uint32_t {  // code | extra bits, n << 24 (n <= 10 + 13)
        int dc, ne;
        uint32_t ev;
        dist_sym(4u * dv, dc, ne, ev);
        const uint32_t cd = S.ld[dc];
        return ((uint32_t)S.kd[dc] | (ev << cd)) | ((cd + (uint32_t)ne) << 24);
    };
    auto op_bits = [&](uint32_t rec) -> uint32_t {
        if (rec >> 31) return (S.u.f.litlo[rec & 31u] >> 24) + (S.u.f.lithi[rec & 31u] >> 24);
        return (S.u.f.lenw[rec & 127u] >> 24) + (dist_w(rec >> 7) >> 24);
    };
    uint32_t mine = 0;
#pragma unroll 4
    for (uint32_t o = o_lo; o < o_hi; ++o) mine += op_bits(ops[o]);
    uint32_t tot;
    const uint32_t pos0 = H + block_scan<kNT>(mine, S.scan, &tot);
    if (tid == 0) S.total_bits = H + tot;
    const uint32_t D = (uint32_t)(kHdrFixed + 4 * nseg);  // header bytes (a multiple of 4)
    uint32_t* const slot = reinterpret_cast<uint32_t*>(a.slots + (int64_t)blockIdx.x * a.slot_bytes);
    uint32_t* const dw = slot + D / 4;                    // the deflate data's words
    {
        const uint32_t nw = (H + tot + 15u + 7u + 64u + 31u) / 32u + 1u;
        for (uint32_t i = tid; i < nw; i += kNT) dw[i] = 0;
    }
    __syncthreads();
    if (tid == 0)
        for (uint32_t i = 0; i < (H + 31u) / 32u; ++i) atomicOr(&dw[i], S.u.f.hdrw[i]);
    {
        // the segments whose first op lies in this thread's range get their
        // bit offset here, as the emission passes that op
        int sidx = 0;
        while (sidx < nseg && S.segop[sidx] < o_lo) ++sidx;
        uint32_t next_seg = sidx < nseg ? S.segop[sidx] : 0xffffffffu;
        uint64_t acc = 0;
        int nb = (int)(pos0 & 31u);
        uint32_t wi = pos0 >> 5;
        bool first = true;
        auto put = [&](uint32_t w) {  // code | extra bits, n << 24 (n <= 24)
            acc |= (uint64_t)(w & 0xffffffu) << nb;
            nb += (int)(w >> 24);
            if (nb >= 32) {
                if (first) { atomicOr(&dw[wi], (uint32_t)acc); first = false; }
                else dw[wi] = (uint32_t)acc;
                ++wi;
                acc >>= 32;
                nb -= 32;
            }
        };
#pragma unroll 2
        for (uint32_t o = o_lo; o < o_hi; ++o) {
            if (o == next_seg) {
                S.segbit[sidx++] = 32u * wi + (uint32_t)nb;
                next_seg = sidx < nseg ? S.segop[sidx] : 0xffffffffu;
            }
            const uint32_t rec = ops[o];
            if (rec >> 31) {
                put(S.u.f.litlo[rec & 31u]);
                put(S.u.f.lithi[rec & 31u]);
            } else {
                put(S.u.f.lenw[rec & 127u]);
                put(dist_w(rec >> 7));
            }
        }
        if (nb > 0) atomicOr(&dw[wi], (uint32_t)acc);
    }
    __syncthreads();
    // ---- I: end of block, CRC-32, ISIZE, the member header ----
    if (tid == 0) {
        uint32_t p = S.total_bits;
        put_bits(dw, p, S.kl[256], S.ll[256]);
        p += S.ll[256];
        p = (p + 7u) & ~7u;
        const uint32_t crc32 = crc_adv(0xffffffffu, 4u * (uint32_t)ntok) ^ S.crc_raw ^ 0xffffffffu;
        put_bits(dw, p, crc32, 32);
        p += 32;
        put_bits(dw, p, 4u * (uint32_t)ntok, 32);
        p += 32;
        const uint32_t bytes = D + p / 8u;
        uint8_t* hb = S.u.f.hb;
        const uint32_t len = 12u + 4u * (uint32_t)nseg, xlen = 4u + len;
        const uint8_t fixed[16] = {0x1f, 0x8b, 0x08, 0x04, 0, 0, 0, 0, 0x00, 0xff, (uint8_t)xlen, (uint8_t)(xlen >> 8),
                                   'O', 'Z', (uint8_t)len, (uint8_t)(len >> 8)};
        for (int i = 0; i < 16; ++i) hb[i] = fixed[i];
        hb[16] = 1;
        hb[17] = (uint8_t)kSegLog;
        hb[18] = (uint8_t)nseg;
        hb[19] = (uint8_t)(nseg >> 8);
        for (int i = 0; i < 4; ++i) {
            hb[20 + i] = (uint8_t)(bytes >> (8 * i));
            hb[24 + i] = (uint8_t)((uint32_t)ntok >> (8 * i));
        }
        for (int s = 0; s < nseg; ++s)
            for (int i = 0; i < 4; ++i) hb[kHdrFixed + 4 * s + i] = (uint8_t)(S.segbit[s] >> (8 * i));
        for (uint32_t i = 0; i < D / 4; ++i) slot[i] = reinterpret_cast<const uint32_t*>(hb)[i];
        a.sizes[blockIdx.x] = bytes;
    }
    PH(9);
    if (ph_on)
        for (int k = 0; k < kEncPhases; ++k) a.phases[k] = ph_acc[k];
}

// ---- inflate --------------------------------------------------------------
constexpr int kDecLitBits = kLitMax, kDecDistBits = kDistMax;
using DecLit = InfCodeT<kDecLitBits, 288>;
using DecDist = InfCodeT<kDecDistBits, 32>;
struct DecSmem {
    DecLit lit;
    DecDist dist;
    uint8_t lens[320];
};
struct DecArgs {
    // device stream: readable, and already landed, 64 bytes past every
    // member's trailer (BitIn's look-ahead at the end bound; the pipelined
    // inflate launches a member only once the H2D piece holding its end plus
    // those 64 bytes has landed, lossy.gunzip_device / _INFLATE_LOOKAHEAD;
    // the last piece is followed by 128 bytes of padding)
    const uint8_t* src;
    const int64_t* idx;      // per member: data offset, data length | kind << 62, output offset, isize | crc << 32
    int64_t nmem;
    uint8_t* out;
    uint64_t out_cap;
    uint32_t* cnt;           // [nmem][kMemSeg] ops per segment
    int* status;
    // the fused LUT decode (k_tlz_resolve<true>): the values stored are
    // lut_tab[t][rank] for the element's tensor t (elements [lut_start[t],
    // lut_end[t]) of the stream's float32 output, sorted); elements between
    // tensors store the rank itself
    const float* lut_tab;
    const int64_t* lut_start;
    const int64_t* lut_end;
    int32_t lut_n;
    int32_t dbg;             // diagnostics (OFL_TLZ_DEC_STATS): timing printf of every 256th member
};

// bytes of the stream (any alignment) through a 128-bit block register pair
struct BitIn {
    const uint4* base;       // 16-byte aligned
    uint4 cur, nxt;
    int64_t blk;             // block index of cur
    int wi;                  // next word of cur
    uint64_t bb;
    int bc;
    DEVI uint32_t word(int k) const { return k == 0 ? cur.x : k == 1 ? cur.y : k == 2 ? cur.z : cur.w; }
    DEVI void start(const uint8_t* src, uint64_t bit) {  // src 16-byte aligned
        base = reinterpret_cast<const uint4*>(src);
        blk = (int64_t)(bit >> 7);
        cur = base[blk];
        nxt = base[blk + 1];
        wi = (int)((bit >> 5) & 3u);
        const int sk = (int)(bit & 31u);
        bb = (uint64_t)(word(wi) >> sk);
        bc = 32 - sk;
        adv();
        fill();
    }
    DEVI void adv() {
        if (++wi == 4) { cur = nxt; ++blk; nxt = base[blk + 1]; wi = 0; }
    }
    DEVI void fill() {  // >= 33 bits in bb
        while (bc <= 32) {
            bb |= (uint64_t)word(wi) << bc;
            bc += 32;
            adv();
        }
    }
    DEVI uint32_t peek() const { return (uint32_t)bb; }
    DEVI void drop(int n) { bb >>= n; bc -= n; }
    DEVI uint32_t get(int n) { const uint32_t v = (uint32_t)(bb & ((1ull << n) - 1ull)); drop(n); return v; }
    DEVI uint64_t pos() const { return (uint64_t)(blk * 128 + wi * 32) - (uint64_t)bc; }
};

// K1: one wavefront per member; the block header on all lanes (wave-uniform),
// then lane s decodes segment s's symbols into op records written over that
// segment's own output bytes (kSeg values = 8 KiB >= 4 bytes per op).
__global__ __launch_bounds__(64) void k_tlz_ops(DecArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    DecSmem& S = *reinterpret_cast<DecSmem*>(smem_raw);
    const int lane = threadIdx.x;
    const int64_t m = blockIdx.x;
    if (m >= a.nmem) return;
    const int64_t* ix = a.idx + 4 * m;
    const int64_t doff = ix[0];
    const uint32_t in_len = (uint32_t)ix[1];
    const int64_t out_off = ix[2];
    const uint32_t isize = (uint32_t)((uint64_t)ix[3] & 0xffffffffu);
    const uint8_t* data = a.src + doff;
    const uint32_t ntok = isize / 4u;
    const int nseg = (int)((ntok + kSeg - 1) >> kSegLog);
    int err = 0;
    if ((isize & 3u) || ntok == 0 || nseg > kMemSeg || (out_off & 3) || (uint64_t)out_off + isize > a.out_cap) err = kInfRange;
    // the 'OZ' subfield ends where the deflate data starts
    const uint8_t* oz = data - 4 * nseg - 16;
    if (!err) {
        auto u32at = [&](const uint8_t* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24); };
        if (oz[0] != 'O' || oz[1] != 'Z' || oz[4] != 1 || oz[5] != kSegLog || ((uint32_t)oz[6] | ((uint32_t)oz[7] << 8)) != (uint32_t)nseg ||
            u32at(oz + 12) != ntok)
            err = kInfCorrupt;
    }
    if (err) {
        if (lane == 0) atomicOr(a.status, err);
        return;
    }
    auto seg_bit = [&](int s) -> uint32_t {
        const uint8_t* p = data - 4 * nseg + 4 * s;
        return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
    };
    const uint64_t dbit = 8ull * (uint64_t)doff;  // the data's first bit in the stream
    // the segment table is untrusted input: every entry must lie inside the
    // member's data and the entries must increase, or no lane may start a
    // decoder there (a bad entry would send BitIn far outside the stream)
    const uint64_t ebit = dbit + 8ull * (uint64_t)in_len;  // one past the data's last bit
    {
        const uint32_t sb = lane < nseg ? seg_bit(lane) : 0u;
        const uint32_t sp = lane > 0 && lane < nseg ? seg_bit(lane - 1) : 0u;
        const bool bad = lane < nseg && ((uint64_t)sb >= 8ull * (uint64_t)in_len || (lane > 0 && sb <= sp));
        if (__ballot(bad)) {
            if (lane == 0) atomicOr(a.status, kInfCorrupt);
            return;
        }
    }
    const uint64_t t_start = a.dbg ? wall_clock64() : 0;
    // ---- the block header, on every lane (wave-uniform) ----
    BitIn in;
    in.start(a.src, dbit);
    if (in.get(1) != 1u || in.get(2) != 2u) err = kInfCorrupt;  // BFINAL, dynamic
    int nlit = 0, ndist = 0;
    if (!err) {
        nlit = (int)in.get(5) + 257;
        ndist = (int)in.get(5) + 1;
        const int ncl = (int)in.get(4) + 4;
        if (nlit > 286 || ndist > 30) err = kInfCorrupt;
        for (int i = lane; i < 19; i += 64) S.lens[i] = 0;
        __builtin_amdgcn_wave_barrier();
        for (int i = 0; i < ncl && !err; ++i) {
            in.fill();
            const uint32_t v = in.get(3);
            if (lane == 0) S.lens[c_clord[i]] = (uint8_t)v;
        }
        __builtin_amdgcn_wave_barrier();
        if (!err && !inf_build(S.lit, S.lens, 19, kAlphaPlain)) err = kInfCorrupt;
        const int total = nlit + ndist;
        int i = 0;
        while (!err && i < total) {
            if (in.pos() > ebit) { err = kInfCorrupt; break; }  // ran past the data (wave-uniform)
            in.fill();
            const uint32_t e = S.lit.fast[in.peek() & (uint32_t)(DecLit::kSize - 1)];
            const int l = (int)(e & 15u);
            if (!l || (e & 0x300u)) { err = kInfCorrupt; break; }
            in.drop(l);
            const int sy = (int)(e >> 16);
            if (sy < 16) {
                if (lane == 0) S.lens[i] = (uint8_t)sy;
                ++i;
                continue;
            }
            int rep, val = 0;
            if (sy == 16) {
                if (i == 0) { err = kInfCorrupt; break; }
                __builtin_amdgcn_wave_barrier();
                val = S.lens[i - 1];
                rep = 3 + (int)in.get(2);
            } else if (sy == 17) {
                rep = 3 + (int)in.get(3);
            } else {
                rep = 11 + (int)in.get(7);
            }
            if (i + rep > total) { err = kInfCorrupt; break; }
            __builtin_amdgcn_wave_barrier();
            for (int k = lane; k < rep; k += 64) S.lens[i + k] = (uint8_t)val;
            __builtin_amdgcn_wave_barrier();
            i += rep;
        }
        __builtin_amdgcn_wave_barrier();
        if (!err) {
            // every code must fit the first-level tables (the encoder limits them)
            bool longc = false;
            for (int k = lane; k < total; k += 64) longc |= S.lens[k] > (k < nlit ? kDecLitBits : kDecDistBits);
            if (__ballot(longc) || S.lens[256] == 0) err = kInfCorrupt;
        }
        if (!err) {
            const uint8_t dl = lane < ndist ? S.lens[nlit + lane] : 0;
            __builtin_amdgcn_wave_barrier();
            for (int k = nlit + lane; k < 288; k += 64) S.lens[k] = 0;
            __builtin_amdgcn_wave_barrier();
            if (lane < 32) S.lens[288 + lane] = lane < ndist ? dl : 0;
            __builtin_amdgcn_wave_barrier();
            if (!inf_build(S.lit, S.lens, nlit, kAlphaLit) || !inf_build(S.dist, S.lens + 288, ndist, kAlphaDist)) err = kInfCorrupt;
        }
        if (!err && in.pos() != dbit + seg_bit(0)) err = kInfCorrupt;  // the ops start where the table says
    }
    if (err) {
        if (lane == 0) atomicOr(a.status, err);
        return;
    }
    __builtin_amdgcn_wave_barrier();
    const uint64_t t_hdr = a.dbg ? wall_clock64() : 0;
    // ---- lane s: segment s ----
    const int s = lane;
    if (s < nseg) {
        const uint32_t T = min((uint32_t)kSeg, ntok - ((uint32_t)s << kSegLog));
        uint32_t* const opo = reinterpret_cast<uint32_t*>(a.out + out_off + ((int64_t)s << (kSegLog + 2)));
        in.start(a.src, dbit + seg_bit(s));
        uint32_t produced = 0, nops = 0;
        const uint32_t before = (uint32_t)s << kSegLog;  // values of the member before this segment
        // op records are collected four at a time and stored as one 16-byte
        // write: every lane writes its own segment's region, so a store
        // instruction is 64 scattered transactions, and one per record made
        // the stores the kernel's limit
        uint32_t b0 = 0, b1 = 0, b2 = 0, b3 = 0;
        const bool al16 = (reinterpret_cast<uintptr_t>(opo) & 15u) == 0;
        auto emit = [&](uint32_t rec) {
            const uint32_t k = nops & 3u;
            b0 = k == 0 ? rec : b0;
            b1 = k == 1 ? rec : b1;
            b2 = k == 2 ? rec : b2;
            b3 = k == 3 ? rec : b3;
            if (k == 3) {
                if (al16) {
                    reinterpret_cast<uint4*>(opo)[nops >> 2] = make_uint4(b0, b1, b2, b3);
                } else {  // a member whose output does not start 16-byte aligned
                    opo[nops - 3] = b0; opo[nops - 2] = b1; opo[nops - 1] = b2; opo[nops] = b3;
                }
            }
            ++nops;
        };
        // a corrupt segment must not decode on past its member: the lane
        // stops once its bit window's block passes the data's last block + 1
        // (reads stay within ~48 bytes past the data; the stream is padded
        // for that), checked on the block index instead of the bit position
        const int64_t blim = (int64_t)(ebit >> 7) + 1;
        while (produced < T) {
            if (in.blk > blim) { err = kInfCorrupt; break; }
            in.fill();
            uint32_t e = S.lit.fast[in.peek() & (uint32_t)(DecLit::kSize - 1)];
            int l = (int)(e & 15u);
            if (!l) { err = kInfCorrupt; break; }
            in.drop(l);
            uint32_t kind = (e >> 8) & 3u;
            if (kind == (uint32_t)kKindLit) {  // a value's 4 literal bytes
                uint32_t bytes = e >> 16;
                in.fill();
#pragma unroll
                for (int y = 1; y < 4; ++y) {
                    e = S.lit.fast[in.peek() & (uint32_t)(DecLit::kSize - 1)];
                    l = (int)(e & 15u);
                    if (!l || ((e >> 8) & 3u) != (uint32_t)kKindLit) { err = kInfCorrupt; break; }
                    in.drop(l);
                    bytes |= (e >> 16) << (8 * y);
                }
                if (err) break;
                const float f = __uint_as_float(bytes);
                const int id = (int)f;
                if (!(id >= 0 && id < 32 && __float_as_uint((float)id) == bytes)) { err = kInfCorrupt; break; }
                emit(0x80000000u | (uint32_t)id);
                produced += 1;
            } else if (kind == (uint32_t)kKindCopy) {
                const uint32_t len = (e >> 16) + in.get((int)((e >> 4) & 15u));
                in.fill();
                const uint32_t f = S.dist.fast[in.peek() & (uint32_t)(DecDist::kSize - 1)];
                const int l2 = (int)(f & 15u);
                in.drop(l2);  // (l2 == 0 or a wrong kind fails below, before anything is used)
                const uint32_t d = (f >> 16) + in.get((int)((f >> 4) & 15u));
                const uint32_t lt = len >> 2, dt = d >> 2;
                // every check at once: one branch out instead of one per test
                const bool bad = (l2 == 0) | (((f >> 8) & 3u) != (uint32_t)kKindCopy) | (((len | d) & 3u) != 0u) |
                                 (lt - (uint32_t)kMinL > (uint32_t)(kMaxL - kMinL)) | (produced + lt > T) |
                                 (dt > before + produced) | (dt > (uint32_t)kWin);
                if (bad) { err = kInfCorrupt; break; }
                emit(lt | (dt << 7));
                produced += lt;
            } else {
                err = kInfCorrupt;
                break;
            }
        }
        if (!err) {
            if (s + 1 < nseg) {
                if (in.pos() != dbit + seg_bit(s + 1)) err = kInfCorrupt;
            } else {  // end of block, then the data ends at the next byte boundary
                in.fill();
                const uint32_t e = S.lit.fast[in.peek() & (uint32_t)(DecLit::kSize - 1)];
                const int l = (int)(e & 15u);
                if (!l || ((e >> 8) & 3u) != (uint32_t)kKindEnd) err = kInfCorrupt;
                else {
                    in.drop(l);
                    if ((in.pos() - dbit + 7u) / 8u != in_len) err = kInfCorrupt;
                }
            }
        }
        {  // the last < 4 records
            const uint32_t k = nops & 3u, q = nops & ~3u;
            if (k > 0) opo[q] = b0;
            if (k > 1) opo[q + 1] = b1;
            if (k > 2) opo[q + 2] = b2;
        }
        a.cnt[m * kMemSeg + s] = nops;
        if (err) atomicOr(a.status, err);
        if (a.dbg && (m & 255) == 0) {
            uint32_t dt = (uint32_t)(wall_clock64() - t_hdr), no = nops;
            for (int o = 32; o > 0; o >>= 1) {
                dt = max(dt, (uint32_t)__shfl_xor((int)dt, o, 64));
                no = max(no, (uint32_t)__shfl_xor((int)no, o, 64));
            }
            if (lane == 0)
                printf("tlz_ops m=%lld hdr_ticks=%u lanes_max_ticks=%u lane0_ops=%u max_ops=%u\n", (long long)m,
                       (uint32_t)(t_hdr - t_start), dt, nops, no);
        }
    }
}

// K2: one block per member; per segment: op positions (block scan), each
// value's source (pointer jumping in LDS; sources before the segment are in
// the value ring), the values as float32, CRC-32 of the member, ISIZE.
constexpr int kRNT = 256, kRPer = kSeg / kRNT;     // resolve: threads per member block, values per thread
constexpr int kLutSlots = 4;                       // fused LUT: tensor tables per segment in LDS
// resolve's CRC advances: table i advances by 2^(5 + i) bytes for i < 7 (a
// thread's 32 bytes .. a wave's 2 KiB), table 7 by a segment's 8 KiB
static_assert(kSegLog == 11, "resolve's CRC tables assume 2048-value segments");
static_assert(kRPer * 32 == kRNT, "one thread per (value slot, id) entry of the resolve's CRC table");
DEVI int adv_k(int i) { return i < 7 ? 5 + i : 13; }
// the resolve's value ring: the window and one segment (LDS per block decides
// how many member blocks share a CU: 4 at < 40 KiB)
constexpr uint32_t kVRing = kWin + kSeg;
struct ResSmem {
    uint32_t adv[8][8][16];        // CRC advance by 2^adv_k(i) bytes, per input nibble (table form of c_adv)
    uint32_t cid[kRPer][32];       // raw CRC of a thread's 32 bytes with only value q = id (from 0)
    alignas(16) uint8_t v[kVRing];  // ids by member position mod kVRing
    uint32_t opr[kSeg];            // the segment's op records
    alignas(16) uint16_t e[kSeg];   // 0x8000 | id (resolved) or the distance to the source
    uint32_t cnt[kMemSeg];         // ops per segment (k_tlz_ops)
    uint32_t crct[1][256];
    uint32_t scan[kRNT / 64];
    uint32_t crc_w[kRNT / 64];
    uint32_t crc_raw;
    float lt[kLutSlots][32];       // fused LUT: the tables of kLutSlots tensors from the segment's first
    int64_t lsa[kLutSlots], lea[kLutSlots];  // their element ranges in the stream
    int32_t ls[kLutSlots], le[kLutSlots];    // the same relative to the segment start (clamped)
    int32_t lt0, ln;               // the first of those tensors, how many
};
// the tensor of element g (-1: none), by binary search over the sorted starts
DEVI int lut_find(const DecArgs& a, int64_t g) {
    int lo = 0, hi = a.lut_n - 1, t = -1;
    while (lo <= hi) {
        const int mid = (lo + hi) >> 1;
        if (a.lut_start[mid] <= g) { t = mid; lo = mid + 1; } else hi = mid - 1;
    }
    return t >= 0 && g < a.lut_end[t] ? t : -1;
}
template <bool LUT>
__global__ __launch_bounds__(kRNT) void k_tlz_resolve(DecArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    ResSmem& S = *reinterpret_cast<ResSmem*>(smem_raw);
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int64_t m = blockIdx.x;
    if (m >= a.nmem) return;
    if (*reinterpret_cast<volatile int*>(a.status)) return;  // K1 found corrupt data (block-uniform)
    const int64_t* ix = a.idx + 4 * m;
    const int64_t out_off = ix[2];
    const uint32_t isize = (uint32_t)((uint64_t)ix[3] & 0xffffffffu), want_crc = (uint32_t)((uint64_t)ix[3] >> 32);
    const uint32_t ntok = isize / 4u;
    const int nseg = (int)((ntok + kSeg - 1) >> kSegLog);
    {
        uint32_t r = (uint32_t)tid;
        for (int k = 0; k < 8; ++k) r = (r & 1u) ? (r >> 1) ^ 0xEDB88320u : r >> 1;
        S.crct[0][tid] = r;
    }
    if (tid == 0) S.crc_raw = 0;
    // the advances as nibble tables: adv(x) = XOR_j T[j][nibble j of x], 8
    // independent LDS reads instead of a 32-step loop over the matrix columns
    for (int e = tid; e < 8 * 8 * 16; e += kRNT) {
        const int i = e >> 7, j = (e >> 4) & 7, v = e & 15;
        uint32_t r = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) r ^= ((v >> b) & 1) ? c_adv[adv_k(i)][4 * j + b] : 0u;
        S.adv[i][j][v] = r;
    }
    if (tid < kMemSeg) S.cnt[tid] = tid < nseg ? a.cnt[m * kMemSeg + tid] : 0u;
    __syncthreads();
    {  // the raw CRC is linear: a thread's 32 bytes hash to the XOR of one entry per value
        const int q = tid >> 5;
        const uint32_t bits = __float_as_uint((float)(tid & 31));
        uint32_t cr = 0;
#pragma unroll
        for (int k = 0; k < kRPer; ++k) cr = crc4(S.crct, cr, k == q ? bits : 0u);
        S.cid[q][tid & 31] = cr;
    }
    __syncthreads();
    auto advt = [&](uint32_t x, int i) -> uint32_t {
        uint32_t r = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) r ^= S.adv[i][j][(x >> (4 * j)) & 15u];
        return r;
    };
    int bad = 0;
    // a segment's op records (over its own output bytes) are loaded one
    // segment ahead, into registers, so that their latency overlaps the
    // previous segment's resolve (they were the loop's first dependent loads)
    constexpr int kOpPer = kSeg / kRNT;  // >= one op per value: nops <= kSeg
    uint32_t pre[kOpPer];
    auto fetch = [&](int sg) {
        const uint32_t n = sg < nseg ? S.cnt[sg] : 0u;
        const uint32_t* opi = reinterpret_cast<const uint32_t*>(a.out + out_off) + ((int64_t)sg << kSegLog);
#pragma unroll
        for (int i = 0; i < kOpPer; ++i) {
            const uint32_t k = (uint32_t)(tid + i * kRNT);
            pre[i] = k < n ? opi[k] : 0u;
        }
    };
    fetch(0);
    uint64_t t_a = a.dbg ? wall_clock64() : 0, d_pre = 0, d_jump = 0, d_val = 0;
    uint32_t jumps = 0;
    for (int s = 0; s < nseg; ++s) {
        const int c0 = s << kSegLog;
        const int T = (int)min((uint32_t)kSeg, ntok - (uint32_t)c0);
        const uint32_t nops = S.cnt[s];
        if (nops > (uint32_t)T) { bad = kInfCorrupt; break; }  // (block-uniform)
        float* const yo = reinterpret_cast<float*>(a.out + out_off) + c0;
#pragma unroll
        for (int i = 0; i < kOpPer; ++i) S.opr[tid + i * kRNT] = pre[i];
        fetch(s + 1);
        const int64_t g0 = out_off / 4 + c0;  // the segment's first element of the stream
        if (LUT) {
            // the slots hold the tensors from the one holding (or following)
            // the segment's first element: loaded for the member's first
            // segment, then moved on only where a tensor ended before this
            // segment (a global search per segment cost ~6 us of dependent
            // loads on every block's critical path)
            if (tid == 0) {
                int t = -1;
                if (s == 0 || (S.ln > 0 && S.lea[0] <= g0 && S.lt0 + 1 < a.lut_n)) {
                    int lo = s == 0 ? 0 : S.lt0, hi = a.lut_n - 1;
                    t = a.lut_n;
                    while (lo <= hi) {  // the first tensor ending after g0
                        const int mid = (lo + hi) >> 1;
                        if (a.lut_end[mid] > g0) { t = mid; hi = mid - 1; } else lo = mid + 1;
                    }
                    S.lt0 = t;
                    S.ln = min(kLutSlots, a.lut_n - t);
                }
                S.scan[0] = t >= 0 ? 1u : 0u;  // reload (the scan words are free until the block scan)
            }
            __syncthreads();
            const int t0 = S.lt0, ln = S.ln;
            if (S.scan[0]) {
                for (int k = tid; k < ln * 32; k += kRNT) S.lt[k >> 5][k & 31] = a.lut_tab[(int64_t)(t0 + (k >> 5)) * 32 + (k & 31)];
                if (tid < ln) { S.lsa[tid] = a.lut_start[t0 + tid]; S.lea[tid] = a.lut_end[t0 + tid]; }
            }
            __syncthreads();
            if (tid < ln) {
                S.ls[tid] = (int32_t)max<int64_t>(-1, min<int64_t>(kSeg + 1, S.lsa[tid] - g0));
                S.le[tid] = (int32_t)max<int64_t>(-1, min<int64_t>(kSeg + 1, S.lea[tid] - g0));
            }
        }
        __syncthreads();
        // positions: each thread a contiguous run of ops
        const uint32_t o_lo = nops * tid / kRNT, o_hi = nops * (tid + 1) / kRNT;
        uint32_t run = 0;
        for (uint32_t o = o_lo; o < o_hi; ++o) { const uint32_t r = S.opr[o]; run += (r >> 31) ? 1u : (r & 127u); }
        uint32_t tot;
        uint32_t p = block_scan<kRNT>(run, S.scan, &tot);
        if (tot != (uint32_t)T) { bad = kInfCorrupt; break; }  // block-uniform
        for (uint32_t o = o_lo; o < o_hi; ++o) {
            const uint32_t r = S.opr[o];
            if (r >> 31) {
                S.e[p++] = (uint16_t)(0x8000u | (r & 31u));
            } else {
                const uint32_t l = r & 127u, d = r >> 7;
                for (uint32_t k = 0; k < l; ++k) S.e[p + k] = (uint16_t)d;
                p += l;
            }
        }
        __syncthreads();
        uint64_t t_b = a.dbg ? wall_clock64() : 0;
        if (a.dbg) d_pre += t_b - t_a;
        // pointer jumping: an unresolved entry points at its source; a source
        // before the segment is a value of the ring
        const int rb0 = (int)((uint32_t)c0 % kVRing);
        // (a resolved entry stays resolved: each thread skips the ones it
        // saw resolved, so later rounds read only the 43 %, 7 %, ... left)
        uint32_t um = (1u << kRPer) - 1u;
#pragma unroll 1
        for (;;) {
            ++jumps;
            int pend = 0;
            uint32_t nm = 0;
#pragma unroll
            for (int i = 0; i < kRPer; ++i) {
                const int k = tid + i * kRNT;
                if (!((um >> i) & 1u) || k >= T) continue;
                const uint32_t e = S.e[k];
                if (e & 0x8000u) continue;
                const int src = k - (int)e;
                uint32_t ne;
                if (src < 0) {  // a value before the segment: ring slot (c0 + src) mod kVRing, src >= -kWin
                    const int r = rb0 + src;
                    ne = 0x8000u | S.v[r < 0 ? r + (int)kVRing : r];
                }
                else {
                    const uint32_t es = S.e[src];
                    ne = (es & 0x8000u) ? es : e + es;
                }
                S.e[k] = (uint16_t)ne;
                if (!(ne & 0x8000u)) { pend = 1; nm |= 1u << i; }
            }
            um = nm;
            if (!__syncthreads_or(pend)) break;
        }
        if (a.dbg) { const uint64_t t = wall_clock64(); d_jump += t - t_b; t_b = t; }
        // values: ring, output (float32), raw CRC-32
        {
            const int k0 = kRPer * tid;
            const int nv = max(0, min(kRPer, T - k0));
            uint32_t crc = 0;
            float f[kRPer];
            // the thread's 8 entries as one 16-byte read, its 8 ids into the
            // ring as one 8-byte write (c0 + k0 and kVRing are multiples of 8:
            // the 8 ring slots never wrap)
            static_assert(kRPer == 8 && kVRing % 8 == 0, "one b128 read, one b64 ring write per thread");
            const uint4 ev = *reinterpret_cast<const uint4*>(&S.e[k0]);
            const uint32_t ew[4] = {ev.x, ev.y, ev.z, ev.w};
            uint32_t idw[2] = {0u, 0u};
#pragma unroll
            for (int q = 0; q < kRPer; ++q) {
                const uint32_t id = q < nv ? ((ew[q >> 1] >> (16 * (q & 1))) & 31u) : 0u;
                f[q] = (float)id;
                idw[q >> 2] |= id << (8 * (q & 3));
                if (q < nv) crc ^= S.cid[q][id];
            }
            if (nv == kRPer) {
                *reinterpret_cast<uint2*>(&S.v[(uint32_t)(c0 + k0) % kVRing]) = make_uint2(idw[0], idw[1]);
            } else {
                for (int q = 0; q < nv; ++q) S.v[(uint32_t)(c0 + k0 + q) % kVRing] = (uint8_t)(idw[q >> 2] >> (8 * (q & 3)));
            }
            if (nv < kRPer) {  // a partial last piece: the values' own chain
                crc = 0;
#pragma unroll
                for (int q = 0; q < kRPer; ++q)
                    if (q < nv) crc = crc4(S.crct, crc, __float_as_uint(f[q]));
            }
            if (LUT) {  // the values through the element's tensor table (the CRC above is the ranks')
                const int ln = S.ln;
                int j = 0;  // the slot of this thread's first element (segment-relative k0)
                while (j < ln && k0 >= S.le[j]) ++j;
                if (j < ln && k0 >= S.ls[j] && k0 + kRPer <= S.le[j]) {  // all its values in one tensor
#pragma unroll
                    for (int q = 0; q < kRPer; ++q) f[q] = S.lt[j][(uint32_t)f[q]];
                } else {
#pragma unroll
                    for (int q = 0; q < kRPer; ++q) {
                        const int k = k0 + q;
                        const uint32_t id = (uint32_t)f[q];
                        int jj = 0;
                        while (jj < ln && k >= S.le[jj]) ++jj;
                        float v = f[q];
                        if (jj < ln) {
                            if (k >= S.ls[jj]) v = S.lt[jj][id];
                        } else if (ln == kLutSlots) {  // past the tables in LDS: a segment over many small tensors
                            const int t = lut_find(a, g0 + k);
                            if (t >= 0) v = a.lut_tab[(int64_t)t * 32 + id];
                        }
                        f[q] = v;
                    }
                }
            }
            if (nv == kRPer && (reinterpret_cast<uintptr_t>(yo + k0) & 15u) == 0) {
                float4* y4 = reinterpret_cast<float4*>(yo + k0);
#pragma unroll
                for (int u = 0; u < kRPer / 4; ++u) y4[u] = make_float4(f[4 * u], f[4 * u + 1], f[4 * u + 2], f[4 * u + 3]);
            } else {
                for (int q = 0; q < nv; ++q) yo[k0 + q] = f[q];
            }
            uint32_t wcrc;
            if (T == kSeg) {
                uint32_t x = crc;
#pragma unroll
                for (int l = 0; l < 6; ++l) {
                    const uint32_t o = (uint32_t)__shfl_xor((int)x, 1 << l, 64);
                    const uint32_t sh = advt(x, l);  // 2^(5 + l) bytes
                    x = (lane & (1 << l)) ? x : (sh ^ o);
                }
                wcrc = x;
            } else {
                uint32_t x = nv ? crc_adv(crc, 4u * (uint32_t)(T - k0 - nv)) : 0u;
                for (int o = 32; o > 0; o >>= 1) x ^= (uint32_t)__shfl_xor((int)x, o, 64);
                wcrc = x;
            }
            if (lane == 0) S.crc_w[wv] = wcrc;
        }
        __syncthreads();
        if (tid == 0) {
            uint32_t raw = 0;
            if (T == kSeg) {
                for (int w = 0; w < kRNT / 64; ++w) raw = advt(raw, 6) ^ S.crc_w[w];  // 2^kSegLog bytes
                S.crc_raw = advt(S.crc_raw, 7) ^ raw;                                   // 2^(kSegLog + 2)
            } else {
                for (int w = 0; w < kRNT / 64; ++w) raw ^= S.crc_w[w];
                S.crc_raw = crc_adv(S.crc_raw, 4u * (uint32_t)T) ^ raw;
            }
        }
        __syncthreads();
        if (a.dbg) { const uint64_t t = wall_clock64(); d_val += t - t_b; t_a = t; }
    }
    if (a.dbg && (m & 255) == 0 && tid == 0)
        printf("tlz_resolve m=%lld load_scan_ticks=%llu jump_ticks=%llu values_ticks=%llu jump_rounds=%u segs=%d\n",
               (long long)m, (unsigned long long)d_pre, (unsigned long long)d_jump, (unsigned long long)d_val, jumps, nseg);
    if (tid == 0) {
        if (bad) atomicOr(a.status, bad);
        else if ((crc_adv(0xffffffffu, isize) ^ S.crc_raw ^ 0xffffffffu) != want_crc) atomicOr(a.status, kInfCrc);
    }
}
}  // namespace tlz

// members -> one contiguous stream (slots of any stride).  The destination is
// usually mapped pinned host memory, written across PCIe: every store is an
// aligned 16-byte one (the source realigned with alignbyte; slots are 4-byte
// aligned), only the < 16 bytes at either end of a member are byte stores.
// (Byte stores for the 3 in 4 members that start misaligned ran at 8.5 GB/s.)
// one member's bytes from its slot to dst (256 threads; 16-byte stores)
DEVI void pack_member(const uint8_t* src, uint8_t* dst, uint32_t n) {
    const uint32_t head = (uint32_t)((16u - (reinterpret_cast<uintptr_t>(dst) & 15u)) & 15u);
    if (n <= head + 16u) {
        for (uint32_t i = threadIdx.x; i < n; i += 256) dst[i] = src[i];
        return;
    }
    const uint32_t body = (n - head) >> 4;  // aligned 16-byte stores
    const uint32_t tail0 = head + 16u * body;
    if (threadIdx.x < head) dst[threadIdx.x] = src[threadIdx.x];
    for (uint32_t i = tail0 + threadIdx.x; i < n; i += 256) dst[i] = src[i];
    const uint32_t sh = head & 3u;             // source offset of the body, mod 4
    const uint32_t* s = reinterpret_cast<const uint32_t*>(src + (head & ~3u));
    uint4* d = reinterpret_cast<uint4*>(dst + head);
    for (uint32_t i = threadIdx.x; i < body; i += 256) {
        const uint32_t* q = s + 4u * i;
        uint4 v;
        if (sh == 0) {
            v = make_uint4(q[0], q[1], q[2], q[3]);
        } else {  // the 5th word is within the slot: the body ends >= 1 byte before n
            const uint32_t w0 = q[0], w1 = q[1], w2 = q[2], w3 = q[3], w4 = q[4];
            v.x = __builtin_amdgcn_alignbyte(w1, w0, sh);
            v.y = __builtin_amdgcn_alignbyte(w2, w1, sh);
            v.z = __builtin_amdgcn_alignbyte(w3, w2, sh);
            v.w = __builtin_amdgcn_alignbyte(w4, w3, sh);
        }
        d[i] = v;
    }
}

__global__ __launch_bounds__(256) void k_gzip_pack(const uint8_t* slots, uint64_t stride, const uint32_t* sizes,
                                                   const uint64_t* off, uint8_t* packed) {
    if (off[blockIdx.x] == ~0ull) return;  // the batch does not fit the output (reported by the scan)
    pack_member(slots + (int64_t)blockIdx.x * stride, packed + off[blockIdx.x], sizes[blockIdx.x]);
}

// the batched path's pack, enqueued right behind the batch's scan with no
// host round trip: the batch's first offset and end come from the scan's
// output (off[0], off[nb]); a batch that fits the device staging goes there
// (stage + off - first, then one DMA), a larger one (nearly incompressible
// ranks) straight into the mapped pinned output at its offsets
__global__ __launch_bounds__(256) void k_gzip_pack_batch(const uint8_t* slots, uint64_t stride, const uint32_t* sizes,
                                                         const uint64_t* off, int nb, uint8_t* stage,
                                                         uint64_t stage_cap, uint8_t* mapped) {
    const uint64_t first = off[0], end = off[nb];
    if (first == ~0ull || off[blockIdx.x] == ~0ull) return;  // the batch does not fit the output (reported by the scan)
    uint8_t* dst = end - first <= stage_cap ? stage + (off[blockIdx.x] - first) : mapped + off[blockIdx.x];
    pack_member(slots + (int64_t)blockIdx.x * stride, dst, sizes[blockIdx.x]);
}

}  // namespace gz

namespace {
thread_local std::string g_gzerr;
int gzfail(int code, const std::string& m) { g_gzerr = m; return code; }
#define GZHIP(x)                                                                                        \
    do {                                                                                                \
        hipError_t e_ = (x);                                                                            \
        if (e_ != hipSuccess) return gzfail(OFL_EHIP, std::string(#x " failed: ") + hipGetErrorString(e_)); \
    } while (0)

// Optional per-kernel timing (bench.py's KC line): while enabled, every
// gzip / inflate launch is bracketed by HIP events on its stream; collect
// synchronises them and sums the time per kernel name.
std::mutex g_prof_m;
bool g_prof_on = false;
struct ProfRec { const char* name; hipEvent_t a, b; };
std::vector<ProfRec> g_prof_pending;
thread_local hipEvent_t g_prof_a = nullptr;
void gzprof_begin(hipStream_t st) {
    if (!g_prof_on) return;
    if (hipEventCreate(&g_prof_a) != hipSuccess || hipEventRecord(g_prof_a, st) != hipSuccess) g_prof_a = nullptr;
}
void gzprof_end(hipStream_t st, const char* name) {
    if (!g_prof_on || !g_prof_a) return;
    hipEvent_t b;
    if (hipEventCreate(&b) != hipSuccess) return;
    if (hipEventRecord(b, st) != hipSuccess) { (void)hipEventDestroy(b); return; }
    std::lock_guard<std::mutex> g(g_prof_m);
    g_prof_pending.push_back({name, g_prof_a, b});
    g_prof_a = nullptr;
}

// the device's stream for the gzip's DMA (created once per device): the
// DMA of batch k overlaps the encode of batch k + 1 only from another HW
// queue.  HIP hands normal-priority streams the GPU_MAX_HW_QUEUES queues in
// turn, so a normal stream made late in a busy process can share the
// caller's queue (the DMA then waits behind the next encode: gzip phase
// 11.9 -> 14.9 ms per GiB); a high-priority stream comes from HIP's separate
// high-priority queues (profiles/r05_kc_hw_queues_ab.txt)
hipError_t gz_side_stream(hipStream_t* out) {
    static std::mutex m;
    static hipStream_t side[64] = {};
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    std::lock_guard<std::mutex> g(m);
    if (!side[dev]) {
        int least = 0, greatest = 0;
        e = hipDeviceGetStreamPriorityRange(&least, &greatest);
        if (e == hipSuccess) e = hipStreamCreateWithPriority(&side[dev], hipStreamNonBlocking, greatest);
    }
    *out = side[dev];
    return e;
}

// a small pinned host block per thread (the gzip's per-batch offsets, read by
// the host while the next batch encodes); allocated once, kept
hipError_t gz_pinned_info(uint64_t** out) {
    thread_local uint64_t* p = nullptr;
    if (!p) {
        const hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&p), 64, hipHostMallocDefault);
        if (e != hipSuccess) { p = nullptr; return e; }
    }
    *out = p;
    return hipSuccess;
}

// raw CRC-32 advance matrices for 2^k zero bytes
void crc_matrices(uint32_t (&m)[32][32]) {
    uint32_t tab[256];
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t r = i;
        for (int k = 0; k < 8; ++k) r = (r & 1u) ? (r >> 1) ^ 0xEDB88320u : r >> 1;
        tab[i] = r;
    }
    for (int i = 0; i < 32; ++i) { const uint32_t v = 1u << i; m[0][i] = tab[v & 0xffu] ^ (v >> 8); }
    auto apply = [](const uint32_t* M, uint32_t v) {
        uint32_t r = 0;
        for (int i = 0; i < 32; ++i) if ((v >> i) & 1u) r ^= M[i];
        return r;
    };
    for (int k = 1; k < 32; ++k)
        for (int i = 0; i < 32; ++i) m[k][i] = apply(m[k - 1], apply(m[k - 1], 1u << i));
}
// the members of a member-indexed stream (every header carries its size in
// an RFC 1952 extra subfield: 'BC' (BGZF: size - 1, 16 bits) or 'OZ' (TLZ:
// size, 32 bits, plus the segment table)): deflate data range, output
// offset, ISIZE, CRC-32 and whether it is a TLZ member
struct GzMember { size_t in, in_len, out; uint32_t isize, crc; bool tlz; };
// one member at pos: its size (0 if the bytes there are not a member header
// with a size field) and its record
size_t member_at(const uint8_t* src, size_t n, size_t pos, GzMember& m) {
    const uint8_t* h = src + pos;
    if (n - pos < 26 || h[0] != 0x1f || h[1] != 0x8b || h[2] != 8 || h[3] != 0x04) return 0;
    const size_t xlen = (size_t)h[10] | ((size_t)h[11] << 8);
    if (12 + xlen > n - pos) return 0;
    size_t bsize = 0;
    bool tlz = false;
    const uint8_t* zf = nullptr;  // the OZ subfield's payload
    for (size_t q = 12; q + 4 <= 12 + xlen;) {
        const size_t sl = (size_t)h[q + 2] | ((size_t)h[q + 3] << 8);
        if (q + 4 + sl > 12 + xlen) return 0;
        if (h[q] == 'B' && h[q + 1] == 'C' && sl == 2) bsize = ((size_t)h[q + 4] | ((size_t)h[q + 5] << 8)) + 1;
        if (h[q] == 'O' && h[q + 1] == 'Z' && sl >= 12) {
            const uint8_t* z = h + q + 4;
            const size_t nseg = (size_t)z[2] | ((size_t)z[3] << 8);
            bsize = (size_t)z[4] | ((size_t)z[5] << 8) | ((size_t)z[6] << 16) | ((size_t)z[7] << 24);
            // the segment table must end where the deflate data starts
            tlz = z[0] == 1 && z[1] == gz::tlz::kSegLog && sl == 12 + 4 * nseg && q + 4 + sl == 12 + xlen &&
                  nseg >= 1 && nseg <= (size_t)gz::tlz::kMemSeg;
            zf = tlz ? z : nullptr;
        }
        q += 4 + sl;
    }
    if (bsize < 12 + xlen + 8 || bsize > n - pos) return 0;
    const uint8_t* t = src + pos + bsize - 8;
    m.in = pos + 12 + xlen;
    m.in_len = bsize - 12 - xlen - 8;
    m.crc = (uint32_t)t[0] | ((uint32_t)t[1] << 8) | ((uint32_t)t[2] << 16) | ((uint32_t)t[3] << 24);
    m.isize = (uint32_t)t[4] | ((uint32_t)t[5] << 8) | ((uint32_t)t[6] << 16) | ((uint32_t)t[7] << 24);
    // a TLZ member's value count (the OZ field) must match its ISIZE
    if (tlz) {
        const uint8_t* z = zf;
        const size_t ntok = (size_t)z[8] | ((size_t)z[9] << 8) | ((size_t)z[10] << 16) | ((size_t)z[11] << 24);
        const size_t nseg = (size_t)z[2] | ((size_t)z[3] << 8);
        tlz = (m.isize & 3u) == 0 && ntok == m.isize / 4 && nseg == (ntok + gz::tlz::kSeg - 1) / gz::tlz::kSeg;
    }
    m.tlz = tlz;
    return bsize;
}

// walk the member chain over [pos, end); false if a header is not one.
// out offsets are relative to the walk's start
bool walk_members(const uint8_t* src, size_t n, size_t pos, size_t end, std::vector<GzMember>& mem, size_t& reached) {
    size_t out = 0;
    while (pos < end) {
        GzMember m;
        const size_t bs = member_at(src, n, pos, m);
        if (!bs) return false;
        m.out = out;
        out += m.isize;
        mem.push_back(m);
        pos += bs;
    }
    reached = pos;
    return true;
}

// The chain is a dependent walk (each header gives the next one's offset), so
// one thread pays a cache miss per member.  Large streams are cut in pieces;
// each thread finds the first header at or after its piece's start (the 'BC'
// member signature) and walks to the end of its piece; the pieces are then
// checked to link exactly (thread k's walk ends where thread k+1's starts), so
// a signature found inside compressed data can only send the parse back to
// the serial walk, never give a wrong index.
int parse_members(const uint8_t* src, size_t n, std::vector<GzMember>& mem, size_t& total) {
    mem.clear();
    total = 0;
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const int nt = (int)std::min<size_t>(std::min<unsigned>(hw, 16u), n >> 22);  // >= 4 MiB per piece
    bool par_ok = nt > 1;
    if (par_ok) {
        std::vector<std::vector<GzMember>> part(nt);
        std::vector<size_t> start(nt + 1, n), reached(nt, 0);
        std::vector<char> ok(nt, 0);
        auto work = [&](int t) {
            size_t p = n * t / nt;
            const size_t lim = n * (t + 1) / nt;
            if (t > 0) {  // the first member signature at or after p
                GzMember m;
                while (p < lim) {
                    const uint8_t* h = src + p;
                    if (h[0] == 0x1f && p + 16 <= n && h[1] == 0x8b && h[2] == 8 && h[3] == 4 &&
                        ((h[12] == 'B' && h[13] == 'C') || (h[12] == 'O' && h[13] == 'Z')) && member_at(src, n, p, m))
                        break;
                    ++p;
                }
            }
            start[t] = p;
            ok[t] = p < lim && walk_members(src, n, p, lim, part[t], reached[t]);
        };
        std::vector<std::thread> th;
        for (int t = 1; t < nt; ++t) th.emplace_back(work, t);
        work(0);
        for (auto& x : th) x.join();
        // members are < 1 MiB and pieces >= 4 MiB: every piece holds a
        // header; piece t's walk (from a true header, by induction from 0)
        // ends on a true header, which must be where piece t + 1 starts
        par_ok = start[0] == 0;
        for (int t = 0; t < nt && par_ok; ++t)
            par_ok = ok[t] && !part[t].empty() && reached[t] == (t + 1 < nt ? start[t + 1] : n);
        if (par_ok) {
            size_t cnt = 0;
            for (auto& p : part) cnt += p.size();
            mem.reserve(cnt);
            for (auto& p : part) mem.insert(mem.end(), p.begin(), p.end());
            for (GzMember& m : mem) { m.out = total; total += m.isize; }  // absolute output offsets
            return OFL_OK;
        }
        mem.clear();
        total = 0;
    }
    size_t reached0 = 0;
    if (!walk_members(src, n, 0, n, mem, reached0)) {
        mem.clear();
        return gzfail(OFL_EFORMAT, "gunzip: not a member-indexed gzip stream");
    }
    for (const GzMember& m : mem) total += m.isize;
    return OFL_OK;
}
}  // namespace

extern "C" {

const char* ofl_gzip_last_error(void) { return g_gzerr.c_str(); }

namespace {
struct TlzLayout {
    int64_t members, batch;
    size_t slot, ops_stride;
    size_t stage;  // a batch's device staging for the D2H: 1 byte per value
};
TlzLayout tlz_layout(int64_t n) {
    using namespace gz::tlz;
    TlzLayout L;
    L.members = std::max<int64_t>(1, (n + kMemTok - 1) / kMemTok);
    L.batch = std::min<int64_t>(L.members, kBatch);
    const int64_t per = std::min<int64_t>(std::max<int64_t>(n, 1), kMemTok);
    L.slot = ((size_t)per * kSlotPerTok + kSlotPad + 255) & ~(size_t)255;
    L.ops_stride = ((size_t)per + 63) & ~(size_t)63;
    L.stage = ((size_t)L.batch * (size_t)per + 255) & ~(size_t)255;
    return L;
}
}  // namespace

size_t ofl_gzip_ranks_workspace_bytes(int64_t n) {
    const TlzLayout L = tlz_layout(n);
    // slots x 2 (the second is the pageable path's staging) | ops | sizes x 2 |
    // offsets x 2 | running | bad | D2H staging x 2
    return 2 * (size_t)L.batch * L.slot + 4 * (size_t)L.batch * L.ops_stride + 8 * (size_t)L.batch +
           16 * (size_t)(L.batch + 1) + 1024 + 2 * L.stage;
}

size_t ofl_gzip_ranks_bound(int64_t n) {
    const TlzLayout L = tlz_layout(n);
    return (size_t)L.members * L.slot;
}

// host_dst (optional): a pageable buffer of host_cap bytes that receives the
// stream too, each batch copied on nthreads host threads while the next batch
// encodes (ofl_gzip_ranks_to)
// lab (optional, device): x holds values, labelled through lab_n records as they load
static int gzip_ranks_impl(const float* x, int64_t n, const ofl_label_rec* lab, int lab_n, uint8_t* out,
                           size_t out_cap, uint8_t* host_dst, size_t host_cap, int nthreads, size_t* out_len, void* ws,
                           size_t ws_bytes, void* stream) {
    if (n < 1 || !x || !out || !out_len) return gzfail(OFL_EINVAL, "gzip ranks: empty input");
    if (lab && lab_n < 1) return gzfail(OFL_EINVAL, "gzip label: no label records");
    if (host_dst && host_cap < out_cap) return gzfail(OFL_EINVAL, "gzip ranks: host_cap < out_cap");
    if (!ws || ws_bytes < ofl_gzip_ranks_workspace_bytes(n)) return gzfail(OFL_ESPACE, "gzip ranks: workspace too small");
    GZHIP(ofl_util::per_device_once([] {  // __constant__ tables and attributes are per device
        uint32_t m[32][32];
        crc_matrices(m);
        hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(gz::c_adv), m, sizeof(m));
        if (e == hipSuccess)
            e = hipFuncSetAttribute((const void*)gz::tlz::k_tlz_encode, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)sizeof(gz::tlz::EncSmem));
        return e;
    }));
    hipStream_t st = static_cast<hipStream_t>(stream);
    const TlzLayout L = tlz_layout(n);
    char* w = static_cast<char*>(ws);
    uint8_t* slots2[2];                              // double-buffered member slots (pinned output path)
    slots2[0] = reinterpret_cast<uint8_t*>(w);
    slots2[1] = slots2[0] + (size_t)L.batch * L.slot;
    uint8_t* slots = slots2[0];
    uint8_t* packed = slots2[1];                     // the pageable path's staging
    uint32_t* ops = reinterpret_cast<uint32_t*>(slots2[1] + (size_t)L.batch * L.slot);
    uint32_t* sizes2[2];
    sizes2[0] = ops + (size_t)L.batch * L.ops_stride;
    sizes2[1] = sizes2[0] + L.batch;
    uint32_t* sizes = sizes2[0];
    uint64_t* off = reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(sizes2[1] + L.batch) + 8 -
                                                (reinterpret_cast<uintptr_t>(sizes2[1] + L.batch) & 7u));
    uint64_t* off2[2] = {off, off + L.batch + 1};
    uint64_t* running = off2[1] + L.batch + 1;
    int* bad = reinterpret_cast<int*>(running + 1);
    uint8_t* stage2[2];
    stage2[0] = reinterpret_cast<uint8_t*>((reinterpret_cast<uintptr_t>(bad + 1) + 255) & ~(uintptr_t)255);
    stage2[1] = stage2[0] + L.stage;
    GZHIP(hipMemsetAsync(bad, 0, sizeof(int), st));
    // out is mapped pinned host memory (e.g. torch pin_memory): the pack
    // kernel writes the stream straight into it and the batches run back to
    // back with one synchronisation at the end; otherwise one D2H per batch
    uint8_t* dout = nullptr;
    {
        hipPointerAttribute_t pa;
        if (hipPointerGetAttributes(&pa, out) == hipSuccess && pa.type == hipMemoryTypeHost && pa.devicePointer)
            dout = static_cast<uint8_t*>(pa.devicePointer);
        (void)hipGetLastError();  // a pageable pointer is not an error here
    }
    const int aligned = (reinterpret_cast<uintptr_t>(x) & 15u) == 0;
    // diagnostics: OFL_GZ_PHASES=1 prints block 0's phase times (10 ns ticks,
    // summed over its segments; [11] = Jacobi rounds) of the first launch
    static const bool phases = getenv("OFL_GZ_PHASES") != nullptr;
    uint64_t* d_ph = nullptr;
    if (phases) {
        GZHIP(hipMalloc(&d_ph, 8 * gz::tlz::kEncPhases));
        GZHIP(hipMemsetAsync(d_ph, 0, 8 * gz::tlz::kEncPhases, st));
    }
    auto enc = [&](int64_t c0, int nb, uint8_t* sl, uint32_t* sz) {
        gz::tlz::EncArgs a{x, n, c0, sl, ops, sz, bad, (uint32_t)L.slot, (uint32_t)L.ops_stride, aligned,
                           c0 == 0 ? d_ph : nullptr, lab, lab ? lab_n : 0};
        gzprof_begin(st);
        hipLaunchKernelGGL(gz::tlz::k_tlz_encode, dim3(nb), dim3(gz::tlz::kNT), sizeof(gz::tlz::EncSmem), st, a);
        gzprof_end(st, "tlz::k_tlz_encode");
    };
    size_t total = 0;
    if (dout) {
        // batch k encodes on the caller's stream into slots[k & 1]; its scan,
        // pack and D2H run on the side stream, overlapping the encode of
        // batch k + 1.  The pack goes to device staging and the stream
        // crosses PCIe by DMA (a kernel's stores into mapped host memory are
        // one small PCIe write each: 8.5 GB/s); the host learns a batch's
        // offset and size from the scan while the next batch encodes.  A
        // batch larger than its staging (> 1 byte per value: nearly
        // incompressible ranks) is packed straight into the mapped output.
        hipStream_t sd = nullptr;
        GZHIP(gz_side_stream(&sd));
        uint64_t* hinfo = nullptr;
        GZHIP(gz_pinned_info(&hinfo));  // [2][2]: a batch's first offset and end
        const int64_t nbatch = (L.members + L.batch - 1) / L.batch;
        hipEvent_t ev_pack[2] = {}, ev_scan[2] = {};
        // every exit (the GZHIP / finish error returns included) waits for the
        // work queued on both streams -- scan, pack and D2H read ws and write
        // out -- before the caller may reuse those buffers, then frees the events
        bool drained = false;
        ofl_util::ScopeExit cleanup([&] {
            if (!drained) { (void)hipStreamSynchronize(sd); (void)hipStreamSynchronize(st); }
            for (int i = 0; i < 2; ++i) {
                if (ev_pack[i]) (void)hipEventDestroy(ev_pack[i]);
                if (ev_scan[i]) (void)hipEventDestroy(ev_scan[i]);
            }
        });
        for (int i = 0; i < 2; ++i) {
            GZHIP(hipEventCreateWithFlags(&ev_pack[i], hipEventDisableTiming));
            GZHIP(hipEventCreateWithFlags(&ev_scan[i], hipEventDisableTiming));
        }
        GZHIP(hipMemsetAsync(running, 0, sizeof(uint64_t), st));
        uint64_t copied = 0;  // host_dst holds out[0, copied)
        // diagnostics: OFL_GZ_FILL_TRACE=1 prints the host's wait / copy times per call
        static const bool fill_trace = getenv("OFL_GZ_FILL_TRACE") != nullptr;
        auto now_us = [] {
            return (double)std::chrono::duration_cast<std::chrono::microseconds>(
                       std::chrono::steady_clock::now().time_since_epoch()).count();
        };
        const double t_call = fill_trace ? now_us() : 0.0;
        char trace[512];
        int tn = 0;
        auto host_copy = [&](uint64_t upto) {  // out[copied, upto) -> host_dst (its DMA complete)
            if (host_dst && upto > copied) {
                const double t0 = fill_trace ? now_us() : 0.0;
                void* d = host_dst + copied;
                const void* src = out + copied;
                const int64_t nb = (int64_t)(upto - copied);
                ofl_host_copy_many(1, &d, &src, &nb, nthreads);
                copied = upto;
                if (fill_trace && tn < 400)
                    tn += snprintf(trace + tn, sizeof(trace) - tn, " copy@%.0f+%.0f", t0 - t_call, now_us() - t0);
            }
        };
        auto wait_ev = [&](hipEvent_t e, const char* what) -> hipError_t {
            const double t0 = fill_trace ? now_us() : 0.0;
            const hipError_t r = hipEventSynchronize(e);
            if (fill_trace && tn < 400)
                tn += snprintf(trace + tn, sizeof(trace) - tn, " %s@%.0f+%.0f", what, t0 - t_call, now_us() - t0);
            return r;
        };
        // Batch k on the caller's stream: encode, scan, pack -- the scan and
        // the pack (tens of us with the whole chip free) run before the next
        // batch's encode, so nothing of a batch waits for CUs behind the next
        // one (on a side stream they queued behind its 80 KiB-LDS blocks for
        // up to 2.3 ms).  Only the DMA of batch k (its size is known once the
        // host has read the scan) goes on the side stream, beside the encode
        // of batch k + 1, and the host copies batch k into host_dst meanwhile.
        // The last batch crosses PCIe in pieces, each copied as it lands.
        hipEvent_t ev_dma[2] = {};
        ofl_util::ScopeExit cleanup2([&] {
            for (int i = 0; i < 2; ++i)
                if (ev_dma[i]) (void)hipEventDestroy(ev_dma[i]);
        });
        for (int i = 0; i < 2; ++i) GZHIP(hipEventCreateWithFlags(&ev_dma[i], hipEventDisableTiming));
        constexpr int kTailPieces = 4;
        hipEvent_t ev_tail[kTailPieces] = {};
        ofl_util::ScopeExit cleanup3([&] {
            for (auto& e : ev_tail)
                if (e) (void)hipEventDestroy(e);
        });
        for (auto& e : ev_tail) GZHIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        uint64_t bfirst[2] = {0, 0}, bend[2] = {0, 0};
        // batch k's DMA (after its scan result is on the host); pieces > 1 for the last batch
        auto issue_dma = [&](int64_t k, int pieces) -> int {
            const int b = (int)(k & 1);
            GZHIP(wait_ev(ev_scan[b], "scan"));
            const uint64_t first = hinfo[2 * b], end = hinfo[2 * b + 1];
            bfirst[b] = first == ~0ull ? 0 : first;
            bend[b] = first == ~0ull ? 0 : end;
            GZHIP(hipStreamWaitEvent(sd, ev_pack[b], 0));
            if (first != ~0ull && end > first && end - first <= L.stage) {
                const uint64_t n = end - first;
                for (int p = 0; p < pieces; ++p) {
                    const uint64_t lo = n * (uint64_t)p / (uint64_t)pieces, hi = n * (uint64_t)(p + 1) / (uint64_t)pieces;
                    gzprof_begin(sd);
                    if (hi > lo) GZHIP(hipMemcpyAsync(out + first + lo, stage2[b] + lo, hi - lo, hipMemcpyDeviceToHost, sd));
                    gzprof_end(sd, "gzip D2H (DMA)");
                    if (pieces > 1) GZHIP(hipEventRecord(ev_tail[p], sd));
                }
            }
            GZHIP(hipEventRecord(ev_dma[b], sd));
            return OFL_OK;
        };
        for (int64_t k = 0; k < nbatch; ++k) {
            const int64_t c0 = k * L.batch;
            const int b = (int)(k & 1);
            const int nb = (int)std::min<int64_t>(L.batch, L.members - c0);
            enc(c0, nb, slots2[b], sizes2[b]);
            gzprof_begin(st);
            hipLaunchKernelGGL(gz::k_gzip_scan, dim3(1), dim3(1024), 0, st, sizes2[b], nb, off2[b], running,
                               (uint64_t)out_cap, bad);
            gzprof_end(st, "k_gzip_scan");
            GZHIP(hipMemcpyAsync(hinfo + 2 * b, off2[b], 8, hipMemcpyDeviceToHost, st));
            GZHIP(hipMemcpyAsync(hinfo + 2 * b + 1, off2[b] + nb, 8, hipMemcpyDeviceToHost, st));
            GZHIP(hipEventRecord(ev_scan[b], st));
            if (k >= 2) GZHIP(hipStreamWaitEvent(st, ev_dma[b], 0));  // stage[b]'s previous DMA has read it
            gzprof_begin(st);
            hipLaunchKernelGGL(gz::k_gzip_pack_batch, dim3(nb), dim3(256), 0, st, slots2[b], (uint64_t)L.slot, sizes2[b],
                               off2[b], nb, stage2[b], (uint64_t)L.stage, dout);
            gzprof_end(st, "k_gzip_pack");
            GZHIP(hipEventRecord(ev_pack[b], st));
            if (hipGetLastError() != hipSuccess) return gzfail(OFL_EHIP, "gzip ranks: kernel launch failed");
            if (k >= 1) {  // batch k - 1: its DMA and its bytes to host_dst, beside this batch's encode
                if (int rc = issue_dma(k - 1, 1)) return rc;
                if (host_dst) {
                    GZHIP(wait_ev(ev_dma[(k - 1) & 1], "dma"));
                    host_copy(bend[(k - 1) & 1]);
                }
            }
        }
        if (int rc = issue_dma(nbatch - 1, host_dst ? kTailPieces : 1)) return rc;
        {  // the last batch, piece by piece as its DMA lands
            const int b = (int)((nbatch - 1) & 1);
            const uint64_t first = bfirst[b], end = bend[b];
            if (host_dst && end > first && end - first <= L.stage) {
                const uint64_t n = end - first;
                for (int p = 0; p < kTailPieces; ++p) {
                    GZHIP(wait_ev(ev_tail[p], "tail"));
                    host_copy(first + n * (uint64_t)(p + 1) / (uint64_t)kTailPieces);
                }
            }
        }
        GZHIP(hipEventRecord(ev_pack[0], sd));
        GZHIP(hipStreamWaitEvent(st, ev_pack[0], 0));  // the caller's stream sees every copy
        uint64_t tot = 0;
        int badh = 0;
        GZHIP(hipMemcpyAsync(&tot, running, 8, hipMemcpyDeviceToHost, st));
        GZHIP(hipMemcpyAsync(&badh, bad, sizeof(int), hipMemcpyDeviceToHost, st));
        GZHIP(hipStreamSynchronize(st));
        drained = true;  // st waited for everything sd ran
        if (badh & 1) return gzfail(OFL_EINVAL, "gzip ranks: values must be float32 integers 0..31");
        if (badh & 2) return gzfail(OFL_ESPACE, "gzip ranks: output buffer too small");
        total = tot;
        if (fill_trace && tn < 400) tn += snprintf(trace + tn, sizeof(trace) - tn, " sync@%.0f", now_us() - t_call);
        host_copy(total);
        if (fill_trace) fprintf(stderr, "gzip fill (us):%s end@%.0f\n", trace, now_us() - t_call);
    }
    for (int64_t c0 = 0; !dout && c0 < L.members; c0 += L.batch) {
        const int nb = (int)std::min<int64_t>(L.batch, L.members - c0);
        enc(c0, nb, slots, sizes);
        hipLaunchKernelGGL(gz::k_gzip_scan, dim3(1), dim3(1024), 0, st, sizes, nb, off, (uint64_t*)nullptr,
                           ~0ull, bad);
        hipLaunchKernelGGL(gz::k_gzip_pack, dim3(nb), dim3(256), 0, st, slots, (uint64_t)L.slot, sizes, off, packed);
        GZHIP(hipGetLastError());
        uint64_t tot = 0;
        int badh = 0;
        GZHIP(hipMemcpyAsync(&tot, off + nb, 8, hipMemcpyDeviceToHost, st));
        GZHIP(hipMemcpyAsync(&badh, bad, sizeof(int), hipMemcpyDeviceToHost, st));
        GZHIP(hipStreamSynchronize(st));
        if (badh) return gzfail(OFL_EINVAL, "gzip ranks: values must be float32 integers 0..31");
        if (total + tot > out_cap) return gzfail(OFL_ESPACE, "gzip ranks: output buffer too small");
        GZHIP(hipMemcpyAsync(out + total, packed, tot, hipMemcpyDeviceToHost, st));
        GZHIP(hipStreamSynchronize(st));
        if (host_dst) memcpy(host_dst + total, out + total, tot);
        total += tot;
    }
    if (d_ph) {
        uint64_t h[gz::tlz::kEncPhases];
        GZHIP(hipMemcpy(h, d_ph, sizeof(h), hipMemcpyDeviceToHost));
        GZHIP(hipFree(d_ph));
        fprintf(stderr, "tlz phases (block 0, 10 ns ticks): load %llu chains[B1 %llu rest %llu] frontier %llu dp %llu parse %llu "
                "ops[walk %llu scan %llu rec %llu] model %llu code %llu bits %llu | jacobi rounds %llu\n",
                (unsigned long long)h[1], (unsigned long long)h[12], (unsigned long long)h[2], (unsigned long long)h[3],
                (unsigned long long)h[4], (unsigned long long)h[5], (unsigned long long)h[13], (unsigned long long)h[14],
                (unsigned long long)h[6], (unsigned long long)h[7], (unsigned long long)h[8], (unsigned long long)h[9],
                (unsigned long long)h[11]);
    }
    *out_len = total;
    return OFL_OK;
}

int ofl_gzip_ranks(const float* x, int64_t n, uint8_t* out, size_t out_cap, size_t* out_len, void* ws,
                   size_t ws_bytes, void* stream) {
    return gzip_ranks_impl(x, n, nullptr, 0, out, out_cap, nullptr, 0, 1, out_len, ws, ws_bytes, stream);
}

int ofl_gzip_ranks_to(const float* x, int64_t n, uint8_t* out, size_t out_cap, uint8_t* host_dst, size_t host_cap,
                      int nthreads, size_t* out_len, void* ws, size_t ws_bytes, void* stream) {
    if (!host_dst) return gzfail(OFL_EINVAL, "gzip ranks to: null host_dst");
    return gzip_ranks_impl(x, n, nullptr, 0, out, out_cap, host_dst, host_cap, std::max(1, nthreads), out_len, ws,
                           ws_bytes, stream);
}

int ofl_gzip_label_to(const float* x, int64_t n, const ofl_label_rec* label_tab, int ntensors, uint8_t* out,
                      size_t out_cap, uint8_t* host_dst, size_t host_cap, int nthreads, size_t* out_len, void* ws,
                      size_t ws_bytes, void* stream) {
    if (!label_tab) return gzfail(OFL_EINVAL, "gzip label: null label_tab");
    return gzip_ranks_impl(x, n, label_tab, ntensors, out, out_cap, host_dst, host_cap, std::max(1, nthreads), out_len,
                           ws, ws_bytes, stream);
}

// Host inflate of a member-indexed gzip stream (every member carries the
// 'BC' extra field that k_gzip_members writes): the members are found from
// their headers alone and inflated on nthreads host threads straight into
// dst (each member's ISIZE gives its output offset).  Streams without the
// field (e.g. gzip.compress output) return OFL_EFORMAT so the caller can use
// gzip.decompress instead; dst == nullptr only measures.
int ofl_gunzip_members(const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_len, int nthreads) {
    if (!src || !out_len) return gzfail(OFL_EINVAL, "gunzip: null argument");
    std::vector<GzMember> mem;
    size_t total = 0;
    if (int rc = parse_members(src, n, mem, total)) return rc;
    using M = GzMember;
    *out_len = total;
    if (!dst) return OFL_OK;
    if (total > cap) return gzfail(OFL_ESPACE, "gunzip: output buffer too small");
    const int nt = (int)std::max<size_t>(1, std::min<size_t>((size_t)std::max(nthreads, 1), mem.size()));
    std::vector<int> bad(nt, 0);
    auto work = [&](int t) {
        z_stream z;
        memset(&z, 0, sizeof(z));
        if (inflateInit2(&z, -15) != Z_OK) { bad[t] = 1; return; }
        const size_t m0 = mem.size() * t / nt, m1 = mem.size() * (t + 1) / nt;
        for (size_t i = m0; i < m1 && !bad[t]; ++i) {
            const M& m = mem[i];
            inflateReset(&z);
            z.next_in = const_cast<Bytef*>(src + m.in);
            z.avail_in = (uInt)m.in_len;
            z.next_out = dst + m.out;
            z.avail_out = m.isize;
            if (inflate(&z, Z_FINISH) != Z_STREAM_END || z.total_out != m.isize ||
                crc32(0L, dst + m.out, m.isize) != m.crc)
                bad[t] = 1;
        }
        inflateEnd(&z);
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
    for (int b : bad)
        if (b) return gzfail(OFL_EINVAL, "gunzip: corrupt member (inflate, size or CRC-32 mismatch)");
    return OFL_OK;
}

int ofl_gzip_member_index(const uint8_t* src, size_t n, int64_t* index, int64_t cap_members, int64_t* nmembers,
                          size_t* out_len, uint32_t* max_isize, int* all_tlz) {
    if (!src || !nmembers || !out_len) return gzfail(OFL_EINVAL, "member index: null argument");
    std::vector<GzMember> mem;
    size_t total = 0;
    if (int rc = parse_members(src, n, mem, total)) return rc;
    *nmembers = (int64_t)mem.size();
    *out_len = total;
    uint32_t mx = 0;
    bool tl = !mem.empty();
    for (const GzMember& m : mem) { mx = std::max(mx, m.isize); tl = tl && m.tlz; }
    if (max_isize) *max_isize = mx;
    if (all_tlz) *all_tlz = tl ? 1 : 0;
    if (!index) return OFL_OK;
    if (cap_members < (int64_t)mem.size()) return gzfail(OFL_ESPACE, "member index: index array too small");
    for (size_t i = 0; i < mem.size(); ++i) {
        index[4 * i + 0] = (int64_t)mem[i].in;
        index[4 * i + 1] = (int64_t)mem[i].in_len | (mem[i].tlz ? (int64_t)1 << 62 : 0);
        index[4 * i + 2] = (int64_t)mem[i].out;
        index[4 * i + 3] = (int64_t)((uint64_t)mem[i].isize | ((uint64_t)mem[i].crc << 32));
    }
    return OFL_OK;
}

size_t ofl_inflate_tlz_workspace_bytes(int64_t nmembers) {
    return 256 + 4 * (size_t)std::max<int64_t>(nmembers, 1) * gz::tlz::kMemSeg;
}

struct LutDev { const float* tab; const int64_t* start; const int64_t* end; int32_t n; };
static int inflate_tlz_enqueue(const uint8_t* src, const int64_t* index, int64_t first, int64_t count, uint8_t* out,
                               size_t out_cap, void* ws, size_t ws_bytes, void* stream, bool reset,
                               const LutDev* lut = nullptr) {
    if (first < 0 || count < 0 || (count && (!src || !index || !out))) return gzfail(OFL_EINVAL, "inflate: null argument");
    if (!ws || ws_bytes < ofl_inflate_tlz_workspace_bytes(first + count)) return gzfail(OFL_ESPACE, "inflate: workspace too small");
    GZHIP(ofl_util::per_device_once([] {
        uint32_t m[32][32];
        crc_matrices(m);
        return hipMemcpyToSymbol(HIP_SYMBOL(gz::c_adv), m, sizeof(m));
    }));
    hipStream_t st = static_cast<hipStream_t>(stream);
    int* status = static_cast<int*>(ws);
    uint32_t* cnt = reinterpret_cast<uint32_t*>(static_cast<char*>(ws) + 256) + first * gz::tlz::kMemSeg;
    if (reset) GZHIP(hipMemsetAsync(status, 0, sizeof(int), st));
    if (count == 0) return OFL_OK;
    static const int dbg = getenv("OFL_TLZ_DEC_STATS") != nullptr;
    gz::tlz::DecArgs a{src, index + 4 * first, count, out, (uint64_t)out_cap, cnt, status,
                       lut ? lut->tab : nullptr, lut ? lut->start : nullptr, lut ? lut->end : nullptr, lut ? lut->n : 0,
                       dbg};
    gzprof_begin(st);
    hipLaunchKernelGGL(gz::tlz::k_tlz_ops, dim3((unsigned)count), dim3(64), sizeof(gz::tlz::DecSmem), st, a);
    gzprof_end(st, "tlz::k_tlz_ops");
    gzprof_begin(st);
    if (lut)
        hipLaunchKernelGGL(gz::tlz::k_tlz_resolve<true>, dim3((unsigned)count), dim3(gz::tlz::kRNT), sizeof(gz::tlz::ResSmem),
                           st, a);
    else
        hipLaunchKernelGGL(gz::tlz::k_tlz_resolve<false>, dim3((unsigned)count), dim3(gz::tlz::kRNT),
                           sizeof(gz::tlz::ResSmem), st, a);
    gzprof_end(st, "tlz::k_tlz_resolve");
    GZHIP(hipGetLastError());
    return OFL_OK;
}

int ofl_inflate_tlz_async(const uint8_t* src, const int64_t* index, int64_t first, int64_t count, uint8_t* out,
                          size_t out_cap, void* ws, size_t ws_bytes, void* stream) {
    return inflate_tlz_enqueue(src, index, first, count, out, out_cap, ws, ws_bytes, stream, first == 0);
}

int ofl_inflate_tlz_launch(const uint8_t* src, const int64_t* index, int64_t first, int64_t count, uint8_t* out,
                           size_t out_cap, void* ws, size_t ws_bytes, void* stream) {
    return inflate_tlz_enqueue(src, index, first, count, out, out_cap, ws, ws_bytes, stream, false);
}

int ofl_inflate_tlz_launch_lut(const uint8_t* src, const int64_t* index, int64_t first, int64_t count, uint8_t* out,
                               size_t out_cap, void* ws, size_t ws_bytes, const float* lut_tab, const int64_t* lut_start,
                               const int64_t* lut_end, int32_t lut_n, void* stream) {
    if (lut_n < 1 || !lut_tab || !lut_start || !lut_end) return gzfail(OFL_EINVAL, "inflate lut: empty table");
    const LutDev lut{lut_tab, lut_start, lut_end, lut_n};
    return inflate_tlz_enqueue(src, index, first, count, out, out_cap, ws, ws_bytes, stream, false, &lut);
}

int ofl_inflate_tlz_check(int64_t nmembers, void* ws, size_t ws_bytes, void* stream) {
    if (nmembers == 0) return OFL_OK;
    if (!ws || ws_bytes < ofl_inflate_tlz_workspace_bytes(nmembers)) return gzfail(OFL_ESPACE, "inflate: workspace too small");
    hipStream_t st = static_cast<hipStream_t>(stream);
    int h = 0;
    GZHIP(hipMemcpyAsync(&h, static_cast<int*>(ws), sizeof(int), hipMemcpyDeviceToHost, st));
    GZHIP(hipStreamSynchronize(st));
    if (h & gz::kInfRange) return gzfail(OFL_ESPACE, "inflate: a member's output falls outside out");
    if (h) return gzfail(OFL_EFORMAT, "inflate: the TLZ decoder refused a member (the generic inflate decides)");
    return OFL_OK;
}

int ofl_inflate_tlz_wait(const uint8_t* src, const int64_t* index, int64_t nmembers, uint8_t* out, size_t out_cap,
                         void* ws, size_t ws_bytes, void* stream) {
    if (nmembers == 0) return OFL_OK;
    if (!ws || ws_bytes < ofl_inflate_tlz_workspace_bytes(nmembers)) return gzfail(OFL_ESPACE, "inflate: workspace too small");
    hipStream_t st = static_cast<hipStream_t>(stream);
    int* status = static_cast<int*>(ws);
    int h = 0;
    GZHIP(hipMemcpyAsync(&h, status, sizeof(int), hipMemcpyDeviceToHost, st));
    GZHIP(hipStreamSynchronize(st));
    if (h & gz::kInfRange) return gzfail(OFL_ESPACE, "inflate: a member's output falls outside out");
    if (h) {
        // not what the TLZ decoder expects: the generic inflate decides (any
        // valid deflate data decodes there; corrupt data fails there too)
        uint32_t mx = 0;
        std::vector<int64_t> hidx(4 * (size_t)nmembers);
        GZHIP(hipMemcpy(hidx.data(), index, 8 * hidx.size(), hipMemcpyDeviceToHost));
        for (int64_t i = 0; i < nmembers; ++i) mx = std::max(mx, (uint32_t)((uint64_t)hidx[4 * i + 3] & 0xffffffffu));
        return ofl_inflate_members(src, index, nmembers, mx, out, out_cap, ws, ws_bytes, stream);
    }
    return OFL_OK;
}

int ofl_inflate_tlz(const uint8_t* src, const int64_t* index, int64_t nmembers, uint8_t* out, size_t out_cap, void* ws,
                    size_t ws_bytes, void* stream) {
    if (nmembers < 0 || (nmembers && (!src || !index || !out))) return gzfail(OFL_EINVAL, "inflate: null argument");
    if (int rc = ofl_inflate_tlz_async(src, index, 0, nmembers, out, out_cap, ws, ws_bytes, stream)) return rc;
    return ofl_inflate_tlz_wait(src, index, nmembers, out, out_cap, ws, ws_bytes, stream);
}

int ofl_gzip_profile(int enable) {
    std::lock_guard<std::mutex> g(g_prof_m);
    for (ProfRec& r : g_prof_pending) { (void)hipEventDestroy(r.a); (void)hipEventDestroy(r.b); }
    g_prof_pending.clear();
    g_prof_on = enable != 0;
    return OFL_OK;
}

int ofl_gzip_profile_collect(char* names, size_t names_cap, double* ms, int64_t* launches, int max_kernels, int* nkernels) {
    if (!names || !ms || !launches || !nkernels) return gzfail(OFL_EINVAL, "profile: null argument");
    std::lock_guard<std::mutex> g(g_prof_m);
    std::vector<std::string> nm;
    std::vector<double> t;
    std::vector<int64_t> k;
    for (ProfRec& r : g_prof_pending) {
        float e = 0.f;
        GZHIP(hipEventSynchronize(r.b));
        GZHIP(hipEventElapsedTime(&e, r.a, r.b));
        size_t i = 0;
        while (i < nm.size() && nm[i] != r.name) ++i;
        if (i == nm.size()) { nm.push_back(r.name); t.push_back(0.0); k.push_back(0); }
        t[i] += e;
        k[i] += 1;
        (void)hipEventDestroy(r.a);
        (void)hipEventDestroy(r.b);
    }
    g_prof_pending.clear();
    std::string all;
    const int nk = (int)std::min<size_t>(nm.size(), (size_t)max_kernels);
    for (int i = 0; i < nk; ++i) {
        all += nm[i];
        all += '\n';
        ms[i] = t[i];
        launches[i] = k[i];
    }
    if (all.size() + 1 > names_cap) return gzfail(OFL_ESPACE, "profile: names buffer too small");
    std::memcpy(names, all.c_str(), all.size() + 1);
    *nkernels = nk;
    return OFL_OK;
}

int ofl_inflate_members(const uint8_t* src, const int64_t* index, int64_t nmembers, uint32_t max_isize, uint8_t* out,
                        size_t out_cap, void* ws, size_t ws_bytes, void* stream) {
    if (nmembers < 0 || (nmembers && (!src || !index || !out))) return gzfail(OFL_EINVAL, "inflate: null argument");
    if (!ws || ws_bytes < 256) return gzfail(OFL_ESPACE, "inflate: workspace too small (256 bytes)");
    static const bool window = [] { const char* v = getenv("OFL_GZ_INFLATE"); return v && v[0] == 'w'; }();
    if (window && max_isize > 65536u)
        return gzfail(OFL_EFORMAT, "inflate: members above 64 KiB of output need the ring decoder");
    if (nmembers == 0) return OFL_OK;
    GZHIP(ofl_util::per_device_once([] {
        uint32_t m[32][32];
        crc_matrices(m);
        hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(gz::c_adv), m, sizeof(m));
        if (e == hipSuccess)
            e = hipFuncSetAttribute((const void*)gz::k_inflate_members<65536, false, false>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(gz::InfSmem<65536, false>));
        return e;
    }));
    hipStream_t st = static_cast<hipStream_t>(stream);
    int* status = static_cast<int*>(ws);
    GZHIP(hipMemsetAsync(status, 0, sizeof(int), st));
    gz::InfArgs a{src, index, nmembers, out, (uint64_t)out_cap, status};
    // OFL_GZ_INFLATE=window: whole-member LDS windows (A/B); default: a
    // 1 KiB LDS ring per member, output stored as produced
    // 1 KiB ring: with the table-driven decode the kernel is scalar-unit
    // bound and more members per CU pay (1 / 2 KiB / 512 B: 12.4 / 13.1 /
    // 12.8 ms for the 1 GiB set; before, 1, 2 and 4 KiB measured the same)
    // the (length, distance) pair table: opt-in (OFL_GZ_PAIR=1).  Measured
    // slower on the 1 GiB rank set: 16.8 vs 12.4 ms per inflate launch
    // (profiles/r03_kc_pair_ab.txt): the 4 KiB table per member cuts the
    // members resident per CU from 26 to 15, and the decode is bound by the
    // scalar issue of many members, not by one member's steps
    static const bool pair = [] { const char* v = getenv("OFL_GZ_PAIR"); return v && v[0] == '1'; }();
    gzprof_begin(st);
    if (!window && pair)
        hipLaunchKernelGGL((gz::k_inflate_members<1024, true, true>), dim3((unsigned)nmembers), dim3(64),
                           sizeof(gz::InfSmem<1024, true>), st, a);
    else if (!window)
        hipLaunchKernelGGL((gz::k_inflate_members<1024, true, false>), dim3((unsigned)nmembers), dim3(64),
                           sizeof(gz::InfSmem<1024, false>), st, a);
    else if (max_isize <= 16384u)
        hipLaunchKernelGGL((gz::k_inflate_members<16384, false, false>), dim3((unsigned)nmembers), dim3(64),
                           sizeof(gz::InfSmem<16384, false>), st, a);
    else
        hipLaunchKernelGGL((gz::k_inflate_members<65536, false, false>), dim3((unsigned)nmembers), dim3(64),
                           sizeof(gz::InfSmem<65536, false>), st, a);
    gzprof_end(st, "k_inflate_members");
    GZHIP(hipGetLastError());
    int h = 0;
    GZHIP(hipMemcpyAsync(&h, status, sizeof(int), hipMemcpyDeviceToHost, st));
    GZHIP(hipStreamSynchronize(st));
    if (h & gz::kInfRange) return gzfail(OFL_ESPACE, "inflate: a member's output falls outside out");
    if (h & gz::kInfCorrupt) return gzfail(OFL_EINVAL, "inflate: corrupt deflate data");
    if (h & gz::kInfSize) return gzfail(OFL_EINVAL, "inflate: member size differs from its ISIZE");
    if (h & gz::kInfCrc) return gzfail(OFL_EINVAL, "inflate: CRC-32 mismatch");
    return OFL_OK;
}

}  // extern "C"

