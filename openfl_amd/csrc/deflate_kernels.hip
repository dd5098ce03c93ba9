// deflate_kernels.hip -- gzip on the GPU for the lossy pipelines' rank arrays
// (SURVEY §8(f) row 3).  Reference: GZIPTransformer.forward
// (kc_pipeline.py:128-156, skc_pipeline.py:201-230, stc_pipeline.py:185-215):
// gzip.compress(float32 ranks bytes), decoded by gzip.decompress.  Any valid
// gzip stream decodes to the same bytes, so the wire stays compatible: the
// output here is a multi-member gzip stream (RFC 1952), one member per 4096
// float32 ranks (16 KiB of input), each member one dynamic-Huffman deflate
// block (RFC 1951), which Python's gzip.decompress reads.
//
// The ranks are small integers stored as float32 (0.0, 1.0, ... < 32), i.e.
// tokens of 4 bytes from a tiny alphabet.  LZ77 runs at token granularity:
// the (3-token key, position) pairs of a member are bitonic-sorted in LDS, each
// position takes the longest match among its 8 nearest earlier positions with
// the same key (>= 3 tokens, <= 64), a greedy parse with one-step lazy
// matching picks the matches (thread 0); the positions in between are coded
// as a copy of the token's previous occurrence (length 4, distance 4 x gap;
// per-thread scans + a block prefix max) or, at a first occurrence, as its 4
// literal bytes.  Per member: symbol histograms in LDS,
// Huffman code lengths (limited to 15 / 7 bits by flattening the
// frequencies), canonical codes, the code-length RLE header, a block scan of
// the tokens' bit costs, bits OR-ed into an LDS buffer, CRC-32 from per-thread
// table CRCs combined with GF(2) shift matrices, then one coalesced copy out.
// Deterministic (bit positions come from scans; OR is order-free).
#include <hip/hip_runtime.h>

#include <algorithm>
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

constexpr int kTok = 4096;                 // float32 tokens per gzip member
constexpr int kNT = 256;
constexpr int kPer = kTok / kNT;           // 16 consecutive tokens per thread
constexpr int kTypes = 32;                 // token values 0..31
constexpr int kOutWords = 8192;            // 32 KiB bit buffer >= worst-case member
constexpr int kOutBytes = 4 * kOutWords;
constexpr int kLit = 286, kDist = 30, kCL = 19;
constexpr int kBatch = 4096;               // members per launch (host loop)
constexpr int kHdr = 18;                   // gzip member header incl. the 'BC' extra field

__constant__ uint16_t c_dbase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129,
                                     193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t c_dext[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t c_clord[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
__constant__ uint16_t c_lbase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59,
                                     67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t c_lext[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint32_t c_adv[32][32];       // raw CRC advance by 2^k zero bytes: GF(2) matrix columns

// Huffman scratch (thread 0), overlaid on the token tables once they are consumed
struct HScratch {
    uint32_t w[2 * kLit];
    int16_t parent[2 * kLit];
    int16_t sym[kLit];
    uint8_t dead[2 * kLit];
    uint16_t rle_sym[kLit + kDist];
    uint16_t rle_ext[kLit + kDist];
};
// The member's bit buffer in LDS.  A member is at most 14.7 KiB of dynamic
// Huffman output: its literal/length alphabet has <= 66 symbols in use (<= 36
// literal byte values of float32 integers 0..31, end of block, <= 29 length
// codes), so the optimal code costs at most a uniform 7-bit code, <= 7 bits
// per literal byte (matches and one-token copies cost less than the literals
// they replace), plus a <= 600-byte header; 17 KiB leaves margin, and a
// member that would not fit is refused (bad flag 4), never truncated.
constexpr int kOutCap = 4352;              // words
constexpr int kHdrW = 160;                 // header words (<= 4642 bits)
struct Smem {
    union {
        struct {
            union {
                int16_t last[kNT][kTypes];  // per thread: last index of each type in its segment; then exclusive prefix max
                uint32_t key[kTok];         // then: (3-token key << 12 | position), sorted
                HScratch h;                 // then: Huffman scratch
            } u;
            alignas(16) uint8_t tk[kTok + 64];  // the member's tokens
        };
        uint32_t out[kOutCap];              // the bit buffer, once the tokens and the Huffman scratch are dead
    };
    uint32_t hdrw[kHdrW];                  // the member header's words (written while the scratch is live)
    uint8_t bestL[kTok];                   // longest earlier match at a position (tokens, 0 = none >= 3)
    union {
        uint32_t crct[256];                // CRC-32 table: only while the tokens are read
        uint16_t bestG[kTok];              // and its distance in tokens
    };
    uint8_t op[kTok];                      // parse: 0 covered, 1 one-token op, 2 match start
    int16_t ptot[8][kTypes];
    uint32_t hl[kLit], hd[kDist], hc[kCL];
    uint8_t ll[kLit], ld[kDist], lc[kCL];
    uint16_t kl[kLit], kd[kDist], kc[kCL];  // bit-reversed canonical codes
    uint32_t scan[kNT / 64];
    uint32_t crc_r[kNT / 64];               // per wave: XOR of its lanes' advanced raw CRCs
    uint32_t hdr_bits, total_bits, nrle, nlit_ndist;
    int bad;
};
static_assert(sizeof(HScratch) <= sizeof(int16_t) * kNT * kTypes, "Huffman scratch fits the token tables");
static_assert(4 * kOutCap <= sizeof(int16_t) * kNT * kTypes + kTok + 64, "bit buffer overlays the token tables");
static_assert(sizeof(Smem) <= 40 * 1024, "four member blocks per CU");

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
// 4 tokens at token offset o (tk is 4-byte aligned and padded)
DEVI uint32_t tk4(const uint8_t* tk, int o) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(tk);
    return __builtin_amdgcn_alignbyte(w[(o >> 2) + 1], w[o >> 2], (uint32_t)(o & 3));
}
constexpr int kMinMatch = 3;    // tokens (12 bytes); shorter runs use the one-token op
constexpr int kMaxMatch = 64;   // tokens (256 of deflate's 258 bytes)
constexpr int kCand = 4;        // nearest earlier positions with the same 3-token key tried (KC ranks: 4 -> ratio 0.1406, 8 -> 0.1390 at 2x the match time, 32 -> 0.1381)

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

struct GzArgs {
    const float* x;
    int64_t n;
    int64_t chunk0;      // first member of this launch
    uint8_t* slots;      // [members][kOutBytes]
    uint32_t* sizes;     // [members]
    int* bad;            // set if a value is not a rank 0..31
    uint64_t* phases;    // diagnostics (OFL_GZ_PHASES): thread 0 of blocks 0..3 stamps each phase; else null
};
constexpr int kPhases = 12;
#define GZ_STAMP(k)                                                                       \
    do {                                                                                  \
        if (a.phases && tid == 0 && blockIdx.x < 4) a.phases[blockIdx.x * kPhases + (k)] = wall_clock64(); \
    } while (0)

__global__ __launch_bounds__(kNT) void k_gzip_members(GzArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    Smem& S = *reinterpret_cast<Smem*>(smem_raw);
    const int tid = threadIdx.x;
    const int64_t c = a.chunk0 + blockIdx.x;
    const int64_t e0 = c * kTok;
    const int ntok = (int)std::min<int64_t>(kTok, a.n - e0);
    GZ_STAMP(0);
    for (int i = tid; i < 256; i += kNT) {
        uint32_t r = (uint32_t)i;
        for (int k = 0; k < 8; ++k) r = (r & 1u) ? (r >> 1) ^ 0xEDB88320u : r >> 1;
        S.crct[i] = r;
    }
    for (int i = tid; i < kLit; i += kNT) S.hl[i] = 0;
    if (tid < kDist) S.hd[tid] = 0;
    if (tid < kCL) S.hc[tid] = 0;
    if (tid == 0) S.bad = 0;
    for (int t = 0; t < kTypes; ++t) S.u.last[tid][t] = -1;
    __syncthreads();

    // ---- tokens, validity, local previous occurrences, raw CRC ----
    const int i0 = tid * kPer;
    const int nv = std::max(0, std::min(kPer, ntok - i0));
    int tok[kPer];
    int prev[kPer];
    uint32_t crc = 0;
    bool bad = false;
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
        tok[q] = 0;
        prev[q] = -1;
        if (q < nv) {
            const float v = a.x[e0 + i0 + q];
            const int t = (int)v;
            const uint32_t bits = __float_as_uint(v);
            if (!(t >= 0 && t < kTypes && bits == __float_as_uint((float)t))) bad = true;
            const int tt = (t >= 0 && t < kTypes) ? t : 0;
            tok[q] = tt;
            S.tk[i0 + q] = (uint8_t)tt;
            prev[q] = S.u.last[tid][tt];
            S.u.last[tid][tt] = (int16_t)(i0 + q);
            for (int b = 0; b < 4; ++b) crc = S.crct[(crc ^ (bits >> (8 * b))) & 0xffu] ^ (crc >> 8);
        }
    }
    if (bad) atomicOr(&S.bad, 1);
    // raw CRC of the member: crc(A | B) = adv(crc(A), |B|) ^ crc(B)
    if (ntok == kTok) {
        // full member, 64 bytes per thread: a tree over the lanes whose level-l
        // shift (64 * 2^l bytes) is the same for every lane (scalar matrix)
        const int lane = tid & 63;
        uint32_t v = crc;
#pragma unroll
        for (int l = 0; l < 6; ++l) {
            const uint32_t o = (uint32_t)__shfl_xor((int)v, 1 << l, 64);
            const uint32_t sh = crc_adv_pow2(v, 6 + l);  // adv over 2^(6+l) bytes
            // the lower lane of a pair holds the earlier bytes
            v = (lane & (1 << l)) ? v : (sh ^ o);
        }
        if (lane == 0) S.crc_r[tid >> 6] = v;
    } else {  // ragged last member: each thread advances over the bytes after it
        uint32_t v = crc_adv(crc, 4u * (uint32_t)std::max(0, ntok - i0 - nv));
        for (int o = 32; o > 0; o >>= 1) v ^= (uint32_t)__shfl_xor((int)v, o, 64);
        if ((tid & 63) == 0) S.crc_r[tid >> 6] = v;
    }
    __syncthreads();
    if (S.bad) {  // block-uniform
        if (tid == 0) { atomicOr(a.bad, 1); a.sizes[blockIdx.x] = 0; }
        return;
    }
    GZ_STAMP(1);
    // exclusive prefix max of the per-thread last indices, per type (in place):
    // thread (type t, part p) walks rows 32p..32p+31, then parts are combined
    {
        const int t = tid & 31, p = tid >> 5;
        int run = -1;
        for (int r = 32 * p; r < 32 * p + 32; ++r) {
            const int v = S.u.last[r][t];
            S.u.last[r][t] = (int16_t)run;
            run = v > run ? v : run;
        }
        S.ptot[p][t] = (int16_t)run;
        __syncthreads();
        int off = -1;
        for (int pp = 0; pp < p; ++pp) off = S.ptot[pp][t] > off ? S.ptot[pp][t] : off;
        for (int r = 32 * p; r < 32 * p + 32; ++r) if (off > S.u.last[r][t]) S.u.last[r][t] = (int16_t)off;
        __syncthreads();
    }
    // one-token op of each position: gap to the previous occurrence (-1: none)
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
        if (q < nv) {
            const int pv = prev[q] >= 0 ? prev[q] : S.u.last[tid][tok[q]];
            prev[q] = pv >= 0 ? i0 + q - pv : -1;
        }
    }
    __syncthreads();  // the last-occurrence tables are dead from here
    GZ_STAMP(2);
    // ---- LZ77 at token granularity: sort (3-token key, position) ----
    // Bitonic network over index tid * kPer + q with the keys in registers:
    // partners < kPer apart are in the same thread, < 64 kPer apart in the
    // same wave (shfl_xor), only the 3 stages with partners 1024 / 2048 apart
    // go through LDS.  Keys are unique (the position is in the low bits), so the
    // order is total.
    for (int i = tid; i < kTok; i += kNT) {
        S.bestL[i] = 0;
        S.bestG[i] = 0;
        S.op[i] = 0;
    }
    uint32_t kv[kPer];
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
        const int i = i0 + q;
        const bool k3 = i + 2 < ntok;
        const uint32_t key = k3 ? ((uint32_t)S.tk[i] | ((uint32_t)S.tk[i + 1] << 5) | ((uint32_t)S.tk[i + 2] << 10)) : 0x7fffu;
        kv[q] = (key << 12) | (uint32_t)i;
    }
#pragma unroll
    for (int k = 2; k <= kTok; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            if (j >= 64 * kPer) {  // across waves: through LDS
                __syncthreads();
#pragma unroll
                for (int q = 0; q < kPer; ++q) S.u.key[i0 + q] = kv[q];
                __syncthreads();
#pragma unroll
                for (int q = 0; q < kPer; ++q) {
                    const int i = i0 + q;
                    const uint32_t o = S.u.key[i ^ j];
                    const bool lower = (i & j) == 0, up = (i & k) == 0;
                    kv[q] = (lower == up) ? min(kv[q], o) : max(kv[q], o);
                }
            } else if (j >= kPer) {  // across lanes of this wave
#pragma unroll
                for (int q = 0; q < kPer; ++q) {
                    const int i = i0 + q;
                    const uint32_t o = (uint32_t)__shfl_xor((int)kv[q], j / kPer, 64);
                    const bool lower = (i & j) == 0, up = (i & k) == 0;
                    kv[q] = (lower == up) ? min(kv[q], o) : max(kv[q], o);
                }
            } else {  // inside this thread
#pragma unroll
                for (int q = 0; q < kPer; ++q) {
                    if ((q & j) == 0) {
                        const bool up = ((i0 + q) & k) == 0;
                        const uint32_t lo = min(kv[q], kv[q + j]), hi = max(kv[q], kv[q + j]);
                        kv[q] = up ? lo : hi;
                        kv[q + j] = up ? hi : lo;
                    }
                }
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kPer; ++q) S.u.key[i0 + q] = kv[q];
    __syncthreads();
    GZ_STAMP(3);
    // longest match among the kCand nearest earlier positions with the same key
    for (int sidx = tid; sidx < kTok; sidx += kNT) {
        const uint32_t me = S.u.key[sidx];
        if ((me >> 12) == 0x7fffu) continue;
        const int i = (int)(me & 0xfffu);
        const int lim = std::min(kMaxMatch, ntok - i);
        int bl = 0, bg = 0;
        for (int c2 = 1; c2 <= kCand && sidx - c2 >= 0; ++c2) {
            const uint32_t o = S.u.key[sidx - c2];
            if ((o >> 12) != (me >> 12)) break;
            const int jj = (int)(o & 0xfffu);
            int L = 3;  // the keys are equal: 3 tokens match
            while (L < lim) {
                const uint32_t d = tk4(S.tk, i + L) ^ tk4(S.tk, jj + L);
                if (d) { L += __builtin_ctz(d) >> 3; break; }
                L += 4;
            }
            L = min(L, lim);
            if (L > bl) { bl = L; bg = i - jj; }
            if (bl == lim) break;
        }
        if (bl >= kMinMatch) { S.bestL[i] = (uint8_t)bl; S.bestG[i] = (uint16_t)bg; }
    }
    __syncthreads();
    GZ_STAMP(4);
    // greedy parse with one-step lazy matching: from position i the parse
    // moves to nxt(i) = i + L(i) if a match starts there (L(i) >= 3 and not
    // L(i+1) > L(i)), else i + 1.  In parallel: thread t's segment
    // [kPer t, kPer t + kPer) maps every entry position to the first parse
    // position past the segment (a match can jump over whole segments);
    // thread 0 chains the kNT segments (kNT dependent steps instead of up to
    // kTok); each thread then walks its segment from its entry and marks the
    // ops.  The ops are exactly the sequential parse's.
    {
        int16_t (*fent)[kPer] = reinterpret_cast<int16_t (*)[kPer]>(S.u.key);  // sort keys are dead
        int16_t* entry = reinterpret_cast<int16_t*>(S.u.key) + kNT * kPer;
        auto nxt = [&](int i) -> int {
            const int L = S.bestL[i];
            return (L >= kMinMatch && !(i + 1 < ntok && S.bestL[i + 1] > L)) ? i + L : i + 1;
        };
        const int s0 = tid * kPer, s1 = s0 + kPer;
        for (int e = kPer - 1; e >= 0; --e) {  // backwards: fent of a later entry is known
            const int p = s0 + e;
            int f = p;
            if (p < ntok) {
                const int q = nxt(p);
                f = (q < s1 && q < ntok) ? fent[tid][q - s0] : q;
            }
            fent[tid][e] = (int16_t)f;
        }
        __syncthreads();
        if (tid == 0) {
            int p = 0;
            for (int t = 0; t < kNT; ++t) {
                entry[t] = (int16_t)p;
                if (p < t * kPer + kPer && p < ntok) p = fent[t][p - t * kPer];
            }
        }
        __syncthreads();
        for (int p = entry[tid]; p < s1 && p < ntok;) {
            const int q = nxt(p);
            S.op[p] = q - p > 1 ? 2 : 1;
            p = q;
        }
    }
    __syncthreads();
    GZ_STAMP(5);
    __syncthreads();
    GZ_STAMP(6);
    // ---- symbol histograms of this thread's ops ----
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
        const int p = i0 + q, o = q < nv ? S.op[p] : 0;
        const bool match = o == 2, copy = o == 1 && prev[q] > 0, lit = o == 1 && !copy;
        const uint32_t bits = __float_as_uint((float)tok[q]);
        const int sa = match ? 257 + len_code(4u * S.bestL[p]) : copy ? 258 : (int)(bits & 0xffu);
        const int sd = dist_code(match ? 4u * S.bestG[p] : copy ? 4u * (uint32_t)prev[q] : 1u);
        // the one-token copy (symbol 258) is most positions' op: counted by
        // ballot; the rest by LDS atomics
        const uint64_t nc = __ballot(copy);
        if ((tid & 63) == 0 && nc) atomicAdd(&S.hl[258], (uint32_t)__popcll(nc));
        if (o != 0 && !copy) atomicAdd(&S.hl[sa], 1u);
        if (match || copy) atomicAdd(&S.hd[sd], 1u);
        if (lit)
#pragma unroll
            for (int b = 1; b < 4; ++b) atomicAdd(&S.hl[(bits >> (8 * b)) & 0xffu], 1u);
    }
    __syncthreads();
    GZ_STAMP(7);
    // ---- wave 0: code lengths and codes (lane 0: the code-length RLE and the
    // header bits) ----
    // (wave 0: literal/length code, wave 1: distance code, concurrently; the
    // serial fallback for > 64 literal symbols uses h.w..h.dead, wave 1's
    // scratch is h.rle_ext, free until the RLE below)
    const int wv = tid >> 6, ln = tid & 63;
    if (wv == 0) {
        HScratch& h = S.u.h;
        if (ln == 0) S.hl[256] = 1;  // end of block
        __builtin_amdgcn_wave_barrier();
        if (!huff_lengths_wave(S.hl, kLit, 15, S.ll, h.w, true) && ln == 0) huff_lengths(S.hl, kLit, 15, S.ll, h, true);
    } else if (wv == 1) {
        HScratch& h = S.u.h;
        const bool anyd = __ballot(ln < kDist && S.hd[ln] != 0u) != 0ull;
        if (!anyd && ln == 0) S.hd[0] = 1;  // one (unused) distance code
        __builtin_amdgcn_wave_barrier();
        huff_lengths_wave(S.hd, kDist, 15, S.ld, reinterpret_cast<uint32_t*>(h.rle_ext), false);  // <= 30 symbols
    }
    __syncthreads();
    if (wv == 1) huff_codes_wave(S.ll, kLit, S.kl);
    if (wv == 2) huff_codes_wave(S.ld, kDist, S.kd);
    if (wv == 0) {
        // run-length code of the concatenated code lengths: the wave finds
        // the used lengths' extents and the run starts by ballots; lane 0
        // then walks the runs (a few dozen) instead of every length
        HScratch& h = S.u.h;
        int nlit = 257, ndist = 1;
        for (int c = 0; c < (kLit + 63) / 64; ++c) {
            const int i = 64 * c + ln;
            const uint64_t m = __ballot(i < kLit && S.ll[i] != 0);
            if (m) nlit = max(nlit, 64 * c + 64 - __builtin_clzll(m));
        }
        {
            const uint64_t m = __ballot(ln < kDist && S.ld[ln] != 0);
            if (m) ndist = max(ndist, 64 - __builtin_clzll(m));
        }
        const int N = nlit + ndist;
        auto val = [&](int i) -> int { return i < nlit ? S.ll[i] : S.ld[i - nlit]; };
        uint64_t starts[(kLit + kDist + 63) / 64];
#pragma unroll
        for (int c = 0; c < (kLit + kDist + 63) / 64; ++c) {
            const int i = 64 * c + ln;
            starts[c] = __ballot(i < N && (i == 0 || val(i) != val(i - 1)));
        }
        if (ln == 0) {
            int nr = 0;
            int c = 0;
            uint64_t m = starts[0];
            int s0 = 0;  // the run start being emitted (position 0 always starts one)
            m &= m - 1;
            for (;;) {
                while (!m && c + 1 < (kLit + kDist + 63) / 64) m = starts[++c];
                const int s1 = m ? 64 * c + __builtin_ctzll(m) : N;
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
        HScratch& h = S.u.h;
        huff_lengths_wave(S.hc, kCL, 7, S.lc, h.w, true);  // <= 19 symbols
        huff_codes_wave(S.lc, kCL, S.kc);
    }
    if (tid == 0) {
        HScratch& h = S.u.h;
        const int nr = (int)S.nrle, nlit = (int)(S.nlit_ndist & 0xffffu), ndist = (int)(S.nlit_ndist >> 16);
        int ncl = kCL;
        while (ncl > 4 && S.lc[c_clord[ncl - 1]] == 0) --ncl;
        // thread 0 owns the header's words: a 64-bit accumulator and plain
        // stores (the ops' first word is OR-ed in after the barrier)
        uint64_t acc = 0;
        int nb = 0;
        uint32_t wi = 0, pos = 0;
        auto put = [&](uint32_t v, int n) {
            acc |= (uint64_t)v << nb;
            nb += n;
            pos += (uint32_t)n;
            if (nb >= 32) { S.hdrw[wi++] = (uint32_t)acc; acc >>= 32; nb -= 32; }
        };
        // member header with a BGZF-style extra field (RFC 1952 FEXTRA,
        // subfield 'BC' = member size - 1, filled in at the end): a reader
        // can find every member without inflating (ofl_gunzip_members);
        // gzip.decompress skips the field
        const uint8_t hdr[kHdr] = {0x1f, 0x8b, 0x08, 0x04, 0, 0, 0, 0, 0x00, 0xff, 6, 0, 'B', 'C', 2, 0, 0, 0};
        for (int i = 0; i < kHdr; ++i) put(hdr[i], 8);
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
        if (nb > 0) S.hdrw[wi] = (uint32_t)acc;
        S.hdr_bits = pos;
    }
    __syncthreads();
    GZ_STAMP(8);
    // the tokens and the Huffman scratch are dead: the bit buffer takes their
    // place, header words first (the ops' first word is OR-ed in after the
    // scan's barrier)
    {
        const uint32_t hw = (S.hdr_bits + 31u) >> 5;
        for (int i = tid; i < kOutCap; i += kNT) S.out[i] = (uint32_t)i < hw ? S.hdrw[i] : 0u;
    }
    // ---- op bits: block scan of the costs, then OR into the buffer ----
    uint32_t mine = 0;
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
        if (q < nv) {
            const int p = i0 + q, o = S.op[p];
            if (o == 2) {
                const int lc = len_code(4u * S.bestL[p]), dc = dist_code(4u * S.bestG[p]);
                mine += S.ll[257 + lc] + c_lext[lc] + S.ld[dc] + c_dext[dc];
            } else if (o == 1 && prev[q] > 0) {
                const int dc = dist_code(4u * (uint32_t)prev[q]);
                mine += S.ll[258] + S.ld[dc] + c_dext[dc];
            } else if (o == 1) {
                const uint32_t bits = __float_as_uint((float)tok[q]);
                for (int b = 0; b < 4; ++b) mine += S.ll[(bits >> (8 * b)) & 0xffu];
            }
        }
    }
    const int lane = tid & 63, w = tid >> 6;
    uint32_t inc = mine;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(inc, o, 64);
        if (lane >= o) inc += t;
    }
    if (lane == 63) S.scan[w] = inc;
    __syncthreads();
    uint32_t pos = S.hdr_bits + inc - mine;
    for (int j = 0; j < w; ++j) pos += S.scan[j];
    if (tid == kNT - 1) S.total_bits = pos + mine;
    // room for the ops, end of block, padding, CRC-32 and ISIZE (see kOutCap)
    const bool fits = pos + mine + 15u + 7u + 64u <= 32u * (uint32_t)kOutCap;
    if (!fits) atomicOr(&S.bad, 2);
    // this thread's ops are one contiguous bit range: gather them in a 64-bit
    // accumulator and store whole words; only the first and the last word
    // can be shared with a neighbour (OR-ed atomically)
    if (fits) {
        uint64_t acc = 0;
        int nb = (int)(pos & 31u);
        uint32_t wi = pos >> 5;
        bool first = true;
        auto put = [&](uint32_t v, int n) {
            acc |= (uint64_t)v << nb;
            nb += n;
            if (nb >= 32) {
                if (first) { atomicOr(&S.out[wi], (uint32_t)acc); first = false; }
                else S.out[wi] = (uint32_t)acc;
                ++wi;
                acc >>= 32;
                nb -= 32;
            }
        };
#pragma unroll
        for (int q = 0; q < kPer; ++q) {
            if (q < nv) {
                const int p = i0 + q, o = S.op[p];
                if (o == 2) {
                    const uint32_t l = 4u * S.bestL[p], d = 4u * S.bestG[p];
                    const int lc = len_code(l), dc = dist_code(d);
                    put(S.kl[257 + lc], S.ll[257 + lc]);
                    put(l - c_lbase[lc], c_lext[lc]);
                    put(S.kd[dc], S.ld[dc]);
                    put(d - c_dbase[dc], c_dext[dc]);
                } else if (o == 1 && prev[q] > 0) {
                    const uint32_t d = 4u * (uint32_t)prev[q];
                    const int dc = dist_code(d);
                    put(S.kl[258], S.ll[258]);
                    put(S.kd[dc], S.ld[dc]);
                    put(d - c_dbase[dc], c_dext[dc]);
                } else if (o == 1) {
                    const uint32_t bits = __float_as_uint((float)tok[q]);
#pragma unroll
                    for (int b = 0; b < 4; ++b) {
                        const uint32_t by = (bits >> (8 * b)) & 0xffu;
                        put(S.kl[by], S.ll[by]);
                    }
                }
            }
        }
        if (nb > 0) atomicOr(&S.out[wi], (uint32_t)acc);
    }
    __syncthreads();
    GZ_STAMP(9);
    // ---- end of block, byte padding, CRC-32 and ISIZE ----
    if (S.bad) {  // block-uniform: the member would not fit the bit buffer
        if (tid == 0) { atomicOr(a.bad, 4); a.sizes[blockIdx.x] = 0; }
        return;
    }
    if (tid == 0) {
        uint32_t p = S.total_bits;
        put_bits(S.out, p, S.kl[256], S.ll[256]); p += S.ll[256];
        p = (p + 7u) & ~7u;
        uint32_t raw = 0;  // full member: waves cover 4096 bytes each; ragged: already advanced
        for (int j = 0; j < kNT / 64; ++j) raw = (ntok == kTok ? crc_adv_pow2(raw, 12) : raw) ^ S.crc_r[j];
        const uint32_t crc32 = crc_adv(0xffffffffu, 4u * (uint32_t)ntok) ^ raw ^ 0xffffffffu;
        put_bits(S.out, p, crc32, 32); p += 32;
        put_bits(S.out, p, 4u * (uint32_t)ntok, 32); p += 32;
        S.total_bits = p;
        put_bits(S.out, 8 * (kHdr - 2), (p >> 3) - 1u, 16);  // BSIZE
        a.sizes[blockIdx.x] = p >> 3;
    }
    __syncthreads();
    const uint32_t nbytes = S.total_bits >> 3;
    uint32_t* dst = reinterpret_cast<uint32_t*>(a.slots + (int64_t)blockIdx.x * kOutBytes);
    for (uint32_t i = tid; i < (nbytes + 3u) / 4u; i += kNT) dst[i] = S.out[i];
    GZ_STAMP(10);
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

// members -> one contiguous stream
__global__ __launch_bounds__(256) void k_gzip_pack(const uint8_t* slots, const uint32_t* sizes, const uint64_t* off,
                                                   uint8_t* packed) {
    if (off[blockIdx.x] == ~0ull) return;  // the batch does not fit the output (reported by the scan)
    const uint8_t* src = slots + (int64_t)blockIdx.x * kOutBytes;
    uint8_t* dst = packed + off[blockIdx.x];
    for (uint32_t i = threadIdx.x; i < sizes[blockIdx.x]; i += 256) dst[i] = src[i];
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
constexpr int kFast = 1 << kFastBits;

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

}  // namespace gz

namespace {
thread_local std::string g_gzerr;
int gzfail(int code, const std::string& m) { g_gzerr = m; return code; }
#define GZHIP(x)                                                                                        \
    do {                                                                                                \
        hipError_t e_ = (x);                                                                            \
        if (e_ != hipSuccess) return gzfail(OFL_EHIP, std::string(#x " failed: ") + hipGetErrorString(e_)); \
    } while (0)

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
// the members of a member-indexed stream (every header carries the 'BC'
// size field): deflate data range, output offset, ISIZE and CRC-32 of each
struct GzMember { size_t in, in_len, out; uint32_t isize, crc; };
// one member at pos: its size (0 if the bytes there are not a member header
// with the 'BC' field) and its record
size_t member_at(const uint8_t* src, size_t n, size_t pos, GzMember& m) {
    const uint8_t* h = src + pos;
    if (n - pos < 26 || h[0] != 0x1f || h[1] != 0x8b || h[2] != 8 || h[3] != 0x04) return 0;
    const size_t xlen = (size_t)h[10] | ((size_t)h[11] << 8);
    size_t bsize = 0;
    for (size_t q = 12; q + 4 <= 12 + xlen && 12 + xlen <= n - pos;) {
        const size_t sl = (size_t)h[q + 2] | ((size_t)h[q + 3] << 8);
        if (h[q] == 'B' && h[q + 1] == 'C' && sl == 2) bsize = ((size_t)h[q + 4] | ((size_t)h[q + 5] << 8)) + 1;
        q += 4 + sl;
    }
    if (bsize < 12 + xlen + 8 || bsize > n - pos) return 0;
    const uint8_t* t = src + pos + bsize - 8;
    m.in = pos + 12 + xlen;
    m.in_len = bsize - 12 - xlen - 8;
    m.crc = (uint32_t)t[0] | ((uint32_t)t[1] << 8) | ((uint32_t)t[2] << 16) | ((uint32_t)t[3] << 24);
    m.isize = (uint32_t)t[4] | ((uint32_t)t[5] << 8) | ((uint32_t)t[6] << 16) | ((uint32_t)t[7] << 24);
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
                    if (h[0] == 0x1f && p + 16 <= n && h[1] == 0x8b && h[2] == 8 && h[3] == 4 && h[12] == 'B' &&
                        h[13] == 'C' && member_at(src, n, p, m))
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
        // members are <= 64 KiB and pieces >= 4 MiB: every piece holds a
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

size_t ofl_gzip_ranks_workspace_bytes(int64_t n) {
    const int64_t members = std::max<int64_t>(1, std::min<int64_t>((n + gz::kTok - 1) / gz::kTok, gz::kBatch));
    return 2 * (size_t)members * gz::kOutBytes + 4 * (size_t)members + 8 * (size_t)(members + 1) + 1024;
}

size_t ofl_gzip_ranks_bound(int64_t n) {
    const int64_t members = std::max<int64_t>(1, (n + gz::kTok - 1) / gz::kTok);
    return (size_t)members * gz::kOutBytes;
}

int ofl_gzip_ranks(const float* x, int64_t n, uint8_t* out, size_t out_cap, size_t* out_len, void* ws,
                   size_t ws_bytes, void* stream) {
    if (n < 1 || !x || !out || !out_len) return gzfail(OFL_EINVAL, "gzip ranks: empty input");
    if (!ws || ws_bytes < ofl_gzip_ranks_workspace_bytes(n)) return gzfail(OFL_ESPACE, "gzip ranks: workspace too small");
    GZHIP(ofl_util::per_device_once([] {  // __constant__ tables and attributes are per device
        uint32_t m[32][32];
        crc_matrices(m);
        hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(gz::c_adv), m, sizeof(m));
        if (e == hipSuccess)
            e = hipFuncSetAttribute((const void*)gz::k_gzip_members, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)sizeof(gz::Smem));
        return e;
    }));
    hipStream_t st = static_cast<hipStream_t>(stream);
    const int64_t members = (n + gz::kTok - 1) / gz::kTok;
    const int64_t batch = std::min<int64_t>(members, gz::kBatch);
    char* w = static_cast<char*>(ws);
    uint8_t* slots = reinterpret_cast<uint8_t*>(w);
    uint8_t* packed = slots + (size_t)batch * gz::kOutBytes;
    uint32_t* sizes = reinterpret_cast<uint32_t*>(packed + (size_t)batch * gz::kOutBytes);
    uint64_t* off = reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(sizes) + ((4 * (size_t)batch + 7) & ~(size_t)7));
    uint64_t* running = off + batch + 1;
    int* bad = reinterpret_cast<int*>(running + 1);
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
    // diagnostics: OFL_GZ_PHASES=1 prints the phase stamps (10 ns ticks) of
    // blocks 0..3 of the first launch to stderr
    static const bool phases = getenv("OFL_GZ_PHASES") != nullptr;
    uint64_t* d_ph = nullptr;
    if (phases) GZHIP(hipMalloc(&d_ph, 8 * 4 * gz::kPhases));
    if (phases) GZHIP(hipMemsetAsync(d_ph, 0, 8 * 4 * gz::kPhases, st));
    size_t total = 0;
    if (dout) {
        GZHIP(hipMemsetAsync(running, 0, sizeof(uint64_t), st));
        for (int64_t c0 = 0; c0 < members; c0 += batch) {
            const int nb = (int)std::min<int64_t>(batch, members - c0);
            gz::GzArgs a{x, n, c0, slots, sizes, bad, c0 == 0 ? d_ph : nullptr};
            hipLaunchKernelGGL(gz::k_gzip_members, dim3(nb), dim3(gz::kNT), sizeof(gz::Smem), st, a);
            hipLaunchKernelGGL(gz::k_gzip_scan, dim3(1), dim3(1024), 0, st, sizes, nb, off, running,
                               (uint64_t)out_cap, bad);
            hipLaunchKernelGGL(gz::k_gzip_pack, dim3(nb), dim3(256), 0, st, slots, sizes, off, dout);
            GZHIP(hipGetLastError());
        }
        uint64_t tot = 0;
        int badh = 0;
        GZHIP(hipMemcpyAsync(&tot, running, 8, hipMemcpyDeviceToHost, st));
        GZHIP(hipMemcpyAsync(&badh, bad, sizeof(int), hipMemcpyDeviceToHost, st));
        GZHIP(hipStreamSynchronize(st));
        if (badh & 1) return gzfail(OFL_EINVAL, "gzip ranks: values must be float32 integers 0..31");
        if (badh & 4) return gzfail(OFL_EHIP, "gzip ranks: a member exceeded the device bit buffer");
        if (badh & 2) return gzfail(OFL_ESPACE, "gzip ranks: output buffer too small");
        total = tot;
    }
    for (int64_t c0 = 0; !dout && c0 < members; c0 += batch) {
        const int nb = (int)std::min<int64_t>(batch, members - c0);
        gz::GzArgs a{x, n, c0, slots, sizes, bad, c0 == 0 ? d_ph : nullptr};
        hipLaunchKernelGGL(gz::k_gzip_members, dim3(nb), dim3(gz::kNT), sizeof(gz::Smem), st, a);
        hipLaunchKernelGGL(gz::k_gzip_scan, dim3(1), dim3(1024), 0, st, sizes, nb, off, (uint64_t*)nullptr,
                           ~0ull, bad);
        hipLaunchKernelGGL(gz::k_gzip_pack, dim3(nb), dim3(256), 0, st, slots, sizes, off, packed);
        GZHIP(hipGetLastError());
        uint64_t tot = 0;
        int badh = 0;
        GZHIP(hipMemcpyAsync(&tot, off + nb, 8, hipMemcpyDeviceToHost, st));
        GZHIP(hipMemcpyAsync(&badh, bad, sizeof(int), hipMemcpyDeviceToHost, st));
        GZHIP(hipStreamSynchronize(st));
        if (badh & 4) return gzfail(OFL_EHIP, "gzip ranks: a member exceeded the device bit buffer");
        if (badh) return gzfail(OFL_EINVAL, "gzip ranks: values must be float32 integers 0..31");
        if (total + tot > out_cap) return gzfail(OFL_ESPACE, "gzip ranks: output buffer too small");
        GZHIP(hipMemcpyAsync(out + total, packed, tot, hipMemcpyDeviceToHost, st));
        GZHIP(hipStreamSynchronize(st));
        total += tot;
    }
    if (d_ph) {
        uint64_t h[4 * gz::kPhases];
        GZHIP(hipMemcpy(h, d_ph, sizeof(h), hipMemcpyDeviceToHost));
        GZHIP(hipFree(d_ph));
        for (int b = 0; b < 4; ++b) {
            fprintf(stderr, "gz phases block %d:", b);
            for (int k = 1; k <= 10; ++k) fprintf(stderr, " %llu", (unsigned long long)(h[b * gz::kPhases + k] - h[b * gz::kPhases + k - 1]));
            fprintf(stderr, "\n");
        }
    }
    *out_len = total;
    return OFL_OK;
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
                          size_t* out_len, uint32_t* max_isize) {
    if (!src || !nmembers || !out_len) return gzfail(OFL_EINVAL, "member index: null argument");
    std::vector<GzMember> mem;
    size_t total = 0;
    if (int rc = parse_members(src, n, mem, total)) return rc;
    *nmembers = (int64_t)mem.size();
    *out_len = total;
    uint32_t mx = 0;
    for (const GzMember& m : mem) mx = std::max(mx, m.isize);
    if (max_isize) *max_isize = mx;
    if (!index) return OFL_OK;
    if (cap_members < (int64_t)mem.size()) return gzfail(OFL_ESPACE, "member index: index array too small");
    for (size_t i = 0; i < mem.size(); ++i) {
        index[4 * i + 0] = (int64_t)mem[i].in;
        index[4 * i + 1] = (int64_t)mem[i].in_len;
        index[4 * i + 2] = (int64_t)mem[i].out;
        index[4 * i + 3] = (int64_t)((uint64_t)mem[i].isize | ((uint64_t)mem[i].crc << 32));
    }
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

