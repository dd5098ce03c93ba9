// eden_kernels.hip -- gfx950 (MI355X / CDNA4) kernels of the Eden codec.
//
// Eden (reference: /root/reference/openfl/pipelines/eden_pipeline.py) encodes
// a slice x of P = 2^p fp32 values as
//     y = H D2 H D1 x / P           (rht twice, :548-549, :475-488)
//     bins = bucketize(y sqrt(P) / |y|, B)  scale = |y|^2 / <C[bins], y>  (:505-525)
// with H the Sylvester Hadamard matrix (:451-473), D1/D2 the rand_diag sign
// diagonals for seed and seed+1 (:403-449), and packs bins into the global
// bit-plane layout (:661-690).  Decode is x' = scale * D1 H D2 H C[bins] / P
// (:613-630).
//
// MI355X design (see DESIGN.md for the roofline):
//  * Every transform is a sequence of FWHT "stages" (one per index bit).  A
//    workgroup owns a tile of up to 2^15 elements; each thread keeps 32
//    elements in VGPRs ("layout" = which 5 index bits live in registers) and
//    runs the stages of those bits as register butterflies.  Between layouts
//    the tile is transposed through LDS with an XOR swizzle that keeps every
//    ds_write / ds_read_b32 wave access bank-conflict-free.
//  * Slices with P <= 2^15 are done in ONE kernel, one workgroup per slice,
//    straight from HBM to bit planes (encode) or planes to HBM (decode).
//  * Larger slices use H_P = H_rows (x) H_cols: a row pass (contiguous 2^15
//    rows), column passes over the remaining bits (2^15-element tiles of
//    2^M rows x 2^(15-M) contiguous columns) and a final row pass.  The two
//    Hadamards meet in the middle column pass, which fuses F1's last stages,
//    D2 and F2's first stages, so a 2-Hadamard encode is 3 HBM passes for
//    P <= 2^25 (5 passes for 2^26..2^29).
//  * D1/D2 signs are regenerated on the fly (no sign tensors in HBM); the two
//    LCG steps are folded into one affine map r2 = A*j + B(seed).
//  * Normalisation uses exact powers of two (2^-floor(p/2) at D2, 2^-ceil(p/2)
//    at the end) instead of the reference's two divisions by float32(sqrt P):
//    identical for even p, < 1e-7 relative apart for odd p.
//  * bucketize is exact with one compare: a 1/64 grid over z (every cell
//    holds <= 1 boundary) stored in LDS with {count, 64*B, C_lo, C_hi}.
//  * Bit planes are produced by in-register 8x8 bit-matrix transposes of 32
//    contiguous bins per thread -> one 32-bit store per plane per thread.
//  * Global addressing: uniform 64-bit base + 32-bit per-lane offsets.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <string>
#include <vector>

#include "eden_tables.h"
#include "ofl_codec.h"
#include "ofl_util.h"

#define DEVI __device__ __forceinline__

#ifndef OFL_COL_SC1
#define OFL_COL_SC1 1
#endif
// cache policy of the large slices' arena I/O (kIoLdAux / kIoStAux below):
// nt both ways -- at MALL-sized waves the streamed x / y / plane bytes then
// do not push a wave's intermediates out of the Infinity Cache (Llama-3-8B
// 444-447 -> 471-472 GiB/s, the 1 GiB set 473-475 -> 508-509,
// profiles/r06_io_nt_ab.txt)
#ifndef OFL_IO_LD_AUX
#define OFL_IO_LD_AUX 2
#endif
#ifndef OFL_IO_ST_AUX
#define OFL_IO_ST_AUX 2
#endif

namespace ofl {

// ---------------------------------------------------------------------------
// Descriptors (host-built once per plan, uploaded on first use)
// ---------------------------------------------------------------------------
struct SliceDesc {
    int64_t x_off;      // encode: element offset of the slice's input in the fp32 arena
    int64_t y_off;      // decode: element offset of the slice's output in the fp32 arena
    int64_t ylen;       // decode: elements of this slice that land in the output
    int64_t ws_off;     // element offset of the slice's intermediate in ws (large slices)
    int64_t pl_off;     // byte offset of the slice's first byte of plane 0
    int64_t pl_stride;  // bytes between planes of this tensor (= P_tot(t) / 8)
    int64_t len;        // encode: valid input elements (<= P), zero padded to P
    int32_t logp;
    int32_t tensor;
    int32_t scale_idx;
    int32_t part_off;   // offset of this slice's partials (large slices)
    int32_t perm;       // ws layout of a 2^25 slice: element bit 15 stored at bit 5 (ws_pos)
    int32_t pad_;
};

struct KArgs {
    const SliceDesc* d;
    const int32_t* list;    // slice indices for this launch
    const int32_t* tstart;  // per-list-entry tile prefix (count + 1), multi-tile kernels
    int32_t count;
    int32_t nbits;
    int32_t lo;             // column passes: first transformed bit
    int32_t do_nu;          // column passes: tile 0 of each slice writes the slice norm
    const float* xin;       // fp32 arena in (encode)
    float* xout;            // fp32 arena out (decode)
    float* ws;              // intermediate buffer base
    const uint8_t* pin;     // planes in (decode)
    uint8_t* pout;          // planes out (encode)
    const uint32_t* seeds;
    float* scales;          // encode: out
    const float* scales_in; // decode: in
    float* part;            // partial sums
    float* nu;              // per-slice norms (large)
    const float* yadd;      // decode: nullable, y = yadd + decoded (apply_delta, float32 add)
    const int32_t* btab;    // column launches: per block {slice, tile << 3 | group} (nullable)
    // round-end fused encode (ofl_eden_encode_wavg): the large slices' x is
    // the float32-rounded delta (sum_c f64(x_c) * w_c) / wsum - f64(base),
    // computed from the collaborators' arenas as the row pass loads it
    const float* const* wx; // collaborator arenas (device array of wc pointers), nullable
    const double* ww;       // their weights (device)
    const float* wbase;     // base model arena, nullable
    double wsum;            // NumPy's float64 sum of the weights
    int32_t wc;             // collaborators (1..16)
    // fused column + small-set launches (k_enc_colm_set / k_dec_colm_set):
    // blocks < sset_first run the small-set groups of table sset
    const int32_t* sset;
    int32_t sset_first;
    // paired row launches (k_enc_rowA2<false> / k_dec_rowC2, row_locate):
    // btab holds npair entries {slice, tile << 3 | pair}; pair = 1: the block
    // also runs tile + 2^(p-18), whose D1 words are the same (0: tstart).
    // The two-blocks-per-CU row kernels all take such a list (pair bits 0
    // but in those two) for a split 5-pass slice's sub-waves
    int32_t npair;
};

// Eden centroids in global memory (copied to LDS per workgroup); the
// bucketize boundaries live in the quantiser table below
__device__ const float g_centroids[8][256] = {
#include "eden_centroids.inc"
};

// ---------------------------------------------------------------------------
// rand_diag (eden_pipeline.py:403-449)
// ---------------------------------------------------------------------------
constexpr uint32_t kLcgA = (uint32_t)(1140671485ull * 1103515245ull);

DEVI uint32_t seed_hash(uint32_t seed) {
    uint32_t s = seed * 1664525u + 1013904223u;  // & mask32 (:423)
    return s * 8121u + 28411u;                    // & mask32 (:424)
}
// r2 = LCG2(LCG1(j + s)) = A*j + B(s)  (:426-430)
DEVI uint32_t seed_b(uint32_t seed) {
    uint32_t s = seed_hash(seed);
    return 1140671485u * (1103515245u * s + 12345u + s) + 12820163u + s;
}
// SplitMix finaliser with the reference's unmasked 33-bit add (:433-436)
DEVI uint32_t rd_mix(uint32_t r2) {
    uint32_t lo = r2 + 0x9E3779B9u;
    uint32_t carry = lo < r2 ? 1u : 0u;
    uint32_t t = lo ^ (lo >> 16) ^ (carry << 16);
    t *= 0x85EBCA6Bu;
    t = (t ^ (t >> 13)) * 0xC2B2AE35u;
    return t ^ (t >> 16);
}
DEVI uint32_t rd_word(uint32_t j, uint32_t b) { return rd_mix(kLcgA * j + b); }
// the 8 sign bits of word j: bit k = 1 <=> nibble k >= 8 <=> element k*S+j is +1 (:440-447)
DEVI uint32_t rd_byte(uint32_t j, uint32_t b) {
    uint32_t x = (rd_word(j, b) >> 3) & 0x11111111u;  // sign bits at 4k
    x = (x | (x >> 3)) & 0x03030303u;                  // -> bits 8m, 8m+1
    x = (x | (x >> 6)) & 0x000F000Fu;                  // -> bits 16m .. 16m+3
    return (x | (x >> 12)) & 0xFFu;                    // -> bits 0 .. 7
}
DEVI float flip_unless(float v, uint32_t plus) {  // plus = 1 -> +v, 0 -> -v
    return __uint_as_float(__float_as_uint(v) ^ ((plus ^ 1u) << 31));
}
DEVI float sgn_elem(float v, uint32_t e, int p, uint32_t b) {
    const uint32_t jm = (1u << (p - 3)) - 1u;
    return flip_unless(v, (rd_word(e & jm, b) >> (4u * (e >> (p - 3)) + 3u)) & 1u);
}

// ---------------------------------------------------------------------------
// Register-layout engine
// ---------------------------------------------------------------------------
// A layout: tile of 2^nb elements; element bit r_i lives in register bit i
// (5 or 6 register bits: 32 or 64 elements per thread); the other element
// bits are the thread index, lowest first.
struct Lay { int nb, r0, r1, r2, r3, r4, r5 = -1; };

template <Lay L> struct LT {
    static constexpr int NR = L.r5 < 0 ? 5 : 6;
    static constexpr int E = 1 << NR;
    static constexpr int rb(int i) {
        return i == 0 ? L.r0 : i == 1 ? L.r1 : i == 2 ? L.r2 : i == 3 ? L.r3 : i == 4 ? L.r4 : L.r5;
    }
    static constexpr uint32_t rmask() { uint32_t m = 0; for (int i = 0; i < NR; ++i) m |= 1u << rb(i); return m; }
    static constexpr uint32_t off(int r) {
        uint32_t o = 0;
        for (int i = 0; i < NR; ++i) if ((r >> i) & 1) o |= 1u << rb(i);
        return o;
    }
    // deposit tid into the non-register bit positions, lowest first
    DEVI static uint32_t base(uint32_t tid) {
        uint32_t b = 0;
        int t = 0;
#pragma unroll
        for (int q = 0; q < L.nb; ++q) {
            if (!((rmask() >> q) & 1u)) { b |= ((tid >> t) & 1u) << q; ++t; }
        }
        return b;
    }
};

// LDS address of tile element e: one pad word per 32 and per 1024 elements.
// Additive over disjoint bit sets (pad(b | o) = pad(b) + pad(o)), so register
// offsets become DS immediates, and conflict-free for every half-wave lane
// pattern the layouts use: lanes varying index bits {0..4}, {5..9}, {2..6},
// {0,1,7,8,9} or {6..10} hit 32 distinct banks (bank = address mod 32).
constexpr uint32_t cpad(uint32_t e) { return e + (e >> 5) + (e >> 10); }
DEVI uint32_t pad(uint32_t e) { return e + (e >> 5) + (e >> 10); }
constexpr size_t lds_floats(int nb) { return ((size_t)1 << nb) + ((size_t)1 << nb >> 5) + ((size_t)1 << nb >> 10); }

// butterflies on every register bit whose element bit is in ACT.  Registers
// (r, r+1) are treated as one 2-wide value so the butterflies issue as packed
// fp32 adds (v_pk_add_f32: two butterflies per instruction; register bit 0
// is the in-pair butterfly, a+b / a-b of the two halves).
typedef float f2v __attribute__((ext_vector_type(2)));
template <Lay L, uint32_t ACT>
DEVI void stages(float (&v)[LT<L>::E]) {
#pragma unroll
    for (int i = 0; i < LT<L>::NR; ++i) {
        if (!((ACT >> LT<L>::rb(i)) & 1u)) continue;
        if (i == 0) {
#pragma unroll
            for (int r = 0; r < LT<L>::E; r += 2) {
                const f2v a = {v[r], v[r]}, b = {v[r + 1], -v[r + 1]};
                const f2v o = a + b;
                v[r] = o.x;
                v[r + 1] = o.y;
            }
        } else {
#pragma unroll
            for (int r = 0; r < LT<L>::E; r += 2) {
                if ((r >> i) & 1) continue;
                const int q = r | (1 << i);
                const f2v a = {v[r], v[r + 1]}, b = {v[q], v[q + 1]};
                const f2v s = a + b, d = a - b;
                v[r] = s.x; v[r + 1] = s.y;
                v[q] = d.x; v[q + 1] = d.y;
            }
        }
    }
}

// a value the compiler cannot hoist or CSE (keeps per-register addresses out of
// loop-invariant code motion: they would pin dozens of VGPRs)
DEVI uint32_t opaque(uint32_t v) { asm volatile("" : "+v"(v)); return v; }

template <Lay A, Lay B>
DEVI void exchange(float (&v)[LT<A>::E], float* s, uint32_t tid) {
    static_assert(LT<A>::E == LT<B>::E, "layouts differ in register count");
    const uint32_t ba = opaque(pad(LT<A>::base(tid)));
#pragma unroll
    for (int r = 0; r < LT<A>::E; ++r) s[ba + cpad(LT<A>::off(r))] = v[r];
    __syncthreads();
    const uint32_t bb = opaque(pad(LT<B>::base(tid)));
#pragma unroll
    for (int r = 0; r < LT<B>::E; ++r) v[r] = s[bb + cpad(LT<B>::off(r))];
    __syncthreads();
}

constexpr uint32_t bits_mask(std::initializer_list<int> l) { uint32_t m = 0; for (int b : l) m |= 1u << b; return m; }

// ---------------------------------------------------------------------------
// Reductions
// ---------------------------------------------------------------------------
DEVI float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
template <int NT>
DEVI float block_sum(float v, float* red) {
    v = wave_sum(v);
    const int w = (threadIdx.x >> 6) & (NT / 64 - 1);  // within an NT-thread (sub-)block
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) t += red[i];
    __syncthreads();
    return t;
}

// ---------------------------------------------------------------------------
// Quantiser tables in LDS.  Grid cell k of z*64 in [k-288, k-287):
//   QEnt{lo = #B < (k-288)/64, 64*B[lo]}  (+inf when lo = 2^b - 1)
// then bin = lo + (64 B[lo] < 64 z) exactly, and C[bin] from a 256-entry table.
// ---------------------------------------------------------------------------
// Bucketize table: one 16-byte entry per grid cell of width 1/64 holds the
// only boundary inside the cell and the centroids on either side, so a bin and
// its centroid cost one LDS read and one compare.
struct QEnt { float b64; int lo; float clo; float chi; };
struct QTab { QEnt grid[EDEN_GRID_CELLS]; };

// The entries are built at compile time from the same generated tables, so a
// workgroup's copy into LDS is independent 16-byte loads (one memory latency)
// instead of a grid -> bounds/centroids chain of dependent loads per entry.
namespace qtab_gen {
constexpr float centroids[8][256] = {
#include "eden_centroids.inc"
};
constexpr unsigned char grid[8][EDEN_GRID_CELLS] = {
#include "eden_grid.inc"
};
constexpr float bounds[8][256] = {
#include "eden_bounds.inc"
};
struct QTabs { QTab t[8]; };
constexpr QTabs make() {
    QTabs r{};
    for (int n = 0; n < 8; ++n) {
        const int nb = (1 << (n + 1)) - 1;
        for (int k = 0; k < EDEN_GRID_CELLS; ++k) {
            const int lo = grid[n][k];
            const bool top = lo >= nb;
            r.t[n].grid[k] = QEnt{top ? __builtin_huge_valf() : bounds[n][lo] * 64.0f, lo, centroids[n][lo],
                                  top ? centroids[n][lo] : centroids[n][lo + 1]};
        }
    }
    return r;
}
}  // namespace qtab_gen
__device__ const qtab_gen::QTabs g_qtabs = qtab_gen::make();

template <int NT>
DEVI void load_qtable(QTab* q, int nbits) {
    const float4* src = reinterpret_cast<const float4*>(&g_qtabs.t[nbits - 1]);
    float4* dst = reinterpret_cast<float4*>(q);
    for (int k = threadIdx.x; k < EDEN_GRID_CELLS; k += NT) dst[k] = src[k];
}

// bucketize + centroid (exact, one compare): returns bin, writes centroid.
// The clamp comes first so NaN lands in a valid cell (fmax(NaN, lo) = lo).
DEVI int quant(float z64, const QTab* q, float& c) {
    const float zc = fminf(fmaxf(z64, -(float)EDEN_GRID_OFF), (float)(EDEN_GRID_OFF - 1));
    const int k = (int)floorf(zc) + EDEN_GRID_OFF;
    const QEnt e = q->grid[k];
    const bool gt = e.b64 < z64;
    c = gt ? e.chi : e.clo;
    return e.lo + (gt ? 1 : 0);
}

// ---------------------------------------------------------------------------
// bins <-> bit planes.  A group is 8 contiguous elements, bins as bytes of a
// 64-bit word (lo = elements 0..3, hi = 4..7).  tr8x8h transposes the 8x8 bit
// matrix (afterwards byte i = plane-i bits of the group, bit t = element t);
// the byte transposes then gather byte i of every group into plane word i.
// ---------------------------------------------------------------------------
DEVI void tr8x8h(uint32_t& lo, uint32_t& hi) {
    uint32_t t;
    t = (lo ^ (lo >> 7)) & 0x00AA00AAu;  lo ^= t ^ (t << 7);
    t = (hi ^ (hi >> 7)) & 0x00AA00AAu;  hi ^= t ^ (t << 7);
    t = (lo ^ (lo >> 14)) & 0x0000CCCCu; lo ^= t ^ (t << 14);
    t = (hi ^ (hi >> 14)) & 0x0000CCCCu; hi ^= t ^ (t << 14);
    t = (lo ^ (hi << 4)) & 0xF0F0F0F0u;  lo ^= t; hi ^= t >> 4;
}
// 4x4 byte transpose: o[i] byte j = r[j] byte i (8 v_perm_b32)
DEVI void t4x4(uint32_t r0, uint32_t r1, uint32_t r2, uint32_t r3, uint32_t& o0, uint32_t& o1, uint32_t& o2,
               uint32_t& o3) {
    const uint32_t t0 = __builtin_amdgcn_perm(r1, r0, 0x05010400u), t1 = __builtin_amdgcn_perm(r1, r0, 0x07030602u);
    const uint32_t t2 = __builtin_amdgcn_perm(r3, r2, 0x05010400u), t3 = __builtin_amdgcn_perm(r3, r2, 0x07030602u);
    o0 = __builtin_amdgcn_perm(t2, t0, 0x05040100u);
    o1 = __builtin_amdgcn_perm(t2, t0, 0x07060302u);
    o2 = __builtin_amdgcn_perm(t3, t1, 0x05040100u);
    o3 = __builtin_amdgcn_perm(t3, t1, 0x07060302u);
}
// 8x8 byte transpose of 64-bit rows given as lo/hi dwords: out row i byte g =
// in row g byte i (an involution)
DEVI void tr_bytes8(const uint32_t (&il)[8], const uint32_t (&ih)[8], uint32_t (&ol)[8], uint32_t (&oh)[8]) {
    t4x4(il[0], il[1], il[2], il[3], ol[0], ol[1], ol[2], ol[3]);
    t4x4(il[4], il[5], il[6], il[7], oh[0], oh[1], oh[2], oh[3]);
    t4x4(ih[0], ih[1], ih[2], ih[3], ol[4], ol[5], ol[6], ol[7]);
    t4x4(ih[4], ih[5], ih[6], ih[7], oh[4], oh[5], oh[6], oh[7]);
}

// quantise one group of 8 contiguous values -> (lo, hi) plane bytes; adds
// <C[bins], y> / ysc.  ysc is a power of two, so z = v * (ysc * zm64) and
// (sum c * v) * ysc round exactly like (v * ysc) * zm64 and sum c * (v * ysc).
// The 8 table reads are issued before any is consumed (LDS latency overlaps).
DEVI void quant_group(const float* vg, float m64, const QTab* q, uint32_t& lo, uint32_t& hi, float& dotv) {
    float z[8];
    uint32_t addr[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        z[t] = vg[t] * m64;
        const float zc = __builtin_amdgcn_fmed3f(z[t], -(float)EDEN_GRID_OFF, (float)(EDEN_GRID_OFF - 1));
        addr[t] = (uint32_t)((int)floorf(zc) + EDEN_GRID_OFF);
    }
    QEnt e[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) e[t] = q->grid[addr[t]];
    __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);  // the 8 DS reads first
    __builtin_amdgcn_sched_group_barrier(0x002, 64, 0); // then the VALU
    lo = 0;
    hi = 0;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        const bool gt = e[t].b64 < z[t];
        dotv = fmaf(gt ? e[t].chi : e[t].clo, vg[t], dotv);
        const uint32_t b = (uint32_t)e[t].lo + (gt ? 1u : 0u);
        if (t < 4) lo |= b << (8 * t); else hi |= b << (8 * (t - 4));
    }
    tr8x8h(lo, hi);
}
// volatile pins order the groups: no group's index math is hoisted ahead of
// the previous group's (all 64 live indices would spill)
template <int N>
DEVI void pin_group(const float* v, float (&vg)[8]) {
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        vg[t] = v[t];
        asm volatile("" : "+v"(vg[t]));
    }
}

// Sum of squares of a thread's values, each square rounded, then added in
// register order: contraction off, so every kernel variant (and context the
// body is inlined into) rounds the same way -- bit-identical partials.
template <int N>
DEVI float sum_sq(const float (&v)[N], float mul = 1.0f) {
#pragma clang fp contract(off)
    float ss = 0.f;
#pragma unroll
    for (int r = 0; r < N; ++r) {
        const float y = v[r] * mul;
        ss += y * y;
    }
    return ss;
}

// 32 contiguous values -> 8 plane words of 32 bits (bit t = element t)
DEVI float quant_pack32(const float (&v)[32], float ysc, float zm64, const QTab* q, uint32_t (&w)[8]) {
    float dot = 0.f;
    const float m64 = ysc * zm64;
    uint32_t xl[4], xh[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        float vg[8];
        pin_group<8>(&v[8 * g], vg);
        quant_group(vg, m64, q, xl[g], xh[g], dot);
        asm volatile("" : "+v"(xl[g]), "+v"(xh[g]), "+v"(dot) :: "memory");  // group done before the next
    }
    t4x4(xl[0], xl[1], xl[2], xl[3], w[0], w[1], w[2], w[3]);
    t4x4(xh[0], xh[1], xh[2], xh[3], w[4], w[5], w[6], w[7]);
    return dot * ysc;
}
// centroids of a group's plane bytes (lo, hi as produced by quant_group)
DEVI void unpack_group(uint32_t lo, uint32_t hi, const float* cen, float* v) {
    tr8x8h(lo, hi);  // involution: byte t = bin of element t
#pragma unroll
    for (int t = 0; t < 4; ++t) v[t] = cen[(lo >> (8 * t)) & 0xffu];
#pragma unroll
    for (int t = 0; t < 4; ++t) v[4 + t] = cen[(hi >> (8 * t)) & 0xffu];
}
// plane words -> centroid values of 32 contiguous elements
DEVI void unpack_centroids32(const uint32_t (&w)[8], const float* cen, float (&v)[32]) {
    uint32_t xl[4], xh[4];
    t4x4(w[0], w[1], w[2], w[3], xl[0], xl[1], xl[2], xl[3]);
    t4x4(w[4], w[5], w[6], w[7], xh[0], xh[1], xh[2], xh[3]);
#pragma unroll
    for (int g = 0; g < 4; ++g) unpack_group(xl[g], xh[g], cen, &v[8 * g]);
}
// 64 contiguous values -> 8 plane words of 64 bits (bit t = element t)
DEVI float quant_pack64(const float (&v)[64], float ysc, float zm64, const QTab* q, uint64_t (&w)[8]) {
    float dot = 0.f;
    const float m64 = ysc * zm64;
    uint32_t xl[8], xh[8];
#pragma unroll
    for (int g = 0; g < 8; ++g) {
        float vg[8];
        pin_group<8>(&v[8 * g], vg);
        quant_group(vg, m64, q, xl[g], xh[g], dot);
        asm volatile("" : "+v"(xl[g]), "+v"(xh[g]), "+v"(dot) :: "memory");  // group done before the next
    }
    uint32_t wl[8], wh[8];
    tr_bytes8(xl, xh, wl, wh);
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = (uint64_t)wl[i] | ((uint64_t)wh[i] << 32);
    return dot * ysc;
}
DEVI void unpack_centroids64(const uint64_t (&w)[8], const float* cen, float (&v)[64]) {
    uint32_t il[8], ih[8], xl[8], xh[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) { il[i] = (uint32_t)w[i]; ih[i] = (uint32_t)(w[i] >> 32); }
    tr_bytes8(il, ih, xl, xh);
#pragma unroll
    for (int g = 0; g < 8; ++g) unpack_group(xl[g], xh[g], cen, &v[8 * g]);
}
DEVI void store_plane_word64(uint8_t* p, uint64_t w) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    if ((a & 7u) == 0) {
        *reinterpret_cast<uint64_t*>(p) = w;
    } else if ((a & 3u) == 0) {
        reinterpret_cast<uint32_t*>(p)[0] = (uint32_t)w;
        reinterpret_cast<uint32_t*>(p)[1] = (uint32_t)(w >> 32);
    } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) p[q] = (uint8_t)(w >> (8 * q));
    }
}
DEVI uint64_t load_plane_word64(const uint8_t* p) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    if ((a & 7u) == 0) return *reinterpret_cast<const uint64_t*>(p);
    if ((a & 3u) == 0) {
        return (uint64_t)reinterpret_cast<const uint32_t*>(p)[0] | ((uint64_t)reinterpret_cast<const uint32_t*>(p)[1] << 32);
    }
    uint64_t r = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) r |= (uint64_t)p[q] << (8 * q);
    return r;
}
DEVI void store_planes64(uint8_t* plane0, uint32_t e, int64_t stride, int nbits, const uint64_t (&w)[8]) {
    uint8_t* p = plane0 + (e >> 3);
    for (int i = 0; i < nbits; ++i) store_plane_word64(p + (int64_t)i * stride, w[i]);
}
DEVI void load_planes64(const uint8_t* plane0, uint32_t e, int64_t stride, int nbits, uint64_t (&w)[8]) {
    const uint8_t* p = plane0 + (e >> 3);
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = 0;
    for (int i = 0; i < nbits; ++i) w[i] = load_plane_word64(p + (int64_t)i * stride);
}

DEVI void store_plane_word(uint8_t* p, uint32_t w) {
    if ((reinterpret_cast<uintptr_t>(p) & 3u) == 0) {
        if constexpr ((OFL_IO_ST_AUX & 2) != 0) __builtin_nontemporal_store(w, reinterpret_cast<uint32_t*>(p));
        else *reinterpret_cast<uint32_t*>(p) = w;
    } else {
        p[0] = (uint8_t)w; p[1] = (uint8_t)(w >> 8); p[2] = (uint8_t)(w >> 16); p[3] = (uint8_t)(w >> 24);
    }
}
DEVI uint32_t load_plane_word(const uint8_t* p) {
    if ((reinterpret_cast<uintptr_t>(p) & 3u) == 0) return *reinterpret_cast<const uint32_t*>(p);
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
// planes at plane0 + byte (e >> 3), stride between planes
DEVI void store_planes(uint8_t* plane0, uint32_t e, int64_t stride, int nbits, const uint32_t (&w)[8]) {
    uint8_t* p = plane0 + (e >> 3);
    for (int i = 0; i < nbits; ++i) store_plane_word(p + (int64_t)i * stride, w[i]);
}
DEVI void load_planes(const uint8_t* plane0, uint32_t e, int64_t stride, int nbits, uint32_t (&w)[8]) {
    const uint8_t* p = plane0 + (e >> 3);
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = 0;
    for (int i = 0; i < nbits; ++i) w[i] = load_plane_word(p + (int64_t)i * stride);
}

DEVI float pow2i(int e) { return __int_as_float((127 + e) << 23); }  // 2^e, |e| < 127

// Hide a value from the optimiser so per-register addresses are recomputed
// (cheap ALU) instead of being kept live across a whole pass (32 VGPRs).

// ---------------------------------------------------------------------------
// fp32 element I/O with valid-length bound (zero padding, :541-546); base is
// block-uniform, offsets 32-bit.
// ---------------------------------------------------------------------------
DEVI void load4(const float* base, uint32_t i, int64_t len, float* v) {
    if ((int64_t)i + 3 < len && ((reinterpret_cast<uintptr_t>(base) & 15u) == 0)) {
        const float4 f = *reinterpret_cast<const float4*>(base + i);
        v[0] = f.x; v[1] = f.y; v[2] = f.z; v[3] = f.w;
    } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = ((int64_t)i + q < len) ? base[i + q] : 0.0f;
    }
}
DEVI void store4(float* base, uint32_t i, int64_t len, const float* v) {
    if ((int64_t)i + 3 < len && ((reinterpret_cast<uintptr_t>(base) & 15u) == 0)) {
        *reinterpret_cast<float4*>(base + i) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) if ((int64_t)i + q < len) base[i + q] = v[q];
    }
}

// y = base + decoded as two rounded float32 operations (apply_delta,
// tensor_codec.py:211: the decoded delta is a float32 array first)
DEVI float add_rn(float b, float d) {
#pragma clang fp contract(off)
    return b + d;
}

// block-uniform slice lookup for multi-tile launches (tile b of the launch)
DEVI void find_tile_at(const KArgs& a, int b, int& slice, uint32_t& tile) {
    if (a.btab) {  // one load instead of a search over the launch's tile prefix
        slice = a.btab[2 * b];
        tile = (uint32_t)a.btab[2 * b + 1] >> 3;
        return;
    }
    int lo = 0, hi = a.count - 1;
    while (lo < hi) {
        int mid = (lo + hi + 1) >> 1;
        if (a.tstart[mid] <= b) lo = mid; else hi = mid - 1;
    }
    slice = a.list[lo];
    tile = (uint32_t)(b - a.tstart[lo]);
}
DEVI void find_tile(const KArgs& a, int& slice, uint32_t& tile) {
    const int b = (int)blockIdx.x;
    if (a.btab) {
        slice = a.btab[2 * b];
        tile = (uint32_t)a.btab[2 * b + 1] >> 3;
        return;
    }
    int lo = 0, hi = a.count - 1;
    while (lo < hi) {
        int mid = (lo + hi + 1) >> 1;
        if (a.tstart[mid] <= b) lo = mid; else hi = mid - 1;
    }
    slice = a.list[lo];
    tile = (uint32_t)(b - a.tstart[lo]);
}

// ===========================================================================
// Layout sets.  Small slices: one set per p in 11..15 (tile = slice, NT =
// 2^(p-5)).  Row passes of large slices reuse the p = 15 set.
//   encode: L1 (load, D1) F1 -> L2 F1 -> L3 F1 | D2 | L3 F2 -> L4 F2 -> L5 F2 (pack)
//   decode: the reverse.
// Lanes 0..31 of every layout vary index bits {0..4}, {5..9}, {2..6} or
// {0,1,7,8,9}, so pad() keeps every exchange bank-conflict-free.
// ===========================================================================
template <int P> struct SmallSet;
template <> struct SmallSet<11> {
    static constexpr Lay L1{11, 0, 1, 8, 9, 10}, L2{11, 2, 3, 4, 5, 6}, L3{11, 5, 7, 8, 9, 10},
                         L4{11, 6, 7, 8, 9, 10}, L5{11, 0, 1, 2, 3, 4};
    static constexpr uint32_t F1a = bits_mask({0, 1, 8, 9, 10}), F1b = bits_mask({2, 3, 4, 5, 6}),
                              F1c = bits_mask({7}), F2c = bits_mask({5, 7, 8, 9, 10}),
                              F2d = bits_mask({6}), F2e = bits_mask({0, 1, 2, 3, 4});
};
template <> struct SmallSet<12> {
    static constexpr Lay L1{12, 0, 1, 9, 10, 11}, L2{12, 2, 3, 4, 5, 6}, L3{12, 7, 8, 9, 10, 11},
                         L4{12, 5, 6, 9, 10, 11}, L5{12, 0, 1, 2, 3, 4};
    static constexpr uint32_t F1a = bits_mask({0, 1, 9, 10, 11}), F1b = bits_mask({2, 3, 4, 5, 6}),
                              F1c = bits_mask({7, 8}), F2c = bits_mask({7, 8, 9, 10, 11}),
                              F2d = bits_mask({5, 6}), F2e = bits_mask({0, 1, 2, 3, 4});
};
template <> struct SmallSet<13> {
    static constexpr Lay L1{13, 0, 1, 10, 11, 12}, L2{13, 2, 3, 4, 5, 6}, L3{13, 7, 8, 9, 10, 11},
                         L4{13, 5, 6, 10, 11, 12}, L5{13, 0, 1, 2, 3, 4};
    static constexpr uint32_t F1a = bits_mask({0, 1, 10, 11, 12}), F1b = bits_mask({2, 3, 4, 5, 6}),
                              F1c = bits_mask({7, 8, 9}), F2c = bits_mask({7, 8, 9, 10, 11}),
                              F2d = bits_mask({5, 6, 12}), F2e = bits_mask({0, 1, 2, 3, 4});
};
template <> struct SmallSet<14> {
    static constexpr Lay L1{14, 0, 1, 11, 12, 13}, L2{14, 2, 3, 4, 5, 6}, L3{14, 7, 8, 9, 10, 11},
                         L4{14, 5, 6, 11, 12, 13}, L5{14, 0, 1, 2, 3, 4};
    static constexpr uint32_t F1a = bits_mask({0, 1, 11, 12, 13}), F1b = bits_mask({2, 3, 4, 5, 6}),
                              F1c = bits_mask({7, 8, 9, 10}), F2c = bits_mask({7, 8, 9, 10, 11}),
                              F2d = bits_mask({5, 6, 12, 13}), F2e = bits_mask({0, 1, 2, 3, 4});
};
template <> struct SmallSet<15> {
    static constexpr Lay L1{15, 0, 1, 12, 13, 14}, L2{15, 2, 3, 4, 5, 6}, L3{15, 7, 8, 9, 10, 11},
                         L4{15, 5, 6, 12, 13, 14}, L5{15, 0, 1, 2, 3, 4};
    static constexpr uint32_t F1a = bits_mask({0, 1, 12, 13, 14}), F1b = bits_mask({2, 3, 4, 5, 6}),
                              F1c = bits_mask({7, 8, 9, 10, 11}), F2c = bits_mask({7, 8, 9, 10, 11}),
                              F2d = bits_mask({5, 6, 12, 13, 14}), F2e = bits_mask({0, 1, 2, 3, 4});
};

// signs of the 32 register elements of layout L from an LDS byte table
// (byte j, bit k = sign of element k*S + j), times mul
template <Lay L>
DEVI void apply_signs_tab(float (&v)[LT<L>::E], uint32_t base, const uint8_t* tab, int p, float mul) {
    const uint32_t jm = (1u << (p - 3)) - 1u;
#pragma unroll
    for (int r = 0; r < LT<L>::E; ++r) {
        const uint32_t e = base | LT<L>::off(r);
        v[r] = flip_unless(v[r] * mul, ((uint32_t)tab[e & jm] >> (e >> (p - 3))) & 1u);
    }
}
// signs of the 32 register elements computed directly (rows of large slices,
// tile start ebase a multiple of 2^15).  For p >= 18 the tile lies inside one
// nibble region (S = 2^(p-3) >= 2^15): j = (ebase mod S) + base + off(r), so
// r2 = A*j + B is one add of the compile-time constant A*off(r) per element.
template <Lay L>
DEVI void apply_signs_direct(float (&v)[LT<L>::E], uint32_t ebase, uint32_t base, int p, uint32_t b, float mul) {
    if (p >= 18) {
        const uint32_t jm = (1u << (p - 3)) - 1u;
        const uint32_t r2b = kLcgA * ((ebase & jm) + base) + b;
        const uint32_t sh = 4u * (ebase >> (p - 3)) + 3u;
#pragma unroll
        for (int r = 0; r < LT<L>::E; ++r)
            v[r] = flip_unless(v[r] * mul, (rd_mix(r2b + kLcgA * LT<L>::off(r)) >> sh) & 1u);
    } else {
#pragma unroll
        for (int r = 0; r < LT<L>::E; ++r) v[r] = sgn_elem(v[r] * mul, ebase + (base | LT<L>::off(r)), p, b);
    }
}

// LDS carve-up of the single-kernel small path
template <int P_LOG> struct SmallSmem {
    static constexpr int NT = 1 << (P_LOG - 5);
    static constexpr int NS = 1 << (P_LOG - 3);
    static constexpr size_t data = (sizeof(float) * lds_floats(P_LOG) + 15) & ~(size_t)15;
    static constexpr size_t tabs = 2 * NS;                                   // bytes
    static constexpr size_t enc = data + tabs + sizeof(QTab) + 4 * 16;
    static constexpr size_t dec = data + tabs + sizeof(float) * 256;
};

// ===========================================================================
// Small slices (2^11 <= P <= 2^15): one NT = 2^(P-5)-thread group per slice,
// whole codec.  The bodies run either as their own workgroup (k_enc_small /
// k_dec_small) or as one of 2^(15-P) sub-blocks of a 1024-thread workgroup of
// the small-set kernels below (every sub-block runs the same P, so they meet
// the same barriers; tid is the thread within the sub-block, sm its LDS).
// st = false: a padding sub-block -- computes, stores nothing.
// ===========================================================================
template <int P_LOG>
DEVI void enc_small_body(const KArgs& a, int si, uint32_t tid, unsigned char* sm, const QTab* qt, float* red,
                         bool st) {
    using S = SmallSet<P_LOG>;
    using SM = SmallSmem<P_LOG>;
    constexpr int NT = SM::NT, NS = SM::NS;
    float* s = reinterpret_cast<float*>(sm);
    uint8_t* tab1 = sm + SM::data;
    uint8_t* tab2 = tab1 + NS;

    const SliceDesc D = a.d[si];
    const uint32_t seed = a.seeds[D.tensor];
    const uint32_t b1 = seed_b(seed), b2 = seed_b(seed + 1u);
    for (int j = tid; j < NS; j += NT) { tab1[j] = (uint8_t)rd_byte(j, b1); tab2[j] = (uint8_t)rd_byte(j, b2); }

    float v[32];
    const float* x = a.xin + D.x_off;
    {
        const uint32_t base = LT<S::L1>::base(tid);
#pragma unroll
        for (int r = 0; r < 32; r += 4) load4(x, base | LT<S::L1>::off(r), D.len, &v[r]);
    }
    __syncthreads();  // tables ready
    apply_signs_tab<S::L1>(v, LT<S::L1>::base(tid), tab1, P_LOG, 1.0f);
    stages<S::L1, S::F1a>(v);
    exchange<S::L1, S::L2>(v, s, tid);
    stages<S::L2, S::F1b>(v);
    exchange<S::L2, S::L3>(v, s, tid);
    stages<S::L3, S::F1c>(v);
    apply_signs_tab<S::L3>(v, LT<S::L3>::base(tid), tab2, P_LOG, pow2i(-(P_LOG / 2)));
    stages<S::L3, S::F2c>(v);
    exchange<S::L3, S::L4>(v, s, tid);
    stages<S::L4, S::F2d>(v);
    exchange<S::L4, S::L5>(v, s, tid);
    stages<S::L5, S::F2e>(v);

    const float ysc = pow2i(-((P_LOG + 1) / 2));
    float ss = sum_sq(v, ysc);
    ss = block_sum<NT>(ss, red);
    const float nu = sqrtf(ss);
    const bool pos = nu > 0.0f;
    const float zm64 = 64.0f * (sqrtf((float)(1 << P_LOG)) / nu);
    uint32_t w[8];
    float dot = quant_pack32(v, ysc, zm64, qt, w);
    if (!pos) dot = 0.f;
    dot = block_sum<NT>(dot, red);
    float scale = pos ? (nu * nu) / dot : 0.0f;
    const bool zero = !pos || isnan(scale);  // reference zero fallback (:517-525)
    if (zero) {
        scale = 0.0f;
#pragma unroll
        for (int i = 0; i < 8; ++i) w[i] = 0;
    }
    if (!st) return;
    store_planes(a.pout + D.pl_off, LT<S::L5>::base(tid), D.pl_stride, a.nbits, w);
    if (tid == 0) a.scales[D.scale_idx] = scale;
}

template <int P_LOG>
DEVI void dec_small_body(const KArgs& a, int si, uint32_t tid, unsigned char* sm, const float* cen, bool st) {
    using S = SmallSet<P_LOG>;
    using SM = SmallSmem<P_LOG>;
    constexpr int NT = SM::NT, NS = SM::NS;
    float* s = reinterpret_cast<float*>(sm);
    uint8_t* tab1 = sm + SM::data;
    uint8_t* tab2 = tab1 + NS;

    const SliceDesc D = a.d[si];
    const uint32_t seed = a.seeds[D.tensor];
    const uint32_t b1 = seed_b(seed), b2 = seed_b(seed + 1u);
    for (int j = tid; j < NS; j += NT) { tab1[j] = (uint8_t)rd_byte(j, b1); tab2[j] = (uint8_t)rd_byte(j, b2); }
    float v[32];
    {
        uint32_t w[8];
        load_planes(a.pin + D.pl_off, LT<S::L5>::base(tid), D.pl_stride, a.nbits, w);
        __syncthreads();
        unpack_centroids32(w, cen, v);
    }
    stages<S::L5, S::F2e>(v);
    exchange<S::L5, S::L4>(v, s, tid);
    stages<S::L4, S::F2d>(v);
    exchange<S::L4, S::L3>(v, s, tid);
    stages<S::L3, S::F2c>(v);
    apply_signs_tab<S::L3>(v, LT<S::L3>::base(tid), tab2, P_LOG, pow2i(-(P_LOG / 2)));
    stages<S::L3, S::F1c>(v);
    exchange<S::L3, S::L2>(v, s, tid);
    stages<S::L2, S::F1b>(v);
    exchange<S::L2, S::L1>(v, s, tid);
    stages<S::L1, S::F1a>(v);
    if (!st) return;
    const float sc = a.scales_in[D.scale_idx];
    const uint32_t base = LT<S::L1>::base(tid);
    apply_signs_tab<S::L1>(v, base, tab1, P_LOG, pow2i(-((P_LOG + 1) / 2)));
#pragma unroll
    for (int r = 0; r < 32; ++r) v[r] = sc * v[r];
    float* y = a.xout + D.y_off;
    if (a.yadd) {
        const float* yb = a.yadd + D.y_off;
#pragma unroll
        for (int r = 0; r < 32; r += 4) {
            float b[4];
            load4(yb, base | LT<S::L1>::off(r), D.ylen, b);
#pragma unroll
            for (int q = 0; q < 4; ++q) v[r + q] = add_rn(b[q], v[r + q]);
        }
    }
#pragma unroll
    for (int r = 0; r < 32; r += 4) store4(y, base | LT<S::L1>::off(r), D.ylen, &v[r]);
}

template <int P_LOG>
__global__ __launch_bounds__(1 << (P_LOG - 5)) void k_enc_small(KArgs a) {
    using SM = SmallSmem<P_LOG>;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    QTab* qt = reinterpret_cast<QTab*>(smem + SM::data + SM::tabs);
    load_qtable<SM::NT>(qt, a.nbits);
    enc_small_body<P_LOG>(a, a.list[blockIdx.x], threadIdx.x, smem, qt, reinterpret_cast<float*>(qt + 1), true);
}

template <int P_LOG>
__global__ __launch_bounds__(1 << (P_LOG - 5)) void k_dec_small(KArgs a) {
    using SM = SmallSmem<P_LOG>;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float* cen = reinterpret_cast<float*>(smem + SM::data + SM::tabs);
    for (int j = threadIdx.x; j < 256; j += SM::NT) cen[j] = g_centroids[a.nbits - 1][j];
    dec_small_body<P_LOG>(a, a.list[blockIdx.x], threadIdx.x, smem, cen, true);
}

// ===========================================================================
// Tiny slices (P <= 2^10): one 256-thread group per slice, LDS-resident
// (latency-bound: more threads per slice shorten every stage).  As above, a
// body runs as its own workgroup or as one of 4 sub-blocks (all of one p) of
// a small-set workgroup.
// ===========================================================================
constexpr int kTinyNT = 256;
DEVI void fwht_lds_generic(float* s, int P, uint32_t tid) {
    for (int h = 1; h < P; h <<= 1) {
        for (int q = tid; q < (P >> 1); q += kTinyNT) {
            const int i = ((q & ~(h - 1)) << 1) | (q & (h - 1));
            const float a = s[i], b = s[i + h];
            s[i] = a + b;
            s[i + h] = a - b;
        }
        __syncthreads();
    }
}
struct TinySmem { float s[1024]; unsigned char bins[1024]; };

DEVI void enc_tiny_body(const KArgs& a, int si, uint32_t tid, TinySmem* ts, const QTab* qt, float* red, bool st) {
    float* s = ts->s;
    unsigned char* bins = ts->bins;
    const SliceDesc D = a.d[si];
    const int p = D.logp, P = 1 << p;
    const uint32_t seed = a.seeds[D.tensor];
    const uint32_t b1 = seed_b(seed), b2 = seed_b(seed + 1u);
    const float* x = a.xin + D.x_off;
    for (int e = tid; e < P; e += kTinyNT) s[e] = sgn_elem(e < D.len ? x[e] : 0.0f, e, p, b1);
    __syncthreads();
    fwht_lds_generic(s, P, tid);
    const float m2 = pow2i(-(p / 2));
    for (int e = tid; e < P; e += kTinyNT) s[e] = sgn_elem(s[e] * m2, e, p, b2);
    __syncthreads();
    fwht_lds_generic(s, P, tid);
    const float ysc = pow2i(-((p + 1) / 2));
    float ss = 0.f;
    for (int e = tid; e < P; e += kTinyNT) {
#pragma clang fp contract(off)
        const float y = s[e] * ysc;
        s[e] = y;
        ss += y * y;
    }
    ss = block_sum<kTinyNT>(ss, red);
    const float nu = sqrtf(ss);
    const bool pos = nu > 0.0f;
    const float zm64 = 64.0f * (sqrtf((float)P) / nu);
    float dot = 0.f;
    for (int e = tid; e < P; e += kTinyNT) {
        float c;
        const int b = pos ? quant(s[e] * zm64, qt, c) : 0;
        if (pos) dot += c * s[e];
        bins[e] = (unsigned char)b;
    }
    dot = block_sum<kTinyNT>(dot, red);
    float scale = pos ? (nu * nu) / dot : 0.0f;
    const bool zero = !pos || isnan(scale);
    if (zero) scale = 0.0f;
    __syncthreads();
    if (!st) return;
    uint8_t* pl = a.pout + D.pl_off;
    for (int q = tid; q < (P >> 3) * a.nbits; q += kTinyNT) {
        const int i = q / (P >> 3), j = q % (P >> 3);
        uint32_t by = 0;
        if (!zero)
            for (int t = 0; t < 8; ++t) by |= ((uint32_t)(bins[8 * j + t] >> i) & 1u) << t;
        pl[(int64_t)i * D.pl_stride + j] = (uint8_t)by;
    }
    if (tid == 0) a.scales[D.scale_idx] = scale;
}

DEVI void dec_tiny_body(const KArgs& a, int si, uint32_t tid, float* s, bool st) {
    const SliceDesc D = a.d[si];
    const int p = D.logp, P = 1 << p;
    const uint32_t seed = a.seeds[D.tensor];
    const uint32_t b1 = seed_b(seed), b2 = seed_b(seed + 1u);
    const uint8_t* pl = a.pin + D.pl_off;
    for (int e = tid; e < P; e += kTinyNT) {
        int b = 0;
        for (int i = 0; i < a.nbits; ++i) b |= ((pl[(int64_t)i * D.pl_stride + (e >> 3)] >> (e & 7)) & 1) << i;
        s[e] = g_centroids[a.nbits - 1][b];
    }
    __syncthreads();
    fwht_lds_generic(s, P, tid);
    const float m2 = pow2i(-(p / 2));
    for (int e = tid; e < P; e += kTinyNT) s[e] = sgn_elem(s[e] * m2, e, p, b2);
    __syncthreads();
    fwht_lds_generic(s, P, tid);
    if (!st) return;
    const float m1 = pow2i(-((p + 1) / 2));
    const float sc = a.scales_in[D.scale_idx];
    float* y = a.xout + D.y_off;
    const float* yb = a.yadd ? a.yadd + D.y_off : nullptr;
    for (int e = tid; e < P; e += kTinyNT)
        if (e < D.ylen) {
            const float d = sc * sgn_elem(s[e] * m1, e, p, b1);
            y[e] = yb ? add_rn(yb[e], d) : d;
        }
}

__global__ __launch_bounds__(kTinyNT) void k_enc_tiny(KArgs a) {
    __shared__ TinySmem ts;
    __shared__ QTab qt[1];
    __shared__ float red[kTinyNT / 64];
    load_qtable<kTinyNT>(qt, a.nbits);
    enc_tiny_body(a, a.list[blockIdx.x], threadIdx.x, &ts, qt, red, true);
}

__global__ __launch_bounds__(kTinyNT) void k_dec_tiny(KArgs a) {
    __shared__ float s[1024];
    dec_tiny_body(a, a.list[blockIdx.x], threadIdx.x, s, true);
}

// ===========================================================================
// Small-set kernels: every tiny and small slice of a call in ONE launch of
// 1024-thread workgroups (instead of one latency-bound launch per size class
// in a chain).  Workgroup b reads its group {P (0: tiny), list offset, count}
// from a.list[3b..3b+2]; a group holds slices of one size: up to 2^(15-P)
// small slices of 2^P elements, or up to 4 tiny slices of one p.  The waves of
// sub-blocks past count end at once.
// ===========================================================================
constexpr int kSetNT = 1024;
template <int P_LOG> struct SetSmem {
    static constexpr int SUB = kSetNT >> (P_LOG - 5);
    static constexpr size_t per = (SmallSmem<P_LOG>::data + SmallSmem<P_LOG>::tabs + 15) & ~(size_t)15;
    static constexpr size_t body = SUB * per;
};
constexpr size_t cmax(size_t a, size_t b) { return a > b ? a : b; }
constexpr size_t kSetBody = cmax(cmax(cmax(SetSmem<11>::body, SetSmem<12>::body), cmax(SetSmem<13>::body, SetSmem<14>::body)),
                                 cmax(SetSmem<15>::body, (kSetNT / kTinyNT) * sizeof(TinySmem)));
constexpr size_t kSetSmemEnc = kSetBody + sizeof(QTab) + sizeof(float) * (kSetNT / 64);
constexpr size_t kSetSmemDec = kSetBody + sizeof(float) * 256;

template <int P_LOG>
DEVI void enc_set_group(const KArgs& a, const int32_t* sl, unsigned char* sm, const QTab* qt, float* red) {
    constexpr int NT = SmallSmem<P_LOG>::NT;
    const uint32_t sub = threadIdx.x / NT;
    enc_small_body<P_LOG>(a, sl[sub], threadIdx.x % NT, sm + sub * SetSmem<P_LOG>::per, qt, red + sub * (NT / 64),
                          true);
}
template <int P_LOG>
DEVI void dec_set_group(const KArgs& a, const int32_t* sl, unsigned char* sm, const float* cen) {
    constexpr int NT = SmallSmem<P_LOG>::NT;
    const uint32_t sub = threadIdx.x / NT;
    dec_small_body<P_LOG>(a, sl[sub], threadIdx.x % NT, sm + sub * SetSmem<P_LOG>::per, cen, true);
}
// threads of a group's sub-blocks (whole waves: every NT >= 64)
DEVI int set_active(int P, int cnt) { return cnt * (P ? (1 << (P - 5)) : kTinyNT); }

// workgroup b of a small-set launch (a.list: its group table)
DEVI void enc_sset_block(const KArgs& a, int b) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    QTab* qt = reinterpret_cast<QTab*>(smem + kSetBody);
    float* red = reinterpret_cast<float*>(qt + 1);
    const int32_t* g = a.list + 3 * b;
    const int P = g[0], cnt = g[2];
    const int32_t* sl = a.list + g[1];
    // waves past the group's sub-blocks end here: a workgroup barrier waits
    // for the waves that have not ended only
    const int act = set_active(P, cnt);
    if ((int)threadIdx.x >= act) return;
    {  // the quantiser table, by the active threads (published by the bodies' first barrier)
        const float4* src = reinterpret_cast<const float4*>(&g_qtabs.t[a.nbits - 1]);
        float4* dst = reinterpret_cast<float4*>(qt);
        for (int k = threadIdx.x; k < EDEN_GRID_CELLS; k += act) dst[k] = src[k];
    }
    switch (P) {
    case 11: enc_set_group<11>(a, sl, smem, qt, red); break;
    case 12: enc_set_group<12>(a, sl, smem, qt, red); break;
    case 13: enc_set_group<13>(a, sl, smem, qt, red); break;
    case 14: enc_set_group<14>(a, sl, smem, qt, red); break;
    case 15: enc_set_group<15>(a, sl, smem, qt, red); break;
    default: {
        const uint32_t sub = threadIdx.x / kTinyNT;
        enc_tiny_body(a, sl[sub], threadIdx.x % kTinyNT, reinterpret_cast<TinySmem*>(smem) + sub, qt,
                      red + sub * (kTinyNT / 64), true);
    }
    }
}
__global__ __launch_bounds__(kSetNT) void k_enc_sset(KArgs a) { enc_sset_block(a, (int)blockIdx.x); }

DEVI void dec_sset_block(const KArgs& a, int b) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float* cen = reinterpret_cast<float*>(smem + kSetBody);
    const int32_t* g = a.list + 3 * b;
    const int P = g[0], cnt = g[2];
    const int32_t* sl = a.list + g[1];
    const int act = set_active(P, cnt);
    if ((int)threadIdx.x >= act) return;  // as in k_enc_sset
    for (int j = threadIdx.x; j < 256; j += act) cen[j] = g_centroids[a.nbits - 1][j];
    switch (P) {
    case 11: dec_set_group<11>(a, sl, smem, cen); break;
    case 12: dec_set_group<12>(a, sl, smem, cen); break;
    case 13: dec_set_group<13>(a, sl, smem, cen); break;
    case 14: dec_set_group<14>(a, sl, smem, cen); break;
    case 15: dec_set_group<15>(a, sl, smem, cen); break;
    default: {
        const uint32_t sub = threadIdx.x / kTinyNT;
        dec_tiny_body(a, sl[sub], threadIdx.x % kTinyNT, reinterpret_cast<TinySmem*>(smem)[sub].s, true);
    }
    }
}
__global__ __launch_bounds__(kSetNT) void k_dec_sset(KArgs a) { dec_sset_block(a, (int)blockIdx.x); }

// ===========================================================================
// Large slices (P >= 2^16): row passes over contiguous 2^15-element rows,
// 512 threads x 64 registers (6 register bits; 2 exchanges per Hadamard)
//   F1: L1 {0,1,11..14} -> L2 {2..6,10} -> L3 {5..10} (F1 does 7,8,9 there)
//   F2: L3 {5..10} -> L4 {11..14,9,10} -> L5 {0..5} (64 contiguous: packing)
// ===========================================================================
struct RowSet6 {
    static constexpr Lay L1{15, 0, 1, 11, 12, 13, 14}, L2{15, 2, 3, 4, 5, 6, 10}, L3{15, 5, 6, 7, 8, 9, 10},
                         L4{15, 11, 12, 13, 14, 9, 10}, L5{15, 0, 1, 2, 3, 4, 5};
    // F1c's layout with element bits 0, 1 in registers: the ws tile moves as
    // float4s (k_enc_rowA's stores, k_dec_rowC's loads); lanes vary bits 2..6,
    // a conflict-free pattern of pad().  Same stages in the same order as L3.
    static constexpr Lay L3F{15, 0, 1, 7, 8, 9, 10};
    static constexpr uint32_t F1a = bits_mask({0, 1, 11, 12, 13, 14}), F1b = bits_mask({2, 3, 4, 5, 6, 10}),
                              F1c = bits_mask({7, 8, 9}), F2c = bits_mask({5, 6, 7, 8, 9, 10}),
                              F2d = bits_mask({11, 12, 13, 14}), F2e = bits_mask({0, 1, 2, 3, 4});
};
using RS = RowSet6;
constexpr int kRowLog = 15;
constexpr int kRowNT = 512;
constexpr size_t kRowSmem = (sizeof(float) * lds_floats(kRowLog) + 15) & ~(size_t)15;
// LDS after the exchange buffer: [tile table][8 wave partials][QTab | centroids]
constexpr int kTabCap = 1024;
struct TileTab { int32_t ts[kTabCap + 1]; int32_t li[kTabCap]; int32_t pad_[3]; };
constexpr size_t kRowTab = kRowSmem;
constexpr size_t kRowRed = kRowTab + sizeof(TileTab);
constexpr size_t kRowExtra = kRowRed + 64;
constexpr size_t kRowSmemA = kRowExtra;
constexpr size_t kRowSmemQ = kRowExtra + sizeof(QTab);
constexpr size_t kRowSmemC = kRowExtra + sizeof(float) * 256;

// block-uniform descriptor/scalar reads: loads issued after the loop's global
// stores are vector loads, so pin their values to SGPRs explicitly (buffer
// resources built from VGPRs turn into waterfall loops)
// Reads through the constant address space are scalar loads (lgkmcnt): vector
// loads would wait on the in-order vmcnt behind the tile prefetch.  Tables are
// written by the host or earlier launches only.
typedef const __attribute__((address_space(4))) uint32_t cu32;
DEVI uint32_t sld(const void* p, int64_t i) { return ((cu32*)p)[i]; }
DEVI SliceDesc udesc(const SliceDesc* d, int si) {
    static_assert(sizeof(SliceDesc) == 80, "SliceDesc layout");
    cu32* p = (cu32*)(d + si);
    uint32_t w[20];
#pragma unroll
    for (int i = 0; i < 20; ++i) w[i] = p[i];
    return __builtin_bit_cast(SliceDesc, w);
}
DEVI float sldf(const float* p, int64_t i) { return __builtin_bit_cast(float, sld(p, i)); }
DEVI uint32_t uu(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// Persistent row launches: one block per CU walks tiles t, t+G, t+2G, ...;
// the next tile's input is in flight in registers while this one computes.
// Persistent row launches: one block per CU walks tiles t, t+G, t+2G, ...
// (G = gridDim.x); the next tile's input is in flight in registers while the
// current one computes.  (Column passes stay one-tile-per-block: their tiles
// read 128 B .. 4 KiB row segments that share DRAM pages with neighbouring
// tiles, and hardware dispatch keeps the tiles in flight a contiguous window;
// persistent column blocks drift apart and measured slower.)
struct TileWalk {
    const KArgs& a;
    TileTab* tab;
    int count, total;
    bool lds;
    DEVI TileWalk(const KArgs& a_, TileTab* tab_, uint32_t tid) : a(a_), tab(tab_) {
        count = a.count;
        lds = count <= kTabCap;
        if (lds) {
            for (int i = (int)tid; i <= count; i += kRowNT) tab->ts[i] = a.tstart[i];
            for (int i = (int)tid; i < count; i += kRowNT) tab->li[i] = a.list[i];
        }
        total = (int)sld(a.tstart, count);
        __syncthreads();
    }
    // LDS and global searches stay separate: a generic (flat) pointer would make
    // every probe wait for all outstanding global loads/stores (vmcnt(0))
    template <typename P>
    static DEVI int search(P ts, int count, int b) {
        int lo = 0, hi = count - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (ts[mid] <= b) lo = mid; else hi = mid - 1;
        }
        return lo;
    }
    DEVI void at(int b, int& slice, uint32_t& tile) const {
        if (lds) {
            const int lo = search(tab->ts, count, b);
            slice = (int)uu((uint32_t)tab->li[lo]);
            tile = uu((uint32_t)(b - tab->ts[lo]));
        } else {
            int lo = 0, hi = count - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if ((int)sld(a.tstart, mid) <= b) lo = mid; else hi = mid - 1;
            }
            slice = (int)sld(a.list, lo);
            tile = (uint32_t)(b - (int)sld(a.tstart, lo));
        }
    }
};

// Tile I/O through raw buffer resources: the tile base and extent live in
// SGPRs, each lane keeps one byte offset (lane bits) and the register part is
// a compile-time soffset/imm (lane and register bits are disjoint, so
// base|off == base+off).  Accesses at or past num_records read 0 / are dropped
// without touching memory; records are kept a multiple of the access width so
// no access straddles the bound, and the <= 3 valid elements of a straddling
// float4 are patched separately.  Nothing here branches on data that is in
// flight: a prefetch must not meet a phi before the tile that consumes it.
// (The clang builtins __builtin_amdgcn_raw_buffer_load_b128 / _b64 of this
// toolchain lower to a 32-bit load; the LLVM intrinsics are bound directly.)
typedef int rsrc_t __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x2 __attribute__((ext_vector_type(2)));
__device__ f32x4 raw_load_f32x4(rsrc_t r, int voff, int soff, int aux) __asm("llvm.amdgcn.raw.buffer.load.v4f32");
__device__ float raw_load_f32(rsrc_t r, int voff, int soff, int aux) __asm("llvm.amdgcn.raw.buffer.load.f32");
__device__ i32x2 raw_load_i32x2(rsrc_t r, int voff, int soff, int aux) __asm("llvm.amdgcn.raw.buffer.load.v2i32");
__device__ uint8_t raw_load_u8(rsrc_t r, int voff, int soff, int aux) __asm("llvm.amdgcn.raw.buffer.load.i8");
__device__ void raw_store_f32x4(f32x4 v, rsrc_t r, int voff, int soff, int aux) __asm("llvm.amdgcn.raw.buffer.store.v4f32");
__device__ void raw_store_f32(float v, rsrc_t r, int voff, int soff, int aux) __asm("llvm.amdgcn.raw.buffer.store.f32");

// Cache policy of the large-slice passes' intermediate (ws) buffer accesses
// (aux operand on gfx950: bit 0 = sc0, bit 1 = nt, bit 4 = sc1).  Tuning
// constants for A/B builds (tools/build_flags_variant.sh ... -DOFL_LD_AUX=2),
// not a platform switch.  Stores sc1: the line leaves the XCD's L2 as it is
// written instead of at the kernel boundary, where a pass would otherwise
// leave up to 32 MiB of dirty L2 behind for the next launch to wait on
// (Llama-3-8B 483.7-483.9 -> 486.5-488.1 GiB/s, the 1 GiB set 514.6-517.5 ->
// 525.2-525.6, profiles/r06_sc1_ab.txt)
#ifndef OFL_LD_AUX
#define OFL_LD_AUX 0
#endif
#ifndef OFL_ST_AUX
#define OFL_ST_AUX 16
#endif
constexpr int kLdAux = OFL_LD_AUX;
constexpr int kStAux = OFL_ST_AUX;
// ... of the large slices' once-read / once-written arena I/O (x loads, y
// stores and the yadd loads, bit-plane loads and stores), separately from
// the intermediates', which MALL-sized waves re-read from the cache
constexpr int kIoLdAux = OFL_IO_LD_AUX;
// k_dec_rowC2's intermediate loads: the decode's last read of a wave's ws
#ifndef OFL_DECC2_LD_AUX
#define OFL_DECC2_LD_AUX 0
#endif
constexpr int kDecC2LdAux = OFL_DECC2_LD_AUX;
constexpr int kIoStAux = OFL_IO_ST_AUX;

// Ladder builds (diagnostics only, WRONG results; tools/r06_ladder.sh):
// -DOFL_LADDER=1 the large-slice passes keep only their tile loads and
// stores (same addresses, layouts and bytes), =2 adds the butterflies and
// the LDS exchanges, =3 adds the sign generation (D1 hashes, the D2 byte
// table); 0 (the product) adds the quantiser / plane pack, the centroid
// unpack and the block reductions.  The partial sums are then written as 1.
#ifndef OFL_LADDER
#define OFL_LADDER 0
#endif
constexpr int kLadder = OFL_LADDER;
// (=5: the product without the sign generation, the bound of cheaper signs)
constexpr bool kLadFly = kLadder == 0 || kLadder >= 2;   // butterflies + exchanges
constexpr bool kLadSign = kLadder == 0 || kLadder == 3;  // sign generation
constexpr bool kLadFull = kLadder == 0 || kLadder == 5;  // quantiser, unpack, reductions
// the memory-only rungs' stand-ins: a plane word from 4 values, values from a plane byte
DEVI uint32_t lad_word(float a, float b, float c, float d) {
    return __float_as_uint(a) ^ __float_as_uint(b) ^ __float_as_uint(c) ^ __float_as_uint(d);
}

// word 3 = 0x00020000: 32-bit data format, as the gfx9 family expects
DEVI rsrc_t mk_rsrc(const void* p, uint32_t bytes) {
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    rsrc_t r;
    r.x = (int)(uint32_t)a;
    r.y = (int)((uint32_t)(a >> 32) & 0xffffu);  // stride 0
    r.z = (int)bytes;
    r.w = 0x00020000;
    return r;
}

// Storage format of the large-slice intermediates.  32 (the product): fp32.
// A/B stubs of narrower intermediates (WRONG results,
// memory pattern only, tools/r06_ws_ab.sh): 16 = the high 16 bits of each
// fp32 (2 B per element), 24 = split planes, the high 16 bits at byte 2e of
// the slice's ws and the next 8 bits at byte 2P + e (3 B per element).
#ifndef OFL_WS_FMT
#define OFL_WS_FMT 32
#endif
constexpr int kWsFmt = OFL_WS_FMT;
static_assert(kWsFmt == 32 || kWsFmt == 24 || kWsFmt == 16, "OFL_WS_FMT: 32, 24 or 16");
__device__ uint16_t raw_load_u16(rsrc_t r, int voff, int soff, int aux) __asm("llvm.amdgcn.raw.buffer.load.i16");
__device__ uint8_t raw_load_u8w(rsrc_t r, int voff, int soff, int aux) __asm("llvm.amdgcn.raw.buffer.load.i8");
__device__ int raw_load_i32w(rsrc_t r, int voff, int soff, int aux) __asm("llvm.amdgcn.raw.buffer.load.i32");
__device__ i32x2 raw_load_i32x2w(rsrc_t r, int voff, int soff, int aux) __asm("llvm.amdgcn.raw.buffer.load.v2i32");
__device__ void raw_store_u16(uint16_t v, rsrc_t r, int voff, int soff, int aux) __asm("llvm.amdgcn.raw.buffer.store.i16");
__device__ void raw_store_u8(uint8_t v, rsrc_t r, int voff, int soff, int aux) __asm("llvm.amdgcn.raw.buffer.store.i8");
__device__ void raw_store_i32(int v, rsrc_t r, int voff, int soff, int aux) __asm("llvm.amdgcn.raw.buffer.store.i32");
__device__ void raw_store_i32x2(i32x2 v, rsrc_t r, int voff, int soff, int aux) __asm("llvm.amdgcn.raw.buffer.store.v2i32");
// a view of the intermediate elements [i0, i0 + bytes / 4) of a slice whose
// ws starts at sw (2^logp elements); offsets below are fp32 byte offsets
struct WsR { rsrc_t h, l; };
DEVI WsR ws_rsrc(const float* sw, int logp, size_t i0, uint32_t bytes) {
    WsR w;
    if constexpr (kWsFmt == 32) {
        w.h = mk_rsrc(sw + i0, bytes);
        w.l = w.h;
    } else {
        const uint8_t* b = reinterpret_cast<const uint8_t*>(sw);
        w.h = mk_rsrc(b + 2 * i0, bytes / 2);
        w.l = mk_rsrc(b + (2ull << logp) + i0, kWsFmt == 24 ? bytes / 4 : 0u);
    }
    return w;
}
DEVI float ws_ld1(const WsR& w, uint32_t vo, uint32_t so, int aux) {
    if constexpr (kWsFmt == 32) return raw_load_f32(w.h, (int)vo, (int)so, aux);
    uint32_t u = (uint32_t)raw_load_u16(w.h, (int)(vo >> 1), (int)(so >> 1), aux) << 16;
    if constexpr (kWsFmt == 24) u |= (uint32_t)raw_load_u8w(w.l, (int)(vo >> 2), (int)(so >> 2), aux) << 8;
    return __uint_as_float(u);
}
DEVI void ws_st1(const WsR& w, uint32_t vo, uint32_t so, float v, int aux) {
    if constexpr (kWsFmt == 32) { raw_store_f32(v, w.h, (int)vo, (int)so, aux); return; }
    const uint32_t u = __float_as_uint(v);
    raw_store_u16((uint16_t)(u >> 16), w.h, (int)(vo >> 1), (int)(so >> 1), aux);
    if constexpr (kWsFmt == 24) raw_store_u8((uint8_t)(u >> 8), w.l, (int)(vo >> 2), (int)(so >> 2), aux);
}
DEVI f32x4 ws_ld4(const WsR& w, uint32_t vo, uint32_t so, int aux) {
    if constexpr (kWsFmt == 32) return raw_load_f32x4(w.h, (int)vo, (int)so, aux);
    const i32x2 h = raw_load_i32x2w(w.h, (int)(vo >> 1), (int)(so >> 1), aux);
    uint32_t l = 0;
    if constexpr (kWsFmt == 24) l = (uint32_t)raw_load_i32w(w.l, (int)(vo >> 2), (int)(so >> 2), aux);
    const uint32_t h0 = (uint32_t)h.x, h1 = (uint32_t)h.y;
    f32x4 q;
    q.x = __uint_as_float((h0 << 16) | ((l & 0xffu) << 8));
    q.y = __uint_as_float((h0 & 0xffff0000u) | (((l >> 8) & 0xffu) << 8));
    q.z = __uint_as_float((h1 << 16) | (((l >> 16) & 0xffu) << 8));
    q.w = __uint_as_float((h1 & 0xffff0000u) | ((l >> 24) << 8));
    return q;
}
DEVI void ws_st4(const WsR& w, uint32_t vo, uint32_t so, f32x4 q, int aux) {
    if constexpr (kWsFmt == 32) { raw_store_f32x4(q, w.h, (int)vo, (int)so, aux); return; }
    const uint32_t a0 = __float_as_uint(q.x), a1 = __float_as_uint(q.y), a2 = __float_as_uint(q.z),
                   a3 = __float_as_uint(q.w);
    const i32x2 h = {(int)((a0 >> 16) | (a1 & 0xffff0000u)), (int)((a2 >> 16) | (a3 & 0xffff0000u))};
    raw_store_i32x2(h, w.h, (int)(vo >> 1), (int)(so >> 1), aux);
    if constexpr (kWsFmt == 24)
        raw_store_i32((int)(((a0 >> 8) & 0xffu) | (a1 & 0xff00u) | ((a2 & 0xff00u) << 8) | ((a3 & 0xff00u) << 16)),
                      w.l, (int)(vo >> 2), (int)(so >> 2), aux);
}
// element i of a slice's intermediate through a plain pointer (k_col)
DEVI float ws_pld(const float* sw, int logp, uint32_t i) {
    if constexpr (kWsFmt == 32) return sw[i];
    const uint8_t* b = reinterpret_cast<const uint8_t*>(sw);
    uint32_t u = (uint32_t)reinterpret_cast<const uint16_t*>(b)[i] << 16;
    if constexpr (kWsFmt == 24) u |= (uint32_t)b[(2ull << logp) + i] << 8;
    return __uint_as_float(u);
}
// SC1: a relaxed agent-scope store, i.e. global_store ... sc1 (as the
// buffer stores' OFL_ST_AUX): the middle passes of col_body (ResNet-50's
// small slices: 0.245 -> 0.239 ms; on the 2^29 slices' outer level-1 passes
// it lost 0.3 %, so those keep plain stores; profiles/r06_colsc1_ab.txt)
template <bool SC1 = false>
DEVI void ws_pst(float* sw, int logp, uint32_t i, float v) {
    if constexpr (kWsFmt == 32 && SC1 && OFL_COL_SC1) {
        __hip_atomic_store(&sw[i], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    if constexpr (kWsFmt == 32) { sw[i] = v; return; }
    uint8_t* b = reinterpret_cast<uint8_t*>(sw);
    const uint32_t u = __float_as_uint(v);
    reinterpret_cast<uint16_t*>(b)[i] = (uint16_t)(u >> 16);
    if constexpr (kWsFmt == 24) b[(2ull << logp) + i] = (uint8_t)(u >> 8);
}
DEVI uint32_t tile_valid(int64_t len) {
    return len <= 0 ? 0u : (len >= (1 << kRowLog) ? (1u << kRowLog) : (uint32_t)len);
}
DEVI float4 bload4(rsrc_t r, uint32_t e, uint32_t k) {
    const f32x4 q = raw_load_f32x4(r, (int)(e * 4u), (int)(k * 4u), kIoLdAux);
    return make_float4(q.x, q.y, q.z, q.w);
}
DEVI void bstore4(rsrc_t r, uint32_t e, uint32_t k, const float* v) {
    const f32x4 q = {v[0], v[1], v[2], v[3]};
    raw_store_f32x4(q, r, (int)(e * 4u), (int)(k * 4u), kIoStAux);
}

// x tile (L1 layout, float4 per register quad); live = false reads nothing
DEVI void fetch_x(const KArgs& a, const SliceDesc& D, uint32_t tile, bool live, uint32_t base1, float (&v)[64]) {
    const uint32_t e0 = tile << kRowLog;
    const uint32_t nv = live ? tile_valid(D.len - (int64_t)e0) : 0u;
    const rsrc_t r = mk_rsrc(a.xin + D.x_off + e0, (nv & ~3u) * 4u);
#pragma unroll
    for (int k = 0; k < 64; k += 4) {
        const float4 f = bload4(r, base1, LT<RS::L1>::off(k));
        v[k] = f.x; v[k + 1] = f.y; v[k + 2] = f.z; v[k + 3] = f.w;
    }
}
// the valid head of a float4 that straddles the slice's input length
// (branch-free per lane: the <= 3 values are block-uniform loads and each
// register takes them by a select, so no register copies or spills)
DEVI void fix_x(const KArgs& a, const SliceDesc& D, uint32_t tile, uint32_t base1, float (&v)[64]) {
    const uint32_t e0 = tile << kRowLog;
    const uint32_t nv = tile_valid(D.len - (int64_t)e0);
    const uint32_t rem = nv & 3u;
    if (rem) {
        const uint32_t eb = nv & ~3u;
        const float* x = a.xin + D.x_off + e0 + eb;
        const float x0 = x[0], x1 = rem > 1u ? x[1] : 0.0f, x2 = rem > 2u ? x[2] : 0.0f;
#pragma unroll
        for (int k = 0; k < 64; k += 4) {
            const bool hit = base1 + LT<RS::L1>::off(k) == eb;
            v[k] = hit ? x0 : v[k];
            v[k + 1] = hit ? x1 : v[k + 1];
            v[k + 2] = hit ? x2 : v[k + 2];
        }
    }
}
DEVI void store_y(const KArgs& a, const SliceDesc& D, uint32_t tile, uint32_t base1, const float (&v)[64]) {
    const uint32_t e0 = tile << kRowLog;
    const uint32_t nv = tile_valid(D.ylen - (int64_t)e0);
    const rsrc_t r = mk_rsrc(a.xout + D.y_off + e0, (nv & ~3u) * 4u);
    if (a.yadd) {  // apply_delta fused: y = base + decoded
        const rsrc_t rb = mk_rsrc(a.yadd + D.y_off + e0, (nv & ~3u) * 4u);
#pragma unroll
        for (int k = 0; k < 64; k += 4) {
            const float4 b = bload4(rb, base1, LT<RS::L1>::off(k));
            const float o[4] = {add_rn(b.x, v[k]), add_rn(b.y, v[k + 1]), add_rn(b.z, v[k + 2]), add_rn(b.w, v[k + 3])};
            bstore4(r, base1, LT<RS::L1>::off(k), o);
        }
    } else {
#pragma unroll
        for (int k = 0; k < 64; k += 4) bstore4(r, base1, LT<RS::L1>::off(k), &v[k]);
    }
    if (nv & 3u) {
        const uint32_t eb = nv & ~3u;
        float* y = a.xout + D.y_off + e0 + eb;
        const float* yb = a.yadd ? a.yadd + D.y_off + e0 + eb : nullptr;
#pragma unroll
        for (int k = 0; k < 64; k += 4)
            if (base1 + LT<RS::L1>::off(k) == eb) {
#pragma unroll
                for (int q = 0; q < 3; ++q)
                    if ((uint32_t)q < (nv & 3u)) y[q] = yb ? add_rn(yb[q], v[k + q]) : v[k + q];
            }
    }
}
// ws tiles are always whole (P is a multiple of the row).
// Interleaved layout of 2^25 slices (D.perm): the element bits (0..4, 15,
// 5..14, 16..) are stored in that order, i.e. bit 15 moves next to the 32
// columns, so the 2^25 middle pass (k_col6<10>: 32 columns x 1024 rows per
// tile) reads and writes 256-B row segments instead of 128-B ones.  A row
// tile t then lives at ((t >> 1) << 16) | ((t & 1) << 5) with a zero bit
// inserted at position 5 of its element index; L3's register bits (5..10)
// simply double.
DEVI constexpr uint32_t ws_row_idx(uint32_t j) { return (j & 31u) | ((j >> 5) << 6); }
DEVI size_t ws_row_i0(const SliceDesc& D, uint32_t tile) {
    return D.perm ? ((size_t)(tile >> 1) << (kRowLog + 1)) + ((tile & 1u) << 5) : ((size_t)tile << kRowLog);
}
DEVI float* ws_row_base(const KArgs& a, const SliceDesc& D, uint32_t tile) { return a.ws + D.ws_off + ws_row_i0(D, tile); }
// the tile's ws view (bytes: fp32 extent of the tile's records)
DEVI WsR ws_row(const KArgs& a, const SliceDesc& D, uint32_t tile, uint32_t bytes) {
    return ws_rsrc(a.ws + D.ws_off, D.logp, ws_row_i0(D, tile), bytes);
}
template <int AUX = kLdAux>
DEVI void fetch_ws(const KArgs& a, const SliceDesc& D, uint32_t tile, bool live, uint32_t base3, float (&v)[64]) {
    if (D.perm) {
        const WsR r = ws_row(a, D, tile, live ? (4u << (kRowLog + 1)) - 128u : 0u);
        const uint32_t b = ws_row_idx(base3);
#pragma unroll
        for (int k = 0; k < 64; ++k) v[k] = ws_ld1(r, b * 4u, (LT<RS::L3>::off(k) << 1) * 4u, AUX);
    } else {
        const WsR r = ws_row(a, D, tile, live ? (4u << kRowLog) : 0u);
#pragma unroll
        for (int k = 0; k < 64; ++k) v[k] = ws_ld1(r, base3 * 4u, LT<RS::L3>::off(k) * 4u, AUX);
    }
}
DEVI void store_ws(const KArgs& a, const SliceDesc& D, uint32_t tile, uint32_t base3, const float (&v)[64]) {
    if (D.perm) {
        const WsR r = ws_row(a, D, tile, (4u << (kRowLog + 1)) - 128u);
        const uint32_t b = ws_row_idx(base3);
#pragma unroll
        for (int k = 0; k < 64; ++k) ws_st1(r, b * 4u, (LT<RS::L3>::off(k) << 1) * 4u, v[k], kStAux);
    } else {
        const WsR r = ws_row(a, D, tile, 4u << kRowLog);
#pragma unroll
        for (int k = 0; k < 64; ++k) ws_st1(r, base3 * 4u, LT<RS::L3>::off(k) * 4u, v[k], kStAux);
    }
}
// ws tile in layout L (element bits 0, 1 in registers 0, 1) as float4s
#ifndef OFL_ROW_WS4
#define OFL_ROW_WS4 1  // A/B builds: 0 = the dword L3 tile I/O in k_enc_rowA / k_dec_rowC
#endif
constexpr bool kRowWs4 = OFL_ROW_WS4 != 0;
template <Lay L>
DEVI void fetch_ws4(const KArgs& a, const SliceDesc& D, uint32_t tile, bool live, uint32_t base, float (&v)[64],
                    int aux = kLdAux) {
    static_assert(LT<L>::rb(0) == 0 && LT<L>::rb(1) == 1, "float4 loads need element bits 0, 1 in registers 0, 1");
    const bool perm = D.perm;
    const WsR r = ws_row(a, D, tile, live ? (perm ? (4u << (kRowLog + 1)) - 128u : 4u << kRowLog) : 0u);
    const uint32_t b = perm ? ws_row_idx(base) : base;
#pragma unroll
    for (int k = 0; k < 64; k += 4) {
        const uint32_t o = LT<L>::off(k);
        const f32x4 f = ws_ld4(r, b * 4u, (perm ? ws_row_idx(o) : o) * 4u, aux);
        v[k] = f.x; v[k + 1] = f.y; v[k + 2] = f.z; v[k + 3] = f.w;
    }
}
template <Lay L>
DEVI void store_ws4(const KArgs& a, const SliceDesc& D, uint32_t tile, uint32_t base, const float (&v)[64]) {
    static_assert(LT<L>::rb(0) == 0 && LT<L>::rb(1) == 1, "float4 stores need element bits 0, 1 in registers 0, 1");
    const bool perm = D.perm;
    const WsR r = ws_row(a, D, tile, perm ? (4u << (kRowLog + 1)) - 128u : 4u << kRowLog);
    const uint32_t b = perm ? ws_row_idx(base) : base;
#pragma unroll
    for (int k = 0; k < 64; k += 4) {
        const uint32_t o = LT<L>::off(k);
        const f32x4 q = {v[k], v[k + 1], v[k + 2], v[k + 3]};
        ws_st4(r, b * 4u, (perm ? ws_row_idx(o) : o) * 4u, q, kStAux);
    }
}

// the memory-only ladder rungs' stand-in for unpack_centroids64: a value per
// byte of the plane words (no bit transposes, no centroid table)
DEVI void lad_unpack64(const uint64_t (&w)[8], float (&v)[64]) {
#pragma unroll
    for (int r = 0; r < 64; ++r) v[r] = (float)((uint32_t)(w[r >> 3] >> (8 * (r & 7))) & 255u);
}

// the tile's 8-byte word of every plane (planes >= nbits read as 0).  A8: the
// launch's plane rows are 8-byte aligned; otherwise bytes.
template <bool A8>
DEVI void fetch_planes(const KArgs& a, const SliceDesc& D, uint32_t tile, bool live, uint32_t base5, uint64_t (&w)[8]) {
    const uint8_t* p0 = a.pin + D.pl_off + ((size_t)tile << (kRowLog - 3));
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const rsrc_t r = mk_rsrc(p0 + (int64_t)i * D.pl_stride, (live && i < a.nbits) ? (1u << (kRowLog - 3)) : 0u);
        if (A8) {
            const i32x2 q = raw_load_i32x2(r, (int)(base5 >> 3), 0, kIoLdAux);
            w[i] = (uint64_t)(uint32_t)q.x | ((uint64_t)(uint32_t)q.y << 32);
        } else {
            uint64_t x = 0;
#pragma unroll
            for (int c = 0; c < 8; ++c)
                x |= (uint64_t)raw_load_u8(r, (int)(base5 >> 3), c, 0) << (8 * c);
            w[i] = x;
        }
    }
}

// encode pass A: x -> D1 -> F1 row stages -> ws ; partial sum of x^2
__global__ __launch_bounds__(kRowNT) void k_enc_rowA(KArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float* s = reinterpret_cast<float*>(smem);
    float* red = reinterpret_cast<float*>(smem + kRowRed);
    const uint32_t tid = threadIdx.x;
    const TileWalk tw(a, reinterpret_cast<TileTab*>(smem + kRowTab), tid);
    int t = (int)blockIdx.x;
    if (t >= tw.total) return;
    const uint32_t base1 = LT<RS::L1>::base(tid), base3 = LT<kRowWs4 ? RS::L3F : RS::L3>::base(tid);
    int si; uint32_t tile;
    tw.at(t, si, tile);
    float nx[64];
    fetch_x(a, udesc(a.d, si), tile, true, base1, nx);
    for (;;) {
        float v[64];
#pragma unroll
        for (int r = 0; r < 64; ++r) v[r] = nx[r];
        const SliceDesc D = udesc(a.d, si);
        const int tn = t + (int)gridDim.x;
        const bool more = tn < tw.total;
        int sn; uint32_t tln;
        tw.at(more ? tn : t, sn, tln);
        fetch_x(a, udesc(a.d, sn), tln, more, base1, nx);
        fix_x(a, D, tile, base1, v);
        const uint32_t b1 = seed_b(sld(a.seeds, D.tensor));
        float ss = kLadFull ? sum_sq(v) : 1.0f;
        if constexpr (kLadSign) apply_signs_direct<RS::L1>(v, tile << kRowLog, base1, D.logp, b1, 1.0f);
        if constexpr (kLadFly) {
            stages<RS::L1, RS::F1a>(v);
            exchange<RS::L1, RS::L2>(v, s, tid);
            stages<RS::L2, RS::F1b>(v);
        }
        if constexpr (kRowWs4) {
            if constexpr (kLadFly) {
                exchange<RS::L2, RS::L3F>(v, s, tid);
                stages<RS::L3F, RS::F1c>(v);
            }
            store_ws4<RS::L3F>(a, D, tile, base3, v);
        } else {
            if constexpr (kLadFly) {
                exchange<RS::L2, RS::L3>(v, s, tid);
                stages<RS::L3, RS::F1c>(v);
            }
            store_ws(a, D, tile, base3, v);
        }
        if constexpr (kLadFull) ss = block_sum<kRowNT>(ss, red);
        if (tid == 0) a.part[D.part_off + tile] = ss;
        if (!more) break;
        t = tn; si = sn; tile = tln;
    }
}

// encode pass C: ws -> F2 row stages -> y -> quantise, pack ; partial dot
__global__ __launch_bounds__(kRowNT) void k_enc_rowC(KArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float* s = reinterpret_cast<float*>(smem);
    float* red = reinterpret_cast<float*>(smem + kRowRed);
    QTab* qt = reinterpret_cast<QTab*>(smem + kRowExtra);
    const uint32_t tid = threadIdx.x;
    load_qtable<kRowNT>(qt, a.nbits);
    const TileWalk tw(a, reinterpret_cast<TileTab*>(smem + kRowTab), tid);  // its barrier publishes qt
    int t = (int)blockIdx.x;
    if (t >= tw.total) return;
    const uint32_t base3 = LT<RS::L3>::base(tid), base5 = LT<RS::L5>::base(tid);
    int si; uint32_t tile;
    tw.at(t, si, tile);
    float nx[64];
    fetch_ws(a, udesc(a.d, si), tile, true, base3, nx);
    for (;;) {
        float v[64];
#pragma unroll
        for (int r = 0; r < 64; ++r) v[r] = nx[r];
        const SliceDesc D = udesc(a.d, si);
        const int tn = t + (int)gridDim.x;
        const bool more = tn < tw.total;
        int sn; uint32_t tln;
        tw.at(more ? tn : t, sn, tln);
        const SliceDesc Dn = udesc(a.d, sn);
        fetch_ws(a, Dn, tln, more, base3, nx);
        if constexpr (kLadFly) {
            stages<RS::L3, RS::F2c>(v);
            exchange<RS::L3, RS::L4>(v, s, tid);
            stages<RS::L4, RS::F2d>(v);
            exchange<RS::L4, RS::L5>(v, s, tid);
            stages<RS::L5, RS::F2e>(v);
        }
        __builtin_amdgcn_sched_barrier(0);  // keep the quantiser out of the butterflies (VGPR cap)
        const float nu = sldf(a.nu, si);
        const float ysc = pow2i(-((D.logp + 1) / 2));
        const float zm64 = 64.0f * (sqrtf((float)(1ll << D.logp)) / nu);
        uint64_t wd[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) wd[i] = 0;
        float dot = 1.0f;
        if constexpr (kLadFull) {
            dot = quant_pack64(v, ysc, zm64, qt, wd);
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i)
                wd[i] = (uint64_t)lad_word(v[8 * i], v[8 * i + 1], v[8 * i + 2], v[8 * i + 3]) |
                        ((uint64_t)lad_word(v[8 * i + 4], v[8 * i + 5], v[8 * i + 6], v[8 * i + 7]) << 32);
        }
        if (!(nu > 0.0f)) {
            dot = 0.f;
#pragma unroll
            for (int i = 0; i < 8; ++i) wd[i] = 0;
        }
        store_planes64(a.pout + D.pl_off, (tile << kRowLog) + base5, D.pl_stride, a.nbits, wd);
        if constexpr (kLadFull) dot = block_sum<kRowNT>(dot, red);
        if (tid == 0) a.part[D.part_off + tile] = dot;
        if (!more) break;
        t = tn; si = sn; tile = tln;
    }
}

// decode pass A: planes -> C[bins] -> G1 row stages -> ws
template <bool A8>
__global__ __launch_bounds__(kRowNT) void k_dec_rowA(KArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float* s = reinterpret_cast<float*>(smem);
    float* cen = reinterpret_cast<float*>(smem + kRowExtra);
    const uint32_t tid = threadIdx.x;
    if (tid < 256) cen[tid] = g_centroids[a.nbits - 1][tid];
    const TileWalk tw(a, reinterpret_cast<TileTab*>(smem + kRowTab), tid);  // its barrier publishes cen
    int t = (int)blockIdx.x;
    if (t >= tw.total) return;
    const uint32_t base3 = LT<RS::L3>::base(tid), base5 = LT<RS::L5>::base(tid);
    int si; uint32_t tile;
    tw.at(t, si, tile);
    uint64_t nw[8];
    fetch_planes<A8>(a, udesc(a.d, si), tile, true, base5, nw);
    for (;;) {
        float v[64];
        if constexpr (kLadFull) unpack_centroids64(nw, cen, v);
        else lad_unpack64(nw, v);
        const SliceDesc D = udesc(a.d, si);
        const int tn = t + (int)gridDim.x;
        const bool more = tn < tw.total;
        int sn; uint32_t tln;
        tw.at(more ? tn : t, sn, tln);
        fetch_planes<A8>(a, udesc(a.d, sn), tln, more, base5, nw);
        if constexpr (kLadFly) {
            stages<RS::L5, RS::F2e>(v);
            exchange<RS::L5, RS::L4>(v, s, tid);
            stages<RS::L4, RS::F2d>(v);
            exchange<RS::L4, RS::L3>(v, s, tid);
            stages<RS::L3, RS::F2c>(v);
        }
        // (one more exchange to L3F for float4 stores: 494 -> 533 us per wave,
        // profiles/r03_deca_ws4_ab.txt)
        store_ws(a, D, tile, base3, v);
        if (!more) break;
        t = tn; si = sn; tile = tln;
    }
}

// decode pass C: ws -> G2 row stages -> D1, scale -> y
__global__ __launch_bounds__(kRowNT) void k_dec_rowC(KArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float* s = reinterpret_cast<float*>(smem);
    const uint32_t tid = threadIdx.x;
    const TileWalk tw(a, reinterpret_cast<TileTab*>(smem + kRowTab), tid);
    int t = (int)blockIdx.x;
    if (t >= tw.total) return;
    const uint32_t base1 = LT<RS::L1>::base(tid), base3 = LT<kRowWs4 ? RS::L3F : RS::L3>::base(tid);
    int si; uint32_t tile;
    tw.at(t, si, tile);
    float nx[64];
    if constexpr (kRowWs4) fetch_ws4<RS::L3F>(a, udesc(a.d, si), tile, true, base3, nx);
    else fetch_ws(a, udesc(a.d, si), tile, true, base3, nx);
    for (;;) {
        float v[64];
#pragma unroll
        for (int r = 0; r < 64; ++r) v[r] = nx[r];
        const SliceDesc D = udesc(a.d, si);
        const int tn = t + (int)gridDim.x;
        const bool more = tn < tw.total;
        int sn; uint32_t tln;
        tw.at(more ? tn : t, sn, tln);
        if constexpr (kRowWs4) fetch_ws4<RS::L3F>(a, udesc(a.d, sn), tln, more, base3, nx);
        else fetch_ws(a, udesc(a.d, sn), tln, more, base3, nx);
        const uint32_t b1 = seed_b(sld(a.seeds, D.tensor));
        if constexpr (kLadFly) {
            if constexpr (kRowWs4) {
                stages<RS::L3F, RS::F1c>(v);
                exchange<RS::L3F, RS::L2>(v, s, tid);
            } else {
                stages<RS::L3, RS::F1c>(v);
                exchange<RS::L3, RS::L2>(v, s, tid);
            }
            stages<RS::L2, RS::F1b>(v);
            exchange<RS::L2, RS::L1>(v, s, tid);
            stages<RS::L1, RS::F1a>(v);
        }
        // scale folded into the 2^-k normalisation: 2^-k is exact, so
        // v * (sc * 2^-k) rounds like (v * 2^-k) * sc (normal range)
        const float sc = sldf(a.scales_in, D.scale_idx);
        if constexpr (kLadSign)
            apply_signs_direct<RS::L1>(v, tile << kRowLog, base1, D.logp, b1, sc * pow2i(-((D.logp + 1) / 2)));
        store_y(a, D, tile, base1, v);
        if (!more) break;
        t = tn; si = sn; tile = tln;
    }
}

// ===========================================================================
// Column passes: tile = 2^M rows (index bits [lo, lo+M)) x 2^(15-M)
// contiguous columns (bits [0, 15-M)), NT = 1024.  MID fuses F1 | D2 | F2.
// ===========================================================================
constexpr int kColLog = 15;
constexpr int kColNT = 1024;
constexpr size_t kColSmem = (sizeof(float) * lds_floats(kColLog) + 15) & ~(size_t)15;
template <int M> struct ColSet {
    static constexpr int K = kColLog - M;
    static constexpr int m1 = M < 5 ? M : 5;
    // L1: rows K..K+m1-1, filled with top columns K-1, K-2, ...
    static constexpr int l1(int i) { return i < m1 ? K + i : K - 1 - (i - m1); }
    static constexpr Lay L1{kColLog, l1(0), l1(1), l1(2), l1(3), l1(4)};
    // L2: rows K+5..K+M-1, filled with rows K, K+1, ...
    static constexpr int l2(int i) { return i < M - 5 ? K + 5 + i : K + (i - (M - 5)); }
    static constexpr Lay L2{kColLog, l2(0), l2(1), l2(2), l2(3), l2(4)};
    static constexpr uint32_t A1 = ((1u << m1) - 1u) << K;
    static constexpr uint32_t A2 = M > 5 ? ((1u << (M - 5)) - 1u) << (K + 5) : 0u;
};

// The middle pass's D2 signs: the tile spans the slice's top three index bits
// (the rand_diag nibble index) whenever M >= 3, so each of its 2^12 distinct
// words j serves 8 elements: one hash per 8 elements, kept as a byte table in
// LDS (bit k of byte = sign of element k*S + j).  M < 3 hashes per element.
constexpr size_t kColTab = 4096;

template <int M, bool MID>
DEVI void col_body(const KArgs& a, int b) {
    using CS = ColSet<M>;
    constexpr int K = CS::K;
    constexpr bool TAB = MID && M >= 3;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float* s = reinterpret_cast<float*>(smem);
    uint8_t* tab = smem + (M > 5 ? kColSmem : 0);
    int si; uint32_t tile;
    find_tile_at(a, b, si, tile);
    const SliceDesc D = a.d[si];
    const uint32_t tid = threadIdx.x;
    const int lo = a.lo;
    // tile -> slice bits: [K, lo) from tile low bits, [lo+M, p) from the rest
    const uint32_t tl = tile & ((1u << (lo - K)) - 1u);
    const uint32_t th = tile >> (lo - K);
    const uint32_t tb = (tl << K) | (th << (lo + M));
    float* w = a.ws + D.ws_off;
    const int lgp = D.logp;
    auto map = [&](uint32_t t) -> uint32_t { return tb | (t & ((1u << K) - 1u)) | ((t >> K) << lo); };
    // sign-table index of tile element t: the tile bits below the nibble bits
    // (columns, then rows lo .. p-4), i.e. t with its top 3 bits removed
    constexpr uint32_t kTabMask = (1u << (kColLog - 3)) - 1u;
    if constexpr (TAB) {
        const uint32_t b2 = seed_b(a.seeds[D.tensor] + 1u);
        for (uint32_t q = tid; q < (1u << (kColLog - 3)); q += kColNT)
            tab[q] = (uint8_t)rd_byte(map(q) & ((1u << (D.logp - 3)) - 1u), b2);
    }
    float v[32];
    const uint32_t base1 = LT<CS::L1>::base(tid);
#pragma unroll
    for (int r = 0; r < 32; ++r) v[r] = ws_pld(w, lgp, map(base1 | LT<CS::L1>::off(r)));
    stages<CS::L1, CS::A1>(v);
    if constexpr (M > 5) {
        exchange<CS::L1, CS::L2>(v, s, tid);  // its barriers also publish tab
        stages<CS::L2, CS::A2>(v);
    } else if constexpr (TAB) {
        __syncthreads();
    }
    if constexpr (MID) {
        const float m2 = pow2i(-(D.logp / 2));
        if constexpr (M > 5) {
            const uint32_t base2 = opaque(LT<CS::L2>::base(tid));
#pragma unroll
            for (int r = 0; r < 32; ++r) {
                const uint32_t t = base2 | LT<CS::L2>::off(r);
                v[r] = flip_unless(v[r] * m2, ((uint32_t)tab[t & kTabMask] >> (t >> (kColLog - 3))) & 1u);
            }
            stages<CS::L2, CS::A2>(v);
            exchange<CS::L2, CS::L1>(v, s, tid);
            stages<CS::L1, CS::A1>(v);
        } else {
            const uint32_t base1s = opaque(base1);
            if constexpr (TAB) {
#pragma unroll
                for (int r = 0; r < 32; ++r) {
                    const uint32_t t = base1s | LT<CS::L1>::off(r);
                    v[r] = flip_unless(v[r] * m2, ((uint32_t)tab[t & kTabMask] >> (t >> (kColLog - 3))) & 1u);
                }
            } else {
                const uint32_t b2 = seed_b(a.seeds[D.tensor] + 1u);
#pragma unroll
                for (int r = 0; r < 32; ++r)
                    v[r] = sgn_elem(v[r] * m2, map(base1s | LT<CS::L1>::off(r)), D.logp, b2);
            }
            stages<CS::L1, CS::A1>(v);
        }
        const uint32_t base1w = opaque(base1);
#pragma unroll
        for (int r = 0; r < 32; ++r) ws_pst<MID>(w, lgp, map(base1w | LT<CS::L1>::off(r)), v[r]);
    } else {
        if constexpr (M > 5) {
            const uint32_t base2 = opaque(LT<CS::L2>::base(tid));
#pragma unroll
            for (int r = 0; r < 32; ++r) ws_pst<MID>(w, lgp, map(base2 | LT<CS::L2>::off(r)), v[r]);
        } else {
            const uint32_t base1w = opaque(base1);
#pragma unroll
            for (int r = 0; r < 32; ++r) ws_pst<MID>(w, lgp, map(base1w | LT<CS::L1>::off(r)), v[r]);
        }
    }
    // The slice norm nu = sqrt(sum of the row pass's partials of x^2)
    // (|H D2 H D1 x| = |x|; eden_pipeline.py:515) for the final row pass: tile
    // 0 of every slice in the slice's first column launch sums them in a fixed
    // order (the same value whatever the launch grouping).
    if (a.do_nu && tile == 0) {
        __shared__ float nred[kColNT / 64];
        const int64_t ntile = 1ll << (D.logp - kRowLog);
        float ss = 0.f;
        for (int64_t t = tid; t < ntile; t += kColNT) ss += a.part[D.part_off + t];
        ss = block_sum<kColNT>(ss, nred);
        if (tid == 0) a.nu[si] = sqrtf(ss);
    }
}
template <int M, bool MID>
__global__ __launch_bounds__(kColNT) void k_col(KArgs a) {
    col_body<M, MID>(a, (int)blockIdx.x);
}

// Several single-level middle passes (heights M = 1..6) in one launch: a
// wave's slices of different sizes share the grid instead of running one
// short launch per height.  a.list -> table of kColGroup ints per group
// {M, list, tstart (both relative to the table), count, first block};
// a.count = groups.  Height 6 needs col_body's exchange buffer: the launch
// takes kColMultiSmem.
constexpr int kColGroup = 5;
constexpr size_t kColMultiSmem = kColSmem + kColTab;
DEVI void col_multi_block(const KArgs& a, int b) {
    int g = 0;
    if (a.btab) {
        g = a.btab[2 * b + 1] & 7;
    } else {
        while (g + 1 < a.count && a.list[kColGroup * (g + 1) + 4] <= b) ++g;
    }
    const int32_t* G = a.list + kColGroup * g;
    KArgs a2 = a;
    a2.list = a.list + G[1];
    a2.tstart = a.list + G[2];
    a2.count = G[3];
    if (a.btab) a2.btab = a.btab + 2 * G[4];  // the group's blocks, indexed from its first
    const int lb = b - G[4];
    switch (G[0]) {
    case 1: col_body<1, true>(a2, lb); break;
    case 2: col_body<2, true>(a2, lb); break;
    case 3: col_body<3, true>(a2, lb); break;
    case 4: col_body<4, true>(a2, lb); break;
    case 5: col_body<5, true>(a2, lb); break;
    default: col_body<6, true>(a2, lb); break;
    }
}
__global__ __launch_bounds__(kColNT) void k_col_multi(KArgs a) { col_multi_block(a, (int)blockIdx.x); }

// One launch for a one-wave plan's small-set groups (blocks < a.sset_first,
// dispatched first: each is longer than a column tile) AND its single-level
// middle passes: the small slices share the CUs with the column tiles, in the
// caller's stream, so the call needs no side
// stream and no cross-queue fork / join (each join cost ~10 us of the caller's
// queue).  Both parts are the bodies of k_col_multi and
// k_enc_sset / k_dec_sset: outputs identical to those launches.
__global__ __launch_bounds__(kColNT) void k_enc_colm_set(KArgs a) {
    const int b = (int)blockIdx.x;
    if (b < a.sset_first) {
        KArgs s = a;
        s.list = a.sset;
        enc_sset_block(s, b);
        return;
    }
    col_multi_block(a, b - a.sset_first);
}
__global__ __launch_bounds__(kColNT) void k_dec_colm_set(KArgs a) {
    const int b = (int)blockIdx.x;
    if (b < a.sset_first) {
        KArgs s = a;
        s.list = a.sset;
        dec_sset_block(s, b);
        return;
    }
    col_multi_block(a, b - a.sset_first);
}

// ===========================================================================
// Column passes for M = 6..10 rows: 512 threads x 64 registers.  L1 keeps
// rows r0..r5 in registers, L2 rows r(M-6)..r(M-1) with r5 last (register
// index 5 in both layouts).  Lanes 0..31 sit on 32 consecutive columns in
// both layouts, so the LDS exchange needs no padding to be conflict-free, and
// it runs in two halves (r5 = 0, then 1) through a 2^14-float buffer: 68 KiB
// of LDS per block, two blocks per CU (one loads while the other computes).
// Tile I/O through a buffer resource over the slice's intermediate: the row
// part of every register's address is a scalar offset.
// ===========================================================================
// TL = log2 of the tile: 15 (512 threads, 2 blocks per CU) or 16 (1024
// threads, one block per CU, twice the columns per row segment).
template <int TL> constexpr int col6_nt() { return 1 << (TL - 6); }
template <int TL> constexpr size_t col6_half() { return sizeof(float) << (TL - 1); }
template <int TL> constexpr size_t col6_tab() { return (size_t)1 << (TL - 3); }
template <int M, int TL> struct Col6Set {
    static_assert(M >= 6 && M <= 10 && (TL == 15 || TL == 16), "Col6Set: 6 <= M <= 10, TL 15 or 16");
    static constexpr int K = TL - M;
    static constexpr int row2(int i) { return (M - 6 + i) + ((M - 6 + i) >= 5 ? 1 : 0); }  // i < 5
    static constexpr Lay L1{TL, K, K + 1, K + 2, K + 3, K + 4, K + 5};
    static constexpr Lay L2{TL, K + row2(0), K + row2(1), K + row2(2), K + row2(3), K + row2(4), K + 5};
    static constexpr uint32_t A1 = 63u << K;
    static constexpr uint32_t A2 = M > 6 ? ((1u << (M - 6)) - 1u) << (K + 6) : 0u;
    static constexpr int HB = K + 5;  // the half bit (row r5)
};
// drop tile bit HB from an index (additive over disjoint bit sets)
template <int HB>
DEVI constexpr uint32_t cidx(uint32_t e) { return (e & ((1u << HB) - 1u)) | ((e >> (HB + 1)) << HB); }

template <Lay A, Lay B, int HB>
DEVI void exchange_half(float (&v)[64], float* s, uint32_t tid) {
    static_assert(LT<A>::rb(5) == HB && LT<B>::rb(5) == HB, "half bit must be register bit 5 of both layouts");
    const uint32_t ba = opaque(cidx<HB>(LT<A>::base(tid)));
    const uint32_t bb = opaque(cidx<HB>(LT<B>::base(tid)));
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int r = 32 * h; r < 32 * h + 32; ++r) s[ba + cidx<HB>(LT<A>::off(r))] = v[r];
        __syncthreads();
#pragma unroll
        for (int r = 32 * h; r < 32 * h + 32; ++r) v[r] = s[bb + cidx<HB>(LT<B>::off(r))];
        __syncthreads();
    }
}

// NTA: the pass streams its intermediate through HBM (the middle pass of a
// split 5-pass slice): nt loads and stores, so it does not evict the other
// stream's MALL-resident waves
template <int M, bool MID, int TL, bool NTA = false>
__global__ __launch_bounds__(col6_nt<TL>(), 4) void k_col6(KArgs a) {
    using CS = Col6Set<M, TL>;
    constexpr int kLd = NTA ? 2 : kLdAux, kSt = NTA ? 2 : kStAux;
    constexpr int NT = col6_nt<TL>();
    constexpr int K = CS::K;
    constexpr bool EXCH = M > 6;
    constexpr Lay LC = EXCH ? CS::L2 : CS::L1;  // layout after the first Hadamard part
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float* s = reinterpret_cast<float*>(smem);
    uint8_t* tab = smem + (EXCH ? col6_half<TL>() : 0);
    int si; uint32_t tile;
    find_tile(a, si, tile);
    const SliceDesc D = udesc(a.d, si);
    const uint32_t tid = threadIdx.x;
    const int lo = a.lo;
    // tile -> slice bits: [K, lo) from tile low bits, [lo+M, p) from the rest
    const uint32_t tl = tile & ((1u << (lo - K)) - 1u);
    const uint32_t th = tile >> (lo - K);
    const uint32_t tb = (tl << K) | (th << (lo + M));
    auto map = [&](uint32_t t) -> uint32_t { return tb | (t & ((1u << K) - 1u)) | ((t >> K) << lo); };
    const WsR rw = ws_rsrc(a.ws + D.ws_off, D.logp, 0, (uint32_t)(4ull << D.logp));
    constexpr uint32_t kTabMask = (1u << (TL - 3)) - 1u;
    if constexpr (MID && kLadSign) {  // D2 sign bytes of the tile's 2^12 rand_diag words (see k_col)
        const uint32_t b2 = seed_b(sld(a.seeds, D.tensor) + 1u);
        for (uint32_t q = tid; q < (1u << (TL - 3)); q += NT)
            tab[q] = (uint8_t)rd_byte(map(q) & ((1u << (D.logp - 3)) - 1u), b2);
    }
    float v[64];
    const uint32_t base1 = LT<CS::L1>::base(tid);
    // interleaved ws layout of 2^25 slices (see ws_row_base): position of
    // element e = ws_pos(e); a row offset (bits 15..20) moves bit 15 to bit 5
    constexpr bool PERM = M == 10 && MID && TL == 15;
    auto ws_pos = [](uint32_t e) -> uint32_t {
        return (e & 31u) | (((e >> 15) & 1u) << 5) | (((e >> 5) & 1023u) << 6) | ((e >> 16) << 16);
    };
    const bool perm = PERM && D.perm;
    if (perm) {
        const uint32_t vo = opaque(ws_pos(map(base1)) * 4u);
#pragma unroll
        for (int r = 0; r < 64; ++r)
            v[r] = ws_ld1(rw, vo, ws_pos((LT<CS::L1>::off(r) >> K) << 15) * 4u, kLd);
    } else {
        const uint32_t vo = opaque(map(base1) * 4u);
#pragma unroll
        for (int r = 0; r < 64; ++r)
            v[r] = ws_ld1(rw, vo, uu((LT<CS::L1>::off(r) >> K) << lo) * 4u, kLd);
    }
    if constexpr (kLadFly) stages<CS::L1, CS::A1>(v);
    if constexpr (EXCH && kLadFly) {
        exchange_half<CS::L1, CS::L2, CS::HB>(v, s, tid);  // its barriers also publish tab
        stages<CS::L2, CS::A2>(v);
    } else if constexpr (MID) {
        __syncthreads();
    }
    if constexpr (MID) {
        const float m2 = pow2i(-(D.logp / 2));
        // the tile's top 3 bits (the sign's nibble index) are register bits of
        // LC, so each register's shift is a constant and its table offset an
        // immediate
        static_assert((LT<LC>::rmask() >> (TL - 3)) == 7u, "top 3 tile bits must be register bits");
        const uint32_t bt = opaque(LT<LC>::base(tid) & kTabMask);
        if constexpr (kLadSign) {
#pragma unroll
            for (int r = 0; r < 64; ++r) {
                const uint32_t o = LT<LC>::off(r);
                v[r] = flip_unless(v[r] * m2, ((uint32_t)tab[bt + (o & kTabMask)] >> (o >> (TL - 3))) & 1u);
            }
        }
        if constexpr (EXCH && kLadFly) {
            stages<CS::L2, CS::A2>(v);
            exchange_half<CS::L2, CS::L1, CS::HB>(v, s, tid);
        }
        if constexpr (kLadFly) stages<CS::L1, CS::A1>(v);
        if (perm) {
            const uint32_t vo = opaque(ws_pos(map(base1)) * 4u);
#pragma unroll
            for (int r = 0; r < 64; ++r)
                ws_st1(rw, vo, ws_pos((LT<CS::L1>::off(r) >> K) << 15) * 4u, v[r], kSt);
        } else {
            const uint32_t vo = opaque(map(base1) * 4u);
            int los = lo;
            asm volatile("" : "+s"(los));  // recompute the row offsets: 64 SGPRs kept live would spill
#pragma unroll
            for (int r = 0; r < 64; ++r)
                ws_st1(rw, vo, uu((LT<CS::L1>::off(r) >> K) << los) * 4u, v[r], kSt);
        }
    } else {
        const uint32_t bcw = LT<LC>::base(tid);
        const uint32_t vo = opaque(map(bcw) * 4u);
        int los = lo;
        asm volatile("" : "+s"(los));
#pragma unroll
        for (int r = 0; r < 64; ++r)
            ws_st1(rw, vo, uu((LT<LC>::off(r) >> K) << los) * 4u, v[r], kSt);
    }
    if (a.do_nu && tile == 0) {  // slice norm, as in k_col
        __shared__ float nred[NT / 64];
        const int64_t ntile = 1ll << (D.logp - kRowLog);
        float ss = 0.f;
        for (int64_t t = tid; t < ntile; t += NT) ss += a.part[D.part_off + t];
        ss = block_sum<NT>(ss, nred);
        if (tid == 0) a.nu[si] = sqrtf(ss);
    }
}

// block-uniform tile lookup of the non-persistent row launches (scalar loads):
// one load from the launch's per-tile table when it has one, else a search
DEVI void row_locate(const KArgs& a, int t, int& si, uint32_t& tile, uint32_t* pair = nullptr) {
    if (a.btab) {
        si = (int)sld(a.btab, 2 * (int64_t)t);
        const uint32_t e = sld(a.btab, 2 * (int64_t)t + 1);
        tile = e >> 3;
        if (pair) *pair = e & 1u;
        return;
    }
    if (pair) *pair = 0u;
    int lo = 0, hi = a.count - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if ((int)sld(a.tstart, mid) <= t) lo = mid; else hi = mid - 1;
    }
    si = (int)sld(a.list, lo);
    tile = (uint32_t)(t - (int)sld(a.tstart, lo));
}

// ===========================================================================
// Encode pass C with two blocks per CU (k_enc_rowC2).  The quantiser makes
// k_enc_rowC latency-bound at one block per CU (LDS table reads, bank
// conflicts, barriers); here the F2 row stages run through layouts that all
// keep element bit 10 at register index 5:
//   L3 {5..10} (F2c) -> L4 {11..14,9,10} (F2d) -> L5 {0..4,10} (F2e),
// so both exchanges go in two halves through a padded 2^14-float buffer
// (68 KiB; pad() keeps lanes 0..31 on distinct banks: they vary bits 0..4
// in L3/L4 and bits 5..9 in L5).  With the 9 KiB quantiser table a block
// takes 77 KiB: two blocks per CU, no register prefetch (the other block
// hides the loads).  Each thread quantises two runs of 32 contiguous
// elements (bit 10 = 0, 1) and stores one 32-bit word per plane per run.
// ===========================================================================
struct RowC2Set {
    static constexpr Lay L3{15, 5, 6, 7, 8, 9, 10}, L4{15, 11, 12, 13, 14, 9, 10}, L5{15, 0, 1, 2, 3, 4, 10};
    static constexpr uint32_t F2c = bits_mask({5, 6, 7, 8, 9, 10}), F2d = bits_mask({11, 12, 13, 14}),
                              F2e = bits_mask({0, 1, 2, 3, 4});
    static constexpr int HB = 10;
};
constexpr size_t kRowC2Ex = (sizeof(float) * lds_floats(kRowLog - 1) + 15) & ~(size_t)15;
constexpr size_t kRowC2Smem = kRowC2Ex + sizeof(QTab) + 64;

template <Lay A, Lay B, int HB>
DEVI void exchange_half_pad(float (&v)[64], float* s, uint32_t tid) {
    static_assert(LT<A>::rb(5) == HB && LT<B>::rb(5) == HB, "half bit must be register bit 5 of both layouts");
    const uint32_t ba = opaque(pad(cidx<HB>(LT<A>::base(tid))));
    const uint32_t bb = opaque(pad(cidx<HB>(LT<B>::base(tid))));
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int r = 32 * h; r < 32 * h + 32; ++r) s[ba + cpad(cidx<HB>(LT<A>::off(r)))] = v[r];
        __syncthreads();
#pragma unroll
        for (int r = 32 * h; r < 32 * h + 32; ++r) v[r] = s[bb + cpad(cidx<HB>(LT<B>::off(r)))];
        __syncthreads();
    }
}

// registers [32 h, 32 h + 32) of a ws tile (L3 layout), as fetch_ws
template <int H, int AUX = kLdAux>
DEVI void fetch_ws_half(const KArgs& a, const SliceDesc& D, uint32_t tile, bool live, uint32_t base3,
                        float (&v)[64]) {
    if (D.perm) {
        const WsR r = ws_row(a, D, tile, live ? (4u << (kRowLog + 1)) - 128u : 0u);
        const uint32_t b = ws_row_idx(base3);
#pragma unroll
        for (int k = 32 * H; k < 32 * H + 32; ++k) v[k] = ws_ld1(r, b * 4u, (LT<RS::L3>::off(k) << 1) * 4u, AUX);
    } else {
        const WsR r = ws_row(a, D, tile, live ? (4u << kRowLog) : 0u);
#pragma unroll
        for (int k = 32 * H; k < 32 * H + 32; ++k) v[k] = ws_ld1(r, base3 * 4u, LT<RS::L3>::off(k) * 4u, AUX);
    }
}

// ROLL: the next tile's intermediate is loaded into the registers the
// quantiser has just freed (its first half after the first 32-element run,
// the second after the second), so the loads are in flight across the second
// run, the plane stores and the dot reduction, with no extra registers (the
// kernel sits at the 128-VGPR cap of two blocks per CU).
// diagnostic builds only (-DOFL_DIAG_ROWC2=mask, wrong results, tools/ab):
// 1 = no F2 exchanges, 2 = no quantiser, 4 = no dot reduction
#ifndef OFL_DIAG_ROWC2
#define OFL_DIAG_ROWC2 0
#endif
constexpr int kDiagRowC2 = OFL_DIAG_ROWC2;
#ifndef OFL_ROWC2_LD_AUX
#define OFL_ROWC2_LD_AUX 0
#endif
// the default policy since the arena I/O went nt (round 6: 478.5-479.2 vs
// 476.7-478.7 GiB/s with nt, profiles/r06_rowc2ld_ab.txt; nt had won at the
// 2 GiB waves of round 3, profiles/r03_nt_ab.txt)
constexpr int kRowC2LdAux = OFL_ROWC2_LD_AUX;
template <bool ROLL>
__global__ __launch_bounds__(kRowNT, 4) void k_enc_rowC2(KArgs a) {
    using R = RowC2Set;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float* s = reinterpret_cast<float*>(smem);
    QTab* qt = reinterpret_cast<QTab*>(smem + kRowC2Ex);
    float* red = reinterpret_cast<float*>(smem + kRowC2Ex + sizeof(QTab));
    const uint32_t tid = threadIdx.x;
    load_qtable<kRowNT>(qt, a.nbits);
    __syncthreads();
    const int total = a.npair ? a.npair : (int)sld(a.tstart, a.count);  // npair: an explicit tile list
    const uint32_t base3 = LT<R::L3>::base(tid), base5 = LT<R::L5>::base(tid);
    auto locate = [&](int t, int& si, uint32_t& tile) { row_locate(a, t, si, tile); };
    int t = (int)blockIdx.x;
    if (t >= total) return;
    int si; uint32_t tile;
    locate(t, si, tile);
    float v[64];
    // the intermediate's last read: kRowC2LdAux (nt won at round 3's 2 GiB
    // waves, the default policy at round 6's MALL-sized ones)
    if (ROLL) fetch_ws<kRowC2LdAux>(a, udesc(a.d, si), tile, true, base3, v);
    for (;;) {
        const SliceDesc D = udesc(a.d, si);
        const int tn = t + (int)gridDim.x;
        const bool more = tn < total;
        int sn; uint32_t tln;
        locate(more ? tn : t, sn, tln);
        if (!ROLL) fetch_ws<kRowC2LdAux>(a, D, tile, true, base3, v);
        if constexpr (kLadFly) {
            stages<R::L3, R::F2c>(v);
            if (!(kDiagRowC2 & 1)) exchange_half_pad<R::L3, R::L4, R::HB>(v, s, tid);
            stages<R::L4, R::F2d>(v);
            if (!(kDiagRowC2 & 1)) exchange_half_pad<R::L4, R::L5, R::HB>(v, s, tid);
            stages<R::L5, R::F2e>(v);
        }
        __builtin_amdgcn_sched_barrier(0);
        const float nu = sldf(a.nu, si);
        const float ysc = pow2i(-((D.logp + 1) / 2));
        const float zm64 = 64.0f * (sqrtf((float)(1ll << D.logp)) / nu);
        const bool pos = nu > 0.0f;
        float dot = 0.f;
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            uint32_t w[8];
            if (!kLadFull) {  // ladder rungs: a plane word from 4 values, no quantiser
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    w[i] = lad_word(v[32 * g + 4 * i], v[32 * g + 4 * i + 1], v[32 * g + 4 * i + 2], v[32 * g + 4 * i + 3]);
                dot = 1.0f;
            } else if (kDiagRowC2 & 2) {  // diagnostic: no quantiser (wrong output)
#pragma unroll
                for (int i = 0; i < 8; ++i) w[i] = __float_as_uint(v[32 * g + 4 * i]) ^ __float_as_uint(v[32 * g + 4 * i + 1]);
                dot += v[32 * g];
            } else {
                dot += quant_pack32(*reinterpret_cast<const float(*)[32]>(&v[32 * g]), ysc, zm64, qt, w);
            }
            if (!pos) {
#pragma unroll
                for (int i = 0; i < 8; ++i) w[i] = 0;
            }
            if (ROLL) {  // this half's registers are free: start the next tile's
                if (g == 0) fetch_ws_half<0, kRowC2LdAux>(a, udesc(a.d, sn), tln, more, base3, v);
                else fetch_ws_half<1, kRowC2LdAux>(a, udesc(a.d, sn), tln, more, base3, v);
            }
            store_planes(a.pout + D.pl_off, (tile << kRowLog) + base5 + ((uint32_t)g << R::HB), D.pl_stride,
                         a.nbits, w);
        }
        if (!pos) dot = 0.f;
        if (!(kDiagRowC2 & 4) && kLadFull) dot = block_sum<kRowNT>(dot, red);
        if (tid == 0) a.part[D.part_off + tile] = dot;
        if (!more) break;
        t = tn; si = sn; tile = tln;
    }
}

// ===========================================================================
// Row passes with two blocks per CU, for waves of few tiles per CU (the
// ResNet-50 class: ~1.5 tiles per CU per pass, where the persistent one-block
// kernels' register prefetch never overlaps anything and half the CUs sit in
// a second-tile tail).  No prefetch: the other block on the CU hides the
// loads.  Every layout keeps one element bit at register index 5 (the half
// bit), so each LDS exchange runs in two halves through a padded 2^14-float
// buffer (68 KiB per block).  The sequence of index bits butterflied is the
// persistent kernel's (an extra layout where needed), and the loads, sums and
// stores are the same, so the outputs are bit-identical to k_enc_rowA /
// k_dec_rowA / k_dec_rowC (tests/test_gpu_parity.py::test_row2_variants_bit_identical).
// ===========================================================================
struct RowA2Set {  // encode pass A, half bit 14: 0,1,11,12,13,14 | 2..6 | 10,7,8,9
    static constexpr Lay A1 = RS::L1, A2{15, 2, 3, 4, 5, 6, 14}, A3{15, 10, 7, 8, 9, 6, 14};
    static constexpr uint32_t F1a = RS::F1a, F1b = bits_mask({2, 3, 4, 5, 6}), F1c = bits_mask({10, 7, 8, 9});
};
struct DecA2Set {  // decode pass A, half bit 5: 0..4 | 11,12,13,14,5 | 6..10
    static constexpr Lay C1 = RS::L5, C2{15, 11, 12, 13, 14, 9, 5}, C3{15, 6, 7, 8, 9, 10, 5};
    static constexpr uint32_t G1 = RS::F2e, G2 = bits_mask({11, 12, 13, 14, 5}), G3 = bits_mask({6, 7, 8, 9, 10});
};
struct DecC2Set {  // decode pass C, half bit 10: 7,8,9 | 2..6,10 | 0,1,11,12,13 | 14
    static constexpr Lay B1 = kRowWs4 ? RS::L3F : RS::L3, B2 = RS::L2, B3{15, 0, 1, 11, 12, 13, 10}, B4{15, 0, 1, 14, 11, 12, 10};
    static constexpr uint32_t H1 = RS::F1c, H2 = RS::F1b, H3 = bits_mask({0, 1, 11, 12, 13}), H4 = bits_mask({14});
};
// apply_signs_direct in groups of 8 registers whose results are pinned before
// the next group starts: at the 128-VGPR cap of two blocks per CU the
// scheduler would otherwise overlap all 64 hash chains and spill
// ADD = false: the general form only (k_enc_rowA2<true>: its weighted-
// average loads leave no registers for the second path)
template <Lay L, bool ADD = true>
DEVI void apply_signs_grouped(float (&v)[64], uint32_t ebase, uint32_t base, int p, uint32_t b, float mul) {
    // the 64 sign bits first in two mask registers pinned per group of 8
    // hashes, then the flips: few live temporaries at the 128-VGPR cap
    const uint32_t jm = (1u << (p - 3)) - 1u;
    const uint32_t ps = (uint32_t)(p - 3);
    uint32_t m[2] = {0u, 0u};
    if (ADD && p >= 18) {
        // a row tile (ebase = tile << 15) lies in one nibble of every word,
        // and its elements' words are j0 + (base | off(r)): the LCG is one
        // add of a compile-time constant per element (as apply_signs_direct),
        // one quarter-rate multiply per element fewer than the general form
        const uint32_t r2b = kLcgA * ((ebase & jm) + base) + b;
        const uint32_t sh = 4u * (ebase >> ps) + 3u;
#pragma unroll
        for (int g = 0; g < 64; g += 8) {
#pragma unroll
            for (int r = g; r < g + 8; ++r)
                m[r >> 5] |= ((rd_mix(r2b + kLcgA * LT<L>::off(r)) >> sh) & 1u) << (r & 31);
            asm volatile("" : "+v"(m[0]), "+v"(m[1]));
        }
    } else {  // the general per-element form of sgn_elem
#pragma unroll
        for (int g = 0; g < 64; g += 8) {
#pragma unroll
            for (int r = g; r < g + 8; ++r) {
                const uint32_t e = ebase + (base | LT<L>::off(r));
                m[r >> 5] |= ((rd_word(e & jm, b) >> (4u * (e >> ps) + 3u)) & 1u) << (r & 31);
            }
            asm volatile("" : "+v"(m[0]), "+v"(m[1]));
        }
    }
#pragma unroll
    for (int r = 0; r < 64; ++r) v[r] = flip_unless(v[r] * mul, (m[r >> 5] >> (r & 31)) & 1u);
}
// the D1 signs of a paired row launch (p >= 18).  Word j of a slice serves
// its elements j + k*2^(p-3), k = 0..7 (bit 4k+3), so the tile one nibble up
// (tile + 2^(p-18)) reuses this tile's words at bit sh + 4.  mode 1 (the
// pair's first tile, nibble even): hash once, flip with bit sh, leave bit
// sh + 4 of the 64 words in the thread's 8 stash bytes; mode 2 (the
// partner, next in the same block): flip with the stash.  Half the hashes of
// the unpaired form.  Each group of 8 hashes leaves its own and its partner
// byte in LDS (bytes 8..15 and 0..7 of the thread's 16), so no mask register
// is live across the hashes (as many live registers as apply_signs_grouped).
template <Lay L>
DEVI void apply_signs_pair(float (&v)[64], uint32_t ebase, uint32_t base, int p, uint32_t b, float mul, uint32_t mode,
                           uint32_t* stash) {
    // stash: the block's stash; a thread's 16 bytes at 16 * tid, the address
    // recomputed at each use (an opaque tid: no register held across the hashes)
    uint32_t m[2];
    if (mode == 2u) {
        const uint2 q = *reinterpret_cast<const uint2*>(stash + 4 * opaque(threadIdx.x));
        m[0] = q.x;
        m[1] = q.y;
    } else {
        const uint32_t jm = (1u << (p - 3)) - 1u;
        const uint32_t r2b = kLcgA * ((ebase & jm) + base) + b;
        const uint32_t sh = 4u * (ebase >> (p - 3)) + 3u;
#pragma unroll
        for (int g = 0; g < 64; g += 8) {
            uint32_t ob = 0u, pb = 0u;
#pragma unroll
            for (int r = g; r < g + 8; ++r) {
                const uint32_t w = rd_mix(r2b + kLcgA * LT<L>::off(r)) >> sh;
                ob |= (w & 1u) << (r & 7);
                pb |= ((w >> 4) & 1u) << (r & 7);
            }
            asm volatile("" : "+v"(ob), "+v"(pb));
            uint8_t* sb = reinterpret_cast<uint8_t*>(stash) + 16 * opaque(threadIdx.x) + (g >> 3);
            sb[0] = (uint8_t)pb;
            sb[8] = (uint8_t)ob;
        }
        const uint2 q = *reinterpret_cast<const uint2*>(stash + 4 * opaque(threadIdx.x) + 2);
        m[0] = q.x;
        m[1] = q.y;
    }
#pragma unroll
    for (int r = 0; r < 64; ++r) v[r] = flip_unless(v[r] * mul, (m[r >> 5] >> (r & 31)) & 1u);
}
// paired row launches: the D1 bits, 16 bytes per thread (thread i at bytes
// 16i..16i+15: partner, own), after the 8 wave partials
constexpr size_t kRow2Stash = kRowC2Ex + 64;
constexpr size_t kRow2Smem = kRow2Stash + 16 * kRowNT;  // half-exchange buffer + partials + stash
constexpr size_t kRow2SmemC = kRowC2Ex + 1024;  // half-exchange buffer + 256 centroids

// ws tile store / y tile store in any layout (as store_ws / store_y)
template <Lay L>
DEVI void store_ws_l(const KArgs& a, const SliceDesc& D, uint32_t tile, uint32_t base, const float (&v)[64]) {
    if (D.perm) {
        const WsR r = ws_row(a, D, tile, (4u << (kRowLog + 1)) - 128u);
        const uint32_t b = ws_row_idx(base);
#pragma unroll
        for (int k = 0; k < 64; ++k) ws_st1(r, b * 4u, (LT<L>::off(k) << 1) * 4u, v[k], kStAux);
    } else {
        const WsR r = ws_row(a, D, tile, 4u << kRowLog);
#pragma unroll
        for (int k = 0; k < 64; ++k) ws_st1(r, base * 4u, LT<L>::off(k) * 4u, v[k], kStAux);
    }
}
template <Lay L>
DEVI void store_y_l(const KArgs& a, const SliceDesc& D, uint32_t tile, uint32_t base, const float (&v)[64]) {
    static_assert(LT<L>::rb(0) == 0 && LT<L>::rb(1) == 1, "float4 stores need element bits 0, 1 in registers 0, 1");
    const uint32_t e0 = tile << kRowLog;
    const uint32_t nv = tile_valid(D.ylen - (int64_t)e0);
    const rsrc_t r = mk_rsrc(a.xout + D.y_off + e0, (nv & ~3u) * 4u);
    if (a.yadd) {
        const rsrc_t rb = mk_rsrc(a.yadd + D.y_off + e0, (nv & ~3u) * 4u);
#pragma unroll
        for (int k = 0; k < 64; k += 4) {
            const float4 b = bload4(rb, base, LT<L>::off(k));
            const float o[4] = {add_rn(b.x, v[k]), add_rn(b.y, v[k + 1]), add_rn(b.z, v[k + 2]), add_rn(b.w, v[k + 3])};
            bstore4(r, base, LT<L>::off(k), o);
        }
    } else {
#pragma unroll
        for (int k = 0; k < 64; k += 4) bstore4(r, base, LT<L>::off(k), &v[k]);
    }
    if (nv & 3u) {
        const uint32_t eb = nv & ~3u;
        float* y = a.xout + D.y_off + e0 + eb;
        const float* yb = a.yadd ? a.yadd + D.y_off + e0 + eb : nullptr;
#pragma unroll
        for (int k = 0; k < 64; k += 4)
            if (base + LT<L>::off(k) == eb) {
#pragma unroll
                for (int q = 0; q < 3; ++q)
                    if ((uint32_t)q < (nv & 3u)) y[q] = yb ? add_rn(yb[q], v[k + q]) : v[k + q];
            }
    }
}

// x tile of the fused round-end encode: per element the delta of the
// weighted average, in k_wavg_delta's operation order (agg_kernels.hip:
// products rounded, summed from the first collaborator on, / wsum, - base,
// FMA contraction off), rounded to float32 -- the values Eden.compress would
// get.  Elements past the slice's valid length are zero (padding).  Loads go
// two float4 chunks x two collaborators at a time (the 128-VGPR budget of two
// blocks per CU; the other block hides the round trips).
DEVI void fetch_x_wavg(const KArgs& a, const SliceDesc& D, uint32_t tile, uint32_t base1, float (&v)[64]) {
#pragma clang fp contract(off)
    const uint32_t e0 = tile << kRowLog;
    const uint32_t nv = tile_valid(D.len - (int64_t)e0);
    const uint32_t rec = (nv & ~3u) * 4u;  // whole float4s; the straddling one below
    const int nc = a.wc;
#pragma unroll
    for (int g = 0; g < 64; g += 8) {
        double s[8];
        for (int c = 0; c < nc; c += 2) {
            const bool two = c + 1 < nc;
            const rsrc_t r0 = mk_rsrc(a.wx[c] + D.x_off + e0, rec);
            const rsrc_t r1 = mk_rsrc(a.wx[two ? c + 1 : c] + D.x_off + e0, two ? rec : 0u);
            const float4 p0 = bload4(r0, base1, LT<RS::L1>::off(g)), p1 = bload4(r0, base1, LT<RS::L1>::off(g + 4));
            const float4 q0 = bload4(r1, base1, LT<RS::L1>::off(g)), q1 = bload4(r1, base1, LT<RS::L1>::off(g + 4));
            const float xp[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
            const float xq[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
            const double w0 = a.ww[c], w1 = two ? a.ww[c + 1] : 0.0;
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                s[t] = c == 0 ? (double)xp[t] * w0 : s[t] + (double)xp[t] * w0;
                if (two) s[t] = s[t] + (double)xq[t] * w1;
            }
        }
        float4 b0 = make_float4(0.f, 0.f, 0.f, 0.f), b1 = b0;
        if (a.wbase) {
            const rsrc_t rb = mk_rsrc(a.wbase + D.x_off + e0, rec);
            b0 = bload4(rb, base1, LT<RS::L1>::off(g));
            b1 = bload4(rb, base1, LT<RS::L1>::off(g + 4));
        }
        const float xb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const double avg = s[t] / a.wsum;
            const double d = a.wbase ? avg - (double)xb[t] : avg;
            const uint32_t i = base1 + LT<RS::L1>::off(g + (t & ~3)) + (uint32_t)(t & 3);
            v[g + t] = i < (nv & ~3u) ? (float)d : 0.0f;
        }
        asm volatile("" : "+v"(v[g]), "+v"(v[g + 1]), "+v"(v[g + 2]), "+v"(v[g + 3]), "+v"(v[g + 4]), "+v"(v[g + 5]),
                     "+v"(v[g + 6]), "+v"(v[g + 7]));
    }
    // the <= 3 valid elements of a float4 that straddles the valid length
    const uint32_t rem = nv & 3u;
    if (rem) {
        const uint32_t eb = nv & ~3u;
        float xs[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            double sq = 0.0;
            const int64_t ei = D.x_off + e0 + eb + q;
            for (int c = 0; c < nc; ++c) sq = c == 0 ? (double)a.wx[c][ei] * a.ww[c] : sq + (double)a.wx[c][ei] * a.ww[c];
            const double avg = sq / a.wsum;
            const double d = a.wbase ? avg - (double)a.wbase[ei] : avg;
            xs[q] = (uint32_t)q < rem ? (float)d : 0.0f;
        }
#pragma unroll
        for (int k = 0; k < 64; k += 4) {
            const bool hit = base1 + LT<RS::L1>::off(k) == eb;
            v[k] = hit ? xs[0] : v[k];
            v[k + 1] = hit ? xs[1] : v[k + 1];
            v[k + 2] = hit ? xs[2] : v[k + 2];
        }
    }
}

// encode pass A (as k_enc_rowA); WAVG: x from the collaborators' arenas
template <bool WAVG>
__global__ __launch_bounds__(kRowNT, 4) void k_enc_rowA2(KArgs a) {
    using R = RowA2Set;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float* s = reinterpret_cast<float*>(smem);
    float* red = reinterpret_cast<float*>(smem + kRowC2Ex);
    uint32_t* stash = reinterpret_cast<uint32_t*>(smem + kRow2Stash);
    const int total = a.npair ? a.npair : (int)sld(a.tstart, a.count);
    for (int t = (int)blockIdx.x; t < total; t += (int)gridDim.x) {
      // a pair: this tile, then the one a nibble up (apply_signs_pair); the
      // entry is re-read per tile (scalar loads: few SGPRs live across tiles)
      for (uint32_t h = 0;; ++h) {
        int si; uint32_t tile0, pair;
        row_locate(a, t, si, tile0, &pair);
        if (WAVG) pair = 0u;
        const SliceDesc D = udesc(a.d, si);
        // thread-derived addresses are recomputed every tile (an opaque tid):
        // hoisted out of the loop they stay live across it and spill
        const uint32_t tid = opaque(threadIdx.x);
        const uint32_t base1 = LT<R::A1>::base(tid), base3 = LT<R::A3>::base(tid);
        const uint32_t tile = h ? tile0 + (1u << (D.logp - 18)) : tile0;
        float v[64];
        if constexpr (WAVG) {
            fetch_x_wavg(a, D, tile, base1, v);
        } else {
            fetch_x(a, D, tile, true, base1, v);
            fix_x(a, D, tile, base1, v);
#pragma unroll
            for (int r = 0; r < 64; r += 8)
                asm volatile("" : "+v"(v[r]), "+v"(v[r + 1]), "+v"(v[r + 2]), "+v"(v[r + 3]), "+v"(v[r + 4]),
                             "+v"(v[r + 5]), "+v"(v[r + 6]), "+v"(v[r + 7]));
        }
        const uint32_t b1 = seed_b(sld(a.seeds, D.tensor));
        float ss = kLadFull ? sum_sq(v) : 1.0f;
        // the sum is taken here, not sunk past the sign flips (which would keep
        // the 64 unflipped values live through the butterflies and spill them)
        asm volatile("" : "+v"(ss));
        if constexpr (kLadSign) {
            if (!WAVG && pair)
                apply_signs_pair<R::A1>(v, tile << kRowLog, base1, D.logp, b1, 1.0f, 1u + h, stash);
            else
                apply_signs_grouped<R::A1, !WAVG>(v, tile << kRowLog, base1, D.logp, b1, 1.0f);
        }
        if constexpr (kLadFly) {
            stages<R::A1, R::F1a>(v);
            exchange_half_pad<R::A1, R::A2, 14>(v, s, tid);
            stages<R::A2, R::F1b>(v);
            exchange_half_pad<R::A2, R::A3, 14>(v, s, tid);
            stages<R::A3, R::F1c>(v);
        }
        store_ws_l<R::A3>(a, D, tile, base3, v);
        if constexpr (kLadFull) ss = block_sum<kRowNT>(ss, red);
        if (tid == 0) a.part[D.part_off + tile] = ss;
        if (h >= pair) break;
      }
    }
}

// decode pass A (as k_dec_rowA)
template <bool A8>
__global__ __launch_bounds__(kRowNT, 4) void k_dec_rowA2(KArgs a) {
    using R = DecA2Set;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float* s = reinterpret_cast<float*>(smem);
    float* cen = reinterpret_cast<float*>(smem + kRowC2Ex);
    if (threadIdx.x < 256) cen[threadIdx.x] = g_centroids[a.nbits - 1][threadIdx.x];
    __syncthreads();
    const int total = a.npair ? a.npair : (int)sld(a.tstart, a.count);  // npair: an explicit tile list
    for (int t = (int)blockIdx.x; t < total; t += (int)gridDim.x) {
        const uint32_t tid = opaque(threadIdx.x);  // as in k_enc_rowA2
        const uint32_t base1 = LT<R::C1>::base(tid), base3 = LT<R::C3>::base(tid);
        int si; uint32_t tile;
        row_locate(a, t, si, tile);
        const SliceDesc D = udesc(a.d, si);
        uint64_t w[8];
        fetch_planes<A8>(a, D, tile, true, base1, w);
        float v[64];
        if constexpr (kLadFull) unpack_centroids64(w, cen, v);
        else lad_unpack64(w, v);
        if constexpr (kLadFly) {
            stages<R::C1, R::G1>(v);
            exchange_half_pad<R::C1, R::C2, 5>(v, s, tid);
            stages<R::C2, R::G2>(v);
            exchange_half_pad<R::C2, R::C3, 5>(v, s, tid);
            stages<R::C3, R::G3>(v);
        }
        store_ws_l<R::C3>(a, D, tile, base3, v);
    }
}

// decode pass C (as k_dec_rowC)
__global__ __launch_bounds__(kRowNT, 4) void k_dec_rowC2(KArgs a) {
    using R = DecC2Set;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float* s = reinterpret_cast<float*>(smem);
    uint32_t* stash = reinterpret_cast<uint32_t*>(smem + kRow2Stash);
    const int total = a.npair ? a.npair : (int)sld(a.tstart, a.count);
    for (int t = (int)blockIdx.x; t < total; t += (int)gridDim.x) {
      for (uint32_t h = 0;; ++h) {  // as in k_enc_rowA2
        int si; uint32_t tile0, pair;
        row_locate(a, t, si, tile0, &pair);
        const SliceDesc D = udesc(a.d, si);
        const uint32_t tid = opaque(threadIdx.x);  // as in k_enc_rowA2
        const uint32_t base1 = LT<R::B1>::base(tid), base4 = LT<R::B4>::base(tid);
        const uint32_t tile = h ? tile0 + (1u << (D.logp - 18)) : tile0;
        float v[64];
        if constexpr (kRowWs4) fetch_ws4<R::B1>(a, D, tile, true, base1, v, kDecC2LdAux);
        else fetch_ws(a, D, tile, true, base1, v);
        const uint32_t b1 = seed_b(sld(a.seeds, D.tensor));
        if constexpr (kLadFly) {
            stages<R::B1, R::H1>(v);
            exchange_half_pad<R::B1, R::B2, 10>(v, s, tid);
            stages<R::B2, R::H2>(v);
            exchange_half_pad<R::B2, R::B3, 10>(v, s, tid);
            stages<R::B3, R::H3>(v);
            exchange_half_pad<R::B3, R::B4, 10>(v, s, tid);
            stages<R::B4, R::H4>(v);
        }
        const float sc = sldf(a.scales_in, D.scale_idx);
        if constexpr (kLadSign) {
            const float mul = sc * pow2i(-((D.logp + 1) / 2));
            if (pair) apply_signs_pair<R::B4>(v, tile << kRowLog, base4, D.logp, b1, mul, 1u + h, stash);
            else apply_signs_grouped<R::B4>(v, tile << kRowLog, base4, D.logp, b1, mul);
        }
        store_y_l<R::B4>(a, D, tile, base4, v);
        if (h >= pair) break;
      }
    }
}

// ===========================================================================
// Per-slice scales (large slices), after every final row pass.
// ===========================================================================

__global__ __launch_bounds__(256) void k_finalize(KArgs a) {
    __shared__ float red[4];
    const int si = a.list[blockIdx.x];
    const SliceDesc D = a.d[si];
    const int64_t ntile = 1ll << (D.logp - kRowLog);
    float dot = 0.f;
    for (int64_t t = threadIdx.x; t < ntile; t += 256) dot += a.part[D.part_off + t];
    dot = block_sum<256>(dot, red);
    const float nu = a.nu[si];
    const bool pos = nu > 0.0f;
    float scale = pos ? (nu * nu) / dot : 0.0f;
    const bool zero = !pos || isnan(scale);
    if (threadIdx.x == 0) a.scales[D.scale_idx] = zero ? 0.0f : scale;
    if (pos && zero) {  // rare: NaN scale -> reference returns all-zero bins (:522-525)
        const int64_t nbytes = 1ll << (D.logp - 3);
        for (int i = 0; i < a.nbits; ++i)
            for (int64_t q = threadIdx.x; q < nbytes; q += 256) a.pout[D.pl_off + i * D.pl_stride + q] = 0;
    }
}

}  // namespace ofl

// ===========================================================================
// Host side: plans and the C ABI
// ===========================================================================
namespace {

thread_local std::string g_err;
int fail(int code, const std::string& msg) { g_err = msg; return code; }
#define HIP_TRY(x)                                                                  \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) return fail(OFL_EHIP, std::string(#x " failed: ") + hipGetErrorString(e_)); \
    } while (0)

struct Launch {
    int kind;        // see enum below
    int param;       // p (small) / M (column)
    int lo;          // column passes
    int mid;         // column: fused middle pass; decode row A: 8-byte plane words
    int list_off;    // into d_list
    int tstart_off;  // into d_tstart (multi-tile kernels), -1 otherwise
    int count;       // list entries
    int64_t blocks;  // grid size
    int nu = 0;      // column: tile 0 of each slice writes the slice norm
    int stream = 0;  // 0: the caller's stream, 1: the plan's side stream, 2 / 3: its small-slice streams
    int join = 0;    // the caller's stream waits for the side stream before this launch
    int tl = 15;     // column: log2 of the tile (16: k_col6 with 1024 threads)
    int btab_off = -1;  // column: per-block {slice, tile << 3 | group} table in ints
    int ptab_off = -1;  // row: the paired table {slice, tile << 3 | pair} in ints (npair entries)
    int npair = 0;
    // a sub-wave launch of a split 5-pass slice (build_schedule): it covers
    // expl_tiles tiles listed in btab_off ({slice, tile << 3}); row launches
    // that apply D1 may take the paired list ptab_off (npair entries) instead
    bool expl = false;
    int64_t expl_tiles = 0;
    bool nt = false;  // column: the intermediate streams through HBM (k_col6<..., true>)
    int sset_off = -1;  // K_COLMSET: the small-set group table in ints
    int sset_groups = 0;  // K_COLMSET: its groups (the launch's first blocks)
    int64_t bytes_moved = 0;  // fp32/plane bytes this launch reads + writes (intermediates included)
    int64_t bytes_alg = 0;    // its share of the SURVEY 8(d) algorithmic bytes (x/y fp32 + planes only)
};
enum Kind { K_TINY, K_SMALL, K_ROWA, K_ROWC, K_COL, K_FINAL, K_COLM, K_SSET, K_COLMSET };

}  // namespace

struct ofl_eden_plan {
    int nbits = 8;
    int ntensors = 0;
    std::vector<ofl::SliceDesc> slices;
    std::vector<int64_t> t_planes_off, t_planes_bytes;
    std::vector<int32_t> t_first, t_nslices;
    int64_t planes_bytes = 0;
    int64_t ws_floats = 0;      // intermediates
    int64_t part_floats = 0;    // partials
    int64_t nlarge = 0;         // large slices (informational)
    int64_t arena = 0;          // fp32 arena length: max over tensors of elem_offset + numel
    // slice ids per kernel class (fixed by the batch) and the schedule built
    // from them (build_schedule)
    std::vector<int32_t> tiny, small[5], large;
    int64_t wave_bytes = 0;     // intermediate bytes per wave of large slices; 0: one wave
    int nstreams = 1;           // 2: waves alternate between the caller's and a side stream
    int nwaves = 0;
    int row2 = -1;              // row launches on the two-blocks-per-CU kernels: -1 auto, 0 never, 1 always
    int pair = -1;              // their tile pairs sharing D1 words: -1 auto, 0 never, 1 whenever possible
    int sset = -1;              // tiny / small slices in one small-set launch: -1 env default, 0 no, 1 yes
    int fuse = -1;              // small-set groups fused into the column launch: -1 env default, 0 no, 1 yes
    bool single = false;        // every launch on the caller's stream (no fork / join) -- K_COLMSET plans
    std::vector<Launch> enc, dec;
    std::vector<int32_t> ints;  // launch lists and tile prefixes (host copy)
    // profiling: events around every launch of every call while enabled
    bool prof = false;
    std::vector<std::vector<hipEvent_t>> prof_ev[2];  // [dec, enc][call][launch+1]
    std::vector<hipEvent_t> ev_pool;
    ofl::SliceDesc* d_slices = nullptr;
    int32_t* d_ints = nullptr;
    int device = -1;
    int ncu = 256;              // persistent row launches: one block per CU
    bool uploaded = false;
    std::mutex mu;
    hipStream_t side = nullptr;  // nstreams == 2: the device's shared side streams (shared_side_streams)
    hipStream_t side2 = nullptr; // the tiny / small slices, beside both wave streams
    hipStream_t side3 = nullptr; // half of the tiny / small launches (use_small_split)
    hipEvent_t ev_fork = nullptr, ev_join = nullptr, ev_join2 = nullptr, ev_join3 = nullptr;
    std::mutex run_mu;          // serialises runs that use the side stream
};

namespace {

// Default large-slice schedule (see build_schedule):
// waves the size of the 256 MiB Infinity Cache's working half on two streams,
// with the two-blocks-per-CU row kernels (1-2 tiles per CU per wave).  Since
// the additive-LCG signs these beat 2 GiB waves on the Llama-3-8B step (429-431
// vs 426-427 GiB/s) and the 1 GiB set (470-474 vs 458-461); 256 MiB waves lose
// (420-422 / 450-452), profiles/r06_sched_ab.txt.  Slices above the wave size
// (the 2^29 ones) are waves of their own and keep the persistent kernels.
constexpr int64_t kDefaultWaveMiB = 128;
constexpr int64_t kDefaultStreams = 2;

int64_t low_po2(int64_t n) { int64_t p = 1; while (p * 2 <= n) p *= 2; return n ? p : 0; }
int64_t high_po2(int64_t n) { int64_t p = 1; while (p < n) p *= 2; return n ? p : 0; }
int ilog2(int64_t v) { int l = 0; while ((1ll << l) < v) ++l; return l; }

template <typename K>
hipError_t launch(K kern, int64_t blocks, int threads, size_t shmem, hipStream_t st, const ofl::KArgs& a) {
    if (blocks <= 0) return hipSuccess;
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(threads), shmem, st, a);
    return hipGetLastError();
}

size_t small_smem(int p, bool enc) {
    switch (p) {
    case 11: return enc ? ofl::SmallSmem<11>::enc : ofl::SmallSmem<11>::dec;
    case 12: return enc ? ofl::SmallSmem<12>::enc : ofl::SmallSmem<12>::dec;
    case 13: return enc ? ofl::SmallSmem<13>::enc : ofl::SmallSmem<13>::dec;
    case 14: return enc ? ofl::SmallSmem<14>::enc : ofl::SmallSmem<14>::dec;
    default: return enc ? ofl::SmallSmem<15>::enc : ofl::SmallSmem<15>::dec;
    }
}

hipError_t set_lds(const void* f, size_t bytes) {
    return hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

template <int P>
hipError_t set_small_attr() {
    hipError_t e = set_lds((const void*)ofl::k_enc_small<P>, ofl::SmallSmem<P>::enc);
    return e != hipSuccess ? e : set_lds((const void*)ofl::k_dec_small<P>, ofl::SmallSmem<P>::dec);
}

size_t col_smem(int M, bool mid) { return (M > 5 ? ofl::kColSmem : 0) + (mid && M >= 3 ? ofl::kColTab : 0); }

template <int M>
hipError_t set_col_attr() {
    hipError_t e = set_lds((const void*)ofl::k_col<M, true>, col_smem(M, true));
    return e != hipSuccess ? e : set_lds((const void*)ofl::k_col<M, false>, col_smem(M, false));
}

size_t col6_smem(int M, bool mid, int tl) {
    return tl == 16 ? (M > 6 ? ofl::col6_half<16>() : 0) + (mid ? ofl::col6_tab<16>() : 0)
                    : (M > 6 ? ofl::col6_half<15>() : 0) + (mid ? ofl::col6_tab<15>() : 0);
}

template <int M, int TL>
hipError_t set_col6_attr() {
    hipError_t e = set_lds((const void*)ofl::k_col6<M, true, TL>, col6_smem(M, true, TL));
    return e != hipSuccess ? e : set_lds((const void*)ofl::k_col6<M, false, TL>, col6_smem(M, false, TL));
}

// 2^16-element tiles for the 2^24 / 2^25 middle column passes: off by default
// (measured slower than two 2^15-tile blocks per CU: 457 vs 432 us, 357 vs
// 307 us per launch); OFL_EDEN_COL16=1 selects them (A/B)
bool use_col16() {
    static const bool on = [] { const char* s = getenv("OFL_EDEN_COL16"); return s && s[0] == '1'; }();
    return on;
}

// encode pass C uses k_enc_rowC2 (OFL_EDEN_ROWC2=0: k_enc_rowC, A/B)
bool use_rowc2() {
    static const bool on = [] { const char* s = getenv("OFL_EDEN_ROWC2"); return !(s && s[0] == '0'); }();
    return on;
}

// k_enc_rowC2 loads the next tile into the quantiser's freed registers
// (OFL_EDEN_ROLL=0: load at the top of each tile, A/B)
bool use_roll() {
    static const bool on = [] { const char* s = getenv("OFL_EDEN_ROLL"); return !(s && s[0] == '0'); }();
    return on;
}

// Row launches of fewer than row2_max_tiles_per_cu() tiles per CU use the
// two-blocks-per-CU kernels (k_enc_rowA2 / k_dec_rowA2 / k_dec_rowC2; outputs
// bit-identical).  OFL_EDEN_ROW2=0: never, =1: always, unset: below the
// threshold (OFL_EDEN_ROW2_TPC tiles per CU, default 5).
int row2_mode() {
    static const int m = [] { const char* s = getenv("OFL_EDEN_ROW2"); return (s && *s) ? (s[0] == '1' ? 1 : 0) : -1; }();
    return m;
}
int64_t row2_max_tiles_per_cu() {
    static const int64_t v = [] { const char* s = getenv("OFL_EDEN_ROW2_TPC"); return (s && *s) ? strtoll(s, nullptr, 10) : 5ll; }();
    return v;
}
bool use_row2(int64_t tiles, int ncu, int plan_mode) {
    const int m = plan_mode >= 0 ? plan_mode : row2_mode();
    return m >= 0 ? m == 1 : tiles < row2_max_tiles_per_cu() * (int64_t)ncu;
}

// column passes with M >= 8 rows, or a middle pass with M >= 6, use k_col6
// (measured: the 1024-thread k_col is ~4 % faster on the plain M = 7 pass);
// OFL_EDEN_COL6=0 forces k_col everywhere (A/B)
bool use_col6() {
    static const bool on = [] { const char* s = getenv("OFL_EDEN_COL6"); return !(s && s[0] == '0'); }();
    return on;
}
// lowest outer (non-middle) column-pass height that runs k_col6
// (OFL_EDEN_COL6_OUTER, default 8: the 5-pass slices' level-1 passes of
// heights 5..7 run k_col)
int col6_outer_min() {
    static const int v = [] { const char* s = getenv("OFL_EDEN_COL6_OUTER"); return (s && *s) ? atoi(s) : 8; }();
    return v;
}
// interleaved ws layout for 2^25 slices (256-B segments in the middle pass)
bool use_perm25() {
    static const bool on = [] { const char* s = getenv("OFL_EDEN_PERM25"); return !(s && s[0] == '0'); }();
    return on;
}
// the tiny / small launches (latency-bound, independent of each other) split
// over two streams instead of one (OFL_EDEN_SMALL2=0: one stream, A/B)
// (opt-in OFL_EDEN_SMALL2=1: measured slower on ResNet-50, 259-269 vs
// 273-276 GiB/s, profiles/r03_resnet50_row2_small2_ab.txt)
bool use_small_split() {
    static const bool on = [] { const char* s = getenv("OFL_EDEN_SMALL2"); return s && s[0] == '1'; }();
    return on;
}
// every tiny / small slice in one small-set launch (k_enc_sset / k_dec_sset)
// instead of a chain of one launch per size class (OFL_EDEN_SSET=0, A/B)
bool use_sset() {
    static const bool on = [] { const char* s = getenv("OFL_EDEN_SSET"); return !(s && s[0] == '0'); }();
    return on;
}
// tiny / small slices on a third stream when the waves use two
bool use_small_stream() {
    static const bool on = [] { const char* s = getenv("OFL_EDEN_SMALLSTREAM"); return !(s && s[0] == '0'); }();
    return on;
}
// two-stream plans whose large slices fit one wave split them into exactly
// two balanced waves (OFL_EDEN_TWOWAVES=0: in-order packing against half the
// total)
bool use_two_waves() {
    static const bool on = [] { const char* s = getenv("OFL_EDEN_TWOWAVES"); return !(s && s[0] == '0'); }();
    return on;
}
// the whole-slice middle pass of a split 5-pass slice streams its
// intermediate with nt loads and stores (OFL_EDEN_MIDNT=0: default policy)
bool use_mid_nt() {
    static const bool on = [] { const char* s = getenv("OFL_EDEN_MIDNT"); return !(s && s[0] == '0'); }();
    return on;
}
int64_t big_sub_mib() {
    static const int64_t v = [] { const char* s = getenv("OFL_EDEN_BIGSUB_MIB"); return (s && *s) ? strtoll(s, nullptr, 10) : 0ll; }();
    return v;
}
// 5-pass slices bigger than a wave run their first two and last two passes
// in MALL-sized sub-waves (OFL_EDEN_BIGSPLIT=0: whole-slice passes)
bool use_big_split() {
    static const bool on = [] { const char* s = getenv("OFL_EDEN_BIGSPLIT"); return !(s && s[0] == '0'); }();
    return on;
}
// multi-wave plans pack their large slices largest first (OFL_EDEN_WAVESORT=0:
// in batch order, =2: smallest first; profiles/r06_sort_roll_ab.txt)
int wave_sort_mode() {
    static const int m = [] { const char* s = getenv("OFL_EDEN_WAVESORT"); return (s && *s) ? (int)(s[0] - '0') : 1; }();
    return m;
}
bool use_wave_sort() { return wave_sort_mode() != 0; }
// column launches find their tile in a per-block table (OFL_EDEN_BTAB=0:
// binary search over the launch's tile prefix, as before)
bool use_btab() {
    static const bool on = [] { const char* s = getenv("OFL_EDEN_BTAB"); return !(s && s[0] == '0'); }();
    return on;
}
// row launches up to this many tiles carry a per-tile table (8 B per tile)
constexpr int64_t kRowTabMax = 1 << 16;
// two-blocks-per-CU row launches of more tiles than block slots run tile
// pairs sharing their D1 words (apply_signs_pair; OFL_EDEN_PAIR=0: never,
// =1: whenever the launch has a paired table)
int pair_mode() {
    static const int m = [] { const char* s = getenv("OFL_EDEN_PAIR"); return (s && *s) ? (s[0] == '1' ? 1 : 0) : -1; }();
    return m;
}
bool use_pair(const Launch& l, int ncu, int plan_mode) {
    if (l.ptab_off < 0 || !use_btab()) return false;
    const int m = plan_mode >= 0 ? plan_mode : pair_mode();
    return m >= 0 ? m == 1 : l.blocks > 2 * (int64_t)ncu;
}
// OFL_EDEN_SPLIT_MIB=m: two-stream plans split their large slices into two
// waves only above m MiB of intermediates; unset (-1): see build_schedule
int64_t split_min_bytes() {
    static const int64_t b = [] {
        const char* s = getenv("OFL_EDEN_SPLIT_MIB");
        const int64_t m = (s && *s) ? strtoll(s, nullptr, 10) : -1;
        return m < 0 ? -1 : m << 20;
    }();
    return b;
}
// one-wave plans with a k_col_multi launch and a small-set launch fuse the
// two into one launch on the caller's stream (OFL_EDEN_FUSESET=0: the
// small-set launch beside the wave on the side stream)
bool use_fuse_sset() {
    static const bool on = [] { const char* s = getenv("OFL_EDEN_FUSESET"); return !(s && s[0] == '0'); }();
    return on;
}
// height-6 middle passes (2^21 slices) run col_body<6> (1024 threads, the
// k_col arithmetic) and join the k_col_multi launch of the smaller heights;
// OFL_EDEN_COLM6=0: their own k_col6<6, true, 15> launch after it (A/B; the
// two differ in the order of the row butterflies after D2, so their bytes
// differ slightly -- every schedule of one setting is bit-identical)
bool use_colm6() {
    static const bool on = [] { const char* s = getenv("OFL_EDEN_COLM6"); return !(s && s[0] == '0'); }();
    return on;
}
// lowest middle-pass height that runs k_col6 (7 when height 6 runs col_body<6>:
// a standalone height-6 launch then uses k_col<6, true> too)
int col6_mid_min() { return use_colm6() ? 7 : 6; }
// k_col6 (else k_col) for a column pass of this height
bool col6_for(int param, bool mid) {
    return (param >= 8 || (mid ? param >= col6_mid_min() : param >= col6_outer_min())) && param >= 6 && use_col6();
}
// one k_col_multi launch per wave for the single-level heights 1..5 (6)
bool use_colmulti() {
    static const bool on = [] { const char* s = getenv("OFL_EDEN_COLMULTI"); return !(s && s[0] == '0'); }();
    return on;
}

hipError_t set_all_attrs() {
    hipError_t e;
    if ((e = set_small_attr<11>()) != hipSuccess) return e;
    if ((e = set_small_attr<12>()) != hipSuccess) return e;
    if ((e = set_small_attr<13>()) != hipSuccess) return e;
    if ((e = set_small_attr<14>()) != hipSuccess) return e;
    if ((e = set_small_attr<15>()) != hipSuccess) return e;
    if ((e = set_lds((const void*)ofl::k_enc_sset, ofl::kSetSmemEnc)) != hipSuccess) return e;
    if ((e = set_lds((const void*)ofl::k_dec_sset, ofl::kSetSmemDec)) != hipSuccess) return e;
    if ((e = set_lds((const void*)ofl::k_enc_colm_set, std::max(ofl::kSetSmemEnc, ofl::kColMultiSmem))) != hipSuccess) return e;
    if ((e = set_lds((const void*)ofl::k_dec_colm_set, std::max(ofl::kSetSmemDec, ofl::kColMultiSmem))) != hipSuccess) return e;
    if ((e = set_lds((const void*)ofl::k_col_multi, ofl::kColMultiSmem)) != hipSuccess) return e;
    if ((e = set_lds((const void*)ofl::k_enc_rowA, ofl::kRowSmemA)) != hipSuccess) return e;
    if ((e = set_lds((const void*)ofl::k_enc_rowC, ofl::kRowSmemQ)) != hipSuccess) return e;
    if ((e = set_lds((const void*)ofl::k_enc_rowC2<true>, ofl::kRowC2Smem)) != hipSuccess) return e;
    if ((e = set_lds((const void*)ofl::k_enc_rowC2<false>, ofl::kRowC2Smem)) != hipSuccess) return e;
    if ((e = set_lds((const void*)ofl::k_dec_rowA<true>, ofl::kRowSmemC)) != hipSuccess) return e;
    if ((e = set_lds((const void*)ofl::k_dec_rowA<false>, ofl::kRowSmemC)) != hipSuccess) return e;
    if ((e = set_lds((const void*)ofl::k_dec_rowC, ofl::kRowSmemA)) != hipSuccess) return e;
    if ((e = set_lds((const void*)ofl::k_enc_rowA2<false>, ofl::kRow2Smem)) != hipSuccess) return e;
    if ((e = set_lds((const void*)ofl::k_enc_rowA2<true>, ofl::kRow2Smem)) != hipSuccess) return e;
    if ((e = set_lds((const void*)ofl::k_dec_rowA2<true>, ofl::kRow2SmemC)) != hipSuccess) return e;
    if ((e = set_lds((const void*)ofl::k_dec_rowA2<false>, ofl::kRow2SmemC)) != hipSuccess) return e;
    if ((e = set_lds((const void*)ofl::k_dec_rowC2, ofl::kRow2Smem)) != hipSuccess) return e;
    if ((e = set_col_attr<6>()) != hipSuccess) return e;
    if ((e = set_col_attr<7>()) != hipSuccess) return e;
    if ((e = set_col_attr<8>()) != hipSuccess) return e;
    if ((e = set_col_attr<9>()) != hipSuccess) return e;
    if ((e = set_col_attr<10>()) != hipSuccess) return e;
    if ((e = set_col6_attr<6, 15>()) != hipSuccess) return e;
    if ((e = set_col6_attr<7, 15>()) != hipSuccess) return e;
    if ((e = set_col6_attr<8, 15>()) != hipSuccess) return e;
    if ((e = set_col6_attr<9, 15>()) != hipSuccess) return e;
    if ((e = set_col6_attr<10, 15>()) != hipSuccess) return e;
    if ((e = set_lds((const void*)ofl::k_col6<7, true, 15, true>, col6_smem(7, true, 15))) != hipSuccess) return e;
    if ((e = set_col6_attr<9, 16>()) != hipSuccess) return e;
    return set_col6_attr<10, 16>();
}

int run(ofl_eden_plan* pl, bool enc, const ofl::KArgs& base, hipStream_t caller) {
    const hipError_t attrs_err = ofl_util::per_device_once([] { return set_all_attrs(); });
    if (attrs_err != hipSuccess) return fail(OFL_EHIP, std::string("hipFuncSetAttribute: ") + hipGetErrorString(attrs_err));
    const std::vector<Launch>& L = enc ? pl->enc : pl->dec;
    // waves on the side stream fork from and join back into the caller's stream
    const bool two = pl->side != nullptr && !pl->single;
    std::unique_lock<std::mutex> lk(pl->run_mu, std::defer_lock);
    if (two) {
        lk.lock();
        HIP_TRY(hipEventRecord(pl->ev_fork, caller));
        HIP_TRY(hipStreamWaitEvent(pl->side, pl->ev_fork, 0));
        if (pl->side2) HIP_TRY(hipStreamWaitEvent(pl->side2, pl->ev_fork, 0));
        if (pl->side3) HIP_TRY(hipStreamWaitEvent(pl->side3, pl->ev_fork, 0));
    }
    const hipStream_t streams[4] = {caller, two ? pl->side : caller, pl->side2 ? pl->side2 : caller,
                                    pl->side3 ? pl->side3 : (pl->side2 ? pl->side2 : caller)};
    bool joined = !two;
    std::vector<hipEvent_t>* evs = nullptr;
    if (pl->prof) {  // one event before and one after every launch, on its stream
        std::lock_guard<std::mutex> g(pl->mu);
        pl->prof_ev[enc].emplace_back();
        evs = &pl->prof_ev[enc].back();
        for (size_t i = 0; i < 2 * L.size(); ++i) {
            hipEvent_t e;
            if (!pl->ev_pool.empty()) { e = pl->ev_pool.back(); pl->ev_pool.pop_back(); }
            else HIP_TRY(hipEventCreate(&e));
            evs->push_back(e);
        }
    }
    for (size_t li = 0; li < L.size(); ++li) {
        const Launch& l = L[li];
        if (l.join && !joined) {
            HIP_TRY(hipEventRecord(pl->ev_join, pl->side));
            HIP_TRY(hipStreamWaitEvent(caller, pl->ev_join, 0));
            joined = true;
        }
        const hipStream_t st = streams[l.stream];
        ofl::KArgs a = base;
        a.list = pl->d_ints + l.list_off;
        a.tstart = l.tstart_off >= 0 ? pl->d_ints + l.tstart_off : nullptr;
        a.btab = l.btab_off >= 0 && use_btab() ? pl->d_ints + l.btab_off : nullptr;
        a.count = l.count;
        a.lo = l.lo;
        a.do_nu = l.nu;
        a.npair = 0;
        if (evs) HIP_TRY(hipEventRecord((*evs)[2 * li], st));
        hipError_t e = hipSuccess;
        switch (l.kind) {
        case K_TINY:
            e = enc ? launch(ofl::k_enc_tiny, l.blocks, ofl::kTinyNT, 0, st, a)
                    : launch(ofl::k_dec_tiny, l.blocks, ofl::kTinyNT, 0, st, a);
            break;
        case K_SSET:
            e = enc ? launch(ofl::k_enc_sset, l.blocks, ofl::kSetNT, ofl::kSetSmemEnc, st, a)
                    : launch(ofl::k_dec_sset, l.blocks, ofl::kSetNT, ofl::kSetSmemDec, st, a);
            break;
        case K_SMALL: {
            const int p = l.param;
            const int nt = 1 << (p - 5);
            const size_t sm = small_smem(p, enc);
#define SMALLCASE(PP)                                                                         \
    case PP:                                                                                  \
        e = enc ? launch(ofl::k_enc_small<PP>, l.blocks, nt, sm, st, a)                       \
                : launch(ofl::k_dec_small<PP>, l.blocks, nt, sm, st, a);                      \
        break;
            switch (p) {
                SMALLCASE(11) SMALLCASE(12) SMALLCASE(13) SMALLCASE(14) SMALLCASE(15)
            default: return fail(OFL_EINVAL, "small slice size out of range");
            }
#undef SMALLCASE
            break;
        }
        case K_ROWA: {
            const bool a8 = l.mid && (reinterpret_cast<uintptr_t>(base.pin) & 7u) == 0;
            if (l.expl) {  // a sub-wave of a split 5-pass slice: its tile list
                const bool paired = enc && !base.wx && l.ptab_off >= 0;
                a.btab = pl->d_ints + (paired ? l.ptab_off : l.btab_off);
                a.npair = paired ? l.npair : (int)l.expl_tiles;
                const int64_t g2 = std::min<int64_t>(a.npair, 2 * pl->ncu);
                e = enc ? (base.wx ? launch(ofl::k_enc_rowA2<true>, g2, ofl::kRowNT, ofl::kRow2Smem, st, a)
                                   : launch(ofl::k_enc_rowA2<false>, g2, ofl::kRowNT, ofl::kRow2Smem, st, a))
                        : a8 ? launch(ofl::k_dec_rowA2<true>, g2, ofl::kRowNT, ofl::kRow2SmemC, st, a)
                             : launch(ofl::k_dec_rowA2<false>, g2, ofl::kRowNT, ofl::kRow2SmemC, st, a);
                break;
            }
            if (enc && base.wx) {  // fused round-end encode: x = the weighted-average delta
                e = launch(ofl::k_enc_rowA2<true>, std::min<int64_t>(l.blocks, 2 * pl->ncu), ofl::kRowNT, ofl::kRow2Smem,
                           st, a);
                break;
            }
            if (use_row2(l.blocks, pl->ncu, pl->row2)) {
                int64_t g2 = std::min<int64_t>(l.blocks, 2 * pl->ncu);
                if (enc && use_pair(l, pl->ncu, pl->pair)) {
                    a.btab = pl->d_ints + l.ptab_off;
                    a.npair = l.npair;
                    g2 = std::min<int64_t>(l.npair, 2 * pl->ncu);
                }
                e = enc ? launch(ofl::k_enc_rowA2<false>, g2, ofl::kRowNT, ofl::kRow2Smem, st, a)
                        : a8 ? launch(ofl::k_dec_rowA2<true>, g2, ofl::kRowNT, ofl::kRow2SmemC, st, a)
                             : launch(ofl::k_dec_rowA2<false>, g2, ofl::kRowNT, ofl::kRow2SmemC, st, a);
                break;
            }
            const int64_t g = std::min<int64_t>(l.blocks, pl->ncu);
            e = enc ? launch(ofl::k_enc_rowA, g, ofl::kRowNT, ofl::kRowSmemA, st, a)
                    : a8 ? launch(ofl::k_dec_rowA<true>, g, ofl::kRowNT, ofl::kRowSmemC, st, a)
                         : launch(ofl::k_dec_rowA<false>, g, ofl::kRowNT, ofl::kRowSmemC, st, a);
            break;
        }
        case K_ROWC: {
            const int64_t g = std::min<int64_t>(l.blocks, pl->ncu);
            if (l.expl) {  // a sub-wave of a split 5-pass slice: its tile list
                const bool paired = !enc && l.ptab_off >= 0;
                a.btab = pl->d_ints + (paired ? l.ptab_off : l.btab_off);
                a.npair = paired ? l.npair : (int)l.expl_tiles;
                const int64_t g2 = std::min<int64_t>(a.npair, 2 * pl->ncu);
                e = !enc ? launch(ofl::k_dec_rowC2, g2, ofl::kRowNT, ofl::kRow2Smem, st, a)
                    : use_roll() ? launch(ofl::k_enc_rowC2<true>, g2, ofl::kRowNT, ofl::kRowC2Smem, st, a)
                                 : launch(ofl::k_enc_rowC2<false>, g2, ofl::kRowNT, ofl::kRowC2Smem, st, a);
                break;
            }
            if (enc && use_rowc2())
                e = use_roll() ? launch(ofl::k_enc_rowC2<true>, std::min<int64_t>(l.blocks, 2 * pl->ncu), ofl::kRowNT,
                                        ofl::kRowC2Smem, st, a)
                               : launch(ofl::k_enc_rowC2<false>, std::min<int64_t>(l.blocks, 2 * pl->ncu), ofl::kRowNT,
                                        ofl::kRowC2Smem, st, a);
            else if (!enc && use_row2(l.blocks, pl->ncu, pl->row2)) {
                int64_t g2 = std::min<int64_t>(l.blocks, 2 * pl->ncu);
                if (use_pair(l, pl->ncu, pl->pair)) {
                    a.btab = pl->d_ints + l.ptab_off;
                    a.npair = l.npair;
                    g2 = std::min<int64_t>(l.npair, 2 * pl->ncu);
                }
                e = launch(ofl::k_dec_rowC2, g2, ofl::kRowNT, ofl::kRow2Smem, st, a);
            }
            else
                e = enc ? launch(ofl::k_enc_rowC, g, ofl::kRowNT, ofl::kRowSmemQ, st, a)
                        : launch(ofl::k_dec_rowC, g, ofl::kRowNT, ofl::kRowSmemA, st, a);
            break;
        }
        case K_COL: {
            if (l.tl == 16) {  // 2^16-element tiles (M = 9, 10)
                const size_t sm = col6_smem(l.param, l.mid != 0, 16);
                e = l.param == 9 ? (l.mid ? launch(ofl::k_col6<9, true, 16>, l.blocks, 1024, sm, st, a)
                                          : launch(ofl::k_col6<9, false, 16>, l.blocks, 1024, sm, st, a))
                                 : (l.mid ? launch(ofl::k_col6<10, true, 16>, l.blocks, 1024, sm, st, a)
                                          : launch(ofl::k_col6<10, false, 16>, l.blocks, 1024, sm, st, a));
                break;
            }
            if (l.nt && l.param == 7 && l.mid && col6_for(7, true)) {
                e = launch(ofl::k_col6<7, true, 15, true>, l.blocks, 512, col6_smem(7, true, 15), st, a);
                break;
            }
            if (col6_for(l.param, l.mid != 0)) {
                const size_t sm = col6_smem(l.param, l.mid != 0, 15);
#define COL6CASE(MM)                                                                                 \
    case MM:                                                                                         \
        e = l.mid ? launch(ofl::k_col6<MM, true, 15>, l.blocks, 512, sm, st, a)                      \
                  : launch(ofl::k_col6<MM, false, 15>, l.blocks, 512, sm, st, a);                    \
        break;
                switch (l.param) {
                    COL6CASE(6) COL6CASE(7) COL6CASE(8) COL6CASE(9) COL6CASE(10)
                default: return fail(OFL_EINVAL, "column pass height out of range");
                }
#undef COL6CASE
                break;
            }
            const size_t sm = col_smem(l.param, l.mid != 0);
#define COLCASE(MM)                                                                                  \
    case MM:                                                                                         \
        e = l.mid ? launch(ofl::k_col<MM, true>, l.blocks, ofl::kColNT, sm, st, a)                   \
                  : launch(ofl::k_col<MM, false>, l.blocks, ofl::kColNT, sm, st, a);                 \
        break;
            switch (l.param) {
                COLCASE(1) COLCASE(2) COLCASE(3) COLCASE(4) COLCASE(5) COLCASE(6) COLCASE(7) COLCASE(8) COLCASE(9)
                COLCASE(10)
            default: return fail(OFL_EINVAL, "column pass height out of range");
            }
#undef COLCASE
            break;
        }
        case K_FINAL: e = launch(ofl::k_finalize, l.blocks, 256, 0, st, a); break;
        case K_COLM: e = launch(ofl::k_col_multi, l.blocks, ofl::kColNT, ofl::kColMultiSmem, st, a); break;
        case K_COLMSET:
            a.sset = pl->d_ints + l.sset_off;
            a.sset_first = (int32_t)l.sset_groups;
            e = enc ? launch(ofl::k_enc_colm_set, l.blocks, ofl::kColNT, std::max(ofl::kSetSmemEnc, ofl::kColMultiSmem), st, a)
                    : launch(ofl::k_dec_colm_set, l.blocks, ofl::kColNT, std::max(ofl::kSetSmemDec, ofl::kColMultiSmem), st, a);
            break;
        }
        if (e != hipSuccess) return fail(OFL_EHIP, std::string("kernel launch failed: ") + hipGetErrorString(e));
        if (evs) HIP_TRY(hipEventRecord((*evs)[2 * li + 1], st));
    }
    if (!joined) {
        HIP_TRY(hipEventRecord(pl->ev_join, pl->side));
        HIP_TRY(hipStreamWaitEvent(caller, pl->ev_join, 0));
    }
    if (two && pl->side2) {
        HIP_TRY(hipEventRecord(pl->ev_join2, pl->side2));
        HIP_TRY(hipStreamWaitEvent(caller, pl->ev_join2, 0));
    }
    if (two && pl->side3) {
        HIP_TRY(hipEventRecord(pl->ev_join3, pl->side3));
        HIP_TRY(hipStreamWaitEvent(caller, pl->ev_join3, 0));
    }
    return OFL_OK;
}

std::string launch_name(const Launch& l, bool enc, int ncu, int row2) {
    const char* d = enc ? "enc" : "dec";
    switch (l.kind) {
    case K_TINY: return std::string("ofl::k_") + d + "_tiny";
    case K_SSET: return std::string("ofl::k_") + d + "_sset";
    case K_SMALL: return std::string("ofl::k_") + d + "_small<" + std::to_string(l.param) + ">";
    case K_ROWA: return std::string("ofl::k_") + d + (use_row2(l.blocks, ncu, row2) ? "_rowA2" : "_rowA");
    case K_ROWC:
        if (enc && use_rowc2()) return std::string("ofl::k_enc_rowC2<") + (use_roll() ? "true" : "false") + ">";
        if (!enc && use_row2(l.blocks, ncu, row2)) return "ofl::k_dec_rowC2";
        return std::string("ofl::k_") + d + "_rowC";
    case K_COL:
        if (l.tl == 16) return "ofl::k_col6<" + std::to_string(l.param) + ", " + (l.mid ? "true" : "false") + ", 16>";
        return std::string(col6_for(l.param, l.mid != 0) ? "ofl::k_col6<" : "ofl::k_col<") +
               std::to_string(l.param) + ", " + (l.mid ? "true" : "false") +
               (col6_for(l.param, l.mid != 0) ? ", 15>" : ">");
    case K_COLM: return "ofl::k_col_multi";
    case K_COLMSET: return std::string("ofl::k_") + d + "_colm_set";
    default: return "ofl::k_finalize";
    }
}

// Large slices run in waves of at most wave_bytes of intermediates (a bigger
// slice is a wave of its own).  A wave runs row pass A, its column passes and
// row pass C back to back, so its intermediates are re-read while they still
// sit in the 256 MiB Infinity Cache; waves share nstreams workspace buffers
// (wave w: buffer and stream w % nstreams).  The scales are finalised once,
// after every wave.
void build_schedule(ofl_eden_plan* pl) {
    std::vector<int32_t>& ints = pl->ints;
    ints.clear();
    pl->enc.clear();
    pl->dec.clear();
    auto add_list = [&](const std::vector<int32_t>& l) {
        const int o = (int)ints.size();
        ints.insert(ints.end(), l.begin(), l.end());
        return o;
    };
    auto add_prefix = [&](const std::vector<int32_t>& l, int log_tile, int64_t& total) {
        const int o = (int)ints.size();
        int64_t acc = 0;
        for (int32_t si : l) { ints.push_back((int32_t)acc); acc += 1ll << (pl->slices[si].logp - log_tile); }
        ints.push_back((int32_t)acc);
        total = acc;
        return o;
    };
    std::vector<Launch> common;
    const bool sset = pl->sset >= 0 ? pl->sset == 1 : use_sset();
    if (sset) {
        // one small-set launch: groups of one size, largest first; table of
        // {P (0: tiny), slice-list offset (from the table), count} per block
        std::vector<std::array<int32_t, 3>> groups;
        std::vector<int32_t> ids;
        auto add_groups = [&](int P, const std::vector<int32_t>& sl, int per) {
            for (size_t i = 0; i < sl.size(); i += per) {
                const int c = (int)std::min<size_t>(per, sl.size() - i);
                groups.push_back({P, (int32_t)ids.size(), c});
                ids.insert(ids.end(), sl.begin() + i, sl.begin() + i + c);
            }
        };
        for (int k = 4; k >= 0; --k) add_groups(11 + k, pl->small[k], ofl::kSetNT >> (6 + k));
        for (int p = 10; p >= 0; --p) {  // tiny slices: groups of one p (same barrier count)
            std::vector<int32_t> sl;
            for (int32_t si : pl->tiny) if (pl->slices[si].logp == p) sl.push_back(si);
            add_groups(0, sl, ofl::kSetNT / ofl::kTinyNT);
        }
        if (!groups.empty()) {
            const int o = (int)ints.size();
            const int nt = 3 * (int)groups.size();
            for (auto& g : groups) { ints.push_back(g[0]); ints.push_back(g[1] + nt); ints.push_back(g[2]); }
            ints.insert(ints.end(), ids.begin(), ids.end());
            common.push_back({K_SSET, 0, 0, 0, o, -1, (int)groups.size(), (int64_t)groups.size()});
        }
    } else {
        if (!pl->tiny.empty())
            common.push_back({K_TINY, 0, 0, 0, add_list(pl->tiny), -1, (int)pl->tiny.size(), (int64_t)pl->tiny.size()});
        for (int k = 0; k < 5; ++k)
            if (!pl->small[k].empty())
                common.push_back({K_SMALL, 11 + k, 0, 0, add_list(pl->small[k]), -1, (int)pl->small[k].size(),
                                  (int64_t)pl->small[k].size()});
    }
    for (auto& D : pl->slices) D.perm = 0;
    std::vector<std::vector<int32_t>> waves;
    int64_t cap = pl->wave_bytes > 0 ? pl->wave_bytes / 4 : INT64_MAX;
    int64_t tot = 0;
    for (int32_t si : pl->large) tot += 1ll << pl->slices[si].logp;
    // more than one wave by size: the large slices largest first (stable), so
    // in-order packing fills each wave with slices of one size -- power-of-two
    // sizes pack whole waves, one column launch per wave (OFL_EDEN_WAVESORT).
    // Llama-3-8B: 210 waves of 1024 tiles (but the two 2^29 ones), 637
    // launches per direction instead of 258 waves of 512-1024 tiles and 909
    // launches; 434.8-435.4 -> 445.7-448.8 GiB/s
    std::vector<int32_t> sorted_large;
    if (tot > cap && use_wave_sort()) {
        sorted_large = pl->large;
        const bool up = wave_sort_mode() == 2;
        std::stable_sort(sorted_large.begin(), sorted_large.end(), [&](int32_t x, int32_t y) {
            return up ? pl->slices[x].logp < pl->slices[y].logp : pl->slices[x].logp > pl->slices[y].logp;
        });
    }
    const std::vector<int32_t>& large = sorted_large.empty() ? pl->large : sorted_large;
    // two streams: at least two waves, so both streams have work -- unless
    // every large slice fits one wave and no small-slice launches could use
    // the second stream (at 2 GiB waves the 1 GiB set ran one wave on one
    // stream, 2.24 vs 2.29 ms; ResNet-50 keeps its two waves beside the small slices: 360
    // vs 369 us with one wave; OFL_EDEN_SPLIT_MIB=m splits above m MiB)
    // With the small-set launch a plan that fits one wave keeps it whole: the
    // one small-set launch runs beside it on the side stream (ResNet-50 0.288
    // vs 0.309 ms with two waves, profiles/r03_resnet50_sset_onewave_ab.txt)
    const int64_t split_min = split_min_bytes();
    const bool split = split_min >= 0 ? 4 * tot > split_min : ((!common.empty() && !sset) || tot > cap);
    // the split only feeds the second stream (everything fits one wave):
    // exactly two waves, cut where the halves are closest (in-order packing
    // against a half-total cap can leave a third wave behind the first on the
    // same stream -- ResNet-50: 417 vs 353 tiles per stream)
    int64_t cut = -1;
    if (pl->nstreams == 2 && split && tot <= cap && large.size() > 1 && use_two_waves()) {
        int64_t pre = 0, best = INT64_MAX;
        for (size_t k = 0; k + 1 < large.size(); ++k) {
            pre += 1ll << pl->slices[large[k]].logp;
            const int64_t d = std::llabs(2 * pre - tot);
            if (d < best) { best = d; cut = (int64_t)k + 1; }
        }
    } else if (pl->nstreams == 2 && split) {
        cap = std::min(cap, std::max<int64_t>(1, (tot + 1) / 2));
    }
    int64_t acc = 0, wmax = 0;
    for (size_t k = 0; k < large.size(); ++k) {
        const int32_t si = large[k];
        const int64_t P = 1ll << pl->slices[si].logp;
        if (waves.empty() || (cut >= 0 ? (int64_t)k == cut : acc + P > cap)) { waves.emplace_back(); acc = 0; }
        waves.back().push_back(si);
        acc += P;
        wmax = std::max(wmax, acc);
    }
    pl->nwaves = (int)waves.size();
    const int nbuf = waves.size() > 1 ? pl->nstreams : 1;
    // the tiny / small slices are independent of the waves: with two wave
    // streams they get a third (or, OFL_EDEN_SMALLSTREAM=0, the wave stream
    // with fewer large-slice elements)
    bool small_own = false;
    if (nbuf == 2) {
        if (use_small_stream()) {  // their own stream(s): latency-bound, they fill CUs beside both waves
            int k = 0;
            for (Launch& l : common) l.stream = use_small_split() && common.size() > 1 ? 2 + (k++ & 1) : 2;
            small_own = true;
        } else {
            int64_t load[2] = {0, 0};
            for (size_t w = 0; w < waves.size(); ++w)
                for (int32_t si : waves[w]) load[w % 2] += 1ll << pl->slices[si].logp;
            for (Launch& l : common) l.stream = load[1] < load[0] ? 1 : 0;
        }
    } else if (pl->nstreams == 2 && !waves.empty() && use_small_stream()) {
        // one wave (too few tiles to split): the small slices run beside it
        // on the side stream
        for (Launch& l : common) l.stream = 1;
        small_own = true;
    }
    // on their own stream the small-slice launches are enqueued after the
    // waves' (the critical path reaches the GPU first; each host enqueue costs
    // microseconds); on a shared stream they go first as before
    const bool small_last = !common.empty() && small_own;
    pl->enc = small_last ? std::vector<Launch>{} : common;
    pl->dec = small_last ? std::vector<Launch>{} : common;
    pl->ws_floats = nbuf * wmax;
    for (size_t w = 0; w < waves.size(); ++w) {
        int64_t off = (int64_t)(w % nbuf) * wmax;
        for (int32_t si : waves[w]) { pl->slices[si].ws_off = off; off += 1ll << pl->slices[si].logp; }
    }
    // decode row A reads 8-byte plane words when every plane row is 8-byte aligned
    int a8 = 1;
    for (int32_t si : large) a8 &= (pl->slices[si].pl_off % 8 == 0) && (pl->slices[si].pl_stride % 8 == 0);
    // one wave with a k_col_multi launch and one small-set launch: fused
    // (k_*_colm_set), everything on the caller's stream
    const int mmax = use_colm6() ? 6 : 5;
    bool fuse = false;
    if ((pl->fuse >= 0 ? pl->fuse == 1 : use_fuse_sset()) && use_colmulti() && waves.size() == 1 && common.size() == 1 && common[0].kind == K_SSET) {
        std::set<int> hs;
        for (int32_t si : waves[0]) {
            const int r = pl->slices[si].logp - ofl::kRowLog;
            if (r >= 1 && r <= mmax) hs.insert(r);
        }
        fuse = hs.size() >= 2;  // the condition for the k_col_multi launch below
    }
    pl->single = fuse;
    if (fuse) {
        pl->enc.clear();
        pl->dec.clear();
        for (Launch& l : common) l.stream = 0;
    }
    for (size_t w = 0; w < waves.size(); ++w) {
        const std::vector<int32_t>& wl = waves[w];
        const int s = (int)(w % nbuf);
        int64_t rows = 0;
        const int lo_l = add_list(wl);
        const int rp = add_prefix(wl, ofl::kRowLog, rows);
        // A 5-pass slice bigger than the wave size (its own wave): passes 1-2
        // (row bits 0..14, column level 1 bits 15..15+m1-1) touch only a
        // sub-block of 2^(15+m1) consecutive elements, and so do passes 4-5,
        // so they run sub-wave by sub-wave (half a wave of nibble-even tiles
        // and their pair partners 2^(p-18) tiles up), each sub-wave's two
        // passes back to back while its intermediate sits in the MALL; the
        // middle pass (column level 2 + D2) spans the slice and runs whole,
        // writing the slice norm (it follows every row-A sub-wave).  Launches
        // of one stream run in order, so no other synchronisation.
        if (wl.size() == 1 && cap != INT64_MAX && use_big_split() && use_rowc2() && use_btab() &&
            pl->slices[wl[0]].logp - ofl::kRowLog >= 11) {
            const int32_t si = wl[0];
            const int p = pl->slices[si].logp, r = p - ofl::kRowLog, m1 = r / 2, m2 = r - m1;
            const int64_t ntile = 1ll << r, sub = 1ll << m1, P = 1ll << (p - 18);
            const int64_t cap_t = cap >> ofl::kRowLog;
            // sub-wave size: the wave size (OFL_EDEN_BIGSUB_MIB overrides, A/B)
            const int64_t sw_t = big_sub_mib() > 0 ? (big_sub_mib() << 20) / 4 >> ofl::kRowLog : cap_t;
            const int64_t half = (sw_t / 2) / sub * sub;
            if (half >= sub && cap_t < ntile && ntile <= kRowTabMax && use_row2(2 * std::min(half, P), pl->ncu, pl->row2)) {
                const bool pair = (pl->pair >= 0 ? pl->pair : pair_mode()) != 0;
                const int lo_c = add_list(wl);
                int64_t tiles_all = 0;
                const int tp = add_prefix(wl, ofl::kColLog, tiles_all);
                struct SubWave { int tab_all, tab_pair; int64_t n_all, n_pair; };
                std::vector<SubWave> sws;
                for (int64_t reg = 0; reg < ntile; reg += 2 * P)
                    for (int64_t c = 0; c < P; c += half) {
                        const int64_t e = std::min(P, c + half);
                        SubWave sw;
                        sw.tab_all = (int)ints.size();
                        for (int64_t h = 0; h < 2; ++h)
                            for (int64_t t = reg + c + h * P; t < reg + e + h * P; ++t) {
                                ints.push_back(si);
                                ints.push_back((int32_t)(t << 3));
                            }
                        sw.n_all = 2 * (e - c);
                        sw.tab_pair = (int)ints.size();
                        for (int64_t t = reg + c; t < reg + e; ++t) {
                            ints.push_back(si);
                            ints.push_back((int32_t)(t << 3) | 1);
                        }
                        sw.n_pair = e - c;
                        sws.push_back(sw);
                    }
                auto rowl = [&](Kind k, const SubWave& sw, bool paired) {
                    Launch l{k, 0, 0, 0, lo_l, rp, 1, sw.n_all};
                    l.expl = true;
                    l.expl_tiles = sw.n_all;
                    l.btab_off = sw.tab_all;
                    if (paired) { l.ptab_off = sw.tab_pair; l.npair = (int)sw.n_pair; }
                    l.stream = s;
                    return l;
                };
                auto coll = [&](const SubWave& sw) {
                    Launch l{K_COL, m1, ofl::kRowLog, 0, lo_c, tp, 1, sw.n_all};
                    l.expl = true;
                    l.expl_tiles = sw.n_all;
                    l.btab_off = sw.tab_all;
                    l.stream = s;
                    return l;
                };
                for (int dir = 0; dir < 2; ++dir) {
                    const bool enc = dir == 1;
                    std::vector<Launch>& L = enc ? pl->enc : pl->dec;
                    for (const SubWave& sw : sws) {
                        Launch ra = rowl(K_ROWA, sw, enc && pair);
                        if (!enc) ra.mid = a8;
                        L.push_back(ra);
                        L.push_back(coll(sw));
                    }
                    Launch mid{K_COL, m2, ofl::kRowLog + m1, 1, lo_c, tp, 1, tiles_all};
                    mid.stream = s;
                    mid.nt = use_mid_nt() && m2 == 7;
                    mid.nu = enc ? 1 : 0;  // after every row-A sub-wave: the slice norm
                    L.push_back(mid);
                    for (const SubWave& sw : sws) {
                        L.push_back(coll(sw));
                        L.push_back(rowl(K_ROWC, sw, !enc && pair));
                    }
                }
                continue;
            }
        }
        std::map<int, std::vector<int32_t>> byp;  // column launches grouped by p
        for (int32_t si : wl) byp[pl->slices[si].logp].push_back(si);
        std::vector<Launch> ce, cd;
        // heights 1..5 (6) -> one k_col_multi
        std::vector<std::pair<int, const std::vector<int32_t>*>> mg;
        if (use_colmulti()) {
            for (auto& kv : byp)
                if (kv.first - ofl::kRowLog >= 1 && kv.first - ofl::kRowLog <= mmax) mg.push_back({kv.first - ofl::kRowLog, &kv.second});
            if (mg.size() < 2) mg.clear();
        }
        if (!mg.empty()) {
            const int gt = (int)ints.size();
            ints.resize(ints.size() + ofl::kColGroup * mg.size());
            int64_t blk = 0, mv = 0;
            for (size_t g = 0; g < mg.size(); ++g) {
                int64_t tiles = 0;
                const int lo_c = add_list(*mg[g].second);
                const int tp = add_prefix(*mg[g].second, ofl::kColLog, tiles);
                int32_t* G = &ints[gt + ofl::kColGroup * g];
                G[0] = mg[g].first;
                G[1] = lo_c - gt;
                G[2] = tp - gt;
                G[3] = (int32_t)mg[g].second->size();
                G[4] = (int32_t)blk;
                blk += tiles;
                for (int32_t si : *mg[g].second) mv += 8ll << pl->slices[si].logp;
            }
            Launch l{K_COLM, 0, ofl::kRowLog, 1, gt, -1, (int)mg.size(), blk};
            l.stream = s;
            l.bytes_moved = mv;
            if (fuse) {  // the small-set groups ride in this launch (its first blocks)
                l.kind = K_COLMSET;
                l.sset_off = common[0].list_off;
                l.sset_groups = common[0].count;
                l.blocks += common[0].count;
            }
            cd.push_back(l);
            l.nu = 1;  // encode: every group is a slice's first (only) column launch
            ce.push_back(l);
        }
        for (auto& kv : byp) {
            const int r = kv.first - ofl::kRowLog;
            if (!mg.empty() && r >= 1 && r <= mmax) continue;  // in the k_col_multi launch
            int64_t tiles = 0;
            const int lo_c = add_list(kv.second);
            const int tp = add_prefix(kv.second, ofl::kColLog, tiles);
            const int cnt = (int)kv.second.size();
            std::vector<Launch> seq;
            if (r <= 10) {
                if ((r == 9 || r == 10) && use_col16()) {  // 2^16-element tiles: 2x longer row segments
                    int64_t t16 = 0;
                    const int tp16 = add_prefix(kv.second, 16, t16);
                    Launch l{K_COL, r, ofl::kRowLog, 1, lo_c, tp16, cnt, t16};
                    l.tl = 16;
                    seq.push_back(l);
                } else {
                    seq.push_back({K_COL, r, ofl::kRowLog, 1, lo_c, tp, cnt, tiles});
                    if (r == 10 && use_col6() && use_perm25())  // k_col6<10, true, 15>: interleaved ws
                        for (int32_t si : kv.second) pl->slices[si].perm = 1;
                }
            } else {  // two column levels; the middle launch carries D2
                const int m1 = r / 2, m2 = r - m1;
                seq.push_back({K_COL, m1, ofl::kRowLog, 0, lo_c, tp, cnt, tiles});
                seq.push_back({K_COL, m2, ofl::kRowLog + m1, 1, lo_c, tp, cnt, tiles});
                seq.push_back({K_COL, m1, ofl::kRowLog, 0, lo_c, tp, cnt, tiles});
            }
            for (Launch& l : seq) l.stream = s;
            cd.insert(cd.end(), seq.begin(), seq.end());
            seq[0].nu = 1;  // encode: the first column launch writes the slice norms
            ce.insert(ce.end(), seq.begin(), seq.end());
        }
        Launch ra{K_ROWA, 0, 0, 0, lo_l, rp, (int)wl.size(), rows};
        Launch rc{K_ROWC, 0, 0, 0, lo_l, rp, (int)wl.size(), rows};
        ra.stream = rc.stream = s;
        pl->enc.push_back(ra);
        pl->enc.insert(pl->enc.end(), ce.begin(), ce.end());
        pl->enc.push_back(rc);
        ra.mid = a8;
        pl->dec.push_back(ra);
        pl->dec.insert(pl->dec.end(), cd.begin(), cd.end());
        pl->dec.push_back(rc);
    }
    if (small_last && !fuse) {
        pl->enc.insert(pl->enc.end(), common.begin(), common.end());
        pl->dec.insert(pl->dec.end(), common.begin(), common.end());
    }
    // scales: one k_finalize per wave stream, after that stream's last row C,
    // over the slices of its own waves.  A single finalize on the caller's
    // stream would need a mid-call join, and a cross-queue wait costs the
    // caller's queue ~10 us even when it is already satisfied (ResNet-50 trace)
    for (int s = 0; s < nbuf; ++s) {
        std::vector<int32_t> fl;
        for (size_t w = s; w < waves.size(); w += nbuf) fl.insert(fl.end(), waves[w].begin(), waves[w].end());
        if (fl.empty()) continue;
        Launch f{K_FINAL, 0, 0, 0, add_list(fl), -1, (int)fl.size(), (int64_t)fl.size()};
        f.stream = s;
        pl->enc.push_back(f);
    }
    // column launches and the two-blocks-per-CU row launches: a per-block
    // (per-tile) {slice, tile << 3 | group} table, so a block finds its tile
    // with one load (a launch of few tiles per CU is latency-bound, and the
    // prefix search is a chain of dependent loads); encode and decode share
    // the table of the same list.  The persistent row kernels search their
    // LDS copy of the prefix and take no table.
    {
        std::map<std::pair<int, int>, int> made;
        auto table = [&](Launch& l) {
            const auto key = std::make_pair(l.list_off, l.tstart_off);
            auto it = made.find(key);
            if (it != made.end()) { l.btab_off = it->second; return; }
            std::vector<int32_t> t;
            t.reserve(2 * (size_t)l.blocks);
            auto add_group = [&](int list_off, int pre_off, int count, int g) {
                for (int i = 0; i < count; ++i)
                    for (int32_t k = 0; k < ints[pre_off + i + 1] - ints[pre_off + i]; ++k) {
                        t.push_back(ints[list_off + i]);
                        t.push_back((k << 3) | g);
                    }
            };
            if (l.kind == K_COL || l.kind == K_ROWA || l.kind == K_ROWC) {
                add_group(l.list_off, l.tstart_off, l.count, 0);
            } else {  // K_COLM / K_COLMSET: l.count groups {M, list, tstart (relative), count, first block}
                for (int g = 0; g < l.count; ++g) {
                    const int32_t* G = &ints[l.list_off + ofl::kColGroup * g];
                    add_group(l.list_off + G[1], l.list_off + G[2], G[3], g);
                }
            }
            if ((int64_t)t.size() != 2 * (l.blocks - l.sset_groups)) return;  // inconsistent: keep the search
            l.btab_off = (int)ints.size();
            made[key] = l.btab_off;
            ints.insert(ints.end(), t.begin(), t.end());
        };
        for (auto* L : {&pl->enc, &pl->dec})
            for (Launch& l : *L)
                if (!l.expl && (l.kind == K_COL || l.kind == K_COLM || l.kind == K_COLMSET ||
                                ((l.kind == K_ROWA || l.kind == K_ROWC) && l.blocks <= kRowTabMax)))
                    table(l);
        // the sign-applying row launches (encode A, decode C): a paired table,
        // one entry per tile of nibble-even position (its partner follows in
        // the same block) and per tile of a slice below 2^18 (unpaired)
        std::map<std::pair<int, int>, std::pair<int, int>> pmade;
        auto ptable = [&](Launch& l) {
            const auto key = std::make_pair(l.list_off, l.tstart_off);
            auto it = pmade.find(key);
            if (it != pmade.end()) { l.ptab_off = it->second.first; l.npair = it->second.second; return; }
            std::vector<int32_t> t;
            bool any = false;
            for (int i = 0; i < l.count; ++i) {
                const int32_t si = ints[l.list_off + i];
                const int p = pl->slices[si].logp;
                const int32_t nt = ints[l.tstart_off + i + 1] - ints[l.tstart_off + i];
                for (int32_t k = 0; k < nt; ++k) {
                    if (p >= 18 && ((k >> (p - 18)) & 1)) continue;  // a partner
                    t.push_back(si);
                    t.push_back((k << 3) | (p >= 18 ? 1 : 0));
                    any = any || p >= 18;
                }
            }
            if (!any) return;
            l.ptab_off = (int)ints.size();
            l.npair = (int)(t.size() / 2);
            pmade[key] = {l.ptab_off, l.npair};
            ints.insert(ints.end(), t.begin(), t.end());
        };
        for (Launch& l : pl->enc)
            if (!l.expl && l.kind == K_ROWA && l.tstart_off >= 0 && l.blocks <= kRowTabMax) ptable(l);
        for (Launch& l : pl->dec)
            if (!l.expl && l.kind == K_ROWC && l.tstart_off >= 0 && l.blocks <= kRowTabMax) ptable(l);
    }
    // per-launch byte accounting (bench / DESIGN.md roofline)
    const int64_t n_bits = pl->nbits;
    for (int dir = 0; dir < 2; ++dir) {
        const bool enc = dir == 1;
        for (Launch& l : enc ? pl->enc : pl->dec) {
            if (l.kind == K_COLM) continue;  // counted when built (its list is a group table)
            int64_t mv = 0, al = 0;
            if (l.kind == K_SSET || l.kind == K_COLMSET) {  // group table {P, offset, count}, then the slice ids
                const int to = l.kind == K_SSET ? l.list_off : l.sset_off;
                const int ng = l.kind == K_SSET ? l.count : l.sset_groups;
                for (int g = 0; g < ng; ++g)
                    for (int i = 0; i < ints[to + 3 * g + 2]; ++i) {
                        const ofl::SliceDesc& D = pl->slices[ints[to + ints[to + 3 * g + 1] + i]];
                        const int64_t pb = n_bits * (1ll << D.logp) / 8;
                        mv += enc ? 4 * D.len + pb : pb + 4 * D.ylen;
                    }
                if (l.kind == K_SSET) l.bytes_moved = mv;
                else l.bytes_moved += mv;  // + the column part, counted when built
                l.bytes_alg = mv;
                continue;
            }
            for (int i = 0; i < l.count; ++i) {
                const ofl::SliceDesc& D = pl->slices[ints[l.list_off + i]];
                const int64_t P = 1ll << D.logp, pb = n_bits * P / 8;
                switch (l.kind) {
                case K_TINY: case K_SMALL:
                    mv += enc ? 4 * D.len + pb : pb + 4 * D.ylen; al = mv; break;
                case K_ROWA:
                    mv += enc ? 4 * D.len + 4 * P : pb + 4 * P; al += enc ? 4 * D.len : pb; break;
                case K_ROWC:
                    mv += enc ? 4 * P + pb : 4 * P + 4 * D.ylen; al += enc ? pb : 4 * D.ylen; break;
                case K_COL: mv += 8 * P; break;
                default: mv += 4 * (P >> ofl::kRowLog); break;
                }
                if (l.expl) {  // a sub-wave: its share of the slice's tiles
                    mv = mv / (P >> ofl::kRowLog) * l.expl_tiles;
                    al = al / (P >> ofl::kRowLog) * l.expl_tiles;
                }
            }
            l.bytes_moved = mv;
            l.bytes_alg = al;
        }
    }
}

int64_t env_i64(const char* name, int64_t dflt) {
    const char* s = getenv(name);
    return (s && *s) ? strtoll(s, nullptr, 10) : dflt;
}

}  // namespace

extern "C" {

const char* ofl_version(void) { return "openfl_amd-codec 0.1 (gfx950)"; }
const char* ofl_last_error(void) { return g_err.c_str(); }

int ofl_eden_slice_plan(int64_t n, int64_t* P_out, int64_t* len_out, int max_slices) {
    if (n <= 0) return 0;
    int64_t rem = n;
    int ns = 0;
    while ((double)(high_po2(rem) - rem) / (double)n > 0.1) {
        const int64_t low = low_po2(rem);
        if (ns < max_slices) {
            if (P_out) P_out[ns] = std::max<int64_t>(low, 8);
            if (len_out) len_out[ns] = low;
        }
        ++ns;
        rem -= low;
    }
    if (ns < max_slices) {
        if (P_out) P_out[ns] = std::max<int64_t>(high_po2(rem), 8);
        if (len_out) len_out[ns] = rem;
    }
    return ns + 1;
}

int ofl_eden_plan_create(int ntensors, const int64_t* numel, const int64_t* elem_offset,
                         const int32_t* nslices, const int64_t* slice_dims, int n_bits,
                         ofl_eden_plan_t* plan_out) {
    if (!plan_out || ntensors < 0 || !numel || !elem_offset) return fail(OFL_EINVAL, "null argument");
    if (n_bits < 1 || n_bits > 8) return fail(OFL_EINVAL, "nbits value is not supported");
    auto* pl = new ofl_eden_plan();
    pl->nbits = n_bits;
    pl->ntensors = ntensors;
    for (int t = 0; t < ntensors; ++t) pl->arena = std::max(pl->arena, elem_offset[t] + numel[t]);
    int64_t dims_pos = 0;
    // per-class slice lists
    std::vector<int32_t>& tiny = pl->tiny;
    std::vector<int32_t>* small = pl->small;
    std::vector<int32_t>& large = pl->large;
    for (int t = 0; t < ntensors; ++t) {
        const int64_t n = numel[t];
        std::vector<int64_t> Ps, Ls;  // padded sizes, valid input lengths
        if (slice_dims) {
            int64_t rem = n;
            for (int k = 0; k < nslices[t]; ++k) {
                const int64_t P = slice_dims[dims_pos + k];
                Ps.push_back(P);
                Ls.push_back(std::max<int64_t>(0, std::min<int64_t>(P, rem)));
                rem -= Ls.back();
            }
            dims_pos += nslices[t];
        } else {
            int ns = ofl_eden_slice_plan(n, nullptr, nullptr, 0);
            Ps.resize(ns);
            Ls.resize(ns);
            ofl_eden_slice_plan(n, Ps.data(), Ls.data(), ns);
        }
        int64_t Ptot = 0;
        for (int64_t P : Ps) {
            if (P < 8 || (P & (P - 1)) || P > (1ll << 29)) {
                delete pl;
                return fail(OFL_EINVAL, "slice size must be a power of two in [8, 2^29]");
            }
            Ptot += P;
        }
        pl->t_first.push_back((int32_t)pl->slices.size());
        pl->t_nslices.push_back((int32_t)Ps.size());
        const int64_t poff = (pl->planes_bytes + 255) & ~255ll;
        pl->t_planes_off.push_back(poff);
        pl->t_planes_bytes.push_back(Ptot / 8 * n_bits);
        pl->planes_bytes = poff + Ptot / 8 * n_bits;
        // Encode reads slice k from input offset sum(len_k') (Eden.compress
        // advances by the valid length, :599-602); decode writes slice k's P
        // outputs at sum(P_k') and truncates to total_dim (:650-657).  The two
        // differ only for n < ~150 with a sub-8 non-final slice (reproduced).
        int64_t off = 0, xoff = 0;
        for (size_t k = 0; k < Ps.size(); ++k) {
            const int64_t P = Ps[k];
            ofl::SliceDesc D{};
            D.x_off = elem_offset[t] + xoff;
            D.len = Ls[k];
            D.y_off = elem_offset[t] + off;
            D.ylen = std::max<int64_t>(0, std::min<int64_t>(P, n - off));
            D.pl_off = poff + off / 8;
            D.pl_stride = Ptot / 8;
            D.logp = ilog2(P);
            D.tensor = t;
            D.scale_idx = (int32_t)pl->slices.size();
            const int si = (int)pl->slices.size();
            if (D.logp <= 10) tiny.push_back(si);
            else if (D.logp <= ofl::kRowLog) small[D.logp - 11].push_back(si);
            else {
                D.part_off = (int32_t)pl->part_floats;  // ws_off: build_schedule
                pl->part_floats += P >> ofl::kRowLog;
                large.push_back(si);
            }
            pl->slices.push_back(D);
            off += P;
            xoff += D.len;
        }
    }
    pl->nlarge = (int64_t)large.size();
    // default schedule (tuning overrides: OFL_EDEN_WAVE_MIB, OFL_EDEN_STREAMS)
    pl->wave_bytes = std::max<int64_t>(0, env_i64("OFL_EDEN_WAVE_MIB", kDefaultWaveMiB)) << 20;
    pl->nstreams = (int)std::min<int64_t>(2, std::max<int64_t>(1, env_i64("OFL_EDEN_STREAMS", kDefaultStreams)));
    build_schedule(pl);
    *plan_out = pl;
    return OFL_OK;
}

// Descriptor tables go to the device on first use (one synchronous copy), so
// plans can be built and inspected on hosts without a GPU.  The first
// encode/decode of a plan must therefore not be inside a graph capture.
// The side streams are shared by every plan of a device (created once):
// each plan owning its own would soon exceed the HW queues (GPU_MAX_HW_QUEUES,
// 4 by default), and streams that share a queue serialise -- the small-slice
// stream then waits behind a wave stream.  Runs of different plans on the
// shared streams stay correct (fork/join events per plan); they may wait for
// each other's work enqueued in between.
// The same streams serve the pipelined inflate's pieces (1, 2)
// (ofl_side_stream): HIP hands streams the HW queues in turn, so the three
// are created together, and every stream the library made instead of sharing
// them pushed a later one onto a queue already in use
// (profiles/r05_kc_hw_queues_ab.txt).
static int side_pool(int dev, hipStream_t (&out)[3]) {
    static std::mutex mu;
    static std::map<int, std::array<hipStream_t, 3>> pool;
    std::lock_guard<std::mutex> g(mu);
    auto& e = pool[dev];
    for (int i = 0; i < 3; ++i)
        if (!e[i]) HIP_TRY(hipStreamCreateWithFlags(&e[i], hipStreamNonBlocking));
    for (int i = 0; i < 3; ++i) out[i] = e[i];
    return OFL_OK;
}
static int shared_side_streams(int dev, bool two, bool three, hipStream_t& s1, hipStream_t& s2, hipStream_t& s3) {
    hipStream_t e[3];
    if (int rc = side_pool(dev, e)) return rc;
    s1 = e[0];
    s2 = two ? e[1] : nullptr;
    s3 = three ? e[2] : nullptr;
    return OFL_OK;
}

static int ensure_device(ofl_eden_plan_t pl) {
    std::lock_guard<std::mutex> g(pl->mu);
    if (pl->uploaded) return OFL_OK;
    HIP_TRY(hipGetDevice(&pl->device));
    HIP_TRY(hipDeviceGetAttribute(&pl->ncu, hipDeviceAttributeMultiprocessorCount, pl->device));
    if (pl->ncu < 1) pl->ncu = 1;
    if (!pl->slices.empty()) {
        HIP_TRY(hipMalloc(&pl->d_slices, sizeof(ofl::SliceDesc) * pl->slices.size()));
        HIP_TRY(hipMemcpy(pl->d_slices, pl->slices.data(), sizeof(ofl::SliceDesc) * pl->slices.size(), hipMemcpyHostToDevice));
    }
    if (!pl->ints.empty()) {
        HIP_TRY(hipMalloc(&pl->d_ints, sizeof(int32_t) * pl->ints.size()));
        HIP_TRY(hipMemcpy(pl->d_ints, pl->ints.data(), sizeof(int32_t) * pl->ints.size(), hipMemcpyHostToDevice));
    }
    bool side = false;
    for (const Launch& l : pl->enc) side |= l.stream != 0;
    for (const Launch& l : pl->dec) side |= l.stream != 0;
    bool side3 = false, side4 = false;
    for (const Launch& l : pl->enc) { side3 |= l.stream >= 2; side4 |= l.stream == 3; }
    for (const Launch& l : pl->dec) { side3 |= l.stream >= 2; side4 |= l.stream == 3; }
    if (side) {
        if (int rc = shared_side_streams(pl->device, side3, side4, pl->side, pl->side2, pl->side3)) return rc;
        HIP_TRY(hipEventCreateWithFlags(&pl->ev_fork, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&pl->ev_join, hipEventDisableTiming));
        if (side3) HIP_TRY(hipEventCreateWithFlags(&pl->ev_join2, hipEventDisableTiming));
        if (side4) HIP_TRY(hipEventCreateWithFlags(&pl->ev_join3, hipEventDisableTiming));
    }
    pl->uploaded = true;
    return OFL_OK;
}

int ofl_side_stream(int index, void** stream) {
    if (index < 0 || index > 2 || !stream) return fail(OFL_EINVAL, "side stream: index 0..2, non-null out");
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    hipStream_t e[3];
    if (int rc = side_pool(dev, e)) return rc;
    *stream = e[index];
    return OFL_OK;
}

void ofl_eden_plan_destroy(ofl_eden_plan_t pl) {
    if (!pl) return;
    ofl_eden_plan_profile(pl, 0);
    for (hipEvent_t e : pl->ev_pool) (void)hipEventDestroy(e);
    if (pl->d_slices) (void)hipFree(pl->d_slices);
    if (pl->d_ints) (void)hipFree(pl->d_ints);
    if (pl->ev_join2) (void)hipEventDestroy(pl->ev_join2);
    if (pl->ev_join3) (void)hipEventDestroy(pl->ev_join3);
    if (pl->ev_fork) (void)hipEventDestroy(pl->ev_fork);
    if (pl->ev_join) (void)hipEventDestroy(pl->ev_join);
    delete pl;
}

int ofl_eden_plan_set_schedule(ofl_eden_plan_t pl, int64_t wave_bytes, int streams) {
    if (!pl) return fail(OFL_EINVAL, "null plan");
    if (streams < 0 || streams > 2) return fail(OFL_EINVAL, "schedule: streams must be 1 or 2 (0 keeps)");
    std::lock_guard<std::mutex> g(pl->mu);
    if (pl->uploaded) return fail(OFL_EINVAL, "schedule must be set before the plan's first encode/decode");
    if (wave_bytes >= 0) pl->wave_bytes = wave_bytes;
    if (streams > 0) pl->nstreams = streams;
    build_schedule(pl);
    return OFL_OK;
}

int ofl_eden_plan_set_row2(ofl_eden_plan_t pl, int mode) {
    if (!pl) return fail(OFL_EINVAL, "null plan");
    if (mode < -1 || mode > 1) return fail(OFL_EINVAL, "row2 mode must be -1 (auto), 0 or 1");
    std::lock_guard<std::mutex> g(pl->mu);
    pl->row2 = mode;
    return OFL_OK;
}

int ofl_eden_plan_set_pair(ofl_eden_plan_t pl, int mode) {
    if (!pl) return fail(OFL_EINVAL, "null plan");
    if (mode < -1 || mode > 1) return fail(OFL_EINVAL, "pair mode must be -1 (auto), 0 or 1");
    std::lock_guard<std::mutex> g(pl->mu);
    pl->pair = mode;
    return OFL_OK;
}

int ofl_eden_plan_set_sset(ofl_eden_plan_t pl, int mode) {
    if (!pl) return fail(OFL_EINVAL, "null plan");
    if (mode < -1 || mode > 1) return fail(OFL_EINVAL, "sset mode must be -1 (default), 0 or 1");
    std::lock_guard<std::mutex> g(pl->mu);
    if (pl->uploaded) return fail(OFL_EINVAL, "sset must be set before the plan's first encode/decode");
    pl->sset = mode;
    build_schedule(pl);
    return OFL_OK;
}

int ofl_eden_plan_set_fuse(ofl_eden_plan_t pl, int mode) {
    if (!pl) return fail(OFL_EINVAL, "null plan");
    if (mode < -1 || mode > 1) return fail(OFL_EINVAL, "fuse mode must be -1 (default), 0 or 1");
    std::lock_guard<std::mutex> g(pl->mu);
    if (pl->uploaded) return fail(OFL_EINVAL, "fuse must be set before the plan's first encode/decode");
    pl->fuse = mode;
    build_schedule(pl);
    return OFL_OK;
}

int ofl_eden_plan_get_schedule(ofl_eden_plan_t pl, int64_t* wave_bytes, int* streams) {
    if (!pl) return fail(OFL_EINVAL, "null plan");
    if (wave_bytes) *wave_bytes = pl->wave_bytes;
    if (streams) *streams = pl->nstreams;
    return OFL_OK;
}

int ofl_eden_plan_num_waves(ofl_eden_plan_t pl) { return pl ? pl->nwaves : -1; }

int64_t ofl_eden_plan_num_slices(ofl_eden_plan_t pl) { return pl ? (int64_t)pl->slices.size() : -1; }
int64_t ofl_eden_plan_planes_bytes(ofl_eden_plan_t pl) { return pl ? pl->planes_bytes : -1; }
int64_t ofl_eden_plan_workspace_bytes(ofl_eden_plan_t pl) {
    if (!pl) return -1;
    // intermediates | partials | norms, each 256-B aligned
    auto al = [](int64_t b) { return (b + 255) & ~255ll; };
    // per-slice norms are indexed by slice id (all slices, not only large ones)
    const int64_t nnu = (int64_t)pl->slices.size();
    return al(pl->ws_floats * 4) + al(pl->part_floats * 4) + al(nnu * 4) + 256;
}

int ofl_eden_plan_tensor_info(ofl_eden_plan_t pl, int t, int64_t* planes_offset, int64_t* planes_bytes,
                              int32_t* first_slice, int32_t* nslices) {
    if (!pl || t < 0 || t >= pl->ntensors) return fail(OFL_EINVAL, "tensor index out of range");
    if (planes_offset) *planes_offset = pl->t_planes_off[t];
    if (planes_bytes) *planes_bytes = pl->t_planes_bytes[t];
    if (first_slice) *first_slice = pl->t_first[t];
    if (nslices) *nslices = pl->t_nslices[t];
    return OFL_OK;
}

int ofl_eden_plan_tensor_dims(ofl_eden_plan_t pl, int t, int64_t* dims_out) {
    if (!pl || t < 0 || t >= pl->ntensors) return fail(OFL_EINVAL, "tensor index out of range");
    for (int k = 0; k < pl->t_nslices[t]; ++k) dims_out[k] = 1ll << pl->slices[pl->t_first[t] + k].logp;
    return OFL_OK;
}

static int prep_args(ofl_eden_plan_t pl, ofl::KArgs& a, void* ws, size_t ws_bytes) {
    if (int rc = ensure_device(pl)) return rc;
    const int64_t need = ofl_eden_plan_workspace_bytes(pl);
    if ((int64_t)ws_bytes < need || (need > 256 && !ws)) return fail(OFL_ESPACE, "workspace too small");
    auto al = [](int64_t b) { return (b + 255) & ~255ll; };
    char* w = static_cast<char*>(ws);
    memset(&a, 0, sizeof(a));
    a.d = pl->d_slices;
    a.nbits = pl->nbits;
    a.ws = reinterpret_cast<float*>(w);
    a.part = reinterpret_cast<float*>(w + al(pl->ws_floats * 4));
    a.nu = reinterpret_cast<float*>(w + al(pl->ws_floats * 4) + al(pl->part_floats * 4));
    return OFL_OK;
}

int ofl_eden_encode(ofl_eden_plan_t pl, const float* x_arena, const uint32_t* seeds, uint8_t* planes_arena,
                    float* scales, void* ws, size_t ws_bytes, void* stream) {
    if (!pl) return fail(OFL_EINVAL, "null plan");
    ofl::KArgs a;
    int rc = prep_args(pl, a, ws, ws_bytes);
    if (rc) return rc;
    a.xin = x_arena;
    a.pout = planes_arena;
    a.seeds = seeds;
    a.scales = scales;
    return run(pl, true, a, static_cast<hipStream_t>(stream));
}

int ofl_eden_encode_wavg(ofl_eden_plan_t pl, const float* const* collab_arenas, const double* weights, int ncollab,
                         double wsum, const float* base_arena, const float* delta_arena, const uint32_t* seeds,
                         uint8_t* planes_arena, float* scales, void* ws, size_t ws_bytes, void* stream) {
    if (!pl) return fail(OFL_EINVAL, "null plan");
    if (!collab_arenas || !weights || ncollab < 1 || ncollab > 16 || !(wsum != 0.0))
        return fail(OFL_EINVAL, "encode_wavg: 1..16 collaborators, their weights and a nonzero weight sum");
    ofl::KArgs a;
    int rc = prep_args(pl, a, ws, ws_bytes);
    if (rc) return rc;
    a.xin = delta_arena;
    a.pout = planes_arena;
    a.seeds = seeds;
    a.scales = scales;
    a.wx = collab_arenas;
    a.ww = weights;
    a.wc = ncollab;
    a.wsum = wsum;
    a.wbase = base_arena;
    return run(pl, true, a, static_cast<hipStream_t>(stream));
}

int ofl_eden_decode(ofl_eden_plan_t pl, const uint8_t* planes_arena, const uint32_t* seeds, const float* scales,
                    float* y_arena, void* ws, size_t ws_bytes, void* stream) {
    return ofl_eden_decode_add(pl, planes_arena, seeds, scales, nullptr, y_arena, ws, ws_bytes, stream);
}

int ofl_eden_decode_add(ofl_eden_plan_t pl, const uint8_t* planes_arena, const uint32_t* seeds, const float* scales,
                        const float* base_arena, float* y_arena, void* ws, size_t ws_bytes, void* stream) {
    if (!pl) return fail(OFL_EINVAL, "null plan");
    ofl::KArgs a;
    int rc = prep_args(pl, a, ws, ws_bytes);
    if (rc) return rc;
    a.pin = planes_arena;
    a.xout = y_arena;
    a.yadd = base_arena;
    a.seeds = seeds;
    a.scales_in = scales;
    return run(pl, false, a, static_cast<hipStream_t>(stream));
}

int ofl_eden_encode_host(ofl_eden_plan_t pl, const void* in_host, void* in_dev, size_t in_bytes, size_t off_seeds,
                         void* out_dev, void* out_host, size_t out_bytes, size_t off_scales, void* ws, size_t ws_bytes,
                         void* stream) {
    if (!pl || !in_host || !in_dev || !out_dev || !out_host) return fail(OFL_EINVAL, "encode_host: null argument");
    if (off_seeds + 4 * (size_t)pl->ntensors > in_bytes || off_seeds < 4 * (size_t)pl->arena ||
        off_scales < (size_t)pl->planes_bytes || off_scales + 4 * pl->slices.size() > out_bytes)
        return fail(OFL_EINVAL, "encode_host: block layout does not fit the plan");
    hipStream_t st = static_cast<hipStream_t>(stream);
    HIP_TRY(hipMemcpyAsync(in_dev, in_host, in_bytes, hipMemcpyHostToDevice, st));
    char* o = static_cast<char*>(out_dev);
    const char* i = static_cast<const char*>(in_dev);
    if (int rc = ofl_eden_encode(pl, reinterpret_cast<const float*>(i), reinterpret_cast<const uint32_t*>(i + off_seeds),
                                 reinterpret_cast<uint8_t*>(o), reinterpret_cast<float*>(o + off_scales), ws, ws_bytes,
                                 stream))
        return rc;
    HIP_TRY(hipMemcpyAsync(out_host, out_dev, out_bytes, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return OFL_OK;
}

int ofl_eden_decode_host(ofl_eden_plan_t pl, const void* in_host, void* in_dev, size_t in_bytes, size_t off_scales,
                         size_t off_seeds, void* out_dev, void* out_host, size_t out_bytes, void* ws, size_t ws_bytes,
                         void* stream) {
    if (!pl || !in_host || !in_dev || !out_dev || !out_host) return fail(OFL_EINVAL, "decode_host: null argument");
    if (off_scales < (size_t)pl->planes_bytes || off_seeds < off_scales + 4 * pl->slices.size() ||
        off_seeds + 4 * (size_t)pl->ntensors > in_bytes || out_bytes > 4 * (size_t)pl->arena)
        return fail(OFL_EINVAL, "decode_host: block layout does not fit the plan");
    hipStream_t st = static_cast<hipStream_t>(stream);
    HIP_TRY(hipMemcpyAsync(in_dev, in_host, in_bytes, hipMemcpyHostToDevice, st));
    const char* i = static_cast<const char*>(in_dev);
    if (int rc = ofl_eden_decode(pl, reinterpret_cast<const uint8_t*>(i), reinterpret_cast<const uint32_t*>(i + off_seeds),
                                 reinterpret_cast<const float*>(i + off_scales), static_cast<float*>(out_dev), ws, ws_bytes,
                                 stream))
        return rc;
    if (out_bytes) HIP_TRY(hipMemcpyAsync(out_host, out_dev, out_bytes, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return OFL_OK;
}

// Zero-copy one-tensor calls: the kernels read and write mapped pinned host
// memory directly (no DMA copies): for plans of tiny / small slices only,
// whose single launch moves a few KiB across the link.
static int mapped_ptr(void* h, void** d) {
    if (hipHostGetDevicePointer(d, h, 0) != hipSuccess || !*d) {
        (void)hipGetLastError();
        return fail(OFL_EINVAL, "mapped call: buffer is not mapped pinned host memory (hipHostMalloc / pin_memory)");
    }
    return OFL_OK;
}

int ofl_eden_encode_mapped(ofl_eden_plan_t pl, const void* in_host, size_t off_seeds, void* out_host,
                           size_t off_scales, void* ws, size_t ws_bytes, void* stream) {
    if (!pl || !in_host || !out_host) return fail(OFL_EINVAL, "encode_mapped: null argument");
    if (!pl->large.empty()) return fail(OFL_EINVAL, "encode_mapped: plans of tiny / small slices (<= 2^15) only");
    if (off_seeds < 4 * (size_t)pl->arena || off_scales < (size_t)pl->planes_bytes)
        return fail(OFL_EINVAL, "encode_mapped: block layout does not fit the plan");
    void *i = nullptr, *o = nullptr;
    if (int rc = mapped_ptr(const_cast<void*>(in_host), &i)) return rc;
    if (int rc = mapped_ptr(out_host, &o)) return rc;
    hipStream_t st = static_cast<hipStream_t>(stream);
    char* oc = static_cast<char*>(o);
    const char* ic = static_cast<const char*>(i);
    if (int rc = ofl_eden_encode(pl, reinterpret_cast<const float*>(ic), reinterpret_cast<const uint32_t*>(ic + off_seeds),
                                 reinterpret_cast<uint8_t*>(oc), reinterpret_cast<float*>(oc + off_scales), ws, ws_bytes,
                                 stream))
        return rc;
    HIP_TRY(hipStreamSynchronize(st));
    return OFL_OK;
}

int ofl_eden_decode_mapped(ofl_eden_plan_t pl, const void* in_host, size_t off_scales, size_t off_seeds, void* y_host,
                           void* ws, size_t ws_bytes, void* stream) {
    if (!pl || !in_host || !y_host) return fail(OFL_EINVAL, "decode_mapped: null argument");
    if (!pl->large.empty()) return fail(OFL_EINVAL, "decode_mapped: plans of tiny / small slices (<= 2^15) only");
    if (off_scales < (size_t)pl->planes_bytes || off_seeds < off_scales + 4 * pl->slices.size())
        return fail(OFL_EINVAL, "decode_mapped: block layout does not fit the plan");
    void *i = nullptr, *y = nullptr;
    if (int rc = mapped_ptr(const_cast<void*>(in_host), &i)) return rc;
    if (int rc = mapped_ptr(y_host, &y)) return rc;
    hipStream_t st = static_cast<hipStream_t>(stream);
    const char* ic = static_cast<const char*>(i);
    if (int rc = ofl_eden_decode(pl, reinterpret_cast<const uint8_t*>(ic), reinterpret_cast<const uint32_t*>(ic + off_seeds),
                                 reinterpret_cast<const float*>(ic + off_scales), static_cast<float*>(y), ws, ws_bytes,
                                 stream))
        return rc;
    HIP_TRY(hipStreamSynchronize(st));
    return OFL_OK;
}

int ofl_eden_encode_seeded(ofl_eden_plan_t pl, void* in_dev, size_t off_seeds, uint32_t seed, void* out_dev,
                           void* out_host, size_t out_bytes, size_t off_scales, void* ws, size_t ws_bytes, void* stream) {
    if (!pl || !in_dev || !out_dev || !out_host) return fail(OFL_EINVAL, "encode_seeded: null argument");
    if (pl->ntensors != 1 || off_seeds < 4 * (size_t)pl->arena || off_scales < (size_t)pl->planes_bytes ||
        off_scales + 4 * pl->slices.size() > out_bytes)
        return fail(OFL_EINVAL, "encode_seeded: one-tensor plans; block layout does not fit the plan");
    hipStream_t st = static_cast<hipStream_t>(stream);
    char* i = static_cast<char*>(in_dev);
    HIP_TRY(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(i + off_seeds), (int)seed, 1, st));
    char* o = static_cast<char*>(out_dev);
    if (int rc = ofl_eden_encode(pl, reinterpret_cast<const float*>(i), reinterpret_cast<const uint32_t*>(i + off_seeds),
                                 reinterpret_cast<uint8_t*>(o), reinterpret_cast<float*>(o + off_scales), ws, ws_bytes,
                                 stream))
        return rc;
    HIP_TRY(hipMemcpyAsync(out_host, out_dev, out_bytes, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return OFL_OK;
}

int ofl_eden_encode_host_x(ofl_eden_plan_t pl, const void* x_host, size_t x_bytes, uint32_t seed, void* in_dev,
                           size_t off_seeds, void* out_dev, void* out_host, size_t out_bytes, size_t off_scales,
                           void* ws, size_t ws_bytes, void* stream) {
    if (!pl || !in_dev || !out_dev || !out_host) return fail(OFL_EINVAL, "encode_host_x: null argument");
    if (pl->ntensors != 1 || off_seeds < 4 * (size_t)pl->arena || (x_host && x_bytes > off_seeds) ||
        off_scales < (size_t)pl->planes_bytes || off_scales + 4 * pl->slices.size() > out_bytes)
        return fail(OFL_EINVAL, "encode_host_x: block layout does not fit the plan");
    hipStream_t st = static_cast<hipStream_t>(stream);
    char* i = static_cast<char*>(in_dev);
    if (x_host && x_bytes) HIP_TRY(hipMemcpyAsync(i, x_host, x_bytes, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(i + off_seeds), (int)seed, 1, st));
    char* o = static_cast<char*>(out_dev);
    if (int rc = ofl_eden_encode(pl, reinterpret_cast<const float*>(i), reinterpret_cast<const uint32_t*>(i + off_seeds),
                                 reinterpret_cast<uint8_t*>(o), reinterpret_cast<float*>(o + off_scales), ws, ws_bytes,
                                 stream))
        return rc;
    HIP_TRY(hipMemcpyAsync(out_host, out_dev, out_bytes, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return OFL_OK;
}

int ofl_eden_decode_host_x(ofl_eden_plan_t pl, const void* planes_host, size_t planes_bytes, const float* scales_host,
                           int nscales, uint32_t seed, void* in_dev, size_t off_scales, size_t off_seeds,
                           void* out_dev, void* y_host, size_t y_bytes, void* ws, size_t ws_bytes, void* stream) {
    if (!pl || !planes_host || !scales_host || !in_dev || !out_dev || !y_host)
        return fail(OFL_EINVAL, "decode_host_x: null argument");
    if (pl->ntensors != 1 || planes_bytes != (size_t)pl->planes_bytes || nscales != (int)pl->slices.size() ||
        off_scales < planes_bytes || off_seeds < off_scales + 4 * (size_t)nscales || y_bytes > 4 * (size_t)pl->arena)
        return fail(OFL_EINVAL, "decode_host_x: block layout does not fit the plan");
    hipStream_t st = static_cast<hipStream_t>(stream);
    char* i = static_cast<char*>(in_dev);
    HIP_TRY(hipMemcpyAsync(i, planes_host, planes_bytes, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(i + off_scales, scales_host, 4 * (size_t)nscales, hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(i + off_seeds), (int)seed, 1, st));
    if (int rc = ofl_eden_decode(pl, reinterpret_cast<const uint8_t*>(i), reinterpret_cast<const uint32_t*>(i + off_seeds),
                                 reinterpret_cast<const float*>(i + off_scales), static_cast<float*>(out_dev), ws, ws_bytes,
                                 stream))
        return rc;
    if (y_bytes) HIP_TRY(hipMemcpyAsync(y_host, out_dev, y_bytes, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return OFL_OK;
}

int ofl_copy_h2d_async(void* dst_dev, const void* src_host, size_t bytes, void* stream) {
    if (!bytes) return OFL_OK;
    if (!dst_dev || !src_host) return fail(OFL_EINVAL, "copy_h2d_async: null argument");
    HIP_TRY(hipMemcpyAsync(dst_dev, src_host, bytes, hipMemcpyHostToDevice, static_cast<hipStream_t>(stream)));
    return OFL_OK;
}

namespace {
// Pinned staging rings of ofl_copy_h2d_staged: a ring is kStageSlots slots
// per thread, each with the event of the DMA that last read it.  Rings belong
// to one device (their events do) and are lent to one call at a time from
// that device's pool: concurrent calls -- on different GPUs, or several on one
// -- take different rings and never hold a common lock while they copy; up to
// kStageRings rings per device are made (a caller beyond that waits for one to
// come back).  Allocated on first use and kept (hipHostMalloc is slow; 64 MiB
// per ring at most).
constexpr size_t kStageChunk = 4u << 20;
constexpr int kStageSlots = 2, kStageMaxThreads = 8, kStageRings = 4;
struct StageRing {
    char* slot[kStageMaxThreads][kStageSlots] = {};
    hipEvent_t ev[kStageMaxThreads][kStageSlots] = {};
    bool used[kStageMaxThreads][kStageSlots] = {};
};
struct StagePool {
    std::mutex mu;
    std::condition_variable cv;
    std::map<int, std::vector<StageRing*>> idle;
    std::map<int, int> made;
    static StagePool& get() {  // a member: the enclosing extern "C" block gives free functions C linkage
        static StagePool* p = new StagePool;  // never destroyed (pinned memory outlives static teardown order)
        return *p;
    }
    StageRing* take(int dev) {
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [&] { return !idle[dev].empty() || made[dev] < kStageRings; });
        if (!idle[dev].empty()) {
            StageRing* r = idle[dev].back();
            idle[dev].pop_back();
            return r;
        }
        ++made[dev];
        return new StageRing;
    }
    void give(int dev, StageRing* r) {
        {
            std::lock_guard<std::mutex> g(mu);
            idle[dev].push_back(r);
        }
        cv.notify_one();
    }
};
}  // namespace

int ofl_copy_h2d_staged(void* dst_dev, const void* src_host, size_t bytes, int nthreads, void* stream) {
    if (!bytes) return OFL_OK;
    if (!dst_dev || !src_host) return fail(OFL_EINVAL, "copy_h2d_staged: null argument");
    if (bytes < 2 * kStageChunk) return ofl_copy_h2d_async(dst_dev, src_host, bytes, stream);
    hipStream_t st = static_cast<hipStream_t>(stream);
    const size_t nchunk = (bytes + kStageChunk - 1) / kStageChunk;
    const int nt = (int)std::min<size_t>(nchunk, (size_t)std::max(1, std::min(nthreads, kStageMaxThreads)));
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    StagePool& P = StagePool::get();
    StageRing& R = *P.take(dev);
    ofl_util::ScopeExit back([&] { P.give(dev, &R); });
    for (int t = 0; t < nt; ++t)
        for (int s = 0; s < kStageSlots; ++s) {
            if (!R.slot[t][s]) HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&R.slot[t][s]), kStageChunk, hipHostMallocDefault));
            if (!R.ev[t][s]) HIP_TRY(hipEventCreateWithFlags(&R.ev[t][s], hipEventDisableTiming));
        }
    // thread t stages chunks t, t + nt, ... through its own slots: the host
    // copies of several threads and the DMAs of earlier chunks run together
    std::atomic<int> err{0};
    auto work = [&](int t) {
        int k = 0;
        for (size_t c = (size_t)t; c < nchunk && !err.load(std::memory_order_relaxed); c += (size_t)nt, ++k) {
            const int s = k % kStageSlots;
            const size_t o = c * kStageChunk, n = std::min(kStageChunk, bytes - o);
            hipError_t e = hipSuccess;
            if (R.used[t][s]) e = hipEventSynchronize(R.ev[t][s]);
            if (e == hipSuccess) {
                memcpy(R.slot[t][s], static_cast<const char*>(src_host) + o, n);
                e = hipMemcpyAsync(static_cast<char*>(dst_dev) + o, R.slot[t][s], n, hipMemcpyHostToDevice, st);
            }
            if (e == hipSuccess) e = hipEventRecord(R.ev[t][s], st);
            if (e != hipSuccess) {
                err.store((int)e);
                return;
            }
            R.used[t][s] = true;
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t)
        th.emplace_back([&, t] {
            (void)hipSetDevice(dev);
            work(t);
        });
    work(0);
    for (auto& x : th) x.join();
    if (err.load()) HIP_TRY(static_cast<hipError_t>(err.load()));
    return OFL_OK;
}

int ofl_eden_plan_profile(ofl_eden_plan_t pl, int enable) {
    if (!pl) return fail(OFL_EINVAL, "null plan");
    std::lock_guard<std::mutex> g(pl->mu);
    for (int d = 0; d < 2; ++d) {
        for (auto& call : pl->prof_ev[d]) pl->ev_pool.insert(pl->ev_pool.end(), call.begin(), call.end());
        pl->prof_ev[d].clear();
    }
    pl->prof = enable != 0;
    return OFL_OK;
}

int ofl_eden_plan_num_launches(ofl_eden_plan_t pl, int encode) {
    if (!pl) return fail(OFL_EINVAL, "null plan");
    return (int)(encode ? pl->enc.size() : pl->dec.size());
}

int ofl_eden_plan_launch_info(ofl_eden_plan_t pl, int encode, int idx, char* name, int cap, int64_t* blocks,
                              int64_t* bytes_moved, int64_t* bytes_alg) {
    if (!pl) return fail(OFL_EINVAL, "null plan");
    const std::vector<Launch>& L = encode ? pl->enc : pl->dec;
    if (idx < 0 || idx >= (int)L.size()) return fail(OFL_EINVAL, "launch index out of range");
    if (name && cap > 0) {
        const std::string s = launch_name(L[idx], encode != 0, pl->ncu, pl->row2);
        snprintf(name, (size_t)cap, "%s", s.c_str());
    }
    if (blocks) *blocks = L[idx].blocks;
    if (bytes_moved) *bytes_moved = L[idx].bytes_moved;
    if (bytes_alg) *bytes_alg = L[idx].bytes_alg;
    return OFL_OK;
}

int ofl_eden_plan_profile_collect(ofl_eden_plan_t pl, int encode, double* ms_sum, int max, int* ncalls) {
    if (!pl) return fail(OFL_EINVAL, "null plan");
    std::lock_guard<std::mutex> g(pl->mu);
    auto& calls = pl->prof_ev[encode ? 1 : 0];
    const int nl = (int)(encode ? pl->enc.size() : pl->dec.size());
    for (int i = 0; i < std::min(nl, max); ++i) ms_sum[i] = 0.0;
    for (auto& call : calls) {
        for (int i = 0; i < nl && i < max; ++i) {
            float ms = 0.f;
            HIP_TRY(hipEventSynchronize(call[2 * i + 1]));
            HIP_TRY(hipEventElapsedTime(&ms, call[2 * i], call[2 * i + 1]));
            ms_sum[i] += ms;
        }
        pl->ev_pool.insert(pl->ev_pool.end(), call.begin(), call.end());
    }
    if (ncalls) *ncalls = (int)calls.size();
    calls.clear();
    return OFL_OK;
}

// strict IEEE order: the library is built without fast-math/reassociation,
// so the compiler keeps the dependent add chain (no vectorised partial sums).
// Arrays of 2^20 elements and more go to the exact multi-threaded evaluation
// of the same chain (csrc/serial_sum.cpp: binade-wise integer prefix sums).
static float serial_sum_f32_loop(const float* x, int64_t n) {
    float s = 0.0f;
    for (int64_t i = 0; i < n; ++i) s = s + x[i];
    return s;
}
constexpr int64_t kSumMtMin = 1 << 20;

float ofl_serial_sum_f32(const float* x, int64_t n) {
    if (n >= kSumMtMin) return ofl::serial_sum_f32_mt_cb(x, n, nullptr, 0, nullptr, nullptr);
    return serial_sum_f32_loop(x, n);
}

float ofl_serial_sum_copy_f32(const float* x, float* dst, int64_t n) {
    if (n >= kSumMtMin) return ofl::serial_sum_f32_mt_cb(x, n, dst, 0, nullptr, nullptr);
    float s = 0.0f;
    int64_t i = 0;
    for (; i + 8 <= n; i += 8) {  // the 8-element block copy issues beside the serial adds
        float v[8];
        memcpy(v, x + i, sizeof(v));
        memcpy(dst + i, v, sizeof(v));
        for (int k = 0; k < 8; ++k) s = s + v[k];
    }
    for (; i < n; ++i) {
        dst[i] = x[i];
        s = s + x[i];
    }
    return s;
}

int ofl_copy_h2d_chunked(const float* x, float* pinned, void* dev, int64_t n, int64_t chunk, int want_sum,
                         float* sum_out, void* stream) {
    if (n < 0 || (n && (!x || !pinned || !dev)) || chunk <= 0) return fail(OFL_EINVAL, "copy_h2d_chunked: bad arguments");
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (want_sum && n >= kSumMtMin) {
        // the copy into pinned staging runs on the sum's threads (its first
        // phase); the one H2D is issued right after it, beside the rest
        struct Ctx { const float* pinned; void* dev; int64_t n; hipStream_t st; hipError_t err; } c{pinned, dev, n, st, hipSuccess};
        const float s = ofl::serial_sum_f32_mt_cb(x, n, pinned, 0, [](void* p) {
            Ctx& c = *static_cast<Ctx*>(p);
            c.err = hipMemcpyAsync(c.dev, c.pinned, 4 * c.n, hipMemcpyHostToDevice, c.st);
        }, &c);
        HIP_TRY(c.err);
        if (sum_out) *sum_out = s;
        return OFL_OK;
    }
    float s = 0.0f;
    for (int64_t o = 0; o < n; o += chunk) {
        const int64_t c = std::min(chunk, n - o);
        if (want_sum) {
            // the serial sum continues from the previous chunk: one dependent chain
            int64_t i = 0;
            const float* xs = x + o;
            float* d = pinned + o;
            for (; i + 8 <= c; i += 8) {
                float v[8];
                memcpy(v, xs + i, sizeof(v));
                memcpy(d + i, v, sizeof(v));
                for (int k = 0; k < 8; ++k) s = s + v[k];
            }
            for (; i < c; ++i) {
                d[i] = xs[i];
                s = s + xs[i];
            }
        } else {
            memcpy(pinned + o, x + o, 4 * c);
        }
        HIP_TRY(hipMemcpyAsync(static_cast<float*>(dev) + o, pinned + o, 4 * c, hipMemcpyHostToDevice, st));
    }
    if (sum_out) *sum_out = s;
    return OFL_OK;
}

double ofl_serial_sum_f64(const double* x, int64_t n) {
    double s = 0.0;
    for (int64_t i = 0; i < n; ++i) s = s + x[i];
    return s;
}

int ofl_serial_sums_many(int n, const void* const* ptrs, const int64_t* lens, int f64, double* out, int nthreads) {
    if (n <= 0) return OFL_OK;
    if (!ptrs || !lens || !out) return fail(OFL_EINVAL, "serial_sums: null arrays");
    std::vector<int> order(n);
    for (int i = 0; i < n; ++i) order[i] = i;
    std::sort(order.begin(), order.end(), [&](int a, int b) { return lens[a] > lens[b]; });  // largest first
    // float32 arrays of 2^22 elements and more: one at a time on all threads
    // (the exact multi-threaded chain); the rest: one array per thread
    int first = 0;
    while (!f64 && first < n && lens[order[first]] >= (1 << 22)) {
        const int i = order[first++];
        out[i] = (double)ofl::serial_sum_f32_mt_cb(static_cast<const float*>(ptrs[i]), lens[i], nullptr, nthreads,
                                                   nullptr, nullptr);
    }
    std::atomic<int> next{first};
    auto work = [&] {
        for (int k = next++; k < n; k = next++) {
            const int i = order[k];
            out[i] = f64 ? ofl_serial_sum_f64(static_cast<const double*>(ptrs[i]), lens[i])
                         : (double)serial_sum_f32_loop(static_cast<const float*>(ptrs[i]), lens[i]);
        }
    };
    const int nt = std::max(1, std::min(nthreads, n - first));
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(work);
    work();
    for (auto& x : th) x.join();
    return OFL_OK;
}

int ofl_host_copy_many(int n, void* const* dst, const void* const* src, const int64_t* bytes, int nthreads) {
    if (n <= 0) return OFL_OK;
    if (!dst || !src || !bytes) return fail(OFL_EINVAL, "copy_many: null arrays");
    int64_t total = 0;
    for (int i = 0; i < n; ++i) total += bytes[i] > 0 ? bytes[i] : 0;
    // split the bytes evenly over the threads (items are cut at thread borders)
    const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(std::max(nthreads, 1), total >> 20));
    auto work = [&](int t) {
        const int64_t lo = total * t / nt, hi = total * (t + 1) / nt;
        int64_t acc = 0;
        for (int i = 0; i < n && acc < hi; ++i) {
            const int64_t b = bytes[i] > 0 ? bytes[i] : 0;
            const int64_t s0 = std::max(acc, lo), s1 = std::min(acc + b, hi);
            if (s1 > s0)
                memcpy(static_cast<char*>(dst[i]) + (s0 - acc), static_cast<const char*>(src[i]) + (s0 - acc),
                       (size_t)(s1 - s0));
            acc += b;
        }
    };
    // on the persistent native pool (a thread start per call cost ~0.1 ms per
    // copy); fresh threads only when every pool is busy with another caller
    if (nt > 1 && ofl::pool_run(nt, nt - 1, work)) return OFL_OK;
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
    return OFL_OK;
}

}  // extern "C"
