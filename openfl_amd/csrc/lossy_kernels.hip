// lossy_kernels.hip -- gfx950 kernels for the k-means / sparsify / ternary
// pipelines of openfl/pipelines (reference: /root/reference):
//   kc_pipeline.py:36-114   KmeansTransformer (sklearn KMeans k=6, n_init=6)
//   skc_pipeline.py:33-187  SparsityTransformer + KmeansTransformer
//   stc_pipeline.py:30-143  SparsityTransformer + TernaryTransformer
//
// Every O(n) pass is a streaming HIP kernel (coalesced 16-B loads, per-block
// LDS/register reduction, one atomic per block and quantity); the O(bins)
// k-means decisions (k-means++ seeding, Lloyd on the histogram) and the
// 2048-bin radix-select walks run on the host side of this library between
// passes.  All entry points are synchronous on `stream` (they return host
// scalars) -- the lossy pipelines are latency-tolerant plugin calls.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <mutex>
#include <random>
#include <string>
#include <vector>

#include "ofl_codec.h"
#include "ofl_util.h"

#define DEVI __device__ __forceinline__

namespace lossy {

constexpr int kNT = 256;
constexpr int kRadixBits = 11;    // radix-select digit
constexpr int kRadix = 1 << kRadixBits;
constexpr int kMaxK = 32;         // clusters supported

DEVI int64_t gtid() { return (int64_t)blockIdx.x * blockDim.x + threadIdx.x; }
DEVI int64_t gstride() { return (int64_t)gridDim.x * blockDim.x; }

template <typename T>
DEVI T wave_sum(T v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
DEVI float wave_min(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
    return v;
}
DEVI float wave_max(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}
// order-preserving float <-> uint32 (for atomic min/max)
DEVI uint32_t fkey(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// LDS histogram increment with wave aggregation for concentrated data: the
// lanes that share the first active lane's bin add once (popcount / wave
// sum), the others add directly.  Sparse or low-entropy inputs (top-k zeros,
// exponent digits) otherwise serialise up to 64 same-address LDS atomics.
DEVI void lds_count(uint32_t* h, int b) {
    const int bl = __builtin_amdgcn_readfirstlane(b);
    const unsigned long long m = __ballot(b == bl);
    if (__popcll(m) >= 8) {
        if (b == bl) {
            if ((int)(threadIdx.x & 63) == __builtin_ffsll((long long)m) - 1) atomicAdd(&h[bl], (uint32_t)__popcll(m));
        } else {
            atomicAdd(&h[b], 1u);
        }
    } else {
        atomicAdd(&h[b], 1u);
    }
}
DEVI void lds_add64(unsigned long long* h, int b, unsigned long long v) {
    const int bl = __builtin_amdgcn_readfirstlane(b);
    const unsigned long long m = __ballot(b == bl);
    if (__popcll(m) >= 8) {
        unsigned long long s = b == bl ? v : 0ull;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
        if (b == bl) {
            if ((int)(threadIdx.x & 63) == __builtin_ffsll((long long)m) - 1) atomicAdd(&h[bl], s);
        } else {
            atomicAdd(&h[b], v);
        }
    } else {
        atomicAdd(&h[b], v);
    }
}

struct KmParams {
    float mids[kMaxK];       // sorted midpoints between consecutive sorted centres (k-1 used)
    float rank[kMaxK];       // label value to write per cluster (float32 rank)
    int k;
};
DEVI int cluster_of(float v, const KmParams& p) {
    int c = 0;
#pragma unroll
    for (int j = 0; j < kMaxK - 1; ++j) c += (j < p.k - 1 && p.mids[j] < v) ? 1 : 0;
    return c;
}

// ---- labels -> float32 ranks -------------------------------------------------
__global__ __launch_bounds__(kNT) void k_km_label(const float* x, int64_t n, KmParams p, float* out) {
    for (int64_t i = gtid(); i < n; i += gstride()) out[i] = p.rank[cluster_of(x[i], p)];
}

// 256-thread exclusive scan of one uint32 per thread (block total in `total`)
DEVI uint32_t block_excl_scan(uint32_t v, uint32_t* tmp, uint32_t& total) {
    // 256 threads: wave-level inclusive scan, then wave offsets
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(inc, o, 64);
        if (lane >= o) inc += t;
    }
    if (lane == 63) tmp[w] = inc;
    __syncthreads();
    uint32_t off = 0;
    total = 0;
#pragma unroll
    for (int j = 0; j < kNT / 64; ++j) { if (j < w) off += tmp[j]; total += tmp[j]; }
    __syncthreads();
    return off + inc - v;
}

// ternary ranks of the sparse array (stc_pipeline.py:105-130): value > 0 ->
// rank_pos, < 0 -> rank_neg, else rank_zero; written as float32 (GZIP input)
__global__ __launch_bounds__(kNT) void k_ternary(const float* sparse, int64_t n, float rneg, float rzero,
                                                 float rpos, float* out) {
    for (int64_t i = gtid(); i < n; i += gstride()) {
        const float v = sparse[i];
        out[i] = v > 0.0f ? rpos : (v < 0.0f ? rneg : rzero);
    }
}

// TernaryTransformer statistics (stc_pipeline.py:120-123): fp64 sum of |x| and
// counts of x > 0, x < 0 (the rest are zeros)
// per-wave partials (sign counts, sum |x| in fp64), then one wave sums them in
// a fixed order: the ternary mean (stc_pipeline.py:120-123) is the same on
// every run (fp64 atomics would make its last bits depend on arrival order)
__global__ __launch_bounds__(kNT) void k_tstats(const float* x, int64_t n, unsigned long long* cnt_p,
                                                 double* abs_p) {
    uint32_t cp = 0, cn = 0;
    double as = 0.0;
    for (int64_t i = gtid(); i < n; i += gstride()) {
        const float v = x[i];
        cp += v > 0.0f;
        cn += v < 0.0f;
        as += fabs((double)v);
    }
    cp = wave_sum(cp); cn = wave_sum(cn); as = wave_sum(as);
    if ((threadIdx.x & 63) == 0) {
        const int64_t w = (int64_t)blockIdx.x * (kNT / 64) + (threadIdx.x >> 6);
        cnt_p[2 * w] = cp;
        cnt_p[2 * w + 1] = cn;
        abs_p[w] = as;
    }
}
__global__ __launch_bounds__(64) void k_tstats_final(const unsigned long long* cnt_p, const double* abs_p, int nw,
                                                     unsigned long long* cnt, double* abs_sum) {
    unsigned long long cp = 0, cn = 0;
    double as = 0.0;
    for (int w = threadIdx.x; w < nw; w += 64) { cp += cnt_p[2 * w]; cn += cnt_p[2 * w + 1]; as += abs_p[w]; }
    cp = wave_sum(cp); cn = wave_sum(cn); as = wave_sum(as);
    if (threadIdx.x == 0) { cnt[0] = cp; cnt[1] = cn; abs_sum[0] = as; }
}

// reference backward (kc_pipeline.py:81-83): for key in order: data[data == key] = value,
// applied in place and in sequence -- emulated exactly per element
struct LutParams { float key[64]; float val[64]; int nk; };
__global__ __launch_bounds__(kNT) void k_lut(const float* in, int64_t n, LutParams p, float* out) {
    for (int64_t i = gtid(); i < n; i += gstride()) {
        float v = in[i];
        for (int j = 0; j < p.nk; ++j) v = (v == p.key[j]) ? p.val[j] : v;
        out[i] = v;
    }
}


// ===========================================================================
// Batched 1-D k-means (KmeansTransformer.forward, kc_pipeline.py:47-63 and
// skc_pipeline.py:127-131, for many tensors of one fp32 arena) entirely on the
// device and deterministic (integer atomics and fixed-order reductions only):
//   k_bkm_minmax  per-tensor min / max                              (1 pass)
//   k_bkm_hist    per-tensor 4096-bin histogram: counts + fixed-point
//                 sums of the position inside the bin               (1 pass)
//   k_bkm_seed    one workgroup per (tensor, restart): weighted k-means++ with
//                 sklearn's 2 + ln(k) local trials, then Lloyd on the bin
//                 means through prefix sums (O(1) cluster edges); n_init
//                 restarts, lowest inertia
//   k_bkm_acc     exact Lloyd statistics on the data: per block, count /
//                 sum / sum of squares above every float32 midpoint (1 pass)
//   k_bkm_update  one wave per tensor: fixed-order sum of the block
//                 partials, new centres; stops when the float32 midpoints
//                 do not move or at sklearn's tolerance (then one more
//                 assignment pass); then counts, inertia, np.unique ranks
//   k_bkm_label   float32 rank of each element's cluster         (1 pass)
// A block covers kBkmChunk consecutive elements of one tensor.
// ===========================================================================
constexpr int kBkmChunk = 1 << 16;
constexpr int kBkmBins = 4096;
constexpr int kBkmMaxInit = 16;  // k-means++ restarts (n_init), one workgroup each

struct BkmTensor { int64_t off; int64_t n; int32_t blk0; int32_t nblk; };
struct BkmState {
    uint32_t mm[2];          // ~key(min), key(max): both reduced by atomicMax from 0
    int32_t converged;       // 0 running, 2 final assignment pass pending, 1 done
    int32_t nuniq;
    double cen[kMaxK];       // sorted centres
    float mids[kMaxK];       // float32 midpoints of consecutive centres (+inf beyond k-1)
    float rank[kMaxK];       // float32 rank of each cluster's value
    double uniq[kMaxK];      // sorted distinct values of the used centres (value dtype)
    long long cnt[kMaxK];
    double inertia;
    double cand[kBkmMaxInit][kMaxK];  // sorted centres of each restart
    double cand_in[kBkmMaxInit];      // and its inertia on the histogram
};
struct BkmArgs {
    const float* x;
    float* out;
    const BkmTensor* td;
    int32_t ntensors;
    int32_t k;
    int32_t n_init;
    int32_t value_f64;       // centre values as float64 (else rounded to float32)
    int32_t final_pass;
    int32_t pad_;
    uint64_t seed;
    BkmState* st;
    uint32_t* hc;            // [T][4096] counts
    unsigned long long* hs;  // [T][4096] sums of (position inside the bin) * 2^32
    double* part;            // [blocks][3][kMaxK] cumulative partials
};

DEVI int bkm_tensor(const BkmArgs& a, int b) {
    int lo = 0, hi = a.ntensors - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (a.td[mid].blk0 <= b) lo = mid; else hi = mid - 1;
    }
    return lo;
}
// this block's tensor and element range
DEVI void bkm_range(const BkmArgs& a, int& t, int64_t& i0, int64_t& i1) {
    t = bkm_tensor(a, (int)blockIdx.x);
    const BkmTensor T = a.td[t];
    i0 = (int64_t)(blockIdx.x - T.blk0) * kBkmChunk;
    i1 = i0 + kBkmChunk < T.n ? i0 + kBkmChunk : T.n;
}
// f(v) for every element of p[i0, i1): 16-B loads over the aligned middle
template <int NT = kNT, typename F>
DEVI void bkm_visit(const float* p, int64_t i0, int64_t i1, F f) {
    int64_t a4 = i0;
    while (a4 < i1 && (reinterpret_cast<uintptr_t>(p + a4) & 15u)) ++a4;
    for (int64_t j = i0 + threadIdx.x; j < a4; j += NT) f(p[j]);
    const int64_t n4 = (i1 - a4) >> 2;
    const float4* q = reinterpret_cast<const float4*>(p + a4);
    for (int64_t j = threadIdx.x; j < n4; j += NT) {
        const float4 v = q[j];
        f(v.x); f(v.y); f(v.z); f(v.w);
    }
    for (int64_t j = a4 + 4 * n4 + threadIdx.x; j < i1; j += NT) f(p[j]);
}

__global__ __launch_bounds__(kNT) void k_bkm_minmax(BkmArgs a) {
    __shared__ float rlo[kNT / 64], rhi[kNT / 64];
    int t; int64_t i0, i1;
    bkm_range(a, t, i0, i1);
    float lo = INFINITY, hi = -INFINITY;
    bkm_visit(a.x + a.td[t].off, i0, i1, [&](float v) { lo = fminf(lo, v); hi = fmaxf(hi, v); });
    lo = wave_min(lo);
    hi = wave_max(hi);
    if ((threadIdx.x & 63) == 0) { rlo[threadIdx.x >> 6] = lo; rhi[threadIdx.x >> 6] = hi; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 0; w < kNT / 64; ++w) { lo = fminf(lo, rlo[w]); hi = fmaxf(hi, rhi[w]); }
        atomicMax(&a.st[t].mm[0], ~fkey(lo));
        atomicMax(&a.st[t].mm[1], fkey(hi));
    }
}
DEVI float bkm_unkey(uint32_t k) { return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k); }
DEVI void bkm_bounds(const BkmState& S, float& lo, float& hi, float& inv_w) {
    lo = bkm_unkey(~S.mm[0]);
    hi = bkm_unkey(S.mm[1]);
    inv_w = hi > lo ? (float)((double)kBkmBins / ((double)hi - (double)lo) * (1.0 - 1e-7)) : 0.0f;
}

// one 64-bit LDS atomic per element: count in bits [47, 64) (a block has at
// most 2^16 elements), the position inside the bin as 2^30 fixed point in
// bits [0, 47) (at most 2^16 * 2^30 = 2^46 per block); flushed as a count
// and a 2^32 fixed-point sum
constexpr int kBkmCntShift = 47;
__global__ __launch_bounds__(kNT) void k_bkm_hist(BkmArgs a) {
    static_assert(kBkmChunk <= (1 << 16), "packed histogram counts");
    __shared__ unsigned long long h[kBkmBins];
    for (int b = threadIdx.x; b < kBkmBins; b += kNT) h[b] = 0;
    int t; int64_t i0, i1;
    bkm_range(a, t, i0, i1);
    float lo, hi, inv_w;
    bkm_bounds(a.st[t], lo, hi, inv_w);
    __syncthreads();
    bkm_visit(a.x + a.td[t].off, i0, i1, [&](float v) {
        const float f = (v - lo) * inv_w;
        int b = (int)f;
        b = b < 0 ? 0 : (b >= kBkmBins ? kBkmBins - 1 : b);
        float fr = f - (float)b;
        fr = fr < 0.f ? 0.f : (fr < 1.f ? fr : 0.99999994f);
        lds_add64(h, b, (1ull << kBkmCntShift) | (unsigned long long)(fr * 1073741824.0f));
    });
    __syncthreads();
    uint32_t* hc = a.hc + (int64_t)t * kBkmBins;
    unsigned long long* hs = a.hs + (int64_t)t * kBkmBins;
    for (int b = threadIdx.x; b < kBkmBins; b += kNT) {
        const unsigned long long v = h[b];
        if (v) {
            atomicAdd(&hc[b], (uint32_t)(v >> kBkmCntShift));
            atomicAdd(&hs[b], (v & ((1ull << kBkmCntShift) - 1)) << 2);
        }
    }
}

DEVI uint64_t bkm_rng(uint64_t& s) {  // xorshift64*
    s ^= s >> 12; s ^= s << 25; s ^= s >> 27;
    return s * 0x2545F4914F6CDD1Dull;
}
DEVI double bkm_uniform(uint64_t& s) { return (double)(bkm_rng(s) >> 11) * (1.0 / 9007199254740992.0); }
// first i in [0, n) with P[i] > u for an inclusive prefix P (last index if none)
template <typename T>
DEVI int bkm_first_above(const T* P, int n, double u) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if ((double)P[mid] > u) hi = mid; else lo = mid + 1;
    }
    return lo;
}
// first i in [0, n] with pts[i] > m (pts ascending)
DEVI int bkm_upper(const float* pts, int n, double m) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if ((double)pts[mid] > m) hi = mid; else lo = mid + 1;
    }
    return lo;
}
DEVI void bkm_set_centres(BkmState& S, const double* c, int k) {
    for (int j = 0; j < kMaxK; ++j) S.cen[j] = j < k ? c[j] : c[k - 1];
    for (int j = 0; j < kMaxK; ++j) S.mids[j] = j + 1 < k ? (float)((c[j] + c[j + 1]) / 2) : INFINITY;
}

// one workgroup per tensor: k-means of the weighted histogram points
// inclusive wave scan of one double per lane; total = the whole wave's sum
DEVI double wscan(double v, double& total) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const double u = __shfl_up(v, o, 64);
        if (lane >= o) v += u;
    }
    total = __shfl(v, 63, 64);
    return v;
}
// block (256 threads) sum / inclusive scan of one double per thread; fixed order
DEVI double bkm_bsum(double v, double* tmp) {
    v = wave_sum(v);
    if ((threadIdx.x & 63) == 0) tmp[threadIdx.x >> 6] = v;
    __syncthreads();
    const double s = (tmp[0] + tmp[1]) + (tmp[2] + tmp[3]);
    __syncthreads();
    return s;
}
DEVI double bkm_bscan(double v, double* tmp, double& total) {
    double t;
    v = wscan(v, t);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) tmp[w] = t;
    __syncthreads();
    double off = 0.0;
    for (int j = 0; j < w; ++j) off += tmp[j];
    total = (tmp[0] + tmp[1]) + (tmp[2] + tmp[3]);
    __syncthreads();
    return off + v;
}

// exclusive running max over the block's threads in thread order (256 threads)
DEVI float bkm_bscan_max_excl(float v, double* tmp) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const float u = __shfl_up(v, o, 64);
        if (lane >= o) v = fmaxf(v, u);
    }
    float ex = __shfl_up(v, 1, 64);
    if (lane == 0) ex = -INFINITY;
    if (lane == 63) tmp[w] = v;
    __syncthreads();
    for (int j = 0; j < w; ++j) ex = fmaxf(ex, (float)tmp[j]);
    __syncthreads();
    return ex;
}

// One workgroup per (tensor, restart): k-means of the 4096 histogram points (bin means,
// weight = count; empty bins keep their centre with weight 0, so the points
// stay sorted and the cluster edge of a midpoint m is found in O(1) from
// (m - lo) * inv_w).  Weighted k-means++ with sklearn's local trials, then
// Lloyd through prefix sums (lane j of wave 0 owns cluster j) to sklearn's
// tolerance.  k_bkm_pick keeps the restart with the lowest histogram inertia.
constexpr int kBkmSeedNT = 256;
constexpr size_t kBkmSeedLds = 4 * sizeof(float) * kBkmBins + 2 * sizeof(double) * kBkmBins;  // 128 KiB
__global__ __launch_bounds__(kBkmSeedNT) void k_bkm_seed(BkmArgs a) {
    static_assert(kBkmSeedNT == 256, "bkm_bsum/bkm_bscan assume 4 waves");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    double* W = reinterpret_cast<double*>(smem);
    double* S1 = W + kBkmBins;
    float* pts = reinterpret_cast<float*>(S1 + kBkmBins);
    float* wts = pts + kBkmBins;
    float* d2 = wts + kBkmBins;
    float* C = d2 + kBkmBins;
    __shared__ double tmp[4];
    __shared__ double cc[kMaxK];
    const int t = blockIdx.x / a.n_init, run = blockIdx.x % a.n_init;
    BkmState& S = a.st[t];
    const int k = a.k;
    auto emit = [&](double in) {  // this restart's result (thread 0)
        for (int j = 0; j < k; ++j) S.cand[run][j] = cc[j];
        S.cand_in[run] = in;
    };
    float lo, hi, inv_w;
    bkm_bounds(S, lo, hi, inv_w);
    if (!(hi > lo)) {  // constant (or non-finite: reported by the host) tensor
        if (threadIdx.x == 0) {
            for (int j = 0; j < k; ++j) cc[j] = lo;
            emit(0.0);
        }
        return;
    }
    constexpr int PER = kBkmBins / kBkmSeedNT;  // 16 consecutive bins per thread
    const int i0 = threadIdx.x * PER;
    const uint32_t* hc = a.hc + (int64_t)t * kBkmBins;
    const unsigned long long* hs = a.hs + (int64_t)t * kBkmBins;
    const double width = 1.0 / (double)inv_w;
    int occ = 0;
    double w0 = 0.0, s0 = 0.0, q0 = 0.0;
    for (int q = 0; q < PER; ++q) {
        const int b = i0 + q;
        const uint32_t cn = hc[b];
        const double fr = cn ? (double)hs[b] / 4294967296.0 / (double)cn : 0.5;
        const float p = (float)((double)lo + ((double)b + fr) * width);
        pts[b] = p;
        wts[b] = (float)cn;
        occ += cn ? 1 : 0;
        w0 += cn;
        s0 += (double)cn * p;
        q0 += (double)cn * p * p;
    }
    double tw, ts;
    double ew = bkm_bscan(w0, tmp, tw) - w0;
    double es = bkm_bscan(s0, tmp, ts) - s0;
    for (int q = 0; q < PER; ++q) { ew += wts[i0 + q]; es += (double)wts[i0 + q] * pts[i0 + q]; W[i0 + q] = ew; S1[i0 + q] = es; }
    const int nocc = (int)bkm_bsum((double)occ, tmp);
    const double sq = bkm_bsum(q0, tmp);  // (also publishes pts / W / S1)
    {  // rounding may break the order of neighbouring bin means: running max (block scan)
        float mx = -INFINITY;
        for (int q = 0; q < PER; ++q) mx = fmaxf(mx, pts[i0 + q]);
        float r = bkm_bscan_max_excl(mx, tmp);
        for (int q = 0; q < PER; ++q) { r = fmaxf(r, pts[i0 + q]); pts[i0 + q] = r; }
    }
    __syncthreads();
    if (nocc <= k) {  // no more occupied bins than clusters: they are the centres
        if (threadIdx.x == 0) {
            int j = 0;
            for (int b = 0; b < kBkmBins && j < k; ++b) if (wts[b] > 0) cc[j++] = pts[b];
            for (; j < k; ++j) cc[j] = cc[j - 1];
            emit(0.0);
        }
        return;
    }
    const double wt = W[kBkmBins - 1];
    const double mu = S1[kBkmBins - 1] / wt;
    const double tol = 1e-4 * fmax(sq / wt - mu * mu, 0.0);  // sklearn's _tolerance
    // first bin whose point lies above m (points sorted, each inside its bin)
    auto edge = [&](double m) -> int {
        int b = (int)floor((m - (double)lo) * (double)inv_w);
        b = b < 0 ? 0 : (b > kBkmBins ? kBkmBins : b);
        while (b > 0 && (double)pts[b - 1] > m) --b;
        while (b < kBkmBins && (double)pts[b] <= m) ++b;
        return b;
    };
    // every thread draws the same numbers
    uint64_t rs = (a.seed ^ (0x9E3779B97F4A7C15ull * (uint64_t)(t + 1)) ^ (0xD1B54A32D192ED03ull * (uint64_t)(run + 1))) | 1ull;
    for (int q = 0; q < 4; ++q) bkm_rng(rs);
    const int trials = 2 + (int)log((double)k);  // sklearn's n_local_trials
    {
        // ---- weighted k-means++ ----
        {
            const int i = bkm_first_above(W, kBkmBins, bkm_uniform(rs) * wt);
            const float c0 = pts[i];
            if (threadIdx.x == 0) cc[0] = c0;
            for (int q = 0; q < PER; ++q) { const float d = pts[i0 + q] - c0; d2[i0 + q] = d * d; }
        }
        for (int j = 1; j < k; ++j) {
            double loc = 0.0;
            for (int q = 0; q < PER; ++q) loc += (double)wts[i0 + q] * d2[i0 + q];
            double pot;
            double e = bkm_bscan(loc, tmp, pot) - loc;
            for (int q = 0; q < PER; ++q) { e += (double)wts[i0 + q] * d2[i0 + q]; C[i0 + q] = (float)e; }
            __syncthreads();
            double bpot = INFINITY;
            int bi = 0;
            for (int tr = 0; tr < trials; ++tr) {
                int ci = pot > 0.0 ? bkm_first_above(C, kBkmBins, bkm_uniform(rs) * pot)
                                   : (int)(bkm_rng(rs) % (uint64_t)kBkmBins);
                while (ci > 0 && wts[ci] == 0) --ci;  // (float rounding of C) never an empty bin
                const float cv = pts[ci];
                double np = 0.0;
                for (int q = 0; q < PER; ++q) { const float d = pts[i0 + q] - cv; np += (double)wts[i0 + q] * fminf(d2[i0 + q], d * d); }
                np = bkm_bsum(np, tmp);
                if (np < bpot) { bpot = np; bi = ci; }
            }
            const float cv = pts[bi];
            if (threadIdx.x == 0) cc[j] = cv;
            for (int q = 0; q < PER; ++q) { const float d = pts[i0 + q] - cv; d2[i0 + q] = fminf(d2[i0 + q], d * d); }
        }
        __syncthreads();
        // ---- Lloyd on the bin means, wave 0, lane j = cluster j ----
        if (threadIdx.x == 0)
            for (int i = 1; i < k; ++i) { const double v = cc[i]; int j = i - 1; while (j >= 0 && cc[j] > v) { cc[j + 1] = cc[j]; --j; } cc[j + 1] = v; }
        __syncthreads();
        if (threadIdx.x < 64) {
            const int lane = threadIdx.x;
            double cj = lane < k ? cc[lane] : 0.0;
            for (int it = 0; it < 300; ++it) {
                const double cn = __shfl_down(cj, 1, 64);
                const int end = lane + 1 < k ? edge((cj + cn) / 2) : kBkmBins;
                int start = __shfl_up(end, 1, 64);
                if (lane == 0) start = 0;
                double nc = cj;
                if (lane < k && end > start) {
                    const double w = W[end - 1] - (start ? W[start - 1] : 0.0);
                    const double sm = S1[end - 1] - (start ? S1[start - 1] : 0.0);
                    if (w > 0) nc = sm / w;
                }
                const double shift = wave_sum(lane < k ? (nc - cj) * (nc - cj) : 0.0);
                cj = nc;
                // an empty cluster keeps its centre and may fall out of order
                const double nx = __shfl_down(cj, 1, 64);
                if (__any(lane + 1 < k && nx < cj)) {
                    if (lane < k) cc[lane] = cj;
                    if (lane == 0)
                        for (int i = 1; i < k; ++i) { const double v = cc[i]; int j = i - 1; while (j >= 0 && cc[j] > v) { cc[j + 1] = cc[j]; --j; } cc[j + 1] = v; }
                    if (lane < k) cj = cc[lane];
                }
                if (shift <= tol) break;
            }
            if (lane < k) cc[lane] = cj;
        }
        __syncthreads();
        // ---- inertia of this run on the histogram ----
        double in = 0.0;
        for (int q = 0; q < PER; ++q) {
            const double p = pts[i0 + q];
            double bd = INFINITY;
            for (int j = 0; j < k; ++j) { const double d = (p - cc[j]) * (p - cc[j]); bd = d < bd ? d : bd; }
            in += (double)wts[i0 + q] * bd;
        }
        in = bkm_bsum(in, tmp);
        if (threadIdx.x == 0) emit(in);
    }
}

// the restart with the lowest histogram inertia (first on ties) seeds the exact passes
__global__ __launch_bounds__(64) void k_bkm_pick(BkmArgs a) {
    const int t = blockIdx.x * 64 + threadIdx.x;
    if (t >= a.ntensors) return;
    BkmState& S = a.st[t];
    int b = 0;
    for (int r = 1; r < a.n_init; ++r) if (S.cand_in[r] < S.cand_in[b]) b = r;
    bkm_set_centres(S, S.cand[b], a.k);
}

// exact Lloyd statistics: per block, cumulative count / sum / sum of squares
// above each of the KM1 midpoints (+ totals); float per thread, double across
constexpr int kBkmAccNT = 1024;  // VALU-heavy per element: 16 waves per block
template <int KM1>
__global__ __launch_bounds__(kBkmAccNT) void k_bkm_acc(BkmArgs a) {
    constexpr int NV = KM1 + 1;
    __shared__ double red[kBkmAccNT / 64][3][NV];
    int t; int64_t i0, i1;
    bkm_range(a, t, i0, i1);
    const BkmState& S = a.st[t];
    if (S.converged == 1) return;
    float m[KM1];
#pragma unroll
    for (int j = 0; j < KM1; ++j) m[j] = S.mids[j];
    uint32_t n[NV];
    float s[NV], q[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) { n[j] = 0; s[j] = 0.f; q[j] = 0.f; }
    bkm_visit<kBkmAccNT>(a.x + a.td[t].off, i0, i1, [&](float v) {
        const float vv = v * v;
        n[0] += 1; s[0] += v; q[0] += vv;
#pragma unroll
        for (int j = 0; j < KM1; ++j) {
            const bool g = v > m[j];
            n[j + 1] += g ? 1u : 0u;
            s[j + 1] += g ? v : 0.f;
            q[j + 1] += g ? vv : 0.f;
        }
    });
    const int w = threadIdx.x >> 6;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const double dn = wave_sum((double)n[j]), ds = wave_sum((double)s[j]), dq = wave_sum((double)q[j]);
        if ((threadIdx.x & 63) == 0) { red[w][0][j] = dn; red[w][1][j] = ds; red[w][2][j] = dq; }
    }
    __syncthreads();
    if (threadIdx.x < 3 * NV) {
        const int r = threadIdx.x / NV, j = threadIdx.x % NV;
        double acc = 0.0;
        for (int ww = 0; ww < kBkmAccNT / 64; ++ww) acc += red[ww][r][j];
        a.part[((int64_t)blockIdx.x * 3 + r) * kMaxK + j] = acc;
    }
}

// one wave per tensor: new centres from the partials.  Lane l sums blocks
// l, l+64, ... in order, then a fixed shuffle tree: deterministic.
__global__ __launch_bounds__(64) void k_bkm_update(BkmArgs a) {
    const int t = blockIdx.x;
    BkmState& S = a.st[t];
    if (S.converged == 1) return;
    const BkmTensor T = a.td[t];
    const int k = a.k;
    __shared__ double g[3][kMaxK + 1];
    for (int j = 0; j < k; ++j)
        for (int r = 0; r < 3; ++r) {
            double acc = 0.0;
            for (int b = T.blk0 + (int)threadIdx.x; b < T.blk0 + T.nblk; b += 64)
                acc += a.part[((int64_t)b * 3 + r) * kMaxK + j];
            acc = wave_sum(acc);
            if (threadIdx.x == 0) g[r][j] = acc;
        }
    if (threadIdx.x != 0) return;
    double cg[kMaxK + 1], sg[kMaxK + 1], qg[kMaxK + 1];
    for (int j = 0; j < k; ++j) { cg[j] = g[0][j]; sg[j] = g[1][j]; qg[j] = g[2][j]; }
    cg[k] = 0.0; sg[k] = 0.0; qg[k] = 0.0;
    // cluster j = (mid[j-1], mid[j]]: cumulative differences
    double N[kMaxK], Sm[kMaxK], Q[kMaxK], nc[kMaxK];
    for (int j = 0; j < k; ++j) {
        N[j] = cg[j] - cg[j + 1];
        Sm[j] = sg[j] - sg[j + 1];
        Q[j] = qg[j] - qg[j + 1];
        nc[j] = N[j] > 0 ? Sm[j] / N[j] : S.cen[j];
    }
    // sort the new centres with their statistics
    for (int i = 1; i < k; ++i) {
        const double v = nc[i], vn = N[i], vs = Sm[i], vq = Q[i];
        int j = i - 1;
        while (j >= 0 && nc[j] > v) { nc[j + 1] = nc[j]; N[j + 1] = N[j]; Sm[j + 1] = Sm[j]; Q[j + 1] = Q[j]; --j; }
        nc[j + 1] = v; N[j + 1] = vn; Sm[j + 1] = vs; Q[j + 1] = vq;
    }
    bool same = true;
    for (int j = 0; j + 1 < k; ++j) same = same && (float)((nc[j] + nc[j + 1]) / 2) == S.mids[j];
    // sklearn's stopping rule: sum of squared centre shifts <= 1e-4 x the
    // data variance; then one more assignment pass with the final centres
    // (converged = 2) so that labels, counts and inertia belong to them
    const double mean = sg[0] / cg[0];
    const double tol = 1e-4 * fmax(qg[0] / cg[0] - mean * mean, 0.0);
    double shift = 0.0;
    for (int j = 0; j < k; ++j) shift += (nc[j] - S.cen[j]) * (nc[j] - S.cen[j]);
    const bool pending = S.converged == 2;
    if (!same && !pending && !a.final_pass) {
        bkm_set_centres(S, nc, k);
        if (shift <= tol) S.converged = 2;
        return;
    }
    // final: counts and inertia of the assignment this pass was made with
    double in = 0.0;
    if (same && !pending) {  // strict convergence: centres = means of the unchanged clusters
        for (int j = 0; j < k; ++j) if (N[j] > 0) in += Q[j] - Sm[j] * Sm[j] / N[j];
        bkm_set_centres(S, nc, k);
    } else {  // keep the centres the assignment was made with
        for (int j = 0; j < k; ++j) {  // (statistics above are sorted by new centre: redo by cluster)
            const double c = S.cen[j];
            N[j] = cg[j] - cg[j + 1]; Sm[j] = sg[j] - sg[j + 1]; Q[j] = qg[j] - qg[j + 1];
            in += Q[j] - 2 * c * Sm[j] + c * c * N[j];
        }
    }
    S.inertia = in > 0 ? in : 0.0;
    // np.unique over the used centres (value dtype) and each cluster's rank
    double vals[kMaxK], uq[kMaxK];
    int nu = 0;
    for (int j = 0; j < k; ++j) {
        vals[j] = a.value_f64 ? S.cen[j] : (double)(float)S.cen[j];
        S.cnt[j] = (long long)(N[j] + 0.5);
    }
    for (int j = 0; j < k; ++j) {
        if (S.cnt[j] <= 0) continue;
        bool dup = false;
        for (int i = 0; i < nu; ++i) dup = dup || uq[i] == vals[j];
        if (!dup) uq[nu++] = vals[j];
    }
    for (int i = 1; i < nu; ++i) { const double v = uq[i]; int j = i - 1; while (j >= 0 && uq[j] > v) { uq[j + 1] = uq[j]; --j; } uq[j + 1] = v; }
    for (int j = 0; j < k; ++j) {
        int r = 0;
        while (r < nu && uq[r] < vals[j]) ++r;
        S.rank[j] = (float)r;
    }
    for (int i = 0; i < kMaxK; ++i) S.uniq[i] = i < nu ? uq[i] : 0.0;
    S.nuniq = nu;
    S.converged = 1;
}

template <int KM1>
__global__ __launch_bounds__(kBkmAccNT) void k_bkm_label(BkmArgs a) {
    int t; int64_t i0, i1;
    bkm_range(a, t, i0, i1);
    const BkmState& S = a.st[t];
    float m[KM1], r[KM1 + 1];
#pragma unroll
    for (int j = 0; j < KM1; ++j) m[j] = S.mids[j];
#pragma unroll
    for (int j = 0; j <= KM1; ++j) r[j] = S.rank[j < a.k ? j : a.k - 1];
    const float* x = a.x + a.td[t].off;
    float* out = a.out + a.td[t].off;
    auto rank_of = [&](float v) {
        float o = r[0];
#pragma unroll
        for (int j = 0; j < KM1; ++j) o = v > m[j] ? r[j + 1] : o;
        return o;
    };
    // x and out share the arena offset, so they are 16-B aligned together
    int64_t a4 = i0;
    while (a4 < i1 && (reinterpret_cast<uintptr_t>(x + a4) & 15u)) ++a4;
    for (int64_t i = i0 + threadIdx.x; i < a4; i += kBkmAccNT) out[i] = rank_of(x[i]);
    const int64_t n4 = (i1 - a4) >> 2;
    const float4* x4 = reinterpret_cast<const float4*>(x + a4);
    float4* o4 = reinterpret_cast<float4*>(out + a4);
    for (int64_t i = threadIdx.x; i < n4; i += kBkmAccNT) {
        const float4 v = x4[i];
        o4[i] = make_float4(rank_of(v.x), rank_of(v.y), rank_of(v.z), rank_of(v.w));
    }
    for (int64_t i = a4 + 4 * n4 + threadIdx.x; i < i1; i += kBkmAccNT) out[i] = rank_of(x[i]);
}

static_assert(sizeof(ofl_label_rec) == 80, "lossy.LabelTable.REC_BYTES");
// each tensor's labelling rule as an ofl_label_rec (k <= 8): what k_bkm_label
// applies, for the gzip encoder to apply as it loads the values
__global__ __launch_bounds__(64) void k_bkm_tab(BkmArgs a, ofl_label_rec* tab) {
    const int t = (int)(blockIdx.x * 64 + threadIdx.x);
    if (t >= a.ntensors) return;
    const BkmState& S = a.st[t];
    ofl_label_rec r;
    r.start = a.td[t].off;
    r.end = a.td[t].off + a.td[t].n;
    for (int j = 0; j < 8; ++j) {
        r.mid[j] = j < 7 ? S.mids[j] : INFINITY;
        r.rank[j] = S.rank[j < a.k ? j : a.k - 1];
    }
    tab[t] = r;
}

// Batched reference backward (kc_pipeline.py:79-83 per tensor): tensor t's
// float32 ranks -> values by the sequential in-place key->value replacement,
// one launch for the whole arena (blocks as in the k-means passes).
struct LutBatchArgs {
    const float* in;
    float* out;
    const BkmTensor* td;
    const int32_t* nk;     // [T]
    const float* keys;     // [T][max_nk]
    const float* vals;     // [T][max_nk]
    int32_t ntensors;
    int32_t max_nk;
};
__global__ __launch_bounds__(kNT) void k_lut_batch(LutBatchArgs a) {
    __shared__ float ks[64], vs[64];
    int lo = 0, hi = a.ntensors - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (a.td[mid].blk0 <= (int)blockIdx.x) lo = mid; else hi = mid - 1;
    }
    const int t = lo;
    const BkmTensor T = a.td[t];
    const int nk = a.nk[t];
    if (threadIdx.x < nk) {
        ks[threadIdx.x] = a.keys[(int64_t)t * a.max_nk + threadIdx.x];
        vs[threadIdx.x] = a.vals[(int64_t)t * a.max_nk + threadIdx.x];
    }
    __syncthreads();
    const int64_t i0 = (int64_t)(blockIdx.x - T.blk0) * kBkmChunk;
    const int64_t i1 = i0 + kBkmChunk < T.n ? i0 + kBkmChunk : T.n;
    const float* x = a.in + T.off;
    float* y = a.out + T.off;
    auto lut = [&](float v) {
        for (int j = 0; j < nk; ++j) v = (v == ks[j]) ? vs[j] : v;
        return v;
    };
    if (((reinterpret_cast<uintptr_t>(x + i0) | reinterpret_cast<uintptr_t>(y + i0)) & 15u) == 0) {
        const int64_t n4 = (i1 - i0) >> 2;
        const float4* x4 = reinterpret_cast<const float4*>(x + i0);
        float4* y4 = reinterpret_cast<float4*>(y + i0);
        for (int64_t i = threadIdx.x; i < n4; i += kNT) {
            const float4 v = x4[i];
            y4[i] = make_float4(lut(v.x), lut(v.y), lut(v.z), lut(v.w));
        }
        for (int64_t i = i0 + 4 * n4 + threadIdx.x; i < i1; i += kNT) y[i] = lut(x[i]);
    } else {
        for (int64_t i = i0 + threadIdx.x; i < i1; i += kNT) y[i] = lut(x[i]);
    }
}
// ===========================================================================
// Batched exact top-k by magnitude (SparsityTransformer._topk_func,
// skc_pipeline.py:72-94 / stc_pipeline.py:53-91, for many tensors of one
// fp32 arena), device-resident and deterministic.  |x| bit patterns order like
// the magnitudes, so the k-th largest is found by a 3-digit radix select over
// the 31 magnitude bits (11 + 11 + 9):
//   k_btk_hist   per-tensor digit histogram of the elements matching the
//                prefix found so far                                 (1 pass)
//   k_btk_digit  one wave per tensor: the digit holding the need-th largest,
//                prefix/need update, histogram cleared for the next pass
// then T = the k-th largest |x| bits and `need` = ties at T kept (lowest index
// first, the reference's argsort order for ties being unspecified):
//   k_btk_ties   per block: ties at T, min kept-for-sure value (|x| > T), min
//                tie value, in-block tie rank of the first negative tie (1 pass)
//   k_btk_scan   one wave per tensor: exclusive prefix of the tie counts and
//                the exact minimum of the kept set -> the +1e-7 shift (:92-93)
//   k_btk_select dense sparse output (kept + shift, else 0) and per-block
//                kept-set statistics (1 pass: read x, write sparse)
//   k_btk_final  one wave per tensor: fixed-order sums of the statistics
// Blocks cover kBkmChunk consecutive elements of one tensor, as in k-means.
// ===========================================================================
struct BtkState {
    int64_t k;            // kept count (ceil(n p))
    int64_t need;         // rank from the top within the current prefix; after pass 3: ties kept
    uint32_t prefix, pmask;
    float kmin;           // min kept value (before the shift)
    float shift;          // 1e-7 or 0
    int64_t n_pos, n_neg, n_zero;
    double abs_sum;       // fp64 sum of |kept + shift|
};
struct BtkBlock {
    uint32_t ties;        // |x| bits == T in this block
    int32_t neg_rank;     // in-block tie rank of the first negative tie, -1 if none
    float smin;           // min value with |x| > T
    float tmin;           // min value with |x| == T
    uint64_t tie_base;    // ties in the tensor's earlier blocks
    uint32_t cpos, cneg, czero, pad_;
    double asum;
};
struct BtkArgs {
    const float* x;
    float* out;
    const BkmTensor* td;
    int32_t ntensors;
    int32_t pass;
    BtkState* st;
    uint32_t* hist;       // [T][kRadix]
    BtkBlock* blk;        // [blocks]
};

DEVI int tensor_of(const BkmTensor* td, int nt, int b) {
    int lo = 0, hi = nt - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (td[mid].blk0 <= b) lo = mid; else hi = mid - 1;
    }
    return lo;
}
// f(v, i) for every element of p[i0, i1) (i = index inside the tensor)
template <typename F>
DEVI void btk_visit(const float* p, int64_t i0, int64_t i1, F f) {
    int64_t a4 = i0;
    while (a4 < i1 && (reinterpret_cast<uintptr_t>(p + a4) & 15u)) ++a4;
    for (int64_t j = i0 + threadIdx.x; j < a4; j += kNT) f(p[j], j);
    const int64_t n4 = (i1 - a4) >> 2;
    const float4* q = reinterpret_cast<const float4*>(p + a4);
    for (int64_t j = threadIdx.x; j < n4; j += kNT) {
        const float4 v = q[j];
        const int64_t i = a4 + 4 * j;
        f(v.x, i); f(v.y, i + 1); f(v.z, i + 2); f(v.w, i + 3);
    }
    for (int64_t j = a4 + 4 * n4 + threadIdx.x; j < i1; j += kNT) f(p[j], j);
}
DEVI int btk_shift(int pass) { return pass == 0 ? 20 : (pass == 1 ? 9 : 0); }
DEVI int btk_width(int pass) { return pass == 2 ? 9 : 11; }

__global__ __launch_bounds__(kNT) void k_btk_hist(BtkArgs a) {
    __shared__ uint32_t h[kRadix];
    for (int b = threadIdx.x; b < kRadix; b += kNT) h[b] = 0;
    const int t = tensor_of(a.td, a.ntensors, (int)blockIdx.x);
    const BkmTensor T = a.td[t];
    const int64_t i0 = (int64_t)(blockIdx.x - T.blk0) * kBkmChunk;
    const int64_t i1 = i0 + kBkmChunk < T.n ? i0 + kBkmChunk : T.n;
    const uint32_t prefix = a.st[t].prefix, pmask = a.st[t].pmask;
    const int sh = btk_shift(a.pass);
    const uint32_t dm = (1u << btk_width(a.pass)) - 1u;
    __syncthreads();
    btk_visit(a.x + T.off, i0, i1, [&](float v, int64_t) {
        const uint32_t m = __float_as_uint(v) & 0x7fffffffu;
        if ((m & pmask) == prefix) lds_count(h, (int)((m >> sh) & dm));  // ballots see the candidates only
    });
    __syncthreads();
    uint32_t* g = a.hist + (int64_t)t * kRadix;
    for (int b = threadIdx.x; b <= (int)dm; b += kNT) if (h[b]) atomicAdd(&g[b], h[b]);
}

__global__ __launch_bounds__(64) void k_btk_digit(BtkArgs a) {
    const int t = blockIdx.x, lane = threadIdx.x;
    BtkState& S = a.st[t];
    uint32_t* h = a.hist + (int64_t)t * kRadix;
    const int width = btk_width(a.pass), sh = btk_shift(a.pass);
    const int per = (1 << width) / 64;
    const int64_t need = S.need;
    int64_t s = 0;
    for (int j = 0; j < per; ++j) s += h[lane * per + j];
    // suffix sums from the top bin: S_l = sum over lanes >= l
    int64_t suf = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int64_t u = __shfl_down(suf, o, 64);
        if (lane + o < 64) suf += u;
    }
    const unsigned long long hit = __ballot(suf >= need);
    const int L = hit ? 63 - __clzll((long long)hit) : 0;   // the need-th largest lies in lane L's bins
    if (lane == L) {
        int64_t acc = suf - s;  // elements in bins above lane L's range
        int d = lane * per;
        for (int b = lane * per + per - 1; b > lane * per; --b) {
            if (acc + (int64_t)h[b] >= need) { d = b; break; }
            acc += h[b];
        }
        S.prefix |= (uint32_t)d << sh;
        S.pmask |= (uint32_t)((1 << width) - 1) << sh;
        S.need = need - acc;
    }
    for (int j = 0; j < per; ++j) h[lane * per + j] = 0;
}

// 256-thread block reductions through a 4-entry LDS array
template <typename V, typename Op>
DEVI V btk_breduce(V v, V* tmp, Op op) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = op(v, __shfl_xor(v, o, 64));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) tmp[threadIdx.x >> 6] = v;
    __syncthreads();
    V r = tmp[0];
#pragma unroll
    for (int w = 1; w < kNT / 64; ++w) r = op(r, tmp[w]);
    return r;
}

__global__ __launch_bounds__(kNT) void k_btk_ties(BtkArgs a) {
    __shared__ uint32_t tu[kNT / 64];
    __shared__ float tf[kNT / 64];
    __shared__ int64_t ti[kNT / 64];
    const int t = tensor_of(a.td, a.ntensors, (int)blockIdx.x);
    const BkmTensor T = a.td[t];
    const int64_t i0 = (int64_t)(blockIdx.x - T.blk0) * kBkmChunk;
    const int64_t i1 = i0 + kBkmChunk < T.n ? i0 + kBkmChunk : T.n;
    const uint32_t Tb = a.st[t].prefix;
    const float* p = a.x + T.off;
    uint32_t c = 0;
    float smin = INFINITY, tmin = INFINITY;
    int64_t neg = INT64_MAX;
    btk_visit(p, i0, i1, [&](float v, int64_t i) {
        const uint32_t m = __float_as_uint(v) & 0x7fffffffu;
        if (m > Tb) smin = fminf(smin, v);
        if (m == Tb) {
            ++c;
            tmin = fminf(tmin, v);
            if (v < 0.0f && i < neg) neg = i;
        }
    });
    c = btk_breduce(c, tu, [](uint32_t x, uint32_t y) { return x + y; });
    smin = btk_breduce(smin, tf, [](float x, float y) { return fminf(x, y); });
    tmin = btk_breduce(tmin, tf, [](float x, float y) { return fminf(x, y); });
    neg = btk_breduce(neg, ti, [](int64_t x, int64_t y) { return x < y ? x : y; });
    int32_t rank = -1;
    if (neg != INT64_MAX) {  // rare: a negative tie -> its rank among the block's ties
        uint32_t r = 0;
        for (int64_t i = i0 + threadIdx.x; i < neg; i += kNT) r += (__float_as_uint(p[i]) & 0x7fffffffu) == Tb;
        rank = (int32_t)btk_breduce(r, tu, [](uint32_t x, uint32_t y) { return x + y; });
    }
    if (threadIdx.x == 0) {
        BtkBlock& B = a.blk[blockIdx.x];
        B.ties = c;
        B.neg_rank = rank;
        B.smin = smin;
        B.tmin = tmin;
    }
}

__global__ __launch_bounds__(64) void k_btk_scan(BtkArgs a) {
    const int t = blockIdx.x, lane = threadIdx.x;
    const BkmTensor T = a.td[t];
    BtkState& S = a.st[t];
    const int64_t need = S.need;
    uint64_t carry = 0;
    float smin = INFINITY, tmin = INFINITY;
    int negkept = 0;
    for (int b0 = 0; b0 < T.nblk; b0 += 64) {
        const int b = b0 + lane;
        BtkBlock* B = a.blk + T.blk0 + b;
        const uint64_t c = b < T.nblk ? B->ties : 0;
        uint64_t inc = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint64_t u = __shfl_up(inc, o, 64);
            if (lane >= o) inc += u;
        }
        if (b < T.nblk) {
            const uint64_t base = carry + inc - c;
            B->tie_base = base;
            smin = fminf(smin, B->smin);
            tmin = fminf(tmin, B->tmin);
            if (B->neg_rank >= 0 && (int64_t)base + B->neg_rank < need) negkept = 1;
        }
        carry += __shfl(inc, 63, 64);
    }
    smin = wave_min(smin);
    tmin = wave_min(tmin);
    negkept = __any(negkept);
    if (lane == 0) {
        float kmin = smin;
        const float Tf = __uint_as_float(S.prefix);
        if (need > 0) kmin = fminf(kmin, (int64_t)carry <= need ? tmin : (negkept ? -Tf : Tf));
        S.kmin = kmin;
        // reference: `if min(topk_mag) - 0 < 10e-8: topk_mag = topk_mag + 10e-8`
        S.shift = ((double)kmin < 10e-8) ? (float)10e-8 : 0.0f;
    }
}

__global__ __launch_bounds__(kNT) void k_btk_select(BtkArgs a) {
    __shared__ uint32_t tu[kNT / 64];
    __shared__ double td[kNT / 64];
    const int t = tensor_of(a.td, a.ntensors, (int)blockIdx.x);
    const BkmTensor T = a.td[t];
    const int64_t i0 = (int64_t)(blockIdx.x - T.blk0) * kBkmChunk;
    const int64_t i1 = i0 + kBkmChunk < T.n ? i0 + kBkmChunk : T.n;
    const uint32_t Tb = a.st[t].prefix;
    const int64_t need = a.st[t].need;
    const float shift = a.st[t].shift;
    BtkBlock& B = a.blk[blockIdx.x];
    const int64_t base = (int64_t)B.tie_base, nt = B.ties;
    const float* p = a.x + T.off;
    float* o = a.out + T.off;
    uint32_t cpos = 0, cneg = 0, czero = 0;
    double as = 0.0;
    auto kept = [&](float v) {
        const float w = v + shift;  // float32 add (NEP 50: python float is weak)
        cpos += w > 0.0f;
        cneg += w < 0.0f;
        czero += w == 0.0f;
        as += fabs((double)w);
        return w;
    };
    if (nt == 0 || base >= need || base + nt <= need) {
        // the block's ties are all dropped or all kept: no ordering needed
        const bool keep_ties = nt > 0 && base + nt <= need;
        auto f = [&](float v) {
            const uint32_t m = __float_as_uint(v) & 0x7fffffffu;
            return (m > Tb || (keep_ties && m == Tb)) ? kept(v) : 0.0f;
        };
        if (((reinterpret_cast<uintptr_t>(p + i0) | reinterpret_cast<uintptr_t>(o + i0)) & 15u) == 0) {
            const int64_t n4 = (i1 - i0) >> 2;
            const float4* x4 = reinterpret_cast<const float4*>(p + i0);
            float4* y4 = reinterpret_cast<float4*>(o + i0);
            for (int64_t j = threadIdx.x; j < n4; j += kNT) {
                const float4 v = x4[j];
                y4[j] = make_float4(f(v.x), f(v.y), f(v.z), f(v.w));
            }
            for (int64_t j = i0 + 4 * n4 + threadIdx.x; j < i1; j += kNT) o[j] = f(p[j]);
        } else {
            for (int64_t j = i0 + threadIdx.x; j < i1; j += kNT) o[j] = f(p[j]);
        }
    } else {
        // the boundary block: in-order tie ranks, kNT elements at a time
        int64_t ties = base;
        for (int64_t c0 = i0; c0 < i1; c0 += kNT) {
            const int64_t i = c0 + threadIdx.x;
            const bool in = i < i1;
            const float v = in ? p[i] : 0.0f;
            const uint32_t m = __float_as_uint(v) & 0x7fffffffu;
            const uint32_t tie = (in && m == Tb) ? 1u : 0u;
            uint32_t tot;
            const uint32_t r = block_excl_scan(tie, tu, tot);
            const bool keep = in && (m > Tb || (tie && ties + (int64_t)r < need));
            ties += tot;
            if (in) o[i] = keep ? kept(v) : 0.0f;
        }
    }
    cpos = btk_breduce(cpos, tu, [](uint32_t x, uint32_t y) { return x + y; });
    cneg = btk_breduce(cneg, tu, [](uint32_t x, uint32_t y) { return x + y; });
    czero = btk_breduce(czero, tu, [](uint32_t x, uint32_t y) { return x + y; });
    as = btk_breduce(as, td, [](double x, double y) { return x + y; });
    if (threadIdx.x == 0) { B.cpos = cpos; B.cneg = cneg; B.czero = czero; B.asum = as; }
}

__global__ __launch_bounds__(64) void k_btk_final(BtkArgs a) {
    const int t = blockIdx.x, lane = threadIdx.x;
    const BkmTensor T = a.td[t];
    uint64_t p = 0, n = 0, z = 0;
    double s = 0.0;
    for (int b = lane; b < T.nblk; b += 64) {
        const BtkBlock& B = a.blk[T.blk0 + b];
        p += B.cpos; n += B.cneg; z += B.czero; s += B.asum;
    }
    p = wave_sum(p); n = wave_sum(n); z = wave_sum(z); s = wave_sum(s);
    if (lane == 0) {
        BtkState& S = a.st[t];
        S.n_pos = (int64_t)p; S.n_neg = (int64_t)n; S.n_zero = (int64_t)z; S.abs_sum = s;
    }
}

// ternary ranks of a sparse arena, per-tensor (rank_neg, rank_zero, rank_pos)
// (stc_pipeline.py:105-130 then _float_to_int)
__global__ __launch_bounds__(kNT) void k_ternary_batch(const float* in, float* out, const BkmTensor* td, int nt,
                                                       const float* ranks3) {
    const int t = tensor_of(td, nt, (int)blockIdx.x);
    const BkmTensor T = td[t];
    const int64_t i0 = (int64_t)(blockIdx.x - T.blk0) * kBkmChunk;
    const int64_t i1 = i0 + kBkmChunk < T.n ? i0 + kBkmChunk : T.n;
    const float rn = ranks3[3 * t], rz = ranks3[3 * t + 1], rp = ranks3[3 * t + 2];
    const float* x = in + T.off;
    float* y = out + T.off;
    auto f = [&](float v) { return v > 0.0f ? rp : (v < 0.0f ? rn : rz); };
    if (((reinterpret_cast<uintptr_t>(x + i0) | reinterpret_cast<uintptr_t>(y + i0)) & 15u) == 0) {
        const int64_t n4 = (i1 - i0) >> 2;
        const float4* x4 = reinterpret_cast<const float4*>(x + i0);
        float4* y4 = reinterpret_cast<float4*>(y + i0);
        for (int64_t i = threadIdx.x; i < n4; i += kNT) {
            const float4 v = x4[i];
            y4[i] = make_float4(f(v.x), f(v.y), f(v.z), f(v.w));
        }
        for (int64_t i = i0 + 4 * n4 + threadIdx.x; i < i1; i += kNT) y[i] = f(x[i]);
    } else {
        for (int64_t i = i0 + threadIdx.x; i < i1; i += kNT) y[i] = f(x[i]);
    }
}
}  // namespace lossy

// ===========================================================================
// Host side
// ===========================================================================
namespace {

thread_local std::string g_lerr;
int lfail(int code, const std::string& m) { g_lerr = m; return code; }
#define LHIP(x)                                                                                       \
    do {                                                                                              \
        hipError_t e_ = (x);                                                                          \
        if (e_ != hipSuccess) return lfail(OFL_EHIP, std::string(#x " failed: ") + hipGetErrorString(e_)); \
    } while (0)

int grid_for(int64_t n) {
    int dev = 0, cus = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int64_t want = (n + lossy::kNT * 16 - 1) / (lossy::kNT * 16);
    return (int)std::max<int64_t>(1, std::min<int64_t>(want, (int64_t)cus * 8));
}

float unkey(uint32_t k) { const uint32_t u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k; float f; memcpy(&f, &u, 4); return f; }

// scratch: small device buffer carved per call (caller workspace)
struct Scratch {
    char* p; size_t left;
    template <typename T> T* take(size_t count) {
        size_t b = (sizeof(T) * count + 255) & ~(size_t)255;
        if (b > left) return nullptr;
        T* r = reinterpret_cast<T*>(p); p += b; left -= b; return r;
    }
};

lossy::KmParams km_params(const std::vector<double>& c) {
    lossy::KmParams p{};
    p.k = (int)c.size();
    for (int j = 0; j + 1 < p.k; ++j) p.mids[j] = (float)((c[j] + c[j + 1]) / 2);
    for (int j = 0; j < p.k; ++j) p.rank[j] = (float)j;
    return p;
}

}  // namespace

extern "C" {

const char* ofl_lossy_last_error(void) { return g_lerr.c_str(); }

size_t ofl_lossy_workspace_bytes(int64_t n) {
    // one-tensor k-means or top-k
    return std::max<size_t>({(size_t)1 << 20, ofl_kmeans1d_batch_workspace_bytes(1, &n),
                             ofl_sparsify_topk_batch_workspace_bytes(1, &n)});
}

// ---- batched 1-D k-means (device-resident; see the kernels above) ---------
}  // extern "C"
namespace {
struct BkmLayout {
    size_t td, st, hc, hs, part, total;
    int64_t blocks;
};
BkmLayout bkm_layout(int T, const int64_t* numels) {
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    BkmLayout L{};
    L.blocks = 0;
    for (int t = 0; t < T; ++t) L.blocks += (numels[t] + lossy::kBkmChunk - 1) / lossy::kBkmChunk;
    L.td = 0;
    L.st = L.td + al(sizeof(lossy::BkmTensor) * T);
    L.hc = L.st + al(sizeof(lossy::BkmState) * T);
    L.hs = L.hc + al(sizeof(uint32_t) * lossy::kBkmBins * T);
    L.part = L.hs + al(sizeof(unsigned long long) * lossy::kBkmBins * T);
    L.total = L.part + al(sizeof(double) * 3 * lossy::kMaxK * (size_t)std::max<int64_t>(L.blocks, 1));
    return L;
}
template <int KM1>
void bkm_launch_acc(int64_t blocks, hipStream_t st, const lossy::BkmArgs& a) {
    hipLaunchKernelGGL(lossy::k_bkm_acc<KM1>, dim3((unsigned)blocks), dim3(lossy::kBkmAccNT), 0, st, a);
}
template <int KM1>
void bkm_launch_label(int64_t blocks, hipStream_t st, const lossy::BkmArgs& a) {
    hipLaunchKernelGGL(lossy::k_bkm_label<KM1>, dim3((unsigned)blocks), dim3(lossy::kBkmAccNT), 0, st, a);
}
}  // namespace
extern "C" {

size_t ofl_kmeans1d_batch_workspace_bytes(int ntensors, const int64_t* numels) {
    if (ntensors < 1 || !numels) return 256;
    return bkm_layout(ntensors, numels).total + 256;
}

int ofl_kmeans1d_batch(int ntensors, const float* x_arena, const int64_t* offsets, const int64_t* numels, int k,
                       int n_init, uint64_t seed, int max_exact, int value_f64, float* ranks_out, double* centres,
                       int64_t* counts, double* inertia, int32_t* nuniq, double* uniq, void* ws, size_t ws_bytes,
                       void* stream) {
    return ofl_kmeans1d_batch_tab(ntensors, x_arena, offsets, numels, k, n_init, seed, max_exact, value_f64, ranks_out,
                                  nullptr, centres, counts, inertia, nuniq, uniq, ws, ws_bytes, stream);
}

int ofl_kmeans1d_batch_tab(int ntensors, const float* x_arena, const int64_t* offsets, const int64_t* numels, int k,
                           int n_init, uint64_t seed, int max_exact, int value_f64, float* ranks_out,
                           ofl_label_rec* label_tab, double* centres, int64_t* counts, double* inertia,
                           int32_t* nuniq, double* uniq, void* ws, size_t ws_bytes, void* stream) {
    if (ntensors < 1 || !x_arena || !offsets || !numels) return lfail(OFL_EINVAL, "kmeans: empty batch");
    if (label_tab) {
        if (k > 8) return lfail(OFL_EINVAL, "kmeans: label records need k <= 8");
        for (int t = 0; t < ntensors; ++t)
            if (offsets[t] < 0 || (t > 0 && offsets[t] < offsets[t - 1] + numels[t - 1]))
                return lfail(OFL_EINVAL, "kmeans: label records need ascending, non-overlapping tensors");
    }
    if (k < 1 || k > lossy::kMaxK) return lfail(OFL_EINVAL, "kmeans: need 1 <= k <= 32");
    if (n_init < 1 || n_init > lossy::kBkmMaxInit || max_exact < 0)
        return lfail(OFL_EINVAL, "kmeans: 1 <= n_init <= 16, max_exact >= 0");
    for (int t = 0; t < ntensors; ++t)
        if (numels[t] < k || numels[t] > (int64_t)lossy::kBkmChunk * 0x7fffffff)
            return lfail(OFL_EINVAL, "kmeans: need n >= k for every tensor");
    const BkmLayout L = bkm_layout(ntensors, numels);
    if (!ws || ws_bytes < L.total) return lfail(OFL_ESPACE, "kmeans: workspace too small");
    if (L.blocks > 0x7fffffff) return lfail(OFL_EINVAL, "kmeans: batch too large");
    LHIP(ofl_util::per_device_once([] {
        return hipFuncSetAttribute((const void*)lossy::k_bkm_seed, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)lossy::kBkmSeedLds);
    }));
    hipStream_t st = static_cast<hipStream_t>(stream);
    char* w = static_cast<char*>(ws);
    std::vector<lossy::BkmTensor> td(ntensors);
    int64_t blk = 0;
    for (int t = 0; t < ntensors; ++t) {
        const int64_t nb = (numels[t] + lossy::kBkmChunk - 1) / lossy::kBkmChunk;
        td[t] = {offsets[t], numels[t], (int32_t)blk, (int32_t)nb};
        blk += nb;
    }
    lossy::BkmArgs a{};
    a.x = x_arena;
    a.out = ranks_out;
    a.td = reinterpret_cast<lossy::BkmTensor*>(w + L.td);
    a.ntensors = ntensors;
    a.k = k;
    a.n_init = n_init;
    a.value_f64 = value_f64 ? 1 : 0;
    a.seed = seed;
    a.st = reinterpret_cast<lossy::BkmState*>(w + L.st);
    a.hc = reinterpret_cast<uint32_t*>(w + L.hc);
    a.hs = reinterpret_cast<unsigned long long*>(w + L.hs);
    a.part = reinterpret_cast<double*>(w + L.part);
    LHIP(hipMemcpyAsync(w + L.td, td.data(), sizeof(lossy::BkmTensor) * ntensors, hipMemcpyHostToDevice, st));
    LHIP(hipMemsetAsync(w + L.st, 0, L.part - L.st, st));  // states + histograms
    const dim3 g((unsigned)L.blocks), b(lossy::kNT);
    hipLaunchKernelGGL(lossy::k_bkm_minmax, g, b, 0, st, a);
    hipLaunchKernelGGL(lossy::k_bkm_hist, g, b, 0, st, a);
    hipLaunchKernelGGL(lossy::k_bkm_seed, dim3(ntensors * n_init), dim3(lossy::kBkmSeedNT), lossy::kBkmSeedLds, st, a);
    hipLaunchKernelGGL(lossy::k_bkm_pick, dim3((ntensors + 63) / 64), dim3(64), 0, st, a);
    for (int pass = 0; pass <= max_exact; ++pass) {
        a.final_pass = pass == max_exact;
        if (k <= 8) bkm_launch_acc<7>(L.blocks, st, a);
        else if (k <= 16) bkm_launch_acc<15>(L.blocks, st, a);
        else bkm_launch_acc<31>(L.blocks, st, a);
        hipLaunchKernelGGL(lossy::k_bkm_update, dim3(ntensors), dim3(64), 0, st, a);
    }
    if (ranks_out) {
        if (k <= 8) bkm_launch_label<7>(L.blocks, st, a);
        else if (k <= 16) bkm_launch_label<15>(L.blocks, st, a);
        else bkm_launch_label<31>(L.blocks, st, a);
    }
    if (label_tab) hipLaunchKernelGGL(lossy::k_bkm_tab, dim3((ntensors + 63) / 64), dim3(64), 0, st, a, label_tab);
    LHIP(hipGetLastError());
    std::vector<lossy::BkmState> sh(ntensors);
    LHIP(hipMemcpyAsync(sh.data(), w + L.st, sizeof(lossy::BkmState) * ntensors, hipMemcpyDeviceToHost, st));
    LHIP(hipStreamSynchronize(st));
    for (int t = 0; t < ntensors; ++t) {
        const float lo = unkey(~sh[t].mm[0]), hi = unkey(sh[t].mm[1]);
        if (!std::isfinite(lo) || !std::isfinite(hi)) return lfail(OFL_EINVAL, "kmeans: non-finite input");
        for (int j = 0; j < k; ++j) {
            if (centres) centres[(int64_t)t * k + j] = sh[t].cen[j];
            if (counts) counts[(int64_t)t * k + j] = sh[t].cnt[j];
            if (uniq) uniq[(int64_t)t * k + j] = j < sh[t].nuniq ? sh[t].uniq[j] : 0.0;
        }
        if (inertia) inertia[t] = sh[t].inertia;
        if (nuniq) nuniq[t] = sh[t].nuniq;
    }
    return OFL_OK;
}

size_t ofl_lut_decode_batch_workspace_bytes(int ntensors, int max_nk) {
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    return al(sizeof(lossy::BkmTensor) * std::max(ntensors, 1)) + al(4 * (size_t)std::max(ntensors, 1)) +
           2 * al(4 * (size_t)std::max(ntensors, 1) * std::max(max_nk, 1)) + 256;
}

int ofl_lut_decode_batch(int ntensors, const float* in_arena, const int64_t* offsets, const int64_t* numels,
                         const int32_t* nk, const float* keys, const float* vals, int max_nk, float* out_arena,
                         void* ws, size_t ws_bytes, void* stream) {
    if (ntensors < 1 || max_nk < 0 || max_nk > 64) return lfail(OFL_EINVAL, "lut: 1+ tensors, at most 64 keys");
    if (ws_bytes < ofl_lut_decode_batch_workspace_bytes(ntensors, max_nk) || !ws)
        return lfail(OFL_ESPACE, "lut: workspace too small");
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    hipStream_t st = static_cast<hipStream_t>(stream);
    char* w = static_cast<char*>(ws);
    const size_t o_nk = al(sizeof(lossy::BkmTensor) * ntensors);
    const size_t o_k = o_nk + al(4 * (size_t)ntensors);
    const size_t o_v = o_k + al(4 * (size_t)ntensors * std::max(max_nk, 1));
    std::vector<lossy::BkmTensor> td(ntensors);
    int64_t blk = 0;
    for (int t = 0; t < ntensors; ++t) {
        if (nk[t] < 0 || nk[t] > max_nk) return lfail(OFL_EINVAL, "lut: key count out of range");
        const int64_t nb = (numels[t] + lossy::kBkmChunk - 1) / lossy::kBkmChunk;
        td[t] = {offsets[t], numels[t], (int32_t)blk, (int32_t)nb};
        blk += nb;
    }
    if (blk == 0) return OFL_OK;
    LHIP(hipMemcpyAsync(w, td.data(), sizeof(lossy::BkmTensor) * ntensors, hipMemcpyHostToDevice, st));
    LHIP(hipMemcpyAsync(w + o_nk, nk, 4 * (size_t)ntensors, hipMemcpyHostToDevice, st));
    if (max_nk) {
        LHIP(hipMemcpyAsync(w + o_k, keys, 4 * (size_t)ntensors * max_nk, hipMemcpyHostToDevice, st));
        LHIP(hipMemcpyAsync(w + o_v, vals, 4 * (size_t)ntensors * max_nk, hipMemcpyHostToDevice, st));
    }
    lossy::LutBatchArgs a{in_arena, out_arena, reinterpret_cast<lossy::BkmTensor*>(w),
                          reinterpret_cast<int32_t*>(w + o_nk), reinterpret_cast<float*>(w + o_k),
                          reinterpret_cast<float*>(w + o_v), ntensors, std::max(max_nk, 1)};
    hipLaunchKernelGGL(lossy::k_lut_batch, dim3((unsigned)blk), dim3(lossy::kNT), 0, st, a);
    LHIP(hipGetLastError());
    return OFL_OK;
}

// single tensor, no labels: sorted centres, counts and inertia (replaces
// sklearn KMeans.fit in kc_pipeline.py:49-56 / skc_pipeline.py:127-131)
int ofl_kmeans1d_fit(const float* x, int64_t n, int k, int n_init, uint64_t seed, int max_exact,
                     double* centres, int64_t* counts, double* inertia, void* ws, size_t ws_bytes,
                     void* stream) {
    const int64_t off = 0;
    return ofl_kmeans1d_batch(1, x, &off, &n, k, n_init, seed, max_exact, 1, nullptr, centres, counts, inertia,
                              nullptr, nullptr, ws, ws_bytes, stream);
}

// labels as float32 values: out[i] = rank_of_cluster[nearest sorted centre]
int ofl_kmeans1d_label(const float* x, int64_t n, const double* centres, int k, const float* rank_of_cluster,
                       float* out, void* stream) {
    if (k < 1 || k > lossy::kMaxK) return lfail(OFL_EINVAL, "kmeans: bad k");
    std::vector<double> c(centres, centres + k);
    lossy::KmParams p = km_params(c);
    for (int j = 0; j < k; ++j) p.rank[j] = rank_of_cluster[j];
    hipLaunchKernelGGL(lossy::k_km_label, dim3(grid_for(n)), dim3(lossy::kNT), 0, static_cast<hipStream_t>(stream),
                       x, n, p, out);
    LHIP(hipGetLastError());
    return OFL_OK;
}

// ---- batched top-k by magnitude (kernels k_btk_*) -------------------------
}  // extern "C"
namespace {
struct BtkLayout {
    size_t td, st, hist, blk, total;
    int64_t blocks;
};
BtkLayout btk_layout(int T, const int64_t* numels) {
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    BtkLayout L{};
    for (int t = 0; t < T; ++t) L.blocks += (numels[t] + lossy::kBkmChunk - 1) / lossy::kBkmChunk;
    L.td = 0;
    L.st = L.td + al(sizeof(lossy::BkmTensor) * T);
    L.hist = L.st + al(sizeof(lossy::BtkState) * T);
    L.blk = L.hist + al(sizeof(uint32_t) * lossy::kRadix * T);
    L.total = L.blk + al(sizeof(lossy::BtkBlock) * (size_t)std::max<int64_t>(L.blocks, 1));
    return L;
}
}  // namespace
extern "C" {

size_t ofl_sparsify_topk_batch_workspace_bytes(int ntensors, const int64_t* numels) {
    if (ntensors < 1 || !numels) return 256;
    return btk_layout(ntensors, numels).total + 256;
}

int ofl_sparsify_topk_batch(int ntensors, const float* x_arena, const int64_t* offsets, const int64_t* numels,
                            const int64_t* ks, float* sparse_arena, float* kept_min, int64_t* n_pos, int64_t* n_neg,
                            int64_t* n_zero, double* abs_sum, int32_t* shifted, void* ws, size_t ws_bytes,
                            void* stream) {
    if (ntensors < 1 || !x_arena || !sparse_arena || !offsets || !numels || !ks)
        return lfail(OFL_EINVAL, "sparsify: empty batch");
    for (int t = 0; t < ntensors; ++t)
        if (ks[t] < 1 || ks[t] > numels[t] || numels[t] > (int64_t)lossy::kBkmChunk * 0x7fffffff)
            return lfail(OFL_EINVAL, "sparsify: need 1 <= k <= n");
    const BtkLayout L = btk_layout(ntensors, numels);
    if (!ws || ws_bytes < L.total) return lfail(OFL_ESPACE, "sparsify: workspace too small");
    if (L.blocks > 0x7fffffff) return lfail(OFL_EINVAL, "sparsify: batch too large");
    hipStream_t st = static_cast<hipStream_t>(stream);
    char* w = static_cast<char*>(ws);
    std::vector<lossy::BkmTensor> td(ntensors);
    std::vector<lossy::BtkState> sh(ntensors);
    int64_t blk = 0;
    for (int t = 0; t < ntensors; ++t) {
        const int64_t nb = (numels[t] + lossy::kBkmChunk - 1) / lossy::kBkmChunk;
        td[t] = {offsets[t], numels[t], (int32_t)blk, (int32_t)nb};
        blk += nb;
        sh[t] = lossy::BtkState{};
        sh[t].k = sh[t].need = ks[t];
    }
    lossy::BtkArgs a{};
    a.x = x_arena;
    a.out = sparse_arena;
    a.td = reinterpret_cast<lossy::BkmTensor*>(w + L.td);
    a.ntensors = ntensors;
    a.st = reinterpret_cast<lossy::BtkState*>(w + L.st);
    a.hist = reinterpret_cast<uint32_t*>(w + L.hist);
    a.blk = reinterpret_cast<lossy::BtkBlock*>(w + L.blk);
    LHIP(hipMemcpyAsync(w + L.td, td.data(), sizeof(lossy::BkmTensor) * ntensors, hipMemcpyHostToDevice, st));
    LHIP(hipMemcpyAsync(w + L.st, sh.data(), sizeof(lossy::BtkState) * ntensors, hipMemcpyHostToDevice, st));
    LHIP(hipMemsetAsync(w + L.hist, 0, L.blk - L.hist, st));
    const dim3 g((unsigned)L.blocks), b(lossy::kNT);
    for (int pass = 0; pass < 3; ++pass) {
        a.pass = pass;
        hipLaunchKernelGGL(lossy::k_btk_hist, g, b, 0, st, a);
        hipLaunchKernelGGL(lossy::k_btk_digit, dim3(ntensors), dim3(64), 0, st, a);
    }
    hipLaunchKernelGGL(lossy::k_btk_ties, g, b, 0, st, a);
    hipLaunchKernelGGL(lossy::k_btk_scan, dim3(ntensors), dim3(64), 0, st, a);
    hipLaunchKernelGGL(lossy::k_btk_select, g, b, 0, st, a);
    hipLaunchKernelGGL(lossy::k_btk_final, dim3(ntensors), dim3(64), 0, st, a);
    LHIP(hipGetLastError());
    LHIP(hipMemcpyAsync(sh.data(), w + L.st, sizeof(lossy::BtkState) * ntensors, hipMemcpyDeviceToHost, st));
    LHIP(hipStreamSynchronize(st));
    for (int t = 0; t < ntensors; ++t) {
        if (kept_min) kept_min[t] = sh[t].kmin;
        if (shifted) shifted[t] = sh[t].shift != 0.0f;
        if (n_pos) n_pos[t] = sh[t].n_pos;
        if (n_neg) n_neg[t] = sh[t].n_neg;
        if (n_zero) n_zero[t] = sh[t].n_zero;
        if (abs_sum) abs_sum[t] = sh[t].abs_sum;
    }
    return OFL_OK;
}

// top-k by magnitude of one tensor (skc/stc SparsityTransformer._topk_func,
// skc_pipeline.py:72-94): the batched path with T = 1.  Exact k-th largest
// |x|; ties at the threshold kept lowest index first; dense float32 sparse
// array (kept values + shift, zeros elsewhere; shift = 1e-7 iff min(kept) <
// 1e-7, :92-93) and the kept-set statistics of the ternary / k-means stages.
int ofl_sparsify_topk(const float* x, int64_t n, int64_t k, float* sparse_out, float* kept_min,
                      int64_t* n_pos, int64_t* n_neg, int64_t* n_zero, double* abs_sum, int* shifted,
                      void* ws, size_t ws_bytes, void* stream) {
    const int64_t off = 0;
    int32_t sh = 0;
    const int rc = ofl_sparsify_topk_batch(1, x, &off, &n, &k, sparse_out, kept_min, n_pos, n_neg, n_zero, abs_sum,
                                           &sh, ws, ws_bytes, stream);
    if (rc == OFL_OK && shifted) *shifted = sh;
    return rc;
}

size_t ofl_ternary_ranks_batch_workspace_bytes(int ntensors) {
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    return al(sizeof(lossy::BkmTensor) * std::max(ntensors, 1)) + al(12 * (size_t)std::max(ntensors, 1)) + 256;
}

int ofl_ternary_ranks_batch(int ntensors, const float* sparse_arena, const int64_t* offsets, const int64_t* numels,
                            const float* ranks3, float* out_arena, void* ws, size_t ws_bytes, void* stream) {
    if (ntensors < 1 || !offsets || !numels || !ranks3) return lfail(OFL_EINVAL, "ternary: empty batch");
    if (!ws || ws_bytes < ofl_ternary_ranks_batch_workspace_bytes(ntensors))
        return lfail(OFL_ESPACE, "ternary: workspace too small");
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    hipStream_t st = static_cast<hipStream_t>(stream);
    char* w = static_cast<char*>(ws);
    const size_t o_r = al(sizeof(lossy::BkmTensor) * ntensors);
    std::vector<lossy::BkmTensor> td(ntensors);
    int64_t blk = 0;
    for (int t = 0; t < ntensors; ++t) {
        const int64_t nb = (numels[t] + lossy::kBkmChunk - 1) / lossy::kBkmChunk;
        td[t] = {offsets[t], numels[t], (int32_t)blk, (int32_t)nb};
        blk += nb;
    }
    if (blk == 0) return OFL_OK;
    if (blk > 0x7fffffff) return lfail(OFL_EINVAL, "ternary: batch too large");
    LHIP(hipMemcpyAsync(w, td.data(), sizeof(lossy::BkmTensor) * ntensors, hipMemcpyHostToDevice, st));
    LHIP(hipMemcpyAsync(w + o_r, ranks3, 12 * (size_t)ntensors, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(lossy::k_ternary_batch, dim3((unsigned)blk), dim3(lossy::kNT), 0, st, sparse_arena, out_arena,
                       reinterpret_cast<lossy::BkmTensor*>(w), ntensors, reinterpret_cast<float*>(w + o_r));
    LHIP(hipGetLastError());
    return OFL_OK;
}

int ofl_ternary_stats(const float* x, int64_t n, int64_t* n_pos, int64_t* n_neg, double* abs_sum, void* ws,
                      size_t ws_bytes, void* stream) {
    hipStream_t st = static_cast<hipStream_t>(stream);
    Scratch sc{static_cast<char*>(ws), ws_bytes};
    const int grid = grid_for(n), nw = grid * (lossy::kNT / 64);
    unsigned long long* c = sc.take<unsigned long long>(2);
    double* a = sc.take<double>(1);
    unsigned long long* cp = sc.take<unsigned long long>(2 * (size_t)nw);
    double* ap = sc.take<double>((size_t)nw);
    if (!c || !a || !cp || !ap) return lfail(OFL_ESPACE, "ternary: workspace too small");
    hipLaunchKernelGGL(lossy::k_tstats, dim3(grid), dim3(lossy::kNT), 0, st, x, n, cp, ap);
    hipLaunchKernelGGL(lossy::k_tstats_final, dim3(1), dim3(64), 0, st, cp, ap, nw, c, a);
    unsigned long long ch[2];
    LHIP(hipMemcpyAsync(ch, c, 16, hipMemcpyDeviceToHost, st));
    LHIP(hipMemcpyAsync(abs_sum, a, 8, hipMemcpyDeviceToHost, st));
    LHIP(hipStreamSynchronize(st));
    *n_pos = (int64_t)ch[0];
    *n_neg = (int64_t)ch[1];
    return OFL_OK;
}

int ofl_ternary_ranks(const float* sparse, int64_t n, float rank_neg, float rank_zero, float rank_pos, float* out,
                      void* stream) {
    hipLaunchKernelGGL(lossy::k_ternary, dim3(grid_for(n)), dim3(lossy::kNT), 0, static_cast<hipStream_t>(stream),
                       sparse, n, rank_neg, rank_zero, rank_pos, out);
    LHIP(hipGetLastError());
    return OFL_OK;
}

// in-place sequential key -> value replacement of the reference backward,
// emulated per element (kc_pipeline.py:81-83, stc_pipeline.py:139-142)
int ofl_lut_decode(const float* in, int64_t n, const float* keys, const float* vals, int nk, float* out,
                   void* stream) {
    if (nk < 0 || nk > 64) return lfail(OFL_EINVAL, "lut: at most 64 keys");
    lossy::LutParams p{};
    p.nk = nk;
    for (int j = 0; j < nk; ++j) { p.key[j] = keys[j]; p.val[j] = vals[j]; }
    hipLaunchKernelGGL(lossy::k_lut, dim3(grid_for(n)), dim3(lossy::kNT), 0, static_cast<hipStream_t>(stream),
                       in, n, p, out);
    LHIP(hipGetLastError());
    return OFL_OK;
}

}  // extern "C"
