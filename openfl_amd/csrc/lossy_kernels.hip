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
#include <random>
#include <string>
#include <vector>

#include "ofl_codec.h"

#define DEVI __device__ __forceinline__

namespace lossy {

constexpr int kNT = 256;
constexpr int kHistBins = 4096;   // k-means histogram resolution
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

// ---- min / max (NaN-free input assumed by callers; NaN propagates as max) --
__global__ __launch_bounds__(kNT) void k_minmax(const float* x, int64_t n, uint32_t* out) {
    float lo = INFINITY, hi = -INFINITY;
    for (int64_t i = gtid(); i < n; i += gstride()) { const float v = x[i]; lo = fminf(lo, v); hi = fmaxf(hi, v); }
    lo = wave_min(lo);
    hi = wave_max(hi);
    if ((threadIdx.x & 63) == 0) { atomicMin(&out[0], fkey(lo)); atomicMax(&out[1], fkey(hi)); }
}

// ---- value histogram: count + fp64 sum per bin over [lo, lo + nb/inv_w) ----
__global__ __launch_bounds__(kNT) void k_hist(const float* x, int64_t n, float lo, float inv_w,
                                              unsigned long long* cnt, double* sum) {
    __shared__ unsigned int c[kHistBins];
    __shared__ double s[kHistBins];
    for (int b = threadIdx.x; b < kHistBins; b += kNT) { c[b] = 0; s[b] = 0.0; }
    __syncthreads();
    for (int64_t i = gtid(); i < n; i += gstride()) {
        const float v = x[i];
        int b = (int)((v - lo) * inv_w);
        b = b < 0 ? 0 : (b >= kHistBins ? kHistBins - 1 : b);
        atomicAdd(&c[b], 1u);
        atomicAdd(&s[b], (double)v);
    }
    __syncthreads();
    for (int b = threadIdx.x; b < kHistBins; b += kNT) {
        if (c[b]) { atomicAdd(&cnt[b], (unsigned long long)c[b]); atomicAdd(&sum[b], s[b]); }
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

// ---- exact Lloyd statistics: per-cluster count, fp64 sum and sum of squares --
__global__ __launch_bounds__(kNT) void k_km_accum(const float* x, int64_t n, KmParams p,
                                                  unsigned long long* cnt, double* sum, double* sq) {
    __shared__ unsigned int c[kMaxK];
    __shared__ double s[kMaxK], q[kMaxK];
    if (threadIdx.x < kMaxK) { c[threadIdx.x] = 0; s[threadIdx.x] = 0.0; q[threadIdx.x] = 0.0; }
    __syncthreads();
    for (int64_t i = gtid(); i < n; i += gstride()) {
        const float v = x[i];
        const int k = cluster_of(v, p);
        atomicAdd(&c[k], 1u);
        atomicAdd(&s[k], (double)v);
        atomicAdd(&q[k], (double)v * (double)v);
    }
    __syncthreads();
    if (threadIdx.x < p.k && c[threadIdx.x]) {
        atomicAdd(&cnt[threadIdx.x], (unsigned long long)c[threadIdx.x]);
        atomicAdd(&sum[threadIdx.x], s[threadIdx.x]);
        atomicAdd(&sq[threadIdx.x], q[threadIdx.x]);
    }
}

// ---- labels -> float32 ranks -------------------------------------------------
__global__ __launch_bounds__(kNT) void k_km_label(const float* x, int64_t n, KmParams p, float* out) {
    for (int64_t i = gtid(); i < n; i += gstride()) out[i] = p.rank[cluster_of(x[i], p)];
}

// ---- radix select on |x| bits (float32 magnitudes order like their bits) ----
// digit d of the 31 magnitude bits: pass 0 -> bits [20,31), 1 -> [9,20), 2 -> [0,9)
__global__ __launch_bounds__(kNT) void k_abs_radix(const float* x, int64_t n, uint32_t prefix,
                                                   uint32_t prefix_mask, int shift, uint32_t digit_mask,
                                                   uint32_t* hist) {
    __shared__ uint32_t h[kRadix];
    for (int b = threadIdx.x; b < kRadix; b += kNT) h[b] = 0;
    __syncthreads();
    for (int64_t i = gtid(); i < n; i += gstride()) {
        const uint32_t m = __float_as_uint(x[i]) & 0x7fffffffu;
        if ((m & prefix_mask) == prefix) atomicAdd(&h[(m >> shift) & digit_mask], 1u);
    }
    __syncthreads();
    for (int b = threadIdx.x; b < kRadix; b += kNT) if (h[b]) atomicAdd(&hist[b], h[b]);
}

// per-block count of elements with |x| bits == T (tie rank by index)
__global__ __launch_bounds__(kNT) void k_tie_count(const float* x, int64_t n, int64_t per_block, uint32_t T,
                                                   uint32_t* block_ties) {
    const int64_t b0 = (int64_t)blockIdx.x * per_block, b1 = std::min<int64_t>(n, b0 + per_block);
    uint32_t c = 0;
    for (int64_t i = b0 + threadIdx.x; i < b1; i += kNT) c += ((__float_as_uint(x[i]) & 0x7fffffffu) == T) ? 1u : 0u;
    c = wave_sum(c);
    if ((threadIdx.x & 63) == 0) atomicAdd(&block_ties[blockIdx.x], c);
}

// kept-element flag for element i of block b (ties kept lowest index first):
// |x| > T, or |x| == T and its index rank among ties < tie_keep.  The in-block
// tie rank needs an ordered scan: each block walks its range in kNT-chunks.
struct SelParams {
    uint32_t T;
    int64_t tie_keep;     // how many |x| == T elements are kept (lowest index)
    int64_t per_block;
    float shift;          // 1e-7 or 0 added to kept values (skc_pipeline.py:92-93)
};

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

// stats of the kept set after the shift: min kept value (pre-shift), counts of
// kept values that end up > 0, < 0, == 0, and fp64 sum of |kept + shift|
__global__ __launch_bounds__(kNT) void k_select(const float* x, int64_t n, SelParams sp, const uint64_t* tie_base,
                                                float* sparse_out, float* kmin, unsigned long long* counts,
                                                double* abs_sum) {
    __shared__ uint32_t tmp[kNT / 64];
    const int64_t b0 = (int64_t)blockIdx.x * sp.per_block, b1 = std::min<int64_t>(n, b0 + sp.per_block);
    int64_t ties = (int64_t)tie_base[blockIdx.x];
    float mn = INFINITY;
    uint32_t cpos = 0, cneg = 0, czero = 0;
    double as = 0.0;
    for (int64_t base = b0; base < b1; base += kNT) {
        const int64_t i = base + threadIdx.x;
        const bool in = i < b1;
        const float v = in ? x[i] : 0.0f;
        const uint32_t m = __float_as_uint(v) & 0x7fffffffu;
        const uint32_t tie = (in && m == sp.T) ? 1u : 0u;
        uint32_t tot;
        const uint32_t rank = block_excl_scan(tie, tmp, tot);
        const bool keep = in && (m > sp.T || (tie && ties + (int64_t)rank < sp.tie_keep));
        ties += tot;
        float outv = 0.0f;
        if (keep) {
            mn = fminf(mn, v);
            outv = v + sp.shift;  // float32 add (NEP 50: python float is weak)
            cpos += outv > 0.0f;
            cneg += outv < 0.0f;
            czero += outv == 0.0f;
            as += fabs((double)outv);
        }
        if (sparse_out && in) sparse_out[i] = outv;
    }
    mn = wave_min(mn);
    cpos = wave_sum(cpos); cneg = wave_sum(cneg); czero = wave_sum(czero);
    as = wave_sum(as);
    if ((threadIdx.x & 63) == 0) {
        atomicMin(reinterpret_cast<uint32_t*>(kmin), fkey(mn));
        atomicAdd(&counts[0], (unsigned long long)cpos);
        atomicAdd(&counts[1], (unsigned long long)cneg);
        atomicAdd(&counts[2], (unsigned long long)czero);
        atomicAdd(abs_sum, as);
    }
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
__global__ __launch_bounds__(kNT) void k_tstats(const float* x, int64_t n, unsigned long long* cnt, double* abs_sum) {
    uint32_t cp = 0, cn = 0;
    double as = 0.0;
    for (int64_t i = gtid(); i < n; i += gstride()) {
        const float v = x[i];
        cp += v > 0.0f;
        cn += v < 0.0f;
        as += fabs((double)v);
    }
    cp = wave_sum(cp); cn = wave_sum(cn); as = wave_sum(as);
    if ((threadIdx.x & 63) == 0) { atomicAdd(&cnt[0], (unsigned long long)cp); atomicAdd(&cnt[1], (unsigned long long)cn); atomicAdd(abs_sum, as); }
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

double weighted_inertia(const std::vector<double>& c, const std::vector<double>& w, const std::vector<double>& m,
                        const std::vector<double>& q) {
    // sum over bins of sum_{x in bin} (x - c_nearest)^2 using count/sum/sumsq per bin
    double tot = 0.0;
    const int k = (int)c.size();
    for (size_t b = 0; b < w.size(); ++b) {
        if (w[b] == 0) continue;
        const double mu = m[b] / w[b];
        int best = 0; double bd = std::abs(mu - c[0]);
        for (int j = 1; j < k; ++j) { double d = std::abs(mu - c[j]); if (d < bd) { bd = d; best = j; } }
        tot += q[b] - 2 * c[best] * m[b] + w[b] * c[best] * c[best];
    }
    return tot;
}

// Lloyd on weighted 1-D points (bin means), from k-means++ seeding; returns centres
std::vector<double> km_hist(const std::vector<double>& pts, const std::vector<double>& wts, int k, int n_init,
                            uint64_t seed, int max_iter) {
    std::mt19937_64 rng(seed);
    std::vector<int> nz;
    for (size_t i = 0; i < pts.size(); ++i) if (wts[i] > 0) nz.push_back((int)i);
    std::vector<double> best;
    double best_in = std::numeric_limits<double>::infinity();
    const int trials = 2 + (int)std::log((double)k);  // sklearn's n_local_trials
    for (int run = 0; run < n_init; ++run) {
        std::vector<double> c;
        // k-means++ (weighted)
        std::discrete_distribution<int> pick0(wts.begin(), wts.end());
        c.push_back(pts[pick0(rng)]);
        std::vector<double> d2(pts.size());
        for (size_t i = 0; i < pts.size(); ++i) d2[i] = (pts[i] - c[0]) * (pts[i] - c[0]);
        while ((int)c.size() < k) {
            double pot = 0.0;
            std::vector<double> pw(pts.size());
            for (size_t i = 0; i < pts.size(); ++i) { pw[i] = wts[i] * d2[i]; pot += pw[i]; }
            if (!(pot > 0)) { c.push_back(pts[nz[rng() % nz.size()]]); continue; }
            std::discrete_distribution<int> pk(pw.begin(), pw.end());
            int bestc = -1; double bestpot = std::numeric_limits<double>::infinity();
            for (int t = 0; t < trials; ++t) {
                const int cand = pk(rng);
                double np = 0.0;
                for (size_t i = 0; i < pts.size(); ++i) {
                    const double d = pts[i] - pts[cand];
                    np += wts[i] * std::min(d2[i], d * d);
                }
                if (np < bestpot) { bestpot = np; bestc = cand; }
            }
            c.push_back(pts[bestc]);
            for (size_t i = 0; i < pts.size(); ++i) { const double d = pts[i] - pts[bestc]; d2[i] = std::min(d2[i], d * d); }
        }
        std::sort(c.begin(), c.end());
        // Lloyd
        for (int it = 0; it < max_iter; ++it) {
            std::vector<double> sw(k, 0.0), sx(k, 0.0);
            for (size_t i = 0; i < pts.size(); ++i) {
                if (wts[i] == 0) continue;
                int j = 0;
                while (j + 1 < k && (c[j] + c[j + 1]) / 2 < pts[i]) ++j;
                sw[j] += wts[i]; sx[j] += wts[i] * pts[i];
            }
            double shift = 0.0;
            for (int j = 0; j < k; ++j) if (sw[j] > 0) { const double nc = sx[j] / sw[j]; shift += (nc - c[j]) * (nc - c[j]); c[j] = nc; }
            std::sort(c.begin(), c.end());
            if (shift == 0.0) break;
        }
        double in = 0.0;
        for (size_t i = 0; i < pts.size(); ++i) {
            if (wts[i] == 0) continue;
            double bd = std::numeric_limits<double>::infinity();
            for (int j = 0; j < k; ++j) bd = std::min(bd, (pts[i] - c[j]) * (pts[i] - c[j]));
            in += wts[i] * bd;
        }
        if (in < best_in) { best_in = in; best = c; }
    }
    return best;
}

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
    (void)n;
    return 1 << 20;  // histograms, counters, per-block tie counts (<= 2048 blocks)
}

// 1-D k-means of x (n fp32 on device): k-means++ (n_init restarts) + Lloyd on a
// 4096-bin histogram, then exact Lloyd passes on the data until the
// assignment is stable (or max_exact passes).  Outputs the sorted centres
// (host doubles, k of them; empty clusters keep their histogram position),
// per-cluster counts and the exact inertia.  Replaces sklearn KMeans.fit in
// kc_pipeline.py:49-56 / skc_pipeline.py:127-131.
int ofl_kmeans1d_fit(const float* x, int64_t n, int k, int n_init, uint64_t seed, int max_exact,
                     double* centres, int64_t* counts, double* inertia, void* ws, size_t ws_bytes,
                     void* stream) {
    if (k < 1 || k > lossy::kMaxK || n < k) return lfail(OFL_EINVAL, "kmeans: need 1 <= k <= 32 and n >= k");
    hipStream_t st = static_cast<hipStream_t>(stream);
    Scratch sc{static_cast<char*>(ws), ws_bytes};
    uint32_t* mm = sc.take<uint32_t>(2);
    unsigned long long* hc = sc.take<unsigned long long>(lossy::kHistBins);
    double* hs = sc.take<double>(lossy::kHistBins);
    unsigned long long* kc = sc.take<unsigned long long>(lossy::kMaxK);
    double* ks = sc.take<double>(lossy::kMaxK);
    double* kq = sc.take<double>(lossy::kMaxK);
    if (!kq) return lfail(OFL_ESPACE, "kmeans: workspace too small");
    const int g = grid_for(n);
    const uint32_t init[2] = {0xffffffffu, 0u};
    LHIP(hipMemcpyAsync(mm, init, 8, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(lossy::k_minmax, dim3(g), dim3(lossy::kNT), 0, st, x, n, mm);
    uint32_t mmh[2];
    LHIP(hipMemcpyAsync(mmh, mm, 8, hipMemcpyDeviceToHost, st));
    LHIP(hipStreamSynchronize(st));
    const float lo = unkey(mmh[0]), hi = unkey(mmh[1]);
    if (!std::isfinite(lo) || !std::isfinite(hi)) return lfail(OFL_EINVAL, "kmeans: non-finite input");
    std::vector<double> c;
    if (hi > lo) {
        const float inv_w = (float)(lossy::kHistBins / ((double)hi - (double)lo) * (1.0 - 1e-7));
        LHIP(hipMemsetAsync(hc, 0, 8 * lossy::kHistBins, st));
        LHIP(hipMemsetAsync(hs, 0, 8 * lossy::kHistBins, st));
        hipLaunchKernelGGL(lossy::k_hist, dim3(g), dim3(lossy::kNT), 0, st, x, n, lo, inv_w, hc, hs);
        std::vector<unsigned long long> hch(lossy::kHistBins);
        std::vector<double> hsh(lossy::kHistBins);
        LHIP(hipMemcpyAsync(hch.data(), hc, 8 * lossy::kHistBins, hipMemcpyDeviceToHost, st));
        LHIP(hipMemcpyAsync(hsh.data(), hs, 8 * lossy::kHistBins, hipMemcpyDeviceToHost, st));
        LHIP(hipStreamSynchronize(st));
        std::vector<double> pts, wts;
        for (int b = 0; b < lossy::kHistBins; ++b)
            if (hch[b]) { pts.push_back(hsh[b] / (double)hch[b]); wts.push_back((double)hch[b]); }
        int distinct = (int)pts.size();
        if (distinct <= k) {  // fewer occupied bins than clusters: seed on them directly
            c = pts;
            while ((int)c.size() < k) c.push_back(c.back());
        } else {
            c = km_hist(pts, wts, k, n_init, seed, 300);
        }
    } else {
        c.assign(k, (double)lo);
    }
    // exact Lloyd refinement on the full data
    std::vector<unsigned long long> cnt(k);
    std::vector<double> sum(k), sq(k);
    for (int pass = 0; pass <= max_exact; ++pass) {
        const lossy::KmParams p = km_params(c);
        LHIP(hipMemsetAsync(kc, 0, 8 * lossy::kMaxK, st));
        LHIP(hipMemsetAsync(ks, 0, 8 * lossy::kMaxK, st));
        LHIP(hipMemsetAsync(kq, 0, 8 * lossy::kMaxK, st));
        hipLaunchKernelGGL(lossy::k_km_accum, dim3(g), dim3(lossy::kNT), 0, st, x, n, p, kc, ks, kq);
        LHIP(hipMemcpyAsync(cnt.data(), kc, 8 * k, hipMemcpyDeviceToHost, st));
        LHIP(hipMemcpyAsync(sum.data(), ks, 8 * k, hipMemcpyDeviceToHost, st));
        LHIP(hipMemcpyAsync(sq.data(), kq, 8 * k, hipMemcpyDeviceToHost, st));
        LHIP(hipStreamSynchronize(st));
        if (pass == max_exact) break;
        std::vector<double> nc = c;
        for (int j = 0; j < k; ++j) if (cnt[j]) nc[j] = sum[j] / (double)cnt[j];
        std::sort(nc.begin(), nc.end());
        // stable when the float32 midpoints (the assignment) do not change
        const lossy::KmParams pn = km_params(nc);
        bool same = true;
        for (int j = 0; j + 1 < k; ++j) same = same && pn.mids[j] == p.mids[j];
        c = nc;
        if (same) { pass = max_exact - 1; }  // one more accumulate for final stats
    }
    double in = 0.0;
    for (int j = 0; j < k; ++j) {
        centres[j] = c[j];
        if (counts) counts[j] = (int64_t)cnt[j];
        in += sq[j] - 2 * c[j] * sum[j] + (double)cnt[j] * c[j] * c[j];
    }
    if (inertia) *inertia = std::max(0.0, in);
    return OFL_OK;
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

// top-k by magnitude (skc/stc SparsityTransformer._topk_func, skc_pipeline.py:72-94):
// exact k-th largest |x| by 3-pass radix select; ties at the threshold are
// kept lowest index first.  Writes the dense float32 sparse array (kept values
// + shift, zeros elsewhere; shift = 1e-7 iff min(kept) < 1e-7, :92-93) and
// returns the kept-set statistics used by the ternary / k-means stages.
int ofl_sparsify_topk(const float* x, int64_t n, int64_t k, float* sparse_out, float* kept_min,
                      int64_t* n_pos, int64_t* n_neg, int64_t* n_zero, double* abs_sum, int* shifted,
                      void* ws, size_t ws_bytes, void* stream) {
    if (k < 1 || k > n) return lfail(OFL_EINVAL, "sparsify: need 1 <= k <= n");
    hipStream_t st = static_cast<hipStream_t>(stream);
    Scratch sc{static_cast<char*>(ws), ws_bytes};
    uint32_t* hist = sc.take<uint32_t>(lossy::kRadix);
    const int g = grid_for(n);
    const int64_t per_block = (n + g - 1) / g;
    uint32_t* bt = sc.take<uint32_t>(g);
    uint64_t* tb = sc.take<uint64_t>(g);
    uint32_t* kmin = sc.take<uint32_t>(1);
    unsigned long long* cnts = sc.take<unsigned long long>(3);
    double* as = sc.take<double>(1);
    if (!as) return lfail(OFL_ESPACE, "sparsify: workspace too small");
    // radix select: the k-th largest magnitude (31 bits: 11 + 11 + 9)
    uint32_t prefix = 0, pmask = 0;
    int64_t need = k;  // rank from the top within the current prefix
    const int shifts[3] = {20, 9, 0};
    const int widths[3] = {11, 11, 9};
    std::vector<uint32_t> h(lossy::kRadix);
    for (int pass = 0; pass < 3; ++pass) {
        LHIP(hipMemsetAsync(hist, 0, 4 * lossy::kRadix, st));
        hipLaunchKernelGGL(lossy::k_abs_radix, dim3(g), dim3(lossy::kNT), 0, st, x, n, prefix, pmask, shifts[pass],
                           (uint32_t)((1 << widths[pass]) - 1), hist);
        LHIP(hipMemcpyAsync(h.data(), hist, 4 * lossy::kRadix, hipMemcpyDeviceToHost, st));
        LHIP(hipStreamSynchronize(st));
        const int nb = 1 << widths[pass];
        int d = nb - 1;
        for (; d > 0; --d) { if ((int64_t)h[d] >= need) break; need -= h[d]; }
        prefix |= (uint32_t)d << shifts[pass];
        pmask |= (uint32_t)(nb - 1) << shifts[pass];
    }
    const uint32_t T = prefix;  // exact bits of the k-th largest |x|; `need` ties at T are kept
    // per-block tie counts -> exclusive prefix (host)
    LHIP(hipMemsetAsync(bt, 0, 4 * g, st));
    hipLaunchKernelGGL(lossy::k_tie_count, dim3(g), dim3(lossy::kNT), 0, st, x, n, per_block, T, bt);
    std::vector<uint32_t> bth(g);
    LHIP(hipMemcpyAsync(bth.data(), bt, 4 * g, hipMemcpyDeviceToHost, st));
    LHIP(hipStreamSynchronize(st));
    std::vector<uint64_t> tbh(g);
    uint64_t acc = 0;
    for (int b = 0; b < g; ++b) { tbh[b] = acc; acc += bth[b]; }
    LHIP(hipMemcpyAsync(tb, tbh.data(), 8 * g, hipMemcpyHostToDevice, st));
    lossy::SelParams sp{T, need, per_block, 0.0f};
    // pass 1: kept min (decides the shift); pass 2: with the shift, write + stats
    for (int pass = 0; pass < 2; ++pass) {
        const uint32_t kinit = 0xffffffffu;
        LHIP(hipMemcpyAsync(kmin, &kinit, 4, hipMemcpyHostToDevice, st));
        LHIP(hipMemsetAsync(cnts, 0, 24, st));
        LHIP(hipMemsetAsync(as, 0, 8, st));
        hipLaunchKernelGGL(lossy::k_select, dim3(g), dim3(lossy::kNT), 0, st, x, n, sp, tb,
                           pass == 1 ? sparse_out : nullptr, reinterpret_cast<float*>(kmin), cnts, as);
        uint32_t km;
        unsigned long long ch[3];
        double ash;
        LHIP(hipMemcpyAsync(&km, kmin, 4, hipMemcpyDeviceToHost, st));
        LHIP(hipMemcpyAsync(ch, cnts, 24, hipMemcpyDeviceToHost, st));
        LHIP(hipMemcpyAsync(&ash, as, 8, hipMemcpyDeviceToHost, st));
        LHIP(hipStreamSynchronize(st));
        const float mn = unkey(km);
        if (pass == 0) {
            // reference: `if min(topk_mag) - 0 < 10e-8: topk_mag = topk_mag + 10e-8`
            sp.shift = ((double)mn < 10e-8) ? (float)10e-8 : 0.0f;
            if (kept_min) *kept_min = mn;
            if (shifted) *shifted = sp.shift != 0.0f;
        } else {
            if (n_pos) *n_pos = (int64_t)ch[0];
            if (n_neg) *n_neg = (int64_t)ch[1];
            if (n_zero) *n_zero = (int64_t)ch[2];
            if (abs_sum) *abs_sum = ash;
        }
    }
    return OFL_OK;
}

int ofl_ternary_stats(const float* x, int64_t n, int64_t* n_pos, int64_t* n_neg, double* abs_sum, void* ws,
                      size_t ws_bytes, void* stream) {
    hipStream_t st = static_cast<hipStream_t>(stream);
    Scratch sc{static_cast<char*>(ws), ws_bytes};
    unsigned long long* c = sc.take<unsigned long long>(2);
    double* a = sc.take<double>(1);
    if (!a) return lfail(OFL_ESPACE, "ternary: workspace too small");
    LHIP(hipMemsetAsync(c, 0, 16, st));
    LHIP(hipMemsetAsync(a, 0, 8, st));
    hipLaunchKernelGGL(lossy::k_tstats, dim3(grid_for(n)), dim3(lossy::kNT), 0, st, x, n, c, a);
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
