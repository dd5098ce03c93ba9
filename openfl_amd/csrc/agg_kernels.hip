// agg_kernels.hip -- the aggregator's end-of-round arithmetic around the codec
// (reference: /root/reference/openfl):
//   interface/aggregation_functions/weighted_average.py:12-14
//       np.average(tensors, weights=weights, axis=0)
//   pipelines/tensor_codec.py:150-211  generate_delta (new - base),
//                                      apply_delta (base + delta)
//   component/aggregator/aggregator.py:780-865  _prepare_trained: average ->
//       delta -> compress -> decompress -> apply, per tensor
//
// Bit-exact with NumPy: np.average promotes to float64, multiplies every
// collaborator's tensor by its weight (one rounding), sums the products over
// the collaborator axis in order (axis-0 reductions accumulate row by row,
// starting from the first row), divides by the float64 sum of the weights
// (computed on the host with NumPy), then generate_delta subtracts the float32
// base in float64.  FMA contraction is disabled in these kernels so that every
// product and sum is rounded exactly as NumPy rounds it.  The codec then sees
// the delta rounded to float32 (torch.Tensor(float64 array), Eden.compress
// :579); apply_delta is a float32 add of the decoded delta.
//
// All tensors of a model update live in one flat arena; the kernels are
// elementwise over it (16-B vector I/O where the arena is aligned).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>

#include "ofl_codec.h"

namespace agg {

constexpr int kNT = 256;
constexpr int kMaxC = 16;  // collaborators per launch (more: chained through agg_out)

struct WavgArgs {
    const float* x[kMaxC];
    double w[kMaxC];
    int nc;            // collaborators in this launch
    int first, last;   // first launch starts from the first product; last divides
    double wsum;       // float64 sum of all weights (NumPy's)
    const float* base; // nullable: delta = average when absent
    double* acc;       // nullable unless chained: running float64 sums / average
    double* delta64;   // nullable
    float* delta32;    // nullable
    int64_t n;
};

// running sum over this launch's collaborators, continuing from s0 (first
// launch: from the first product) -- the sequence NumPy performs, rounded
// after every operation
__device__ __forceinline__ double wavg_sum(const WavgArgs& a, int64_t i, double s0) {
#pragma clang fp contract(off)
    double s = a.first ? (double)a.x[0][i] * a.w[0] : s0;
    for (int c = a.first ? 1 : 0; c < a.nc; ++c) s = s + (double)a.x[c][i] * a.w[c];
    return s;
}
__device__ __forceinline__ double wavg_delta(const WavgArgs& a, int64_t i, double s, double& avg) {
#pragma clang fp contract(off)
    avg = s / a.wsum;
    return a.base ? avg - (double)a.base[i] : avg;
}

__device__ __forceinline__ void wavg_elem(const WavgArgs& a, int64_t i) {
    const double s = wavg_sum(a, i, a.first ? 0.0 : a.acc[i]);
    if (!a.last) { a.acc[i] = s; return; }
    double avg;
    const double d = wavg_delta(a, i, s, avg);
    if (a.acc) a.acc[i] = avg;
    if (a.delta64) a.delta64[i] = d;
    if (a.delta32) a.delta32[i] = (float)d;
}

// 4 consecutive elements per thread: 16-B loads of every collaborator's
// tensor (the kernel reads 4 C + 4 bytes and writes 4 per element)
__device__ __forceinline__ void wavg_quad(const WavgArgs& a, int64_t i) {
#pragma clang fp contract(off)
    double s[4];
    if (a.first) {
        const float4 v = *reinterpret_cast<const float4*>(a.x[0] + i);
        s[0] = (double)v.x * a.w[0]; s[1] = (double)v.y * a.w[0];
        s[2] = (double)v.z * a.w[0]; s[3] = (double)v.w * a.w[0];
    } else {
        for (int k = 0; k < 4; ++k) s[k] = a.acc[i + k];
    }
    for (int c = a.first ? 1 : 0; c < a.nc; ++c) {
        const float4 v = *reinterpret_cast<const float4*>(a.x[c] + i);
        const double w = a.w[c];
        s[0] = s[0] + (double)v.x * w; s[1] = s[1] + (double)v.y * w;
        s[2] = s[2] + (double)v.z * w; s[3] = s[3] + (double)v.w * w;
    }
    if (!a.last) {
        for (int k = 0; k < 4; ++k) a.acc[i + k] = s[k];
        return;
    }
    float4 b = make_float4(0.f, 0.f, 0.f, 0.f);
    if (a.base) b = *reinterpret_cast<const float4*>(a.base + i);
    const float bb[4] = {b.x, b.y, b.z, b.w};
    double d[4];
    for (int k = 0; k < 4; ++k) {
        const double avg = s[k] / a.wsum;
        if (a.acc) a.acc[i + k] = avg;
        d[k] = a.base ? avg - (double)bb[k] : avg;
    }
    if (a.delta64)
        for (int k = 0; k < 4; ++k) a.delta64[i + k] = d[k];
    if (a.delta32) *reinterpret_cast<float4*>(a.delta32 + i) = make_float4((float)d[0], (float)d[1], (float)d[2], (float)d[3]);
}

__global__ __launch_bounds__(kNT) void k_wavg_delta(WavgArgs a, int vec) {
    const int64_t stride = (int64_t)gridDim.x * kNT;
    const int64_t t0 = (int64_t)blockIdx.x * kNT + threadIdx.x;
    int64_t tail = 0;
    if (vec) {
        const int64_t n4 = a.n >> 2;
        for (int64_t q = t0; q < n4; q += stride) wavg_quad(a, 4 * q);
        tail = 4 * n4;
    }
    for (int64_t i = tail + t0; i < a.n; i += stride) wavg_elem(a, i);
}

// Single-element tensors: NumPy reduces a (C, 1) stack as a 1-D array, i.e.
// pairwise_sum of all C products (numpy/_core/src/umath/loops_utils.h.src:
// < 8 terms summed from +0.0; up to 128 with eight
// accumulators combined ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) then the tail;
// larger blocks split in halves rounded down to a multiple of 8).
struct PointArgs {
    const float* const* x;  // device [nc]
    const double* w;        // device [nc]
    int nc;
    double wsum;
    const float* base;
    const int64_t* idx;     // device [np]
    int np;
    double* acc;
    double* delta64;
    float* delta32;
};
__device__ double np_pairwise(const PointArgs& a, int64_t i, int c0, int n) {
#pragma clang fp contract(off)
    auto p = [&](int c) { return (double)a.x[c][i] * a.w[c]; };
    if (n < 8) {
        double r = 0.0;
        for (int k = 0; k < n; ++k) r = r + p(c0 + k);
        return r;
    }
    if (n <= 128) {
        double r[8];
        for (int k = 0; k < 8; ++k) r[k] = p(c0 + k);
        int k = 8;
        for (; k < n - (n % 8); k += 8)
            for (int j = 0; j < 8; ++j) r[j] = r[j] + p(c0 + k + j);
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; k < n; ++k) res = res + p(c0 + k);
        return res;
    }
    int n2 = n / 2;
    n2 -= n2 % 8;
    return np_pairwise(a, i, c0, n2) + np_pairwise(a, i, c0 + n2, n - n2);
}
__global__ __launch_bounds__(64) void k_wavg_points(PointArgs a) {
#pragma clang fp contract(off)
    for (int j = blockIdx.x * 64 + threadIdx.x; j < a.np; j += gridDim.x * 64) {
        const int64_t i = a.idx[j];
        const double s = np_pairwise(a, i, 0, a.nc);
        const double avg = s / a.wsum;
        if (a.acc) a.acc[i] = avg;
        const double d = a.base ? avg - (double)a.base[i] : avg;
        if (a.delta64) a.delta64[i] = d;
        if (a.delta32) a.delta32[i] = (float)d;
    }
}

// the float64 delta on listed element ranges, packed into out: the values
// the Eden seed's serial sums read (one range per tensor; single-element
// tensors use the pairwise order)
struct RangeArgs {
    PointArgs p;
    const int64_t* start;   // device [nr]
    const int64_t* dst;     // device [nr + 1] exclusive prefix of the counts
    const int32_t* single;  // device [nr]
    int nr;
};
__global__ __launch_bounds__(kNT) void k_wavg_ranges(RangeArgs r, double* out) {
#pragma clang fp contract(off)
    const int64_t total = r.dst[r.nr];
    for (int64_t j = (int64_t)blockIdx.x * kNT + threadIdx.x; j < total; j += (int64_t)gridDim.x * kNT) {
        int lo = 0, hi = r.nr - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (r.dst[mid] <= j) lo = mid; else hi = mid - 1;
        }
        const int64_t i = r.start[lo] + (j - r.dst[lo]);
        double s;
        if (r.single[lo]) {
            s = np_pairwise(r.p, i, 0, r.p.nc);
        } else {
            s = (double)r.p.x[0][i] * r.p.w[0];
            for (int c = 1; c < r.p.nc; ++c) s = s + (double)r.p.x[c][i] * r.p.w[c];
        }
        const double avg = s / r.p.wsum;
        out[j] = r.p.base ? avg - (double)r.p.base[i] : avg;
    }
}

// serial float64 sum of each packed range, left to right like Python's sum()
// over NumPy scalars: one 256-thread block per range stages 2048 values at a
// time in LDS, then one lane runs the dependent add chain from LDS (loads
// issued eight ahead of the adds)
__global__ __launch_bounds__(256) void k_range_sums(const double* packed, const int64_t* dst, double* sums) {
    __shared__ double v[2048];
    const int r = blockIdx.x;
    const int64_t j0 = dst[r], j1 = dst[r + 1];
    double s = 0.0;
    for (int64_t c0 = j0; c0 < j1; c0 += 2048) {
        const int m = (int)(j1 - c0 < 2048 ? j1 - c0 : 2048);
        __syncthreads();
        for (int k = threadIdx.x; k < m; k += 256) v[k] = packed[c0 + k];
        __syncthreads();
        if (threadIdx.x == 0) {
            int k = 0;
            for (; k + 8 <= m; k += 8) {
                double t[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) t[q] = v[k + q];
#pragma unroll
                for (int q = 0; q < 8; ++q) s = s + t[q];
            }
            for (; k < m; ++k) s = s + v[k];
        }
    }
    if (threadIdx.x == 0) sums[r] = s;
}

// CPython's hash of a finite float (Objects/object.c _Py_HashDouble, modulus
// 2^61 - 1): the 28-bit chunks of the mantissa folded with a rotation, then the
// exponent as a rotation, the sign, and -1 -> -2.  inf -> +-314159; NaN (an
// object-id hash in CPython >= 3.10, not reproducible) -> 0.
__device__ int64_t py_hash_double(double v) {
    const uint64_t MOD = (1ull << 61) - 1ull;
    if (isinf(v)) return v > 0 ? 314159 : -314159;
    if (isnan(v)) return 0;
    int e;
    double m = frexp(v, &e);
    int sign = 1;
    if (m < 0) { sign = -1; m = -m; }
    uint64_t x = 0;
    while (m != 0.0) {
        x = ((x << 28) & MOD) | x >> (61 - 28);
        m *= 268435456.0;
        e -= 28;
        const uint64_t y = (uint64_t)m;
        m -= (double)y;
        x += y;
        if (x >= MOD) x -= MOD;
    }
    e = e >= 0 ? e % 61 : 61 - 1 - ((-1 - e) % 61);
    x = ((x << e) & MOD) | x >> (61 - e);
    x = x * (uint64_t)(int64_t)sign;
    if (x == ~0ull) x = ~0ull - 1ull;
    return (int64_t)x;
}
// the Eden seed of each tensor from its serial float64 sum and its np.random
// draw (eden_pipeline.py:771-772): (hash(sum * 13 + 7) + draw) % 2^16
__global__ __launch_bounds__(64) void k_seeds(const double* sums, const int64_t* draws, int n, uint32_t* seeds) {
#pragma clang fp contract(off)
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= n) return;
    const double t = sums[i] * 13.0 + 7.0;
    const int64_t h = py_hash_double(t) + draws[i];
    seeds[i] = (uint32_t)(((h % 65536) + 65536) % 65536);
}

// apply_delta: out = base + delta (float32)
__global__ __launch_bounds__(kNT) void k_apply(const float* base, const float* delta, int64_t n, float* out) {
    const int64_t stride = (int64_t)gridDim.x * kNT;
    const int64_t n4 = ((reinterpret_cast<uintptr_t>(base) | reinterpret_cast<uintptr_t>(delta) |
                         reinterpret_cast<uintptr_t>(out)) & 15u) ? 0 : n >> 2;
    const float4* b4 = reinterpret_cast<const float4*>(base);
    const float4* d4 = reinterpret_cast<const float4*>(delta);
    float4* o4 = reinterpret_cast<float4*>(out);
    for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < n4; i += stride) {
        const float4 b = b4[i], d = d4[i];
        o4[i] = make_float4(b.x + d.x, b.y + d.y, b.z + d.z, b.w + d.w);
    }
    for (int64_t i = 4 * n4 + (int64_t)blockIdx.x * kNT + threadIdx.x; i < n; i += stride) out[i] = base[i] + delta[i];
}

// RandomShiftTransformer.backward with wire metadata (random_shift_pipeline.py:
// 45-68): data (float32) - shift (float64) in float64, as NumPy promotes
__global__ __launch_bounds__(kNT) void k_unshift64(const float* data, const double* shift, int64_t n, double* out) {
    for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kNT)
        out[i] = (double)data[i] - shift[i];
}

// apply_delta on listed ranges (device tables): the tensors the codec does
// not touch when the decode itself adds the base (ofl_eden_decode_add)
__global__ __launch_bounds__(kNT) void k_apply_ranges(const float* base, const float* delta, float* out,
                                                      const int64_t* start, const int64_t* dst, int nr) {
    const int64_t total = dst[nr];
    for (int64_t j = (int64_t)blockIdx.x * kNT + threadIdx.x; j < total; j += (int64_t)gridDim.x * kNT) {
        int lo = 0, hi = nr - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (dst[mid] <= j) lo = mid; else hi = mid - 1;
        }
        const int64_t i = start[lo] + (j - dst[lo]);
        out[i] = base[i] + delta[i];
    }
}

// the float32 delta (as k_wavg_delta writes it) on listed ranges only: the
// elements the fused round-end encode does not compute itself
// (ofl_eden_encode_wavg: slices of <= 2^15 elements and the tensors the codec
// does not touch)
__global__ __launch_bounds__(kNT) void k_wavg_delta32_ranges(WavgArgs a, const int64_t* start, const int64_t* dst,
                                                             int nr) {
    const int64_t total = dst[nr];
    for (int64_t j = (int64_t)blockIdx.x * kNT + threadIdx.x; j < total; j += (int64_t)gridDim.x * kNT) {
        int lo = 0, hi = nr - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (dst[mid] <= j) lo = mid; else hi = mid - 1;
        }
        const int64_t i = start[lo] + (j - dst[lo]);
        double avg;
        a.delta32[i] = (float)wavg_delta(a, i, wavg_sum(a, i, 0.0), avg);
    }
}

__global__ __launch_bounds__(64) void k_py_hash(const double* v, int n, int64_t* out) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i < n) out[i] = py_hash_double(v[i]);
}

}  // namespace agg

namespace {
thread_local std::string g_aerr;
int afail(int code, const std::string& m) { g_aerr = m; return code; }
#define AHIP(x)                                                                                        \
    do {                                                                                               \
        hipError_t e_ = (x);                                                                           \
        if (e_ != hipSuccess) return afail(OFL_EHIP, std::string(#x " failed: ") + hipGetErrorString(e_)); \
    } while (0)

int grid_for(int64_t n, int per_thread) {
    int dev = 0, cus = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int64_t want = (n + (int64_t)agg::kNT * per_thread - 1) / ((int64_t)agg::kNT * per_thread);
    return (int)std::max<int64_t>(1, std::min<int64_t>(want, (int64_t)cus * 16));
}

int fill_args(agg::WavgArgs& a, int ncollab, const float* const* xs, const double* weights, double wsum,
              const float* base, int64_t n) {
    // shared checks; the per-launch collaborator slots are filled by the caller
    if (ncollab < 1 || !xs || !weights) return afail(OFL_EINVAL, "wavg: need at least one collaborator");
    if (n < 0) return afail(OFL_EINVAL, "wavg: negative size");
    a = agg::WavgArgs{};
    a.wsum = wsum;
    a.base = base;
    a.n = n;
    return OFL_OK;
}
}  // namespace

extern "C" {

const char* ofl_agg_last_error(void) { return g_aerr.c_str(); }

int ofl_wavg_delta(int ncollab, const float* const* xs, const double* weights, double wsum, const float* base,
                   int64_t n, double* agg_out, double* delta64_out, float* delta32_out, void* stream) {
    agg::WavgArgs a;
    if (int rc = fill_args(a, ncollab, xs, weights, wsum, base, n)) return rc;
    if (ncollab > agg::kMaxC && !agg_out)
        return afail(OFL_EINVAL, "wavg: more than 16 collaborators need agg_out (running sums)");
    if (n == 0) return OFL_OK;
    hipStream_t st = static_cast<hipStream_t>(stream);
    const int g = grid_for(n, 4);
    for (int c0 = 0; c0 < ncollab; c0 += agg::kMaxC) {
        a.nc = std::min(agg::kMaxC, ncollab - c0);
        for (int c = 0; c < a.nc; ++c) {
            if (!xs[c0 + c]) return afail(OFL_EINVAL, "wavg: null collaborator tensor");
            a.x[c] = xs[c0 + c];
            a.w[c] = weights[c0 + c];
        }
        a.first = c0 == 0;
        a.last = c0 + a.nc == ncollab;
        a.acc = agg_out;
        a.delta64 = a.last ? delta64_out : nullptr;
        a.delta32 = a.last ? delta32_out : nullptr;
        uintptr_t al = reinterpret_cast<uintptr_t>(a.base) | reinterpret_cast<uintptr_t>(a.delta32) |
                       reinterpret_cast<uintptr_t>(a.acc) | reinterpret_cast<uintptr_t>(a.delta64);
        for (int c = 0; c < a.nc; ++c) al |= reinterpret_cast<uintptr_t>(a.x[c]);
        hipLaunchKernelGGL(agg::k_wavg_delta, dim3(g), dim3(agg::kNT), 0, st, a, (al & 15u) ? 0 : 1);
        AHIP(hipGetLastError());
    }
    return OFL_OK;
}

size_t ofl_wavg_ranges_workspace_bytes(int ncollab, int nranges) {
    return 16 * (size_t)std::max(ncollab, 1) + 20 * (size_t)(std::max(nranges, 1) + 1) + 512;
}

int ofl_wavg_delta_ranges(int ncollab, const float* const* xs, const double* weights, double wsum,
                          const float* base, int nranges, const int64_t* starts, const int64_t* counts,
                          const int32_t* single, double* out, void* ws, size_t ws_bytes, void* stream) {
    if (ncollab < 1 || ncollab > 2048 || !xs || !weights)
        return afail(OFL_EINVAL, "wavg ranges: 1 <= collaborators <= 2048");
    if (nranges < 1) return OFL_OK;
    if (!starts || !counts || !ws || ws_bytes < ofl_wavg_ranges_workspace_bytes(ncollab, nranges))
        return afail(OFL_ESPACE, "wavg ranges: workspace too small");
    const size_t o_w = 8 * (size_t)ncollab, o_s = 16 * (size_t)ncollab;
    const size_t o_d = o_s + 8 * (size_t)nranges, o_f = o_d + 8 * (size_t)(nranges + 1);
    std::string host(o_f + 4 * (size_t)nranges, '\0');
    memcpy(host.data(), xs, 8 * (size_t)ncollab);
    memcpy(host.data() + o_w, weights, 8 * (size_t)ncollab);
    int64_t* hs = reinterpret_cast<int64_t*>(host.data() + o_s);
    int64_t* hd = reinterpret_cast<int64_t*>(host.data() + o_d);
    int32_t* hf = reinterpret_cast<int32_t*>(host.data() + o_f);
    int64_t acc = 0;
    for (int i = 0; i < nranges; ++i) {
        if (counts[i] < 0 || starts[i] < 0) return afail(OFL_EINVAL, "wavg ranges: negative range");
        hs[i] = starts[i];
        hd[i] = acc;
        hf[i] = single ? single[i] : 0;
        acc += counts[i];
    }
    hd[nranges] = acc;
    if (acc == 0) return OFL_OK;
    hipStream_t st = static_cast<hipStream_t>(stream);
    char* w = static_cast<char*>(ws);
    AHIP(hipMemcpyAsync(w, host.data(), host.size(), hipMemcpyHostToDevice, st));
    agg::RangeArgs r{};
    r.p.x = reinterpret_cast<const float* const*>(w);
    r.p.w = reinterpret_cast<const double*>(w + o_w);
    r.p.nc = ncollab;
    r.p.wsum = wsum;
    r.p.base = base;
    r.start = reinterpret_cast<const int64_t*>(w + o_s);
    r.dst = reinterpret_cast<const int64_t*>(w + o_d);
    r.single = reinterpret_cast<const int32_t*>(w + o_f);
    r.nr = nranges;
    hipLaunchKernelGGL(agg::k_wavg_ranges, dim3(grid_for(acc, 1)), dim3(agg::kNT), 0, st, r, out);
    AHIP(hipGetLastError());
    AHIP(hipStreamSynchronize(st));  // the staging string must outlive the copy
    return OFL_OK;
}

size_t ofl_wavg_range_sums_workspace_bytes(int ncollab, int nranges, int64_t total) {
    return ofl_wavg_ranges_workspace_bytes(ncollab, nranges) + 8 * (size_t)(std::max<int64_t>(total, 1) + nranges) + 512;
}

int ofl_wavg_delta_range_sums(int ncollab, const float* const* xs, const double* weights, double wsum,
                              const float* base, int nranges, const int64_t* starts, const int64_t* counts,
                              const int32_t* single, double* sums, void* ws, size_t ws_bytes, void* stream) {
    if (nranges < 1) return OFL_OK;
    if (!sums || !counts) return afail(OFL_EINVAL, "wavg range sums: null output");
    int64_t total = 0;
    for (int i = 0; i < nranges; ++i) total += counts[i] > 0 ? counts[i] : 0;
    if (!ws || ws_bytes < ofl_wavg_range_sums_workspace_bytes(ncollab, nranges, total))
        return afail(OFL_ESPACE, "wavg range sums: workspace too small");
    const size_t head = (ofl_wavg_ranges_workspace_bytes(ncollab, nranges) + 255) & ~(size_t)255;
    char* w = static_cast<char*>(ws);
    double* packed = reinterpret_cast<double*>(w + head);
    double* dsums = packed + std::max<int64_t>(total, 1);
    const int rc = ofl_wavg_delta_ranges(ncollab, xs, weights, wsum, base, nranges, starts, counts, single, packed,
                                         ws, head, stream);
    if (rc != OFL_OK) return rc;
    hipStream_t st = static_cast<hipStream_t>(stream);
    // the range table the ranges call staged: dst prefix after the pointers, weights and starts
    const int64_t* dst = reinterpret_cast<const int64_t*>(w + 16 * (size_t)ncollab + 8 * (size_t)nranges);
    hipLaunchKernelGGL(agg::k_range_sums, dim3(nranges), dim3(256), 0, st, packed, dst, dsums);
    AHIP(hipGetLastError());
    AHIP(hipMemcpyAsync(sums, dsums, 8 * (size_t)nranges, hipMemcpyDeviceToHost, st));
    AHIP(hipStreamSynchronize(st));
    return OFL_OK;
}

int ofl_wavg_delta_seeds(int ncollab, const float* const* xs_dev, const double* weights_dev, double wsum,
                         const float* base, int nranges, const int64_t* starts_dev, const int64_t* dst_dev,
                         const int32_t* single_dev, int64_t total, const int64_t* draws_dev, uint32_t* seeds_dev,
                         double* sums_dev, double* packed_dev, void* stream) {
    if (ncollab < 1 || ncollab > 2048 || nranges < 1) return afail(OFL_EINVAL, "wavg seeds: bad sizes");
    if (!xs_dev || !weights_dev || !starts_dev || !dst_dev || !single_dev || !draws_dev || !seeds_dev || !sums_dev ||
        (total > 0 && !packed_dev))
        return afail(OFL_EINVAL, "wavg seeds: null pointer");
    hipStream_t st = static_cast<hipStream_t>(stream);
    agg::RangeArgs r{};
    r.p.x = xs_dev;
    r.p.w = weights_dev;
    r.p.nc = ncollab;
    r.p.wsum = wsum;
    r.p.base = base;
    r.start = starts_dev;
    r.dst = dst_dev;
    r.single = single_dev;
    r.nr = nranges;
    if (total > 0) hipLaunchKernelGGL(agg::k_wavg_ranges, dim3(grid_for(total, 1)), dim3(agg::kNT), 0, st, r, packed_dev);
    hipLaunchKernelGGL(agg::k_range_sums, dim3(nranges), dim3(256), 0, st, packed_dev, dst_dev, sums_dev);
    hipLaunchKernelGGL(agg::k_seeds, dim3((nranges + 63) / 64), dim3(64), 0, st, sums_dev, draws_dev, nranges, seeds_dev);
    AHIP(hipGetLastError());
    return OFL_OK;
}

int ofl_py_hash_doubles(const double* v_dev, int n, int64_t* out_dev, void* stream) {
    if (n <= 0) return OFL_OK;
    hipLaunchKernelGGL(agg::k_py_hash, dim3((n + 63) / 64), dim3(64), 0, static_cast<hipStream_t>(stream), v_dev, n,
                       out_dev);
    AHIP(hipGetLastError());
    return OFL_OK;
}

size_t ofl_wavg_points_workspace_bytes(int ncollab, int npoints) {
    return 16 * (size_t)std::max(ncollab, 1) + 8 * (size_t)std::max(npoints, 1) + 512;
}

int ofl_wavg_delta_points(int ncollab, const float* const* xs, const double* weights, double wsum, const float* base,
                          int npoints, const int64_t* idx, double* agg_out, double* delta64_out, float* delta32_out,
                          void* ws, size_t ws_bytes, void* stream) {
    if (ncollab < 1 || ncollab > 2048 || !xs || !weights)
        return afail(OFL_EINVAL, "wavg points: 1 <= collaborators <= 2048");
    if (npoints < 1) return OFL_OK;
    if (!idx || !ws || ws_bytes < ofl_wavg_points_workspace_bytes(ncollab, npoints))
        return afail(OFL_ESPACE, "wavg points: workspace too small");
    std::string host(16 * (size_t)ncollab + 8 * (size_t)npoints, '\0');
    memcpy(host.data(), xs, 8 * (size_t)ncollab);
    memcpy(host.data() + 8 * (size_t)ncollab, weights, 8 * (size_t)ncollab);
    memcpy(host.data() + 16 * (size_t)ncollab, idx, 8 * (size_t)npoints);
    hipStream_t st = static_cast<hipStream_t>(stream);
    char* w = static_cast<char*>(ws);
    AHIP(hipMemcpyAsync(w, host.data(), host.size(), hipMemcpyHostToDevice, st));
    agg::PointArgs a{};
    a.x = reinterpret_cast<const float* const*>(w);
    a.w = reinterpret_cast<const double*>(w + 8 * (size_t)ncollab);
    a.idx = reinterpret_cast<const int64_t*>(w + 16 * (size_t)ncollab);
    a.nc = ncollab;
    a.wsum = wsum;
    a.base = base;
    a.np = npoints;
    a.acc = agg_out;
    a.delta64 = delta64_out;
    a.delta32 = delta32_out;
    hipLaunchKernelGGL(agg::k_wavg_points, dim3((npoints + 63) / 64), dim3(64), 0, st, a);
    AHIP(hipGetLastError());
    AHIP(hipStreamSynchronize(st));  // the staging string must outlive the copy
    return OFL_OK;
}

int ofl_apply_delta(const float* base, const float* delta, int64_t n, float* out, void* stream) {
    if (n < 0 || (n && (!base || !delta || !out))) return afail(OFL_EINVAL, "apply_delta: bad arguments");
    if (n == 0) return OFL_OK;
    hipLaunchKernelGGL(agg::k_apply, dim3(grid_for(n, 16)), dim3(agg::kNT), 0, static_cast<hipStream_t>(stream), base,
                       delta, n, out);
    AHIP(hipGetLastError());
    return OFL_OK;
}

int ofl_sub_f32_f64(const float* data, const double* shift, int64_t n, double* out, void* stream) {
    if (n < 0 || (n && (!data || !shift || !out))) return afail(OFL_EINVAL, "sub_f32_f64: bad arguments");
    if (n == 0) return OFL_OK;
    hipLaunchKernelGGL(agg::k_unshift64, dim3(grid_for(n, 16)), dim3(agg::kNT), 0, static_cast<hipStream_t>(stream),
                       data, shift, n, out);
    AHIP(hipGetLastError());
    return OFL_OK;
}

int ofl_wavg_delta32_ranges(int ncollab, const float* const* xs, const double* weights, double wsum,
                            const float* base, int nranges, const int64_t* starts, const int64_t* dst, int64_t total,
                            float* delta32_out, void* stream) {
    if (nranges < 1 || total <= 0) return OFL_OK;
    if (ncollab > agg::kMaxC) return afail(OFL_EINVAL, "wavg_delta32_ranges: at most 16 collaborators");
    if (!starts || !dst || !delta32_out) return afail(OFL_EINVAL, "wavg_delta32_ranges: bad arguments");
    agg::WavgArgs a;
    if (int rc = fill_args(a, ncollab, xs, weights, wsum, base, total)) return rc;
    a.nc = ncollab;
    for (int c = 0; c < ncollab; ++c) {
        if (!xs[c]) return afail(OFL_EINVAL, "wavg: null collaborator tensor");
        a.x[c] = xs[c];
        a.w[c] = weights[c];
    }
    a.first = 1;
    a.last = 1;
    a.delta32 = delta32_out;
    hipLaunchKernelGGL(agg::k_wavg_delta32_ranges, dim3(grid_for(total, 1)), dim3(agg::kNT), 0,
                       static_cast<hipStream_t>(stream), a, starts, dst, nranges);
    AHIP(hipGetLastError());
    return OFL_OK;
}

int ofl_apply_delta_ranges(const float* base, const float* delta, float* out, int nranges, const int64_t* starts,
                           const int64_t* dst, int64_t total, void* stream) {
    if (nranges < 1 || total <= 0) return OFL_OK;
    if (!base || !delta || !out || !starts || !dst) return afail(OFL_EINVAL, "apply_delta_ranges: bad arguments");
    hipLaunchKernelGGL(agg::k_apply_ranges, dim3(grid_for(total, 1)), dim3(agg::kNT), 0,
                       static_cast<hipStream_t>(stream), base, delta, out, starts, dst, nranges);
    AHIP(hipGetLastError());
    return OFL_OK;
}

}  // extern "C"
