// 24-bit block-float intermediates, memory side: can the
// large-slice passes move a 3-byte intermediate at the rate they move fp32?
// Format under test ("bf24x4"): 4 consecutive elements share the exponent of
// their largest |value|; each keeps a 22-bit two's-complement mantissa; the
// group is 3 dwords (12 B), the exponent in the top byte of the third.
// Shapes (2^29 elements per launch, the 2 GiB wave of the Llama step):
//   row: persistent 512-thread blocks over 2^15-element tiles, next tile in
//        flight; fp32 copy vs fp32 -> bf24 (pack + dwordx3 stores) vs
//        bf24 -> fp32 (dwordx3 loads + unpack)
//   col: the 2^24 middle pass (512 rows x 64 columns per tile, rows 2^15
//        elements apart): fp32 vs bf24 -> bf24 (192-B row runs that straddle
//        128-B lines), tiles dealt naively or in XCD pairs (blocks b and b + 8
//        share an XCD and take adjacent column groups, so the straddled line
//        meets both halves in one L2)
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/streambench4 tools/streambench4.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CHECK(x)                                                                    \
    do {                                                                            \
        hipError_t e = (x);                                                         \
        if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
    } while (0)

typedef int rsrc_t __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x3 __attribute__((ext_vector_type(3)));
__device__ float raw_load_f32(rsrc_t r, int voff, int soff, int aux) __asm("llvm.amdgcn.raw.buffer.load.f32");
__device__ void raw_store_f32(float v, rsrc_t r, int voff, int soff, int aux) __asm("llvm.amdgcn.raw.buffer.store.f32");
__device__ f32x4 raw_load_f32x4(rsrc_t r, int voff, int soff, int aux) __asm("llvm.amdgcn.raw.buffer.load.v4f32");
__device__ void raw_store_f32x4(f32x4 v, rsrc_t r, int voff, int soff, int aux) __asm("llvm.amdgcn.raw.buffer.store.v4f32");
__device__ i32x3 raw_load_i32x3(rsrc_t r, int voff, int soff, int aux) __asm("llvm.amdgcn.raw.buffer.load.v3i32");
__device__ void raw_store_i32x3(i32x3 v, rsrc_t r, int voff, int soff, int aux) __asm("llvm.amdgcn.raw.buffer.store.v3i32");

#define DEVI __device__ __forceinline__
DEVI rsrc_t mk_rsrc(const void* p, uint32_t bytes) {
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    rsrc_t r;
    r.x = (int)(uint32_t)a;
    r.y = (int)((uint32_t)(a >> 32) & 0xffffu);
    r.z = (int)bytes;
    r.w = 0x00020000;
    return r;
}

// ---- bf24x4 ---------------------------------------------------------------
DEVI i32x3 pack4(float a, float b, float c, float d) {
    const float mx = fmaxf(fmaxf(fabsf(a), fabsf(b)), fmaxf(fabsf(c), fabsf(d)));
    const uint32_t E = max(__float_as_uint(mx) >> 23, 21u);  // 255: Inf / NaN group
    const float s = __uint_as_float((274u - E) << 23);      // 2^(147 - E)
    const int lim = (1 << 21) - 1;
    const int m0 = min(max(__float2int_rn(a * s), -lim), lim), m1 = min(max(__float2int_rn(b * s), -lim), lim);
    const int m2 = min(max(__float2int_rn(c * s), -lim), lim), m3 = min(max(__float2int_rn(d * s), -lim), lim);
    i32x3 w;
    w.x = (int)(((uint32_t)m0 & 0x3fffffu) | ((uint32_t)m1 << 22));
    w.y = (int)((((uint32_t)m1 >> 10) & 0xfffu) | ((uint32_t)m2 << 12));
    w.z = (int)((((uint32_t)m2 >> 20) & 3u) | (((uint32_t)m3 & 0x3fffffu) << 2) | (E << 24));
    return w;
}
DEVI int sx22(uint32_t v) { return ((int)(v << 10)) >> 10; }
DEVI void unpack4(i32x3 w, float& a, float& b, float& c, float& d) {
    const uint32_t x = (uint32_t)w.x, y = (uint32_t)w.y, z = (uint32_t)w.z;
    const uint32_t E = z >> 24;
    const float r = E == 255u ? __uint_as_float(0x7fc00000u) : __uint_as_float((E - 20u) << 23);  // 2^(E - 147)
    a = (float)sx22(x) * r;
    b = (float)sx22(__builtin_amdgcn_alignbit(y, x, 22)) * r;
    c = (float)sx22(__builtin_amdgcn_alignbit(z, y, 12)) * r;
    d = (float)sx22(z >> 2) * r;
}

// ---- row shape --------------------------------------------------------------
// MODE 0: fp32 -> fp32; 1: fp32 -> bf24; 2: bf24 -> fp32
template <int MODE>
__global__ __launch_bounds__(512) void row_k(const void* __restrict__ a, void* __restrict__ b, int ntile) {
    const unsigned t = threadIdx.x;
    int tile = blockIdx.x;
    if (tile >= ntile) return;
    constexpr uint32_t in_eb = MODE == 2 ? 3u : 4u, out_eb = MODE == 1 ? 3u : 4u;
    auto load = [&](int tl, bool live, float (&v)[64]) {
        const rsrc_t r = mk_rsrc((const char*)a + ((size_t)tl << 15) * in_eb, live ? in_eb << 15 : 0u);
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            if (MODE == 2) {
                const i32x3 w = raw_load_i32x3(r, (int)(t * 12u), k * 512 * 12, 0);
                unpack4(w, v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
            } else {
                const f32x4 q = raw_load_f32x4(r, (int)(t * 16u), k * 512 * 16, 0);
                v[4 * k] = q.x; v[4 * k + 1] = q.y; v[4 * k + 2] = q.z; v[4 * k + 3] = q.w;
            }
        }
    };
    float nx[64];
    load(tile, true, nx);
    for (;;) {
        float v[64];
#pragma unroll
        for (int k = 0; k < 64; ++k) v[k] = nx[k] * 1.0001f;
        const int tn = tile + gridDim.x;
        const bool more = tn < ntile;
        load(more ? tn : tile, more, nx);
        const rsrc_t w = mk_rsrc((char*)b + ((size_t)tile << 15) * out_eb, out_eb << 15);
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            if (MODE == 1) {
                raw_store_i32x3(pack4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]), w, (int)(t * 12u), k * 512 * 12, 0);
            } else {
                const f32x4 q = {v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]};
                raw_store_f32x4(q, w, (int)(t * 16u), k * 512 * 16, 0);
            }
        }
        if (!more) break;
        tile = tn;
    }
}

// ---- column shape (2^24 slices: 512 rows x 64 columns per tile) ------------
DEVI unsigned col_tile(unsigned b, bool pair) {
    if (!pair) return b;
    const unsigned x = b & 7u, h = (b >> 3) & 1u, j = b >> 4;
    return 2u * (8u * j + x) + h;
}
template <bool PAIR>
__global__ __launch_bounds__(512, 2) void col32_k(const float* __restrict__ a, float* __restrict__ b) {
    const unsigned t = threadIdx.x, tile = col_tile(blockIdx.x, PAIR);
    const unsigned slice = tile >> 9, cg = tile & 511u;
    const size_t sb = (size_t)slice << 24;
    const rsrc_t ra = mk_rsrc(a + sb + cg * 64u, 4u << 24), rb = mk_rsrc(b + sb + cg * 64u, 4u << 24);
    const unsigned c = t & 63u, r0 = t >> 6;  // 8 rows per instruction
    float v[64];
#pragma unroll
    for (int k = 0; k < 64; ++k) v[k] = raw_load_f32(ra, (int)((c + (r0 << 15)) * 4u), (k << 18) * 4, 0);
#pragma unroll
    for (int k = 0; k < 64; ++k) raw_store_f32(v[k] * 1.0001f, rb, (int)((c + (r0 << 15)) * 4u), (k << 18) * 4, 0);
}
template <bool PAIR>
__global__ __launch_bounds__(512, 2) void col24_k(const uint8_t* __restrict__ a, uint8_t* __restrict__ b) {
    const unsigned t = threadIdx.x, tile = col_tile(blockIdx.x, PAIR);
    const unsigned slice = tile >> 9, cg = tile & 511u;
    const size_t sb = ((size_t)slice << 24) * 3u;
    const rsrc_t ra = mk_rsrc(a + sb + cg * 192u, 3u << 24), rb = mk_rsrc(b + sb + cg * 192u, 3u << 24);
    const unsigned g = t & 15u, r0 = t >> 4;  // 16 groups x 32 rows per 512 threads
    float v[64];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const i32x3 w = raw_load_i32x3(ra, (int)(g * 12u + r0 * (3u << 15)), k * 32 * (3 << 15), 0);
        unpack4(w, v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
    }
#pragma unroll
    for (int k = 0; k < 64; ++k) v[k] *= 1.0001f;
#pragma unroll
    for (int k = 0; k < 16; ++k)
        raw_store_i32x3(pack4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]), rb,
                        (int)(g * 12u + r0 * (3u << 15)), k * 32 * (3 << 15), 0);
}

__global__ void fill(float* p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = (float)((i * 2654435761u) & 0xffff) * 1e-4f - 3.0f;
}

int main() {
    const size_t n = (size_t)1 << 29;  // 2^29 elements
    void *a, *b;
    CHECK(hipMalloc(&a, n * 4));
    CHECK(hipMalloc(&b, n * 4));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (float*)a, n);
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (float*)b, n);
    CHECK(hipDeviceSynchronize());
    int cus = 256;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    auto run = [&](const char* name, double bytes, auto launch) {
        launch();
        CHECK(hipDeviceSynchronize());
        float best = 1e30f, sum = 0;
        for (int rep = 0; rep < 3; ++rep) {
            CHECK(hipEventRecord(e0));
            for (int i = 0; i < 5; ++i) launch();
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
            sum += ms;
        }
        const double us = 1e3 * best / 5, avg = 1e3 * sum / 15;
        printf("%-34s best %8.1f us %6.2f TB/s   avg %8.1f us %6.2f TB/s  (%.2f B/elem)\n", name, us,
               bytes / (us * 1e-6) / 1e12, avg, bytes / (avg * 1e-6) / 1e12, bytes / n);
        fflush(stdout);
    };
    const int ntile = (int)(n >> 15);
    for (int rep = 0; rep < 2; ++rep) {
        run("row fp32->fp32", 8.0 * n, [&] { hipLaunchKernelGGL(row_k<0>, dim3(cus), dim3(512), 0, 0, a, b, ntile); });
        run("row fp32->bf24", 7.0 * n, [&] { hipLaunchKernelGGL(row_k<1>, dim3(cus), dim3(512), 0, 0, a, b, ntile); });
        run("row bf24->fp32", 7.0 * n, [&] { hipLaunchKernelGGL(row_k<2>, dim3(cus), dim3(512), 0, 0, b, a, ntile); });
        run("col2^24 fp32 naive", 8.0 * n,
            [&] { hipLaunchKernelGGL(col32_k<false>, dim3(ntile), dim3(512), 0, 0, (const float*)a, (float*)b); });
        run("col2^24 fp32 xcd-pairs", 8.0 * n,
            [&] { hipLaunchKernelGGL(col32_k<true>, dim3(ntile), dim3(512), 0, 0, (const float*)a, (float*)b); });
        run("col2^24 bf24 naive", 6.0 * n,
            [&] { hipLaunchKernelGGL(col24_k<false>, dim3(ntile), dim3(512), 0, 0, (const uint8_t*)a, (uint8_t*)b); });
        run("col2^24 bf24 xcd-pairs", 6.0 * n,
            [&] { hipLaunchKernelGGL(col24_k<true>, dim3(ntile), dim3(512), 0, 0, (const uint8_t*)a, (uint8_t*)b); });
    }
    return 0;
}
