// Read+write streaming microbenchmark: how fast can a 4 B in / 4 B out pass
// over 2 GiB go on this chip, by access width and lane pattern?  (Sizing the
// ceiling of the codec's row and column passes)
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/streambench tools/streambench.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ws24.h"

#define CHECK(x)                                                                    \
    do {                                                                            \
        hipError_t e = (x);                                                         \
        if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
    } while (0)

// 16 B per lane, grid-stride
__global__ __launch_bounds__(256) void copy4(const float4* __restrict__ a, float4* __restrict__ b, size_t n4) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) b[i] = a[i];
}
// 4 B per lane, 8 independent dwords per thread in flight (256 B per wave-instruction)
__global__ __launch_bounds__(256) void copy1(const float* __restrict__ a, float* __restrict__ b, size_t n) {
    const size_t per = 256ull * 8;
    for (size_t base = blockIdx.x * per; base < n; base += (size_t)gridDim.x * per) {
        float v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = a[base + k * 256 + threadIdx.x];
#pragma unroll
        for (int k = 0; k < 8; ++k) b[base + k * 256 + threadIdx.x] = v[k];
    }
}
// the row passes' ws pattern: a 2^15 tile per block of 512 threads, lanes
// 0..31 on 32 consecutive floats, lane bit 5 -> +2048, waves -> bits 12..14,
// 64 registers at register bits 5..10 (one dword each)
__global__ __launch_bounds__(512) void copy_l3(const float* __restrict__ a, float* __restrict__ b, size_t ntile) {
    const unsigned t = threadIdx.x;
    const unsigned base = (t & 31u) | (((t >> 5) & 1u) << 11) | ((t >> 6) << 12);
    for (size_t tile = blockIdx.x; tile < ntile; tile += gridDim.x) {
        const float* src = a + (tile << 15);
        float* dst = b + (tile << 15);
        float v[64];
#pragma unroll
        for (int r = 0; r < 64; ++r) v[r] = src[base + (r << 5)];
#pragma unroll
        for (int r = 0; r < 64; ++r) dst[base + (r << 5)] = v[r];
    }
}
// the same tile with float4 per lane: register bits 0,1 + 4 more
__global__ __launch_bounds__(512) void copy_l3q(const float* __restrict__ a, float* __restrict__ b, size_t ntile) {
    const unsigned t = threadIdx.x;
    // lanes: bits 2..6 (32 lanes = 128 consecutive floats), lane bit 5 -> bit 11, waves -> 12..14
    const unsigned base = ((t & 31u) << 2) | (((t >> 5) & 1u) << 11) | ((t >> 6) << 12);
    for (size_t tile = blockIdx.x; tile < ntile; tile += gridDim.x) {
        const float4* src = reinterpret_cast<const float4*>(a + (tile << 15));
        float4* dst = reinterpret_cast<float4*>(b + (tile << 15));
        float4 v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = src[(base + ((r & 3) << 7) + ((r >> 2) << 9)) >> 2];
#pragma unroll
        for (int r = 0; r < 16; ++r) dst[(base + ((r & 3) << 7) + ((r >> 2) << 9)) >> 2] = v[r];
    }
}

// 24-bit block-float intermediates (openfl_amd/csrc/ws24.h) in the L3 tile
// pattern: fp32 in -> packed out, and packed in -> fp32 out
__device__ __forceinline__ unsigned l3_base(unsigned t) {
    return (t & 31u) | (((t >> 5) & 1u) << 11) | ((t >> 6) << 12);
}
__global__ __launch_bounds__(512) void pack_l3(const float* __restrict__ a, uint8_t* __restrict__ p, size_t ntile) {
    const unsigned t = threadIdx.x, base = l3_base(t), g = t & 7u;
    for (size_t tile = blockIdx.x; tile < ntile; tile += gridDim.x) {
        const float* src = a + (tile << 15);
        uint8_t* dst = p + 3 * (tile << 15);
        float v[64];
#pragma unroll
        for (int r = 0; r < 64; ++r) v[r] = src[base + (r << 5)];
#pragma unroll
        for (int r = 0; r < 64; ++r) {
            const uint32_t d = ws24::pack(v[r], g);
            if ((g & 3u) != 3u) *reinterpret_cast<uint32_t*>(dst + ws24::boff(base + (r << 5))) = d;
        }
    }
}
__global__ __launch_bounds__(512) void unpack_l3(const uint8_t* __restrict__ p, float* __restrict__ b, size_t ntile) {
    const unsigned t = threadIdx.x, base = l3_base(t), g = t & 7u;
    const unsigned lb = 3u * (base & ~3u) + 4u * min(g & 3u, 2u);  // lane 3 re-reads lane 2's dword
    for (size_t tile = blockIdx.x; tile < ntile; tile += gridDim.x) {
        const uint8_t* src = p + 3 * (tile << 15);
        float* dst = b + (tile << 15);
        uint32_t d[64];
#pragma unroll
        for (int r = 0; r < 64; ++r) d[r] = *reinterpret_cast<const uint32_t*>(src + lb + 3u * (r << 5));
#pragma unroll
        for (int r = 0; r < 64; ++r) dst[base + (r << 5)] = ws24::unpack(d[r], g);
    }
}
// the pack's store pattern alone (no math): 3 of 4 lanes store a dword at 3e + q
__global__ __launch_bounds__(512) void store34_l3(const float* __restrict__ a, uint8_t* __restrict__ p, size_t ntile) {
    const unsigned t = threadIdx.x, base = l3_base(t), g = t & 7u;
    for (size_t tile = blockIdx.x; tile < ntile; tile += gridDim.x) {
        const float* src = a + (tile << 15);
        uint8_t* dst = p + 3 * (tile << 15);
        float v[64];
#pragma unroll
        for (int r = 0; r < 64; ++r) v[r] = src[base + (r << 5)];
#pragma unroll
        for (int r = 0; r < 64; ++r)
            if ((g & 3u) != 3u) *reinterpret_cast<uint32_t*>(dst + ws24::boff(base + (r << 5))) = __float_as_uint(v[r]);
    }
}
// pack with the math but stores through LDS: the tile's packed 96 KiB is
// written to LDS, then streamed out as 16 B per lane (whole 128-B lines)
__global__ __launch_bounds__(512) void pack_l3_lds(const float* __restrict__ a, uint8_t* __restrict__ p, size_t ntile) {
    __shared__ uint32_t sm[3 << 13];  // 96 KiB
    const unsigned t = threadIdx.x, base = l3_base(t), g = t & 7u;
    for (size_t tile = blockIdx.x; tile < ntile; tile += gridDim.x) {
        const float* src = a + (tile << 15);
        uint4* dst = reinterpret_cast<uint4*>(p + 3 * (tile << 15));
        float v[64];
#pragma unroll
        for (int r = 0; r < 64; ++r) v[r] = src[base + (r << 5)];
#pragma unroll
        for (int r = 0; r < 64; ++r) {
            const uint32_t d = ws24::pack(v[r], g);
            if ((g & 3u) != 3u) sm[ws24::boff(base + (r << 5)) >> 2] = d;
        }
        __syncthreads();
        const uint4* s4 = reinterpret_cast<const uint4*>(sm);
#pragma unroll
        for (int k = 0; k < 12; ++k) dst[t + 512 * k] = s4[t + 512 * k];
        __syncthreads();
    }
}
__global__ void fill(float* a, size_t n) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        uint32_t h = (uint32_t)i * 2654435761u ^ (uint32_t)(i >> 32);
        h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
        uint32_t h2 = h * 747796405u + 2891336453u;
        // ~N(0,1) from two uniforms (Box-Muller), spiky tail every 1e6
        const float u1 = (h >> 8) * (1.0f / 16777216.0f) + 1e-9f, u2 = (h2 >> 8) * (1.0f / 16777216.0f);
        float z = sqrtf(-2.0f * logf(u1)) * cosf(6.2831853f * u2);
        if ((i % 1000003) == 7) z *= 1e4f;
        a[i] = z;
    }
}

int main() {
    const size_t n = (size_t)1 << 29;  // 2 GiB of floats
    float *a, *b;
    CHECK(hipMalloc(&a, n * 4));
    CHECK(hipMalloc(&b, n * 4));
    CHECK(hipMemset(a, 0, n * 4));
    int cus = 256;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    // bytes per element moved (read + write): 8 for the copies, 7 for the
    // 4 B <-> 3 B pack / unpack kernels (round 2 printed every line at 8, which
    // overstated the pack rows by 8/7: pack_l3_lds is 5.45 TB/s, not 6.23)
    double bpe = 8.0;
    auto run = [&](const char* name, auto launch) {
        launch();
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(e0));
        for (int i = 0; i < 10; ++i) launch();
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-28s %8.1f us  %6.2f TB/s (read+write)\n", name, 1e3 * ms / 10, bpe * n / (ms / 10 * 1e-3) / 1e12);
    };
    for (int g : {1, 2, 4, 8}) {
        char nm[64];
        snprintf(nm, 64, "copy4 grid %dx", g);
        run(nm, [&] { hipLaunchKernelGGL(copy4, dim3(cus * g), dim3(256), 0, 0, (const float4*)a, (float4*)b, n / 4); });
        snprintf(nm, 64, "copy1 grid %dx", g);
        run(nm, [&] { hipLaunchKernelGGL(copy1, dim3(cus * g), dim3(256), 0, 0, a, b, n); });
    }
    for (int g : {1, 2}) {
        char nm[64];
        snprintf(nm, 64, "copy_l3 (dword) %d/CU", g);
        run(nm, [&] { hipLaunchKernelGGL(copy_l3, dim3(cus * g), dim3(512), 0, 0, a, b, n >> 15); });
        snprintf(nm, 64, "copy_l3q (dwordx4) %d/CU", g);
        run(nm, [&] { hipLaunchKernelGGL(copy_l3q, dim3(cus * g), dim3(512), 0, 0, a, b, n >> 15); });
    }
    uint8_t* pk;
    CHECK(hipMalloc(&pk, n * 3));
    hipLaunchKernelGGL(fill, dim3(cus * 4), dim3(256), 0, 0, a, n);
    bpe = 7.0;
    run("pack_l3 (4 B in, 3 B out)", [&] { hipLaunchKernelGGL(pack_l3, dim3(cus), dim3(512), 0, 0, a, pk, n >> 15); });
    run("store34_l3 (no math)", [&] { hipLaunchKernelGGL(store34_l3, dim3(cus), dim3(512), 0, 0, a, pk, n >> 15); });
    run("pack_l3_lds (LDS-staged)", [&] { hipLaunchKernelGGL(pack_l3_lds, dim3(cus), dim3(512), 0, 0, a, pk, n >> 15); });
    run("pack_l3 2/CU", [&] { hipLaunchKernelGGL(pack_l3, dim3(2 * cus), dim3(512), 0, 0, a, pk, n >> 15); });
    run("unpack_l3 (3 B in, 4 B out)", [&] { hipLaunchKernelGGL(unpack_l3, dim3(cus), dim3(512), 0, 0, pk, b, n >> 15); });
    CHECK(hipDeviceSynchronize());
    // round-trip error on the first 2^24 elements
    const size_t m = (size_t)1 << 24;
    std::vector<float> ha(m), hb(m);
    CHECK(hipMemcpy(ha.data(), a, m * 4, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(hb.data(), b, m * 4, hipMemcpyDeviceToHost));
    double se = 0, sr = 0, worst = 0;
    for (size_t i = 0; i < m; i += 8) {
        float gm = 0;
        for (int k = 0; k < 8; ++k) gm = fmaxf(gm, fabsf(ha[i + k]));
        for (int k = 0; k < 8; ++k) {
            const double e = (double)hb[i + k] - ha[i + k];
            se += e * e; sr += (double)ha[i + k] * ha[i + k];
            if (gm > 0) worst = fmax(worst, fabs(e) / gm);
        }
    }
    printf("ws24 round trip: rel-L2 %.3e, max |err| / group max %.3e (bound 2^-22 = %.3e)\n", sqrt(se / sr), worst,
           ldexp(1.0, -22));
    return 0;
}
