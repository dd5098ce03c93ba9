// Streaming-rate calibration for the codec's pass shapes.
// Why does a plain copy top out near 5.4 TB/s here while the microarch guide
// quotes 6.29 TB/s for a float4 copy and an LDS-staged 4 B -> 3 B pack reaches
// 6.2?  Measures read-only, write-only and mixed streams by read:write ratio,
// access shape, blocks per CU, cache policy (nt) and footprint.
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/streambench2 tools/streambench2.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                    \
    do {                                                                            \
        hipError_t e = (x);                                                         \
        if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
    } while (0)

typedef float f4v __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ float4 ld(const float4* p) {
    if constexpr (NT) {
        const f4v v = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p));
        return make_float4(v.x, v.y, v.z, v.w);
    } else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(float4* p, float4 v) {
    if constexpr (NT) {
        f4v w = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(w, reinterpret_cast<f4v*>(p));
    } else *p = v;
}

// U float4 per lane per iteration, block-contiguous chunks of 256*U float4
template <int U, bool NT>
__global__ __launch_bounds__(256) void rd(const float4* __restrict__ a, float* __restrict__ out, size_t n4) {
    float s = 0.f;
    const size_t per = 256ull * U;
    for (size_t base = blockIdx.x * per; base < n4; base += (size_t)gridDim.x * per) {
        float4 v[U];
#pragma unroll
        for (int k = 0; k < U; ++k) v[k] = ld<NT>(a + base + k * 256 + threadIdx.x);
#pragma unroll
        for (int k = 0; k < U; ++k) s += v[k].x + v[k].y + v[k].z + v[k].w;
    }
    if (s == 12345.678f) out[threadIdx.x] = s;
}
template <int U, bool NT>
__global__ __launch_bounds__(256) void wr(float4* __restrict__ b, size_t n4) {
    const size_t per = 256ull * U;
    const float4 z = make_float4(1.f, 2.f, 3.f, 4.f);
    for (size_t base = blockIdx.x * per; base < n4; base += (size_t)gridDim.x * per) {
#pragma unroll
        for (int k = 0; k < U; ++k) st<NT>(b + base + k * 256 + threadIdx.x, z);
    }
}
// read R float4, write W float4 per "unit" of 256 lanes (R, W in 1..8); the
// written array is W/R the size of the read one
template <int R, int W, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void mix(const float4* __restrict__ a, float4* __restrict__ b, size_t units) {
    for (size_t u = blockIdx.x; u < units; u += gridDim.x) {
        float4 v[R];
#pragma unroll
        for (int k = 0; k < R; ++k) v[k] = ld<NTL>(a + u * (256 * R) + k * 256 + threadIdx.x);
#pragma unroll
        for (int k = 0; k < W; ++k) {
            float4 o = v[k % R];
            if (k >= R) o.x += 1.f;
#pragma unroll
            for (int j = k + W; j < R; j += W) { o.x += v[j].x; o.y += v[j].y; o.z += v[j].z; o.w += v[j].w; }
            st<NTS>(b + u * (256 * W) + k * 256 + threadIdx.x, o);
        }
    }
}
// persistent 512-thread copy over 2^15-float tiles with the next tile's loads
// in flight while the current one is stored (the row passes' pipeline shape)
template <bool NTL, bool NTS>
__global__ __launch_bounds__(512) void copy_tile_pf(const float4* __restrict__ a, float4* __restrict__ b, size_t ntile) {
    const unsigned t = threadIdx.x;
    float4 cur[16], nxt[16];
    size_t tile = blockIdx.x;
    if (tile >= ntile) return;
#pragma unroll
    for (int r = 0; r < 16; ++r) cur[r] = ld<NTL>(a + (tile << 13) + r * 512 + t);
    for (; tile < ntile; tile += gridDim.x) {
        const size_t nt = tile + gridDim.x;
        if (nt < ntile) {
#pragma unroll
            for (int r = 0; r < 16; ++r) nxt[r] = ld<NTL>(a + (nt << 13) + r * 512 + t);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) st<NTS>(b + (tile << 13) + r * 512 + t, cur[r]);
#pragma unroll
        for (int r = 0; r < 16; ++r) cur[r] = nxt[r];
    }
}

int main(int argc, char** argv) {
    const size_t n = (size_t)1 << 29;  // 2 GiB of floats
    float *a, *b, *o;
    CHECK(hipMalloc(&a, n * 4));
    CHECK(hipMalloc(&b, n * 4));
    CHECK(hipMalloc(&o, 4096));
    CHECK(hipMemset(a, 0, n * 4));
    CHECK(hipMemset(b, 0, n * 4));
    int cus = 256;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const int reps = 10;
    auto run = [&](const char* name, double bytes, auto launch) {
        launch();
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(e0));
        for (int i = 0; i < reps; ++i) launch();
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        const double us = 1e3 * ms / reps;
        printf("%-44s %9.1f us  %6.2f TB/s\n", name, us, bytes / (us * 1e-6) / 1e12);
        fflush(stdout);
    };
    const size_t n4 = n / 4;
    char nm[96];
    // read-only / write-only
    for (int g : {2, 4, 8}) {
        snprintf(nm, 96, "read  U8 %d/CU", g);
        run(nm, n * 4.0, [&] { hipLaunchKernelGGL((rd<8, false>), dim3(cus * g), dim3(256), 0, 0, (const float4*)a, o, n4); });
        snprintf(nm, 96, "read  U8 nt %d/CU", g);
        run(nm, n * 4.0, [&] { hipLaunchKernelGGL((rd<8, true>), dim3(cus * g), dim3(256), 0, 0, (const float4*)a, o, n4); });
        snprintf(nm, 96, "write U8 %d/CU", g);
        run(nm, n * 4.0, [&] { hipLaunchKernelGGL((wr<8, false>), dim3(cus * g), dim3(256), 0, 0, (float4*)b, n4); });
        snprintf(nm, 96, "write U8 nt %d/CU", g);
        run(nm, n * 4.0, [&] { hipLaunchKernelGGL((wr<8, true>), dim3(cus * g), dim3(256), 0, 0, (float4*)b, n4); });
    }
    // mixed: 1 GiB read side so every shape fits; units of 256 lanes x R float4
    const size_t rd_f4 = n4 / 2;
    auto mixrun = [&](const char* tag, int R, int W, auto kern) {
        const size_t units = rd_f4 / (256 * R) < n4 / (256 * W) ? rd_f4 / (256 * R) : n4 / (256 * W);
        const double bytes = units * 256.0 * 16.0 * (R + W);
        for (int g : {2, 4, 8}) {
            snprintf(nm, 96, "%s %d:%d %d/CU", tag, R, W, g);
            run(nm, bytes, [&] { hipLaunchKernelGGL(kern, dim3(cus * g), dim3(256), 0, 0, (const float4*)a, (float4*)b, units); });
        }
    };
    mixrun("mix", 4, 4, mix<4, 4, false, false>);
    mixrun("mix nt-st", 4, 4, mix<4, 4, false, true>);
    mixrun("mix nt-ld", 4, 4, mix<4, 4, true, false>);
    mixrun("mix nt-both", 4, 4, mix<4, 4, true, true>);
    mixrun("mix", 8, 8, mix<8, 8, false, false>);
    mixrun("mix", 4, 3, mix<4, 3, false, false>);
    mixrun("mix", 4, 1, mix<4, 1, false, false>);
    mixrun("mix nt-st", 4, 1, mix<4, 1, false, true>);
    mixrun("mix", 1, 4, mix<1, 4, false, false>);
    mixrun("mix", 2, 8, mix<2, 8, false, false>);
    mixrun("mix", 3, 4, mix<3, 4, false, false>);
    // persistent prefetching tile copy, 2 GiB -> 2 GiB
    for (int g : {1, 2}) {
        snprintf(nm, 96, "tile_pf %d/CU", g);
        run(nm, n * 8.0, [&] { hipLaunchKernelGGL((copy_tile_pf<false, false>), dim3(cus * g), dim3(512), 0, 0, (const float4*)a, (float4*)b, n >> 15); });
        snprintf(nm, 96, "tile_pf nt-st %d/CU", g);
        run(nm, n * 8.0, [&] { hipLaunchKernelGGL((copy_tile_pf<false, true>), dim3(cus * g), dim3(512), 0, 0, (const float4*)a, (float4*)b, n >> 15); });
        snprintf(nm, 96, "tile_pf nt-both %d/CU", g);
        run(nm, n * 8.0, [&] { hipLaunchKernelGGL((copy_tile_pf<true, true>), dim3(cus * g), dim3(512), 0, 0, (const float4*)a, (float4*)b, n >> 15); });
    }
    // footprint: the same 4:4 copy over 64 MiB .. 2 GiB read sides
    for (size_t mib : {64, 256, 512, 2048}) {
        const size_t f4 = mib * (1u << 20) / 16;
        const size_t units = f4 / 1024;
        snprintf(nm, 96, "mix 4:4 4/CU read side %zu MiB", mib);
        run(nm, units * 256.0 * 16.0 * 8, [&] { hipLaunchKernelGGL((mix<4, 4, false, false>), dim3(cus * 4), dim3(256), 0, 0, (const float4*)a, (float4*)b, units); });
    }
    (void)argc; (void)argv;
    return 0;
}
