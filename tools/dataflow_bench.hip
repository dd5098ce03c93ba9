// A/B for VERDICT r04 item 3: does a persistent, slice-granular dataflow
// schedule whose FWHT intermediates stay in the 256 MiB Infinity Cache beat
// the codec's per-pass launches over 2 GiB waves?  Memory side only (an upper
// bound for a real kernel: no butterflies, no quantiser), the codec's own
// access shapes and bytes per element, encode direction:
//   A  row pass     x (2^15-float row tile)   -> ws (same tile)          4 + 4 B
//   B  column pass  ws (2^(p-15) rows x 2^(30-p) floats) -> ws in place   4 + 4 B
//   C  row pass     ws (row tile)             -> planes (1 B per element) 4 + 1 B
// (the decode is the mirror: 1 + 4, 4 + 4, 4 + 4).
//
// base:     three persistent launches per wave (2 GiB of ws per wave), as the codec.
// dataflow: ONE persistent launch.  Work items (a pass's tile of a slice) are
//           dequeued in a fixed order -- round r: A(r), B(r-1), C(r-2) -- and
//           a tile waits for the pass it depends on to be complete on its
//           slice (B(s) on A(s), C(s) on B(s), A(s) on C(s - NR): ws is a ring
//           of NR slices, NR x 2^p x 4 B <= 256 MiB).  Hand-off per
//           MI355X_MICROARCH.md "Valid forms" row 1: every ws byte stored sc1
//           (write-through, 16 B per lane), every storing wave drains
//           (vmcnt(0)), a workgroup barrier, then one lane adds to the slice's
//           counter (agent atomic); the consumer polls that counter with sc1
//           loads and reads ws with sc1 loads only.  Items depend only on
//           earlier items, so the persistent grid cannot deadlock; every spin
//           is bounded (a timeout flag ends it).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/dataflow_bench tools/dataflow_bench.hip
//   tools/bin/dataflow_bench [log2_elems=30] [reps=5]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                         \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } \
    } while (0)

typedef int rsrc_t __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned u4 __attribute__((ext_vector_type(4)));
__device__ f4 raw_load_f4(rsrc_t r, int voff, int soff, int aux) __asm("llvm.amdgcn.raw.buffer.load.v4f32");
__device__ void raw_store_f4(f4 v, rsrc_t r, int voff, int soff, int aux) __asm("llvm.amdgcn.raw.buffer.store.v4f32");
__device__ void raw_store_u4(u4 v, rsrc_t r, int voff, int soff, int aux) __asm("llvm.amdgcn.raw.buffer.store.v4i32");

constexpr int kNT = 512, kTile = 1 << 15, kPerT = kTile / 4 / kNT;  // float4s per thread per tile (16)
constexpr int kSC1 = 16;                                          // cache policy: sc1 (write-through / L1 bypass)

__device__ __forceinline__ rsrc_t mk_rsrc(const void* p, uint32_t bytes) {
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    rsrc_t r;
    r.x = (int)(uint32_t)a;
    r.y = (int)((uint32_t)(a >> 32) & 0xffffu);
    r.z = (int)bytes;
    r.w = 0x00020000;
    return r;
}

// one tile of one pass; WS_AUX: the ws loads' and stores' cache policy
template <int WS_AUX>
__device__ __forceinline__ void do_tile(int ph, int p, const float* x, float* ws, uint8_t* planes, int64_t s_elem,
                                        int64_t ws_elem, int t) {
    const unsigned tid = threadIdx.x;
    f4 v[kPerT];
    if (ph == 0) {  // A: x row tile -> ws row tile
        const rsrc_t r = mk_rsrc(x + s_elem + (int64_t)t * kTile, 4u * kTile);
#pragma unroll
        for (int k = 0; k < kPerT; ++k) v[k] = raw_load_f4(r, (int)(16 * tid), k * 16 * kNT, 0);
        const rsrc_t w = mk_rsrc(ws + ws_elem + (int64_t)t * kTile, 4u * kTile);
#pragma unroll
        for (int k = 0; k < kPerT; ++k) raw_store_f4(v[k] * 1.0001f, w, (int)(16 * tid), k * 16 * kNT, WS_AUX);
    } else if (ph == 1) {  // B: column tile in place: R rows x W floats
        const int rbits = p - 15, wl4 = 30 - p - 2;  // float4s per row segment: 2^wl4
        float* base = ws + ws_elem + (int64_t)t * (kTile >> rbits);
        const rsrc_t r = mk_rsrc(base, 4u * (uint32_t)((int64_t)kTile << rbits) - 4u * (uint32_t)(t * (kTile >> rbits)));
#pragma unroll
        for (int k = 0; k < kPerT; ++k) {
            const unsigned f = (unsigned)k * kNT + tid;
            const unsigned row = f >> wl4, c4 = f & ((1u << wl4) - 1u);
            v[k] = raw_load_f4(r, (int)(4u * (row * kTile + 4u * c4)), 0, WS_AUX);
        }
#pragma unroll
        for (int k = 0; k < kPerT; ++k) {
            const unsigned f = (unsigned)k * kNT + tid;
            const unsigned row = f >> wl4, c4 = f & ((1u << wl4) - 1u);
            raw_store_f4(v[k] * 0.9999f, r, (int)(4u * (row * kTile + 4u * c4)), 0, WS_AUX);
        }
    } else {  // C: ws row tile -> planes (1 B per element)
        const rsrc_t r = mk_rsrc(ws + ws_elem + (int64_t)t * kTile, 4u * kTile);
#pragma unroll
        for (int k = 0; k < kPerT; ++k) v[k] = raw_load_f4(r, (int)(16 * tid), k * 16 * kNT, WS_AUX);
        // 64 floats -> 16 dwords -> 4 x 16-B stores of bytes
        const rsrc_t w = mk_rsrc(planes + s_elem + (int64_t)t * kTile, kTile);
#pragma unroll
        for (int k = 0; k < kPerT; k += 4) {
            u4 o;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const f4 a = v[k + u];
                o[u] = ((unsigned)(a.x > 0.5f)) | ((unsigned)(a.y > 0.5f) << 8) | ((unsigned)(a.z > 0.5f) << 16) |
                       ((unsigned)(a.w > 0.5f) << 24);
            }
            raw_store_u4(o, w, (int)(16 * tid), (k / 4) * 16 * kNT, 0);
        }
    }
}

// base: one pass over the slices [s0, s0 + ns) of a wave; ws holds the wave
__global__ __launch_bounds__(kNT, 2) void k_pass(int ph, int p, const float* x, float* ws, uint8_t* planes, int s0,
                                                 int ns) {
    const int T = 1 << (p - 15);
    const int ntile = ns * T;
    for (int i = blockIdx.x; i < ntile; i += gridDim.x) {
        const int s = s0 + i / T, t = i % T;
        do_tile<0>(ph, p, x, ws, planes, (int64_t)s << p, (int64_t)(s - s0) << p, t);
    }
}

struct DfArgs {
    const float* x;
    float* ws;  // NR slices
    uint8_t* planes;
    const uint32_t* items;  // slice << 20 | phase << 16 | tile
    int nitems, p, nr;
    unsigned* next;   // dequeue head
    unsigned* done;   // [S][3] tiles complete per (slice, pass)
    unsigned* tmo;    // timeouts seen
    unsigned long long* waitcyc;  // summed wait cycles (lane 0 of each block)
};

__device__ __forceinline__ unsigned ld_sc1(const unsigned* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(kNT, 2) void k_dataflow(DfArgs a) {
    __shared__ unsigned item_s;
    const int T = 1 << (a.p - 15);
    unsigned long long waited = 0;
    for (;;) {
        if (threadIdx.x == 0) {
            const unsigned i = atomicAdd(a.next, 1u);
            unsigned it = 0xffffffffu;
            if (i < (unsigned)a.nitems) {
                it = a.items[i];
                const int s = (int)(it >> 20), ph = (int)((it >> 16) & 15u);
                const unsigned* w = nullptr;
                if (ph == 0 && s >= a.nr) w = a.done + 3 * (s - a.nr) + 2;
                if (ph == 1) w = a.done + 3 * s + 0;
                if (ph == 2) w = a.done + 3 * s + 1;
                if (w) {
                    const unsigned long long t0 = wall_clock64();
                    unsigned spins = 0;
                    while (ld_sc1(w) < (unsigned)T) {
                        __builtin_amdgcn_s_sleep(2);
                        if (++spins > (1u << 24)) { atomicAdd(a.tmo, 1u); break; }
                    }
                    waited += wall_clock64() - t0;
                }
            }
            item_s = it;
        }
        __syncthreads();
        const unsigned it = item_s;
        if (it == 0xffffffffu) break;
        const int s = (int)(it >> 20), ph = (int)((it >> 16) & 15u), t = (int)(it & 0xffffu);
        do_tile<kSC1>(ph, a.p, a.x, a.ws, a.planes, (int64_t)s << a.p, (int64_t)(s % a.nr) << a.p, t);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave: its stores drained, its loads landed
        __syncthreads();
        if (threadIdx.x == 0) atomicAdd(a.done + 3 * s + ph, 1u);  // agent-scope device atomic
        __syncthreads();  // item_s is rewritten next iteration
    }
    if (threadIdx.x == 0) atomicAdd(a.waitcyc, waited);
}

int main(int argc, char** argv) {
    const int lg = argc > 1 ? atoi(argv[1]) : 30;
    const int reps = argc > 2 ? atoi(argv[2]) : 5;
    const int64_t N = (int64_t)1 << lg;
    int ncu = 0;
    CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    const int grid = 2 * ncu;
    float* x;
    float* ws;
    uint8_t* planes;
    const int64_t wave = (int64_t)1 << 29;  // 2 GiB of ws per wave (the codec's)
    CHECK(hipMalloc(&x, 4 * N));
    CHECK(hipMalloc(&ws, 4 * std::max<int64_t>(wave, (int64_t)1 << 26)));
    CHECK(hipMalloc(&planes, N));
    CHECK(hipMemset(x, 0, 4 * N));
    unsigned *ctr, *d_items;
    unsigned long long* wc;
    const int max_items = 3 * (int)(N >> 15);
    CHECK(hipMalloc(&ctr, 4 * (2 + 3 * (N >> 15))));
    CHECK(hipMalloc(&wc, 8));
    CHECK(hipMalloc(&d_items, 4 * max_items));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const double moved = 21.0 * (double)N;  // bytes per element, encode direction
    printf("# dataflow_bench: %lld elements (x %.1f GiB), %d blocks, 21 B/element moved, %d reps (min ms)\n",
           (long long)N, 4.0 * N / (1 << 30), grid, reps);
    for (int p : {22, 23, 24, 25}) {
        const int S = (int)(N >> p);
        // base: per-pass launches over 2 GiB waves
        {
            float best = 1e30f;
            for (int r = 0; r < reps; ++r) {
                CHECK(hipEventRecord(e0));
                const int per = (int)(wave >> p);
                for (int s0 = 0; s0 < S; s0 += per) {
                    const int ns = std::min(per, S - s0);
                    for (int ph = 0; ph < 3; ++ph)
                        hipLaunchKernelGGL(k_pass, dim3(grid), dim3(kNT), 0, 0, ph, p, x, ws, planes, s0, ns);
                }
                CHECK(hipEventRecord(e1));
                CHECK(hipEventSynchronize(e1));
                float ms = 0;
                CHECK(hipEventElapsedTime(&ms, e0, e1));
                best = std::min(best, ms);
            }
            printf("p=%d base(2GiB waves)      %8.3f ms  %6.2f TB/s moved  %7.1f GiB/s of x\n", p, best,
                   moved / best / 1e9, 4.0 * N / (1 << 30) / (best / 1e3));
        }
        // base with MALL-sized waves (per-pass launches, ws re-read from the cache)
        {
            const int per = std::max(1, (int)(((int64_t)64 << 20) / 4 >> p));
            float best = 1e30f;
            for (int r = 0; r < reps; ++r) {
                CHECK(hipEventRecord(e0));
                for (int s0 = 0; s0 < S; s0 += per) {
                    const int ns = std::min(per, S - s0);
                    for (int ph = 0; ph < 3; ++ph)
                        hipLaunchKernelGGL(k_pass, dim3(grid), dim3(kNT), 0, 0, ph, p, x, ws, planes, s0, ns);
                }
                CHECK(hipEventRecord(e1));
                CHECK(hipEventSynchronize(e1));
                float ms = 0;
                CHECK(hipEventElapsedTime(&ms, e0, e1));
                best = std::min(best, ms);
            }
            printf("p=%d base(%3d MiB waves)   %8.3f ms  %6.2f TB/s moved  %7.1f GiB/s of x\n", p,
                   (int)((4ll * per) << p >> 20), best, moved / best / 1e9, 4.0 * N / (1 << 30) / (best / 1e3));
        }
        for (int cfg = 0; cfg < 4; ++cfg) {
            // lag L between the passes of one slice (round r: A(r), B(r - L),
            // C(r - 2L)); the ring must hold the 2L + 1 slices in flight, so
            // that every item depends only on earlier items
            const int L = cfg < 2 ? 1 : 2, nr = 2 * L + 1 + (cfg & 1);
            if (((int64_t)nr << p) * 4 > ((int64_t)384 << 20)) continue;
            std::vector<uint32_t> items;
            const int T = 1 << (p - 15);
            for (int r = 0; r < S + 2 * L; ++r)
                for (int ph = 0; ph < 3; ++ph) {
                    const int s = r - ph * L;
                    if (s < 0 || s >= S) continue;
                    for (int t = 0; t < T; ++t) items.push_back((uint32_t)s << 20 | (uint32_t)ph << 16 | (uint32_t)t);
                }
            CHECK(hipMemcpy(d_items, items.data(), 4 * items.size(), hipMemcpyHostToDevice));
            float best = 1e30f;
            unsigned tmo = 0;
            unsigned long long wcy = 0;
            for (int r = 0; r < reps; ++r) {
                CHECK(hipMemset(ctr, 0, 4 * (2 + 3 * S)));
                CHECK(hipMemset(wc, 0, 8));
                DfArgs a{x, ws, planes, d_items, (int)items.size(), p, nr, ctr, ctr + 2, ctr + 1, wc};
                CHECK(hipEventRecord(e0));
                hipLaunchKernelGGL(k_dataflow, dim3(grid), dim3(kNT), 0, 0, a);
                CHECK(hipEventRecord(e1));
                CHECK(hipEventSynchronize(e1));
                float ms = 0;
                CHECK(hipEventElapsedTime(&ms, e0, e1));
                unsigned t = 0;
                CHECK(hipMemcpy(&t, ctr + 1, 4, hipMemcpyDeviceToHost));
                tmo += t;
                if (ms < best) {
                    best = ms;
                    CHECK(hipMemcpy(&wcy, wc, 8, hipMemcpyDeviceToHost));
                }
            }
            printf("p=%d dataflow L=%d NR=%d (%3d MiB) %8.3f ms  %6.2f TB/s moved  %7.1f GiB/s of x  wait %.1f%% of block time%s\n",
                   p, L, nr, (int)((4ll * nr) << p >> 20), best, moved / best / 1e9, 4.0 * N / (1 << 30) / (best / 1e3),
                   100.0 * (double)wcy / 100.0 / ((double)grid * best * 1e3), tmo ? "  TIMEOUTS" : "");
        }
        fflush(stdout);
    }
    return 0;
}
