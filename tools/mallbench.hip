// mallbench.hip -- streaming bandwidth vs working-set size on MI355X.
// In-place read-modify-write (the FWHT pass pattern: read 4 B + write 4 B per
// element) over buffers of 8 MiB .. 4 GiB, repeated; also read-only and
// write-only sweeps.  Tells whether pass intermediates that fit the 256 MiB
// Infinity Cache stream faster than HBM.
// Build: hipcc --offload-arch=gfx950 -O3 -o mallbench mallbench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void rmw(float4* p, size_t n4, float a) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    size_t stride = (size_t)gridDim.x * blockDim.x;
    for (; i < n4; i += stride) {
        float4 v = p[i];
        v.x = v.x * a + 1.f; v.y = v.y * a + 1.f; v.z = v.z * a + 1.f; v.w = v.w * a + 1.f;
        p[i] = v;
    }
}
__global__ void rd(const float4* p, size_t n4, float* out) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    size_t stride = (size_t)gridDim.x * blockDim.x;
    float s = 0.f;
    for (; i < n4; i += stride) { float4 v = p[i]; s += v.x + v.y + v.z + v.w; }
    if (s == 12345.678f) out[0] = s;
}
__global__ void wr(float4* p, size_t n4) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    size_t stride = (size_t)gridDim.x * blockDim.x;
    for (; i < n4; i += stride) p[i] = make_float4(1.f, 2.f, 3.f, 4.f);
}

int main() {
    size_t maxb = 4ull << 30;
    float4* buf; float* out;
    hipMalloc(&buf, maxb); hipMalloc(&out, 4);
    hipMemset(buf, 0, maxb);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    const int grid = 256 * 8, block = 256;
    printf("size_MiB  rmw_GBps(r+w)  read_GBps  write_GBps\n");
    for (size_t mb = 8; mb <= 4096; mb *= 2) {
        size_t n4 = (mb << 20) / 16;
        int reps = mb <= 256 ? 50 : 10;
        float res[3];
        for (int k = 0; k < 3; ++k) {
            for (int w = 0; w < 3; ++w) {
                if (k == 0) rmw<<<grid, block>>>(buf, n4, 0.5f);
                else if (k == 1) rd<<<grid, block>>>(buf, n4, out);
                else wr<<<grid, block>>>(buf, n4);
            }
            hipEventRecord(a);
            for (int r = 0; r < reps; ++r) {
                if (k == 0) rmw<<<grid, block>>>(buf, n4, 0.5f);
                else if (k == 1) rd<<<grid, block>>>(buf, n4, out);
                else wr<<<grid, block>>>(buf, n4);
            }
            hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b);
            double bytes = (double)(mb << 20) * reps * (k == 0 ? 2 : 1);
            res[k] = bytes / (ms / 1e3) / 1e9;
        }
        printf("%8zu  %12.0f  %9.0f  %10.0f\n", mb, res[0], res[1], res[2]);
    }
    return 0;
}
