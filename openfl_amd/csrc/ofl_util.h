// ofl_util.h -- small host-side helpers shared by the kernel sources.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <functional>
#include <map>
#include <mutex>

namespace ofl_util {

// f() once per device (kernel attributes, __constant__ uploads are
// per-device state); the result is remembered per device.  Each call site
// (lambda type) has its own table.
template <typename F>
hipError_t per_device_once(F f) {
    static std::mutex mu;
    static std::map<int, hipError_t> done;
    int dev = 0;
    const hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> g(mu);
    auto it = done.find(dev);
    if (it != done.end()) return it->second;
    const hipError_t r = f();
    done[dev] = r;
    return r;
}

// runs f() when the scope ends, on every return path
template <typename F>
struct ScopeExit {
    F f;
    explicit ScopeExit(F fn) : f(fn) {}
    ~ScopeExit() { f(); }
    ScopeExit(const ScopeExit&) = delete;
    ScopeExit& operator=(const ScopeExit&) = delete;
};

}  // namespace ofl_util

namespace ofl {
// f(0..n-1) on the caller and at least `workers` threads of a persistent
// native pool (csrc/serial_sum.cpp); false when every pool is busy with
// another caller (then nothing ran)
bool pool_run(int n, int workers, const std::function<void(int)>& f);
// exact serial float32 sum (csrc/serial_sum.cpp): s <- fl(s + x[i]) left to
// right, evaluated on up to nthreads threads (<= 0: the default); dst (or
// NULL) receives a copy of x, after which after_copy(ctx) (or NULL) runs on
// the calling thread while the sum goes on
float serial_sum_f32_mt_cb(const float* x, int64_t n, float* dst, int nthreads, void (*after_copy)(void*), void* ctx);
}  // namespace ofl
