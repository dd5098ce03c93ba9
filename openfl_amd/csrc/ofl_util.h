// ofl_util.h -- small host-side helpers shared by the kernel sources.
#pragma once
#include <hip/hip_runtime.h>

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

}  // namespace ofl_util
