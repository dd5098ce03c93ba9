// Exact multi-threaded evaluation of the reference seed's serial float32 sum.
//
// The Eden seed (openfl/pipelines/eden_pipeline.py:771) hashes
// `sum(data.flatten())`: a left-to-right float32 sum, s <- fl(s + x_i), whose
// every rounding depends on the previous one.  Its value decides the seed and
// so every byte of the payload; it has to be reproduced exactly.
//
// Within one binade the chain is integer arithmetic.  While |s| stays in
// [2^e, 2^(e+1)) every partial sum is a multiple of u = 2^(e-23), and
//   fl(s + x) = s + u * R,  R = x/u rounded to the nearest integer,
// ties broken so that (s/u + R) is even (round-half-even of the sum's last
// significand bit).  x/u is exact (a power-of-two scaling), so R is the
// integer rint(x/u) except at ties, where the choice depends only on the
// parity of s/u.  A run of elements can therefore be summed as integers in
// parallel and stitched together afterwards:
//   phase A (threads): a float64 sum of every 256-element sub-chunk; the
//           prefix of those estimates the serial sum at each sub-chunk start
//           and so its binade e (the serial sum's rounding drift is far below
//           a binade except right at a boundary, where the check below sends
//           the sub-chunk to the scalar loop);
//   phase B (threads): per sub-chunk, with the estimated e: the prefix sums of
//           R relative to the sub-chunk start, their min / max, and every tie
//           (its relative prefix and the other candidate's direction);
//   phase C (one thread, in order): with the exact s at the sub-chunk start,
//           if s is in the guessed binade and every partial sum
//           S0 + prefix (+- the ties' corrections) stays strictly inside
//           [2^23 + 1, 2^24 - 1] in magnitude -- so the exact s + x is in the
//           binade too and the grid u applies -- the ties are resolved in
//           order by parity and s = (S0 + prefix_end + corrections) * u;
//           otherwise (binade crossing, zero / subnormal / non-finite values,
//           many ties) the sub-chunk runs the plain serial loop.
// Phase C touches each sub-chunk once in O(1 + ties); the serial loop only
// runs where the partial sums cross a binade.  Bit-identical to the plain
// loop by construction (tests/test_serial_sum.py checks it on adversarial
// inputs: ties, binade crossings, zeros, subnormals, Inf / NaN).
#include <algorithm>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "ofl_util.h"

namespace {

constexpr int kG = 256;      // sub-chunk
constexpr int kTieCap = 6;   // ties per sub-chunk resolved in phase C (more: serial loop)
constexpr int64_t kLo = (1ll << 23) + 1, kHi = (1ll << 24) - 1;

struct Sub {
    int64_t pre_end, lo, hi;
    int64_t tpre[kTieCap];
    int8_t tdel[kTieCap];
    int16_t ntie;
    int16_t e;   // guessed binade; kNoBinade: none (phase C runs the serial loop)
    double dsum;
};
constexpr int16_t kNoBinade = -32768;

// A small persistent pool: try_run(n, w, f) calls f(0..n-1) on the caller and
// (at least) w workers.  One job at a time; a caller that finds the pool busy
// gets false and runs serially (concurrent plugin calls keep their own core).
class Pool {
   public:
    static Pool& get() {
        static Pool* p = new Pool;  // never destroyed: its threads live as long as the process
        return *p;
    }
    bool try_run(int n, int workers, const std::function<void(int)>& f) {
        std::unique_lock<std::mutex> busy(run_m_, std::try_to_lock);
        if (!busy.owns_lock()) return false;
        ensure(workers);
        {
            std::lock_guard<std::mutex> g(m_);
            job_ = &f;
            njob_ = n;
            next_.store(1);
            pending_ = (int)th_.size();  // every worker checks in once per job
            ++gen_;
        }
        cv_.notify_all();
        f(0);
        for (int i = next_++; i < n; i = next_++) f(i);  // help with whatever is left
        std::unique_lock<std::mutex> g(m_);
        done_.wait(g, [&] { return pending_ == 0; });
        job_ = nullptr;
        return true;
    }

   private:
    void ensure(int workers) {
        while ((int)th_.size() < workers) th_.emplace_back([this] { loop(); });
    }
    void loop() {
        int seen = 0;
        for (;;) {
            const std::function<void(int)>* f;
            int n;
            {
                std::unique_lock<std::mutex> g(m_);
                cv_.wait(g, [&] { return gen_ != seen; });
                seen = gen_;
                f = job_;
                n = njob_;
            }
            if (f)
                for (int i = next_++; i < n; i = next_++) (*f)(i);
            std::lock_guard<std::mutex> g(m_);
            if (f && --pending_ == 0) done_.notify_all();
        }
    }
    std::mutex run_m_, m_;
    std::condition_variable cv_, done_;
    std::vector<std::thread> th_;
    const std::function<void(int)>* job_ = nullptr;
    int njob_ = 0, pending_ = 0, gen_ = 0;
    std::atomic<int> next_{0};
};

float serial_loop(const float* x, int64_t n, float s) {
    for (int64_t i = 0; i < n; ++i) s = s + x[i];
    return s;
}

void phase_b(const float* x, int len, Sub& b) {
    const float f = (float)b.dsum;  // estimate of the serial sum at the sub-chunk start
    b.e = kNoBinade;
    if (!std::isnormal(f)) return;
    const int e = std::ilogb(f);
    if (e < -103) return;  // u = 2^(e-23) must be a normal float
    const float scale = std::ldexp(1.0f, 23 - e);
    int64_t p = 0, lo = INT64_MAX, hi = INT64_MIN;
    int nt = 0;
    bool nan = false;
    for (int j = 0; j < len; ++j) {
        float q = x[j] * scale;  // exact (power-of-two scaling)
        nan |= q != q;
        // |R| >= 2^25 leaves the range whatever S0 is; the clamp keeps R in int range
        q = q > 0x1p25f ? 0x1p25f : q;
        q = q < -0x1p25f ? -0x1p25f : q;
        // round half even: the 1.5 * 2^23 shift rounds in the FPU's default mode;
        // |q| >= 2^23 is an integer already
        const float m = (q + 0x1.8p23f) - 0x1.8p23f;
        const float r = std::fabs(q) < 0x1p23f ? m : q;
        if (std::fabs(q - r) == 0.5f) {
            if (nt < kTieCap) {
                b.tpre[nt] = p;
                b.tdel[nt] = q > r ? 1 : -1;
            }
            ++nt;
        }
        p += (int64_t)r;
        lo = p < lo ? p : lo;
        hi = p > hi ? p : hi;
    }
    if (nan) return;
    if (nt > kTieCap) return;
    b.pre_end = p;
    b.lo = lo;
    b.hi = hi;
    b.ntie = (int16_t)nt;
    b.e = (int16_t)e;
}

// exact continuation of s over one sub-chunk through its phase-B summary;
// false: the summary does not apply (the caller runs the serial loop)
bool phase_c(const Sub& b, float& s) {
    if (b.e == kNoBinade || !std::isnormal(s) || std::ilogb(s) != b.e) return false;
    const int64_t S0 = (int64_t)std::ldexp(s, 23 - b.e);  // exact integer in [2^23, 2^24)
    const int64_t nt = b.ntie;
    if (S0 > 0 ? !(S0 + b.lo - nt >= kLo && S0 + b.hi + nt <= kHi)
               : !(S0 + b.hi + nt <= -kLo && S0 + b.lo - nt >= -kHi))
        return false;
    int64_t c = 0;
    for (int t = 0; t < nt; ++t)
        if ((S0 + b.tpre[t] + c) & 1) c += b.tdel[t];
    s = std::ldexp((float)(S0 + b.pre_end + c), b.e - 23);  // |S| < 2^24: exact
    return true;
}

int default_threads() {
    static const int n = [] {
        const char* v = std::getenv("OFL_SUM_THREADS");
        int t = v ? std::atoi(v) : 8;
        const int hw = (int)std::thread::hardware_concurrency();
        if (hw > 0) t = std::min(t, hw);
        return std::max(1, std::min(t, 64));
    }();
    return n;
}

}  // namespace

namespace ofl {
float serial_sum_f32_mt_cb(const float* x, int64_t n, float* dst, int nthreads, void (*after_copy)(void*),
                               void* ctx) {
    if (nthreads <= 0) nthreads = default_threads();
    const int64_t K = (n + kG - 1) / kG;
    auto plain = [&] {
        if (dst && n) std::memcpy(dst, x, sizeof(float) * n);
        if (after_copy) after_copy(ctx);
        return serial_loop(x, n, 0.0f);
    };
    if (nthreads <= 1 || K < 64) return plain();
    std::vector<Sub> subs(K);
    const int parts = (int)std::min<int64_t>(nthreads * 4, K);
    auto range = [&](int i, int64_t& k0, int64_t& k1) {
        k0 = K * i / parts;
        k1 = K * (i + 1) / parts;
    };
    // phase A: float64 sums of the sub-chunks (and the copy)
    const std::function<void(int)> fa = [&](int i) {
        int64_t k0, k1;
        range(i, k0, k1);
        if (dst) std::memcpy(dst + k0 * kG, x + k0 * kG, sizeof(float) * (std::min(n, k1 * kG) - k0 * kG));
        for (int64_t k = k0; k < k1; ++k) {
            const float* xs = x + k * kG;
            const int len = (int)std::min<int64_t>(kG, n - k * kG);
            double a0 = 0, a1 = 0, a2 = 0, a3 = 0;
            int j = 0;
            for (; j + 4 <= len; j += 4) {
                a0 += xs[j];
                a1 += xs[j + 1];
                a2 += xs[j + 2];
                a3 += xs[j + 3];
            }
            for (; j < len; ++j) a0 += xs[j];
            subs[k].dsum = (a0 + a1) + (a2 + a3);
        }
    };
    if (!Pool::get().try_run(parts, nthreads - 1, fa)) return plain();
    if (after_copy) after_copy(ctx);
    double run = 0.0;  // dsum -> the estimate at each sub-chunk's start
    for (int64_t k = 0; k < K; ++k) {
        const double d = subs[k].dsum;
        subs[k].dsum = run;
        run += d;
    }
    // phase B: integer prefix summaries in the estimated binades
    const std::function<void(int)> fb = [&](int i) {
        int64_t k0, k1;
        range(i, k0, k1);
        for (int64_t k = k0; k < k1; ++k) phase_b(x + k * kG, (int)std::min<int64_t>(kG, n - k * kG), subs[k]);
    };
    if (!Pool::get().try_run(parts, nthreads - 1, fb))
        for (int i = 0; i < parts; ++i) fb(i);
    // phase C: in order, exact
    float s = 0.0f;
    for (int64_t k = 0; k < K; ++k)
        if (!phase_c(subs[k], s)) s = serial_loop(x + k * kG, std::min<int64_t>(kG, n - k * kG), s);
    return s;
}

}  // namespace ofl

extern "C" {

// exact serial float32 sum of x[0..n) (plus a copy of x into dst if dst is
// not NULL) on up to nthreads threads (<= 0: OFL_SUM_THREADS, default 8)
float ofl_serial_sum_f32_mt(const float* x, int64_t n, float* dst, int nthreads) {
    return ofl::serial_sum_f32_mt_cb(x, n, dst, nthreads, nullptr, nullptr);
}

}  // extern "C"
