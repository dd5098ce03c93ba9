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
//           Where the estimated partial sums leave that binade the
//           sub-chunk is cut into up to three runs at the elements that
//           cross, each summarised in the binade the estimate is in there;
//   phase C (one thread, in order): with the exact s at a run's start,
//           if s is in the guessed binade and every partial sum
//           S0 + prefix (+- the ties' corrections) stays strictly inside
//           [2^23 + 1, 2^24 - 1] in magnitude -- so the exact s + x is in the
//           binade too and the grid u applies -- the ties are resolved in
//           order by parity and s = (S0 + prefix_end + corrections) * u,
//           and the element that crosses into the next run is one scalar
//           add; otherwise (a wrong guess, more crossings, zero / subnormal /
//           non-finite values, many ties) the rest of the sub-chunk runs the
//           plain serial loop (N(0, 0.01) data at 2^21: 1053 -> ~370 of 8192
//           sub-chunks).
// Phase C touches each sub-chunk once in O(1 + ties); the serial loop only
// runs where the partial sums cross a binade.  Bit-identical to the plain
// loop by construction (tests/test_serial_sum.py checks it on adversarial
// inputs: ties, binade crossings, zeros, subnormals, Inf / NaN).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cmath>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>

#include <unistd.h>
#include <vector>

#include "ofl_util.h"

namespace {

constexpr int kG = 256;      // sub-chunk
constexpr int kTieCap = 6;   // ties per sub-chunk resolved in phase C (more: serial loop)
constexpr int64_t kLo = (1ll << 23) + 1, kHi = (1ll << 24) - 1;

// one run of a sub-chunk summarised in one binade: elements [j0, j1); the
// element j1 (if j1 < len) takes the partial sums across a binade boundary and
// is added by one scalar step in phase C
struct Part {
    int64_t pre_end, lo, hi;
    int64_t tpre[kTieCap];
    int8_t tdel[kTieCap];
    int16_t ntie;
    int16_t e;   // guessed binade
    int16_t j0, j1;
    float up, down;  // 2^(23 - e), 2^(e - 23)
};
constexpr int kParts = 3;  // runs per sub-chunk (a sub-chunk crossing more binades runs the serial loop)
struct Sub {
    Part p[kParts];
    int8_t nparts;  // 0: the whole sub-chunk runs the serial loop
    int16_t jend;   // elements from here on (after the parts) run the serial loop
    double dsum;
};
// biased exponent field of a float (1..254: normal)
inline int expo(float f) {
    uint32_t b;
    std::memcpy(&b, &f, 4);
    return (int)((b >> 23) & 0xffu);
}
inline float pow2f(int k) {  // 2^k, -126 <= k <= 127
    const uint32_t b = (uint32_t)(k + 127) << 23;
    float f;
    std::memcpy(&f, &b, 4);
    return f;
}
constexpr int16_t kNoBinade = -32768;

// A small persistent pool: try_run(n, w, f) calls f(0..n-1) on the caller and
// (at least) w workers.  One job at a time per pool; Pool::run tries a few
// pools in turn, so concurrent plugin calls (the gRPC server's threads) each
// get workers of their own, and only a caller that finds every pool busy
// runs serially.  Fork-safe: a fork()ed child inherits the pools' state but
// none of their threads, so a pool created in another process (pid recorded
// at creation) always reports busy and the caller runs serially.
class Pool {
   public:
    static bool run(int n, int workers, const std::function<void(int)>& f) {
        static const int npools = [] {
            const char* e = getenv("OFL_SUM_POOLS");
            return std::max(1, std::min(16, e ? atoi(e) : 4));
        }();
        static std::mutex m;
        static Pool* pools[16] = {};  // never destroyed: their threads live as long as the process
        for (int i = 0; i < npools; ++i) {
            Pool* p;
            {
                std::lock_guard<std::mutex> g(m);
                if (!pools[i]) pools[i] = new Pool;
                p = pools[i];
            }
            if (p->try_run(n, workers, f)) return true;
        }
        return false;
    }
    bool try_run(int n, int workers, const std::function<void(int)>& f) {
        if (getpid() != pid_) return false;
        std::unique_lock<std::mutex> busy(run_m_, std::try_to_lock);
        if (!busy.owns_lock()) return false;
        ensure(workers);
        {
            std::lock_guard<std::mutex> g(m_);
            job_ = &f;
            njob_ = n;
            next_.store(1);
            pending_ = (int)th_.size();  // every worker checks in once per job
            gen_.fetch_add(1, std::memory_order_release);
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
            // a plugin call's phases come back to back: spin briefly (~2000 pauses)
            // before sleeping, so a wake-up does not cost a futex round trip
            for (int i = 0; i < 2000 && gen_.load(std::memory_order_acquire) == seen; ++i) __builtin_ia32_pause();
            const std::function<void(int)>* f;
            int n;
            {
                std::unique_lock<std::mutex> g(m_);
                cv_.wait(g, [&] { return gen_.load(std::memory_order_relaxed) != seen; });
                seen = gen_.load(std::memory_order_relaxed);
                f = job_;
                n = njob_;
            }
            if (f)
                for (int i = next_++; i < n; i = next_++) (*f)(i);
            std::lock_guard<std::mutex> g(m_);
            if (f && --pending_ == 0) done_.notify_all();
        }
    }
    const pid_t pid_ = getpid();
    std::mutex run_m_, m_;
    std::condition_variable cv_, done_;
    std::vector<std::thread> th_;
    const std::function<void(int)>* job_ = nullptr;
    int njob_ = 0, pending_ = 0;
    std::atomic<int> gen_{0};
    std::atomic<int> next_{0};
};

float serial_loop(const float* x, int64_t n, float s) {
    for (int64_t i = 0; i < n; ++i) s = s + x[i];
    return s;
}

// (an AVX2 clone beside the baseline, picked at load time: the two loops
// below are the multi-threaded sum's largest phase.  This file is host code;
// hipcc also runs it through the gfx950 pass, which has no clones.)
#if defined(__HIP_DEVICE_COMPILE__)
#define OFL_HOST_CLONES
#else
#define OFL_HOST_CLONES __attribute__((target_clones("avx2", "default")))
#endif
// R = x / u rounded half-even and each tie's other candidate (+1 / -1, 0: no
// tie), for j in [j0, len); false if some |x / u| > 2^22 (a step of more than
// a quarter of the sum: the relative prefix would leave int32)
OFL_HOST_CLONES bool steps(const float* x, int j0, int len, float scale, int32_t* R, int32_t* tie) {
    int bad = 0;
    for (int j = j0; j < len; ++j) {
        const float q = x[j] * scale;  // exact (power-of-two scaling)
        bad |= !(std::fabs(q) <= 0x1p22f);  // also NaN
        // round half even: the 1.5 * 2^23 shift rounds in the FPU's default mode
        const float qc = std::fabs(q) <= 0x1p22f ? q : 0.0f;
        const float r = (qc + 0x1.8p23f) - 0x1.8p23f;
        tie[j] = std::fabs(qc - r) == 0.5f ? (qc > r ? 1 : -1) : 0;
        R[j] = (int32_t)r;
    }
    return !bad;
}
// the binade of a float estimate (kNoBinade: zero / subnormal / non-finite, or
// a grid u below the normal range)
int binade(double est) {
    const int be = expo((float)est);
    if (be == 0 || be == 255) return kNoBinade;
    const int e = be - 127;
    return e < -103 ? kNoBinade : e;
}
bool inside(double S, int64_t lo, int64_t hi, int64_t nt) {  // a start S's partial sums stay in its binade
    return S > 0 ? (S + (double)(lo - nt) >= (double)kLo && S + (double)(hi + nt) <= (double)kHi)
                 : (S + (double)(hi + nt) <= -(double)kLo && S + (double)(lo - nt) >= -(double)kHi);
}

// Phase B of one sub-chunk: the whole sub-chunk as one run in the binade of
// the estimate at its start (the common case, vectorised); where the
// estimated partial sums leave that binade, up to kParts runs split at the
// elements that cross, each in the binade the estimate is in there.
OFL_HOST_CLONES void phase_b(const float* x, int len, Sub& b) {
    b.nparts = 0;
    b.jend = 0;
    int e = binade(b.dsum);
    if (e == kNoBinade) return;
    float scale = pow2f(23 - e);
    alignas(64) int32_t R[kG + 4];
    alignas(64) int32_t tie[kG + 4];
    if (!steps(x, 0, len, scale, R, tie)) return;
    for (int j = len; j < ((len + 3) & ~3); ++j) R[j] = tie[j] = 0;  // ragged tail: zero steps
    // the inclusive prefix, four lanes at a time, and its envelope
    typedef int32_t i4 __attribute__((ext_vector_type(4)));
    const i4 z = {0, 0, 0, 0};
    i4 carry = z, mn = {INT32_MAX, INT32_MAX, INT32_MAX, INT32_MAX}, mx = {INT32_MIN, INT32_MIN, INT32_MIN, INT32_MIN};
    int anytie = 0;
    alignas(64) int32_t P[kG + 4];
    for (int j = 0; j < len; j += 4) {
        i4 v = *reinterpret_cast<const i4*>(R + j);
        v += __builtin_shufflevector(z, v, 0, 4, 5, 6);
        v += __builtin_shufflevector(z, v, 0, 1, 4, 5);
        v += carry;
        *reinterpret_cast<i4*>(P + j) = v;
        carry = __builtin_shufflevector(v, v, 3, 3, 3, 3);
        mn = v < mn ? v : mn;
        mx = v > mx ? v : mx;
        const i4 t = *reinterpret_cast<const i4*>(tie + j);
        anytie |= (t.x | t.y | t.z | t.w);
    }
    // (lanes past len in a ragged last group hold P[len - 1]: a real partial sum)
    const int64_t lo = std::min(std::min(mn.x, mn.y), std::min(mn.z, mn.w));
    const int64_t hi = std::max(std::max(mx.x, mx.y), std::max(mx.z, mx.w));
    int nt = 0;
    if (anytie)
        for (int j = 0; j < len; ++j) nt += tie[j] != 0;
    if (nt <= kTieCap && inside(b.dsum * (double)scale, lo, hi, nt)) {  // one run
        Part& p = b.p[0];
        int t = 0;
        if (anytie)
            for (int j = 0; j < len; ++j)
                if (tie[j]) {
                    p.tpre[t] = P[j] - R[j];  // the prefix before element j
                    p.tdel[t++] = (int8_t)tie[j];
                }
        p.pre_end = P[len - 1];
        p.lo = lo;
        p.hi = hi;
        p.ntie = (int16_t)nt;
        p.e = (int16_t)e;
        p.up = scale;
        p.down = pow2f(e - 23);
        p.j0 = 0;
        p.j1 = (int16_t)len;
        b.nparts = 1;
        b.jend = (int16_t)len;
        return;
    }
    // runs split where the estimate crosses a binade boundary (scalar: rare)
    double est = b.dsum;
    int j0 = 0;
    while (j0 < len && b.nparts < kParts) {
        if (b.nparts > 0) {  // the grid of this run's binade
            e = binade(est);
            if (e == kNoBinade) break;
            scale = pow2f(23 - e);
            if (!steps(x, j0, len, scale, R, tie)) break;
        }
        Part& p = b.p[b.nparts];
        const double S = est * (double)scale;  // the estimated integer start
        int64_t acc = 0, plo = INT64_MAX, phi = INT64_MIN;
        int t = 0, j = j0;
        for (; j < len; ++j) {
            const int64_t a = acc + R[j];
            const int64_t ntn = t + (tie[j] != 0);
            if (ntn > kTieCap || !inside(S, std::min(plo, a), std::max(phi, a), ntn)) break;
            if (tie[j]) {
                p.tpre[t] = acc;
                p.tdel[t++] = (int8_t)tie[j];
            }
            acc = a;
            plo = std::min(plo, a);
            phi = std::max(phi, a);
        }
        p.pre_end = acc;
        p.lo = j > j0 ? plo : 0;
        p.hi = j > j0 ? phi : 0;
        p.ntie = (int16_t)t;
        p.e = (int16_t)e;
        p.up = scale;
        p.down = pow2f(e - 23);
        p.j0 = (int16_t)j0;
        p.j1 = (int16_t)j;
        ++b.nparts;
        for (int k = j0; k <= j && k < len; ++k) est += (double)x[k];  // through the crossing element
        j0 = j + 1;
        b.jend = (int16_t)std::min(j0, len);
    }
}

// exact continuation of s over one run through its summary; false: the
// summary does not apply (the caller runs the serial loop from the run's start)
bool run_c(const Part& b, float& s) {
    if (b.j1 == b.j0) return true;  // an empty run (the first element crossed)
    if (expo(s) - 127 != b.e) return false;  // also rejects 0 / subnormal / Inf / NaN
    const int64_t S0 = (int64_t)(s * b.up);  // exact integer in [2^23, 2^24) in magnitude
    const int64_t nt = b.ntie;
    if (S0 > 0 ? !(S0 + b.lo - nt >= kLo && S0 + b.hi + nt <= kHi)
               : !(S0 + b.hi + nt <= -kLo && S0 + b.lo - nt >= -kHi))
        return false;
    int64_t c = 0;
    for (int t = 0; t < nt; ++t)
        if ((S0 + b.tpre[t] + c) & 1) c += b.tdel[t];
    s = (float)(S0 + b.pre_end + c) * b.down;  // |S| < 2^24, a power-of-two scale: exact
    return true;
}

// phase C of one sub-chunk of len elements at x; returns false if some of it
// ran the serial loop
bool phase_c(const Sub& b, const float* x, int len, float& s) {
    for (int t = 0; t < b.nparts; ++t) {
        const Part& p = b.p[t];
        if (!run_c(p, s)) {
            s = serial_loop(x + p.j0, len - p.j0, s);
            return false;
        }
        if (p.j1 < len) s = s + x[p.j1];  // the crossing element
    }
    if (b.jend < len) {
        s = serial_loop(x + b.jend, len - b.jend, s);
        return false;
    }
    return true;
}

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
bool debug_on() {
    static const bool on = [] { const char* v = std::getenv("OFL_SUM_DEBUG"); return v && v[0] == '1'; }();
    return on;
}

int default_threads() {
    static const int n = [] {
        const char* v = std::getenv("OFL_SUM_THREADS");
        int t = v ? std::atoi(v) : 16;  // (8 -> 16 on the GPU box's 16 cores: 553 -> 502 us at 2^21)
        const int hw = (int)std::thread::hardware_concurrency();
        if (hw > 0) t = std::min(t, hw);
        return std::max(1, std::min(t, 64));
    }();
    return n;
}

}  // namespace

namespace ofl {
bool pool_run(int n, int workers, const std::function<void(int)>& f) { return Pool::run(n, workers, f); }

float serial_sum_f32_mt_cb(const float* x, int64_t n, float* dst, int nthreads, void (*after_copy)(void*),
                           void* ctx) {
    if (nthreads <= 0) nthreads = default_threads();
    auto plain = [&] {
        if (dst && n) std::memcpy(dst, x, sizeof(float) * n);
        if (after_copy) after_copy(ctx);
        return serial_loop(x, n, 0.0f);
    };
    if (nthreads <= 1 || (n + kG - 1) / kG < 64) return plain();
    // chunks of kChunk elements (the sub-chunk summaries stay a few MB for
    // any n); the estimate and the exact sum carry over from chunk to chunk
    constexpr int64_t kChunk = (int64_t)1 << 24;
    const int64_t Kmax = (std::min(n, kChunk) + kG - 1) / kG;
    thread_local std::vector<Sub> subs_tl;  // kept per calling thread: no fresh pages every call
    if ((int64_t)subs_tl.size() < Kmax) subs_tl.resize(Kmax);
    std::vector<Sub>& subs = subs_tl;
    double run = 0.0;  // float64 running sum: the estimate at each sub-chunk's start
    float s = 0.0f;    // the exact serial sum so far
    int64_t serial = 0;
    double ta = 0, tb = 0, tc = 0;
    for (int64_t c0 = 0; c0 < n; c0 += kChunk) {
        const float* xc = x + c0;
        const int64_t nc = std::min(kChunk, n - c0);
        const int64_t K = (nc + kG - 1) / kG;
        const int parts = (int)std::min<int64_t>(nthreads * 4, K);
        auto range = [&](int i, int64_t& k0, int64_t& k1) {
            k0 = K * i / parts;
            k1 = K * (i + 1) / parts;
        };
        const double t0 = debug_on() ? now_s() : 0.0;
        // phase A: float64 sums of the sub-chunks (and the copy)
        const std::function<void(int)> fa = [&](int i) {
            int64_t k0, k1;
            range(i, k0, k1);
            if (dst) std::memcpy(dst + c0 + k0 * kG, xc + k0 * kG, sizeof(float) * (std::min(nc, k1 * kG) - k0 * kG));
            for (int64_t k = k0; k < k1; ++k) {
                const float* xs = xc + k * kG;
                const int len = (int)std::min<int64_t>(kG, nc - k * kG);
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
        if (!Pool::run(parts, nthreads - 1, fa)) {
            // every pool is busy (other callers): the plain chain for the rest
            if (dst) std::memcpy(dst + c0, xc, sizeof(float) * (n - c0));
            if (after_copy) after_copy(ctx);
            return serial_loop(xc, n - c0, s);
        }
        if (after_copy && c0 + nc == n) after_copy(ctx);
        const double t1 = debug_on() ? now_s() : 0.0;
        for (int64_t k = 0; k < K; ++k) {
            const double d = subs[k].dsum;
            subs[k].dsum = run;
            run += d;
        }
        // phase B: integer prefix summaries in the estimated binades
        const std::function<void(int)> fb = [&](int i) {
            int64_t k0, k1;
            range(i, k0, k1);
            for (int64_t k = k0; k < k1; ++k) phase_b(xc + k * kG, (int)std::min<int64_t>(kG, nc - k * kG), subs[k]);
        };
        if (!Pool::run(parts, nthreads - 1, fb))
            for (int i = 0; i < parts; ++i) fb(i);
        // phase C: in order, exact
        const double t2 = debug_on() ? now_s() : 0.0;
        for (int64_t k = 0; k < K; ++k)
            serial += !phase_c(subs[k], xc + k * kG, (int)std::min<int64_t>(kG, nc - k * kG), s);
        if (debug_on()) {
            ta += t1 - t0;
            tb += t2 - t1;
            tc += now_s() - t2;
        }
    }
    if (debug_on())
        std::fprintf(stderr, "[ofl sum] n=%lld threads=%d A %.1f us B %.1f us C %.1f us serial sub-chunks %lld/%lld\n",
                     (long long)n, nthreads, 1e6 * ta, 1e6 * tb, 1e6 * tc, (long long)serial,
                     (long long)((n + kG - 1) / kG));
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
