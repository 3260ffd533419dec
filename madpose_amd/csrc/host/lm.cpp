// Host LM for LO -- see lm.h.
#include "lm.h"
#include "lm_eval.h"
#include "env.h"

#include <sched.h>

#include <chrono>
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <functional>
#include <mutex>
#include <thread>
#include <cmath>
#include <cstring>

namespace mp {

namespace {


inline void skew(const double *v, double *S) {
    S[0] = 0;
    S[1] = -v[2];
    S[2] = v[1];
    S[3] = v[2];
    S[4] = 0;
    S[5] = -v[0];
    S[6] = -v[1];
    S[7] = v[0];
    S[8] = 0;
}
inline void mm3(const double *A, const double *B, double *C) {
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) C[3 * r + c] = A[3 * r] * B[c] + A[3 * r + 1] * B[3 + c] + A[3 * r + 2] * B[6 + c];
}
inline void mv3(const double *A, const double *v, double *o) {
    for (int r = 0; r < 3; ++r) o[r] = A[3 * r] * v[0] + A[3 * r + 1] * v[1] + A[3 * r + 2] * v[2];
}
inline void mtv3(const double *A, const double *v, double *o) { // A^T v
    for (int r = 0; r < 3; ++r) o[r] = A[r] * v[0] + A[3 + r] * v[1] + A[6 + r] * v[2];
}

struct Params {
    double q[4], R[9], t[3], s, o0, o1, f0, f1;
};

struct Ctx {
    const HostPair *P;
    const std::vector<int> *sample;
    LMSettings S;
    bool has_o0, has_s_o1;
    int col[kNFull]; // full -> active column (-1 inactive)
    int n;
};

// Normal-equation accumulator in the full parameter layout (packed upper triangle).
// Inactive parameters accumulate harmlessly and are dropped by scatter().
struct Acc {
    double H[kNPack];
    double g[kNFull];
    double cost;
    void clear() {
        std::memset(H, 0, sizeof(H));
        std::memset(g, 0, sizeof(g));
        cost = 0.0;
    }
    void add(double r, const double *gf) {
        cost += 0.5 * r * r;
        int q = 0;
        for (int a = 0; a < kNFull; ++a) {
            g[a] += gf[a] * r;
            const double ja = gf[a];
            for (int b = a; b < kNFull; ++b) H[q++] += ja * gf[b];
        }
    }
    void merge(const Acc &o) {
        for (int q = 0; q < kNPack; ++q) H[q] += o.H[q];
        for (int a = 0; a < kNFull; ++a) g[a] += o.g[a];
        cost += o.cost;
    }
    void scatter(const Ctx &C, double *Hn, double *gn) const {
        std::memset(Hn, 0, sizeof(double) * C.n * C.n);
        std::memset(gn, 0, sizeof(double) * C.n);
        int q = 0;
        for (int a = 0; a < kNFull; ++a) {
            const int ca = C.col[a];
            if (ca >= 0) gn[ca] = g[a];
            for (int b = a; b < kNFull; ++b, ++q) {
                const int cb = C.col[b];
                if (ca >= 0 && cb >= 0) Hn[ca * C.n + cb] = Hn[cb * C.n + ca] = H[q];
            }
        }
    }
};

// Evaluates cost (and, when H != nullptr, normal equations) at parameters p.
// Small persistent pool for the residual loop of large LM problems (the LO's
// all-inlier fits, >= kPoolBlocks residual blocks: ~100-500 us per evaluation on one
// core, on the critical path of every LO); smaller problems (~10-100 us of work,
// comparable to a thread wake-up) run inline.  MADPOSE_LO_THREADS sets the pool size
// (default 8, of which 4 take the problems below kPoolWide blocks; 1 = off).  The
// blocks are reduced in fixed chunks in chunk order either way, so the result does not
// depend on the pool.
constexpr size_t kChunk = 256;
constexpr size_t kPoolBlocks = 2048;
// Workers spin (with pause) for a while after each job before they block on the
// condition variable: the evaluations of one LM follow each other within
// microseconds, and a futex wake-up per evaluation would cost about as much as the
// evaluation's share per thread.  The spin is bounded by time, not by a pause count
// (pause latency differs ~10x across x86 generations): MADPOSE_LO_SPIN = microseconds
// (0 = block right away).  Default 1000, or 0 when the process's CPU affinity share is
// smaller than kSpinCpusPerRank per rank on this host (LOCAL_WORLD_SIZE): spinning
// pays while the host has idle CPUs and costs when ranks oversubscribe one share
// (two ranks on one 16-CPU share, 730 pairs/s spinning vs 840 blocking).
// 1000 rather than round 5's 300: with 8 pairs in flight the pool's jobs from different
// pairs come further apart than 300 us, and a worker that has gone to sleep costs a
// wake-up -- ScanNet stand-in +3-6 % (7 of 8 same-box A/B pairs), tf -2.5 %, cal and sf
// within noise (profiles/r06/spin); blocking at once (0) costs the stand-in 15-25 %.
constexpr int kSpinCpusPerRank = 12; // about the threads one rank keeps busy (LO lanes, pool, sampler)
}  // namespace

int lo_spin_us() {
    static const int v = [] {
        if (std::getenv("MADPOSE_LO_SPIN")) return (int)env_int("MADPOSE_LO_SPIN", 0, 0, 1000000);
        int cpus = 0;
        cpu_set_t set;
        CPU_ZERO(&set);
        if (sched_getaffinity(0, sizeof(set), &set) == 0) cpus = CPU_COUNT(&set);
        const char *l = std::getenv("LOCAL_WORLD_SIZE");
        const int ranks = std::max(1, l ? std::atoi(l) : 1);
        return (cpus > 0 && cpus < kSpinCpusPerRank * ranks) ? 0 : 1000;
    }();
    return v;
}

namespace {
// Workers 1..kNarrow-1 take part in every job; the rest (MADPOSE_LO_THREADS beyond
// kNarrow) only in wide jobs -- problems of at least kPoolWide blocks, the two-focal
// all-inlier fits (N = 4000: ~10k blocks), where 8 threads cut the LO's serial fits by
// a third (prefix 257 -> 169-193 us, tf 13.2 -> 11.7-12.1 ms per pair) while the
// calibrated / shared-focal ones (<= ~7.5k blocks) gained nothing from them
// (profiles/r04/lotab, tflo).  The wide workers wait on a counter of their own, so a
// narrow job neither wakes them nor keeps them spinning.
constexpr int kNarrow = 4;
// every pool-sized problem is wide since round 5: the LO's serial all-inlier fit (the
// prefix) 90-93 -> 82-88 us per calibrated LO with 8 threads instead of 4 (3 x 100
// pairs on one box, profiles/r05/r5t); 12 threads oversubscribe the 16-CPU share
// (prefix 132-134 us).  MADPOSE_LM_WIDE overrides the threshold, in blocks.
size_t pool_wide() {
    static const size_t v = [] {
        return (size_t)env_int("MADPOSE_LM_WIDE", 2048, 1, 1ll << 40);
    }();
    return v;
}
class Pool {
  public:
    explicit Pool(int n) {
        spin_ns_ = lo_spin_us() * 1000ll;
        for (int i = 1; i < n; ++i) th_.emplace_back([this, i] { loop(i >= kNarrow); });
        narrow_ = std::min((int)th_.size(), kNarrow - 1);
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
            gen_.fetch_add(1, std::memory_order_release);
            gen_wide_.fetch_add(1, std::memory_order_release);
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
    }
    // runs f(k) for k in [0, n); the calling thread takes part, and the narrow workers
    // (all workers when wide)
    void run(size_t n, const std::function<void(size_t)> &f, bool wide = false) {
        if (th_.empty() || n < 2) {
            for (size_t k = 0; k < n; ++k) f(k);
            return;
        }
        std::lock_guard<std::mutex> job(job_mu_);
        wide = wide && (int)th_.size() > narrow_;
        {
            std::lock_guard<std::mutex> lk(mu_);
            f_ = &f;
            n_ = n;
            next_.store(0);
            active_.store(wide ? (int)th_.size() : narrow_, std::memory_order_relaxed);
            gen_.fetch_add(1, std::memory_order_release);
            if (wide) gen_wide_.fetch_add(1, std::memory_order_release);
        }
        cv_.notify_all();
        work();
        // the workers' share: spin, then block
        if (!spin_until([this] { return active_.load(std::memory_order_acquire) == 0; })) {
            std::unique_lock<std::mutex> lk(mu_);
            done_cv_.wait(lk, [this] { return active_.load(std::memory_order_acquire) == 0; });
        }
        f_ = nullptr;
    }

  private:
    static void pause() {
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
    }
    // polls ready() with pause for at most spin_ns_; true once it held
    template <class F> bool spin_until(const F &ready) const {
        if (spin_ns_ <= 0) return ready();
        const auto t0 = std::chrono::steady_clock::now();
        for (int k = 0;; ++k) {
            if (ready()) return true;
            pause();
            if ((k & 63) == 63 &&
                std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count() >
                    spin_ns_)
                return ready();
        }
    }
    void work() {
        for (size_t k; (k = next_.fetch_add(1)) < n_;) (*f_)(k);
    }
    void loop(bool wide_only) {
        const std::atomic<uint64_t> &g = wide_only ? gen_wide_ : gen_;
        uint64_t seen = 0;
        for (;;) {
            const bool ready = spin_until([&] { return g.load(std::memory_order_acquire) != seen; });
            if (!ready) {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return g.load(std::memory_order_acquire) != seen; });
            }
            {
                std::lock_guard<std::mutex> lk(mu_); // (pairs with run()'s publication)
                if (stop_) return;
                seen = g.load(std::memory_order_relaxed);
            }
            work();
            if (active_.fetch_sub(1, std::memory_order_acq_rel) == 1) {
                std::lock_guard<std::mutex> lk(mu_);
                done_cv_.notify_one();
            }
        }
    }
    std::vector<std::thread> th_;
    int narrow_ = 0;
    std::mutex mu_, job_mu_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(size_t)> *f_ = nullptr;
    size_t n_ = 0;
    std::atomic<size_t> next_{0};
    std::atomic<int> active_{0};
    std::atomic<uint64_t> gen_{0}, gen_wide_{0};
    bool stop_ = false;
    long long spin_ns_ = 0;
};

Pool &lo_pool() {
    static Pool pool([] {
        return (int)env_int("MADPOSE_LO_THREADS", 8, 1, 64);
    }());
    return pool;
}

// the 8-lane residual evaluation runs as AVX-512 when the CPU has it (identical results
// either way, lm_eval.inc); MADPOSE_LM_ISA=avx2 forces the AVX2 build (A/B)
bool lm_eval_avx512() {
    static const bool on = [] {
        if (env_avx2("MADPOSE_LM_ISA")) return false;
        __builtin_cpu_init();
        return __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512dq") &&
               __builtin_cpu_supports("avx512vl");
    }();
    return on;
}

size_t num_blocks(const Ctx &C) {
    return (C.S.use_reproj ? C.sample[0].size() + C.sample[1].size() : 0) +
           (C.S.use_sampson ? C.sample[2].size() : 0);
}

// Evaluates cost (and, when H != nullptr, the active normal equations) at p.  Blocks
// are reduced in fixed chunks in chunk order, so the result does not depend on how
// many worker threads evaluate them.
double evaluate(const Ctx &C, const Params &p, double *H, double *g) {
    const size_t nb = num_blocks(C);
    const size_t nchunks = (nb + kChunk - 1) / kChunk;
    const bool jac = H != nullptr;
    Acc total;
    total.clear();
    const HostPair &P = *C.P;
    LmEvalIn E;
    E.variant = P.variant;
    E.x0 = P.x0.data();
    E.x1 = P.x1.data();
    E.d0 = P.d0.data();
    E.d1 = P.d1.data();
    E.K0 = P.K0;
    E.K1 = P.K1;
    E.K0i = P.K0i;
    E.K1i = P.K1i;
    E.s0 = C.sample[0].data();
    E.s1 = C.sample[1].data();
    E.s2 = C.sample[2].data();
    E.n0 = C.S.use_reproj ? C.sample[0].size() : 0;
    E.n1 = C.S.use_reproj ? C.sample[1].size() : 0;
    E.n2 = C.S.use_sampson ? C.sample[2].size() : 0;
    E.w_sampson = C.S.w_sampson;
    LmEvalParams ep;
    std::memcpy(ep.R, p.R, sizeof(ep.R));
    std::memcpy(ep.t, p.t, sizeof(ep.t));
    ep.s = p.s;
    ep.o0 = p.o0;
    ep.o1 = p.o1;
    ep.f0 = p.f0;
    ep.f1 = p.f1;
    const auto eval = lm_eval_avx512() ? lm_eval_range_w8 : lm_eval_range_w4;
    auto range = [&](size_t a, size_t b, Acc &acc) { eval(E, ep, jac, a, b, acc.H, acc.g, &acc.cost); };
    if (nchunks <= 1) {
        range(0, nb, total);
    } else {
        // (on the stack up to 64 chunks = 16k blocks: no allocation per evaluation)
        Acc stack_parts[64];
        std::vector<Acc> heap_parts(nchunks > 64 ? nchunks : 0);
        Acc *parts = nchunks > 64 ? heap_parts.data() : stack_parts;
        auto chunk = [&](size_t k) {
            parts[k].clear();
            range(k * kChunk, std::min(nb, (k + 1) * kChunk), parts[k]);
        };
        if (nb >= kPoolBlocks)
            lo_pool().run(nchunks, chunk, nb >= pool_wide());
        else
            for (size_t k = 0; k < nchunks; ++k) chunk(k);
        for (size_t k = 0; k < nchunks; ++k) total.merge(parts[k]);
    }
    if (jac) total.scatter(C, H, g);
    return total.cost;
}

// Solves A x = b (n x n, symmetric positive definite) by Cholesky; A and b are
// overwritten (factor, solution).  Returns false if A is not positive definite.
bool chol_solve(double *A, int n, double *b) {
    for (int j = 0; j < n; ++j) {
        double d = A[j * n + j];
        for (int k = 0; k < j; ++k) d -= A[j * n + k] * A[j * n + k];
        if (!(d > 0)) return false;
        d = std::sqrt(d);
        A[j * n + j] = d;
        for (int i = j + 1; i < n; ++i) {
            double s = A[i * n + j];
            for (int k = 0; k < j; ++k) s -= A[i * n + k] * A[j * n + k];
            A[i * n + j] = s / d;
        }
    }
    for (int i = 0; i < n; ++i) {
        double s = b[i];
        for (int k = 0; k < i; ++k) s -= A[i * n + k] * b[k];
        b[i] = s / A[i * n + i];
    }
    for (int i = n - 1; i >= 0; --i) {
        double s = b[i];
        for (int k = i + 1; k < n; ++k) s -= A[k * n + i] * b[k];
        b[i] = s / A[i * n + i];
    }
    return true;
}

void set_rotation(Params &p) { quat_to_rot(p.q, p.R); }

} // namespace

void rot_to_quat(const double *R, double *q) {
    const double tr = R[0] + R[4] + R[8];
    if (tr > 0) {
        double s = std::sqrt(tr + 1.0);
        q[0] = 0.5 * s;
        s = 0.5 / s;
        q[1] = (R[7] - R[5]) * s;
        q[2] = (R[2] - R[6]) * s;
        q[3] = (R[3] - R[1]) * s;
    } else {
        int i = 0;
        if (R[4] > R[0]) i = 1;
        if (R[8] > R[4 * i]) i = 2;
        const int j = (i + 1) % 3, k = (j + 1) % 3;
        double s = std::sqrt(R[4 * i] - R[4 * j] - R[4 * k] + 1.0);
        double v[3];
        v[i] = 0.5 * s;
        s = 0.5 / s;
        q[0] = (R[3 * k + j] - R[3 * j + k]) * s;
        v[j] = (R[3 * j + i] + R[3 * i + j]) * s;
        v[k] = (R[3 * k + i] + R[3 * i + k]) * s;
        q[1] = v[0];
        q[2] = v[1];
        q[3] = v[2];
    }
}

void quat_to_rot(const double *q0, double *R) {
    const double n = std::sqrt(q0[0] * q0[0] + q0[1] * q0[1] + q0[2] * q0[2] + q0[3] * q0[3]);
    const double w = q0[0] / n, x = q0[1] / n, y = q0[2] / n, z = q0[3] / n;
    R[0] = 1 - 2 * (y * y + z * z);
    R[1] = 2 * (x * y - w * z);
    R[2] = 2 * (x * z + w * y);
    R[3] = 2 * (x * y + w * z);
    R[4] = 1 - 2 * (x * x + z * z);
    R[5] = 2 * (y * z - w * x);
    R[6] = 2 * (x * z - w * y);
    R[7] = 2 * (y * z + w * x);
    R[8] = 1 - 2 * (x * x + y * y);
}

thread_local int lm_last_evals = 0;

bool lm_refine(const HostPair &P, const std::vector<int> *sample, const LMSettings &S, Model *m) {
    lm_last_evals = 0;
    Ctx C;
    C.P = &P;
    C.sample = sample;
    C.S = S;
    size_t nres = 0;
    if (S.use_reproj) nres += sample[0].size() + sample[1].size();
    if (S.use_sampson) nres += sample[2].size();
    if (nres == 0) return false;
    C.has_o0 = S.use_reproj && !sample[0].empty();
    C.has_s_o1 = S.use_reproj && !sample[1].empty();
    for (int k = 0; k < kNFull; ++k) C.col[k] = -1;
    int n = 0;
    for (int k = 0; k < 6; ++k) C.col[k] = n++;
    bool has_lo[kNFull] = {false};
    double lo[kNFull] = {0};
    if (C.has_s_o1) {
        C.col[kS] = n++;
        has_lo[kS] = true;
        lo[kS] = 1e-2;
    }
    if (C.has_o0 && S.use_shift) C.col[kO0] = n++;
    if (C.has_s_o1 && S.use_shift) C.col[kO1] = n++;
    if (S.min_depth_constraint) {
        has_lo[kO0] = has_lo[kO1] = true;
        lo[kO0] = -P.min_depth[0] + 1e-2;
        lo[kO1] = -P.min_depth[1] + 1e-2;
    }
    if (P.variant == kSF) C.col[kF0] = n++;
    if (P.variant == kTF) {
        C.col[kF0] = n++;
        C.col[kF1] = n++;
        has_lo[kF0] = has_lo[kF1] = true;
        lo[kF0] = lo[kF1] = 1e-6;
    }
    C.n = n;
    Params x;
    rot_to_quat(m->R, x.q);
    set_rotation(x);
    std::memcpy(x.t, m->t, sizeof(x.t));
    x.s = m->scale;
    x.o0 = m->offset0;
    x.o1 = m->offset1;
    x.f0 = m->focal0;
    x.f1 = m->focal1;
    // constant bounded blocks must start feasible (Ceres Program::IsFeasible)
    if (!S.use_shift && S.min_depth_constraint) {
        if (C.has_o0 && x.o0 < lo[kO0]) return true;
        if (C.has_s_o1 && x.o1 < lo[kO1]) return true;
    }
    auto amb_norm2 = [](const Params &p) {
        return p.q[0] * p.q[0] + p.q[1] * p.q[1] + p.q[2] * p.q[2] + p.q[3] * p.q[3] + p.t[0] * p.t[0] +
               p.t[1] * p.t[1] + p.t[2] * p.t[2] + p.s * p.s + p.o0 * p.o0 + p.o1 * p.o1 + p.f0 * p.f0 + p.f1 * p.f1;
    };
    // (fixed-size storage: n <= kNFull, no allocation inside the iterations)
    double Hbuf[2][kNFull * kNFull], gbuf[2][kNFull];
    double *H = Hbuf[0], *g = gbuf[0], *Hc = Hbuf[1], *gc = gbuf[1];
    double cost = evaluate(C, x, H, g);
    lm_last_evals = 1;
    auto gmax = [&]() {
        double v = 0;
        for (int a = 0; a < n; ++a) v = std::max(v, std::fabs(g[a]));
        return v;
    };
    double radius = 1e4, decrease = 2.0;
    // Ceres TrustRegionStepEvaluator: step quality against the current cost and
    // against a reference cost that may lag behind it for up to 5 consecutive
    // non-monotonic steps (0 when use_nonmonotonic_steps is off, which makes the
    // reference the current cost and the quality the plain relative decrease); the
    // parameters returned are those of the lowest cost reached (Ceres writes the
    // user's parameter blocks only on a new minimum).
    const int max_nonmono = S.nonmonotonic ? 5 : 0;
    double ref_cost = cost, min_cost = cost, cand_cost_ref = cost, acc_ref = 0.0, acc_cand = 0.0;
    int n_nonmono = 0;
    Params best = x;
    if (!(gmax() <= S.gtol)) {
        for (int iter = 0; iter < S.max_iter; ++iter) {
            double sc[kNFull], A[kNFull * kNFull], y[kNFull];
            for (int j = 0; j < n; ++j) sc[j] = 1.0 / (1.0 + std::sqrt(H[j * n + j]));
            for (int a = 0; a < n; ++a) {
                y[a] = -g[a] * sc[a];
                for (int b = 0; b < n; ++b) A[a * n + b] = H[a * n + b] * sc[a] * sc[b];
            }
            for (int j = 0; j < n; ++j) {
                const double dg = std::min(std::max(A[j * n + j], 1e-6), 1e32);
                A[j * n + j] += dg / radius;
            }
            if (!chol_solve(A, n, y)) {
                radius /= decrease;
                decrease *= 2.0;
                if (radius < 1e-32) break;
                continue;
            }
            double d[kNFull];
            for (int j = 0; j < n; ++j) d[j] = y[j] * sc[j];
            // candidate = Plus(x, d), projected onto the bounds
            Params c = x;
            {
                const double dv[3] = {d[0], d[1], d[2]};
                const double nd = std::sqrt(dv[0] * dv[0] + dv[1] * dv[1] + dv[2] * dv[2]);
                if (nd > 0) {
                    const double sn = std::sin(nd) / nd;
                    const double qd[4] = {std::cos(nd), sn * dv[0], sn * dv[1], sn * dv[2]};
                    const double *q = x.q;
                    c.q[0] = qd[0] * q[0] - qd[1] * q[1] - qd[2] * q[2] - qd[3] * q[3];
                    c.q[1] = qd[0] * q[1] + qd[1] * q[0] + qd[2] * q[3] - qd[3] * q[2];
                    c.q[2] = qd[0] * q[2] - qd[1] * q[3] + qd[2] * q[0] + qd[3] * q[1];
                    c.q[3] = qd[0] * q[3] + qd[1] * q[2] - qd[2] * q[1] + qd[3] * q[0];
                }
                for (int k = 0; k < 3; ++k) c.t[k] = x.t[k] + d[3 + k];
                auto upd = [&](int slot, double &v) {
                    if (C.col[slot] < 0) return;
                    v += d[C.col[slot]];
                    if (has_lo[slot] && v < lo[slot]) v = lo[slot];
                };
                upd(kS, c.s);
                upd(kO0, c.o0);
                upd(kO1, c.o1);
                upd(kF0, c.f0);
                upd(kF1, c.f1);
                set_rotation(c);
            }
            double step2 = 0;
            {
                const double dd[12] = {c.q[0] - x.q[0], c.q[1] - x.q[1], c.q[2] - x.q[2], c.q[3] - x.q[3],
                                       c.t[0] - x.t[0], c.t[1] - x.t[1], c.t[2] - x.t[2], c.s - x.s,
                                       c.o0 - x.o0,     c.o1 - x.o1,     c.f0 - x.f0,     c.f1 - x.f1};
                for (double e : dd) step2 += e * e;
            }
            const double step_norm = std::sqrt(step2), xnorm = std::sqrt(amb_norm2(x));
            // the candidate is evaluated with its normal equations: accepted steps
            // (the common case) then need no second pass
            const double cand_cost = evaluate(C, c, Hc, gc);
            ++lm_last_evals;
            if (step_norm <= S.ptol * (xnorm + S.ptol)) break;
            if (std::fabs(cost - cand_cost) <= S.ftol * cost) break;
            double gd = 0, jd2 = 0;
            for (int a = 0; a < n; ++a) {
                gd += g[a] * d[a];
                for (int b = 0; b < n; ++b) jd2 += d[a] * H[a * n + b] * d[b];
            }
            const double mcc = -(gd + 0.5 * jd2);
            const double rho = (mcc > 0 && std::isfinite(cand_cost))
                                   ? std::max((cost - cand_cost) / mcc, (ref_cost - cand_cost) / (acc_ref + mcc))
                                   : -1.0;
            if (rho > 1e-3) {
                x = c;
                cost = cand_cost;
                std::swap(H, Hc);
                std::swap(g, gc);
                // TrustRegionStepEvaluator::StepAccepted
                acc_cand += mcc;
                acc_ref += mcc;
                if (cost < min_cost) {
                    min_cost = cost;
                    n_nonmono = 0;
                    cand_cost_ref = cost;
                    acc_cand = 0.0;
                    best = x;
                } else {
                    ++n_nonmono;
                    if (cost > cand_cost_ref) {
                        cand_cost_ref = cost;
                        acc_cand = 0.0;
                    }
                }
                if (n_nonmono == max_nonmono) {
                    ref_cost = cand_cost_ref;
                    acc_ref = acc_cand;
                }
                radius = std::min(1e16, radius / std::max(1.0 / 3.0, 1.0 - std::pow(2.0 * rho - 1.0, 3)));
                decrease = 2.0;
                if (gmax() <= S.gtol) break;
            } else {
                radius /= decrease;
                decrease *= 2.0;
                if (radius < 1e-32) break;
            }
        }
    }
    quat_to_rot(best.q, m->R);
    std::memcpy(m->t, best.t, sizeof(best.t));
    m->scale = best.s;
    m->offset0 = best.o0;
    m->offset1 = best.o1;
    m->focal0 = best.f0;
    m->focal1 = (P.variant == kSF) ? best.f0 : best.f1;
    return true;
}

} // namespace mp
