// Host LM for LO -- see lm.h.
#include "lm.h"

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

enum Full { kD0 = 0, kD1, kD2, kT0, kT1, kT2, kS, kO0, kO1, kF0, kF1, kNFull };

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
constexpr int kNPack = kNFull * (kNFull + 1) / 2;
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
// (default 4; 1 = off).  The blocks are reduced in fixed chunks in chunk order either
// way, so the result does not depend on the pool.
constexpr size_t kChunk = 256;
constexpr size_t kPoolBlocks = 2048;
// Workers spin (with pause) for a while after each job before they block on the
// condition variable: the evaluations of one LM follow each other within
// microseconds, and a futex wake-up per evaluation would cost about as much as the
// evaluation's share per thread.  The spin is bounded by time, not by a pause count
// (pause latency differs ~10x across x86 generations): MADPOSE_LO_SPIN = microseconds
// (0 = block right away).  Default 300, or 0 when the process's CPU affinity share is
// smaller than kSpinCpusPerRank per rank on this host (LOCAL_WORLD_SIZE): spinning
// pays while the host has idle CPUs and costs when ranks oversubscribe one share
// (two ranks on one 16-CPU share, 730 pairs/s spinning vs 840 blocking).
constexpr int kSpinCpusPerRank = 12; // about the threads one rank keeps busy (LO lanes, pool, sampler)
}  // namespace

int lo_spin_us() {
    static const int v = [] {
        if (const char *e = std::getenv("MADPOSE_LO_SPIN")) return std::max(0, std::atoi(e));
        int cpus = 0;
        cpu_set_t set;
        CPU_ZERO(&set);
        if (sched_getaffinity(0, sizeof(set), &set) == 0) cpus = CPU_COUNT(&set);
        const char *l = std::getenv("LOCAL_WORLD_SIZE");
        const int ranks = std::max(1, l ? std::atoi(l) : 1);
        return (cpus > 0 && cpus < kSpinCpusPerRank * ranks) ? 0 : 300;
    }();
    return v;
}

namespace {
class Pool {
  public:
    explicit Pool(int n) {
        spin_ns_ = lo_spin_us() * 1000ll;
        for (int i = 0; i < n - 1; ++i) th_.emplace_back([this] { loop(); });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
            gen_.fetch_add(1, std::memory_order_release);
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
    }
    // runs f(k) for k in [0, n); the calling thread takes part
    void run(size_t n, const std::function<void(size_t)> &f) {
        if (th_.empty() || n < 2) {
            for (size_t k = 0; k < n; ++k) f(k);
            return;
        }
        std::lock_guard<std::mutex> job(job_mu_);
        {
            std::lock_guard<std::mutex> lk(mu_);
            f_ = &f;
            n_ = n;
            next_.store(0);
            active_.store((int)th_.size(), std::memory_order_relaxed);
            gen_.fetch_add(1, std::memory_order_release);
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
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            const bool ready = spin_until([&] { return gen_.load(std::memory_order_acquire) != seen; });
            if (!ready) {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return gen_.load(std::memory_order_acquire) != seen; });
            }
            {
                std::lock_guard<std::mutex> lk(mu_); // (pairs with run()'s publication)
                if (stop_) return;
                seen = gen_.load(std::memory_order_relaxed);
            }
            work();
            if (active_.fetch_sub(1, std::memory_order_acq_rel) == 1) {
                std::lock_guard<std::mutex> lk(mu_);
                done_cv_.notify_one();
            }
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_, job_mu_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(size_t)> *f_ = nullptr;
    size_t n_ = 0;
    std::atomic<size_t> next_{0};
    std::atomic<int> active_{0};
    std::atomic<uint64_t> gen_{0};
    bool stop_ = false;
    long long spin_ns_ = 0;
};

Pool &lo_pool() {
    static Pool pool([] {
        const char *e = std::getenv("MADPOSE_LO_THREADS");
        const int n = e ? std::atoi(e) : 4;
        return std::max(1, std::min(n, 64));
    }());
    return pool;
}

// Residual blocks [b0, b1) of the concatenated block list (reproj0, reproj1, Sampson)
// into acc; with jac == false only the cost is accumulated (in the same order).
void evaluate_range(const Ctx &C, const Params &p, bool jac, size_t b0, size_t b1, Acc &acc) {
    const HostPair &P = *C.P;
    const bool cal = P.variant == kCal;
    const bool sf = P.variant == kSF;
    const double f0 = p.f0, f1 = sf ? p.f0 : p.f1;
    double &cost = acc.cost;
    const size_t n0 = C.S.use_reproj ? C.sample[0].size() : 0, n1 = C.S.use_reproj ? C.sample[1].size() : 0;
    const size_t n2 = C.S.use_sampson ? C.sample[2].size() : 0;
    const double *R = p.R, *t = p.t;
    if (n0 > 0 && b0 < n0) {
        // LiftProjectionFunctor0 and variants: x1_hat = K1 (R c0 (d0 + o0) + t)
        for (size_t bi = b0; bi < std::min(b1, n0); ++bi) {
            const int i = C.sample[0][bi];
            double c[3];
            const double xh[3] = {P.x0[2 * i], P.x0[2 * i + 1], 1.0};
            if (cal)
                mv3(P.K0i, xh, c);
            else {
                c[0] = xh[0] / f0;
                c[1] = xh[1] / f0;
                c[2] = 1.0;
            }
            const double a = P.d0[i] + p.o0;
            const double pp[3] = {c[0] * a, c[1] * a, c[2] * a};
            double v[3], y[3], h[3];
            mv3(R, pp, v);
            for (int k = 0; k < 3; ++k) y[k] = v[k] + t[k];
            if (cal)
                mv3(P.K1, y, h);
            else {
                h[0] = f1 * y[0];
                h[1] = f1 * y[1];
                h[2] = y[2];
            }
            const double iz = 1.0 / h[2];
            const double r0 = h[0] * iz - P.x1[2 * i], r1 = h[1] * iz - P.x1[2 * i + 1];
            if (!jac) {
                cost += 0.5 * r0 * r0;
                cost += 0.5 * r1 * r1;
                continue;
            }
            // dr/dh
            const double Dh[2][3] = {{iz, 0, -h[0] * iz * iz}, {0, iz, -h[1] * iz * iz}};
            double G[2][3]; // dr/dy
            for (int rr = 0; rr < 2; ++rr)
                for (int k = 0; k < 3; ++k) {
                    if (cal)
                        G[rr][k] = Dh[rr][0] * P.K1[k] + Dh[rr][1] * P.K1[3 + k] + Dh[rr][2] * P.K1[6 + k];
                    else
                        G[rr][k] = Dh[rr][k] * (k < 2 ? f1 : 1.0);
                }
            double Sv[9];
            skew(v, Sv);
            double Rc[3];
            mv3(R, c, Rc);
            double dcf[3] = {0, 0, 0}, Rdcf[3] = {0, 0, 0};
            if (!cal) {
                dcf[0] = -xh[0] / (f0 * f0) * a;
                dcf[1] = -xh[1] / (f0 * f0) * a;
                mv3(R, dcf, Rdcf);
            }
            for (int rr = 0; rr < 2; ++rr) {
                double gf[kNFull] = {0};
                for (int k = 0; k < 3; ++k) {
                    // dy/ddelta = -2 [v]x
                    gf[kD0 + k] = -2.0 * (G[rr][0] * Sv[k] + G[rr][1] * Sv[3 + k] + G[rr][2] * Sv[6 + k]);
                    gf[kT0 + k] = G[rr][k];
                }
                gf[kO0] = G[rr][0] * Rc[0] + G[rr][1] * Rc[1] + G[rr][2] * Rc[2];
                if (!cal) {
                    const double dyf0 = G[rr][0] * Rdcf[0] + G[rr][1] * Rdcf[1] + G[rr][2] * Rdcf[2];
                    const double dhf1 = Dh[rr][0] * y[0] + Dh[rr][1] * y[1];
                    if (sf)
                        gf[kF0] = dyf0 + dhf1;
                    else {
                        gf[kF0] = dyf0;
                        gf[kF1] = dhf1;
                    }
                }
                acc.add(rr == 0 ? r0 : r1, gf);
            }
        }
    }
    if (n1 > 0 && b1 > n0 && b0 < n0 + n1) {
        // LiftProjectionFunctor1: x0_hat = K0 R^T (c1 (d1 + o1) s - t)
        for (size_t bi = std::max(b0, n0); bi < std::min(b1, n0 + n1); ++bi) {
            const int i = C.sample[1][bi - n0];
            double c[3];
            const double xh[3] = {P.x1[2 * i], P.x1[2 * i + 1], 1.0};
            if (cal)
                mv3(P.K1i, xh, c);
            else {
                c[0] = xh[0] / f1;
                c[1] = xh[1] / f1;
                c[2] = 1.0;
            }
            const double dep = P.d1[i] + p.o1;
            const double a = dep * p.s;
            const double u[3] = {c[0] * a - t[0], c[1] * a - t[1], c[2] * a - t[2]};
            double y[3], h[3];
            mtv3(R, u, y);
            if (cal)
                mv3(P.K0, y, h);
            else {
                h[0] = f0 * y[0];
                h[1] = f0 * y[1];
                h[2] = y[2];
            }
            const double iz = 1.0 / h[2];
            const double r0 = h[0] * iz - P.x0[2 * i], r1 = h[1] * iz - P.x0[2 * i + 1];
            if (!jac) {
                cost += 0.5 * r0 * r0;
                cost += 0.5 * r1 * r1;
                continue;
            }
            const double Dh[2][3] = {{iz, 0, -h[0] * iz * iz}, {0, iz, -h[1] * iz * iz}};
            double G[2][3];
            for (int rr = 0; rr < 2; ++rr)
                for (int k = 0; k < 3; ++k) {
                    if (cal)
                        G[rr][k] = Dh[rr][0] * P.K0[k] + Dh[rr][1] * P.K0[3 + k] + Dh[rr][2] * P.K0[6 + k];
                    else
                        G[rr][k] = Dh[rr][k] * (k < 2 ? f0 : 1.0);
                }
            // dy/ddelta = 2 R^T [u]x ; dy/dt = -R^T ; dy/ds = R^T c dep ; dy/do1 = R^T c s
            double Su[9], RtSu[9];
            skew(u, Su);
            for (int r = 0; r < 3; ++r)
                for (int cc = 0; cc < 3; ++cc)
                    RtSu[3 * r + cc] = R[r] * Su[cc] + R[3 + r] * Su[3 + cc] + R[6 + r] * Su[6 + cc];
            double Rtc[3];
            mtv3(R, c, Rtc);
            double Rtdcf[3] = {0, 0, 0};
            if (!cal) {
                const double dcf[3] = {-xh[0] / (f1 * f1) * a, -xh[1] / (f1 * f1) * a, 0.0};
                mtv3(R, dcf, Rtdcf);
            }
            for (int rr = 0; rr < 2; ++rr) {
                double gf[kNFull] = {0};
                for (int k = 0; k < 3; ++k) {
                    gf[kD0 + k] =
                        2.0 * (G[rr][0] * RtSu[k] + G[rr][1] * RtSu[3 + k] + G[rr][2] * RtSu[6 + k]);
                    gf[kT0 + k] = -(G[rr][0] * R[3 * k] + G[rr][1] * R[3 * k + 1] + G[rr][2] * R[3 * k + 2]);
                }
                const double gRtc = G[rr][0] * Rtc[0] + G[rr][1] * Rtc[1] + G[rr][2] * Rtc[2];
                gf[kS] = gRtc * dep;
                gf[kO1] = gRtc * p.s;
                if (!cal) {
                    const double dyf1 = G[rr][0] * Rtdcf[0] + G[rr][1] * Rtdcf[1] + G[rr][2] * Rtdcf[2];
                    const double dhf0 = Dh[rr][0] * y[0] + Dh[rr][1] * y[1];
                    if (sf)
                        gf[kF0] = dyf1 + dhf0;
                    else {
                        gf[kF0] = dhf0;
                        gf[kF1] = dyf1;
                    }
                }
                acc.add(rr == 0 ? r0 : r1, gf);
            }
        }
    }
    if (n2 > 0 && b1 > n0 + n1) {
        // SampsonError*Functor: r = w C / |(e0, e1, g0, g1)|
        double Tx[9], E[9];
        skew(t, Tx);
        mm3(Tx, R, E);
        double s0[3] = {1, 1, 1}, s1[3] = {1, 1, 1};
        if (!cal) {
            s0[0] = s0[1] = 1.0 / f0;
            s1[0] = s1[1] = 1.0 / f1;
        }
        double F[9];
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) F[3 * r + c] = E[3 * r + c] * s1[r] * s0[c];
        // derivative building blocks: dE/dt_k = [e_k]x R, dE/ddelta_k = 2 [t]x [e_k]x R
        double dEt[3][9], dEd[3][9];
        if (jac) {
            for (int k = 0; k < 3; ++k) {
                double ek[3] = {0, 0, 0};
                ek[k] = 1.0;
                double Sk[9];
                skew(ek, Sk);
                mm3(Sk, R, dEt[k]);
                mm3(Tx, dEt[k], dEd[k]);
                for (int e = 0; e < 9; ++e) dEd[k][e] *= 2.0;
            }
        }
        for (size_t bi = std::max(b0, n0 + n1); bi < std::min(b1, n0 + n1 + n2); ++bi) {
            const int i = C.sample[2][bi - n0 - n1];
            double a[3], b[3];
            if (cal) {
                const double xa[3] = {P.x0[2 * i], P.x0[2 * i + 1], 1.0}, xb[3] = {P.x1[2 * i], P.x1[2 * i + 1], 1.0};
                mv3(P.K0i, xa, a);
                mv3(P.K1i, xb, b);
            } else {
                a[0] = P.x0[2 * i];
                a[1] = P.x0[2 * i + 1];
                b[0] = P.x1[2 * i];
                b[1] = P.x1[2 * i + 1];
            }
            a[2] = b[2] = 1.0; // the functor uses the first two coordinates and an implicit 1
            const double e0 = F[0] * a[0] + F[1] * a[1] + F[2];
            const double e1 = F[3] * a[0] + F[4] * a[1] + F[5];
            const double e2 = F[6] * a[0] + F[7] * a[1] + F[8];
            const double g0 = F[0] * b[0] + F[3] * b[1] + F[6];
            const double g1 = F[1] * b[0] + F[4] * b[1] + F[7];
            const double Cc = b[0] * e0 + b[1] * e1 + e2;
            const double D = e0 * e0 + e1 * e1 + g0 * g0 + g1 * g1;
            const double sD = std::sqrt(D);
            const double r = C.S.w_sampson * Cc / sD;
            if (!jac) {
                cost += 0.5 * r * r;
                continue;
            }
            const double ev[3] = {e0, e1, e2}, gv[3] = {g0, g1, 0.0};
            double W[9]; // dr/dF
            const double k1 = C.S.w_sampson / sD, k2 = C.S.w_sampson * Cc / (D * sD);
            for (int ii = 0; ii < 3; ++ii)
                for (int jj = 0; jj < 3; ++jj) {
                    const double dD = (ii < 2 ? ev[ii] * a[jj] : 0.0) + (jj < 2 ? gv[jj] * b[ii] : 0.0);
                    W[3 * ii + jj] = k1 * b[ii] * a[jj] - k2 * dD;
                }
            double WE[9]; // dr/dE
            for (int ii = 0; ii < 3; ++ii)
                for (int jj = 0; jj < 3; ++jj) WE[3 * ii + jj] = W[3 * ii + jj] * s1[ii] * s0[jj];
            double gf[kNFull] = {0};
            for (int k = 0; k < 3; ++k) {
                double dt = 0, dd = 0;
                for (int e = 0; e < 9; ++e) {
                    dt += WE[e] * dEt[k][e];
                    dd += WE[e] * dEd[k][e];
                }
                gf[kT0 + k] = dt;
                gf[kD0 + k] = dd;
            }
            if (!cal) {
                const double ds0[3] = {-1.0 / (f0 * f0), -1.0 / (f0 * f0), 0.0};
                const double ds1[3] = {-1.0 / (f1 * f1), -1.0 / (f1 * f1), 0.0};
                double df0 = 0, df1 = 0;
                for (int ii = 0; ii < 3; ++ii)
                    for (int jj = 0; jj < 3; ++jj) {
                        df0 += W[3 * ii + jj] * E[3 * ii + jj] * s1[ii] * ds0[jj];
                        df1 += W[3 * ii + jj] * E[3 * ii + jj] * ds1[ii] * s0[jj];
                    }
                if (sf)
                    gf[kF0] = df0 + df1;
                else {
                    gf[kF0] = df0;
                    gf[kF1] = df1;
                }
            }
            acc.add(r, gf);
        }
    }
}

// ---------------------------------------------------------------------------
// Four residual blocks at a time (GCC/Clang vector extension; AVX2 on the build
// flags): the per-block Jacobian algebra of evaluate_range with every per-block value
// a 4-lane vector and the parameters broadcast.  Lanes past the end of the block list
// repeat the last block with a zero weight.  NA = number of leading full-layout
// parameters that can be active for the variant (cal 9, sf 10, tf 11).
typedef double V4 __attribute__((vector_size(32)));
inline V4 vs(double a) { return V4{a, a, a, a}; }
inline V4 vsqrt(V4 v) { return V4{std::sqrt(v[0]), std::sqrt(v[1]), std::sqrt(v[2]), std::sqrt(v[3])}; }
inline double hsum(V4 v) { return (v[0] + v[1]) + (v[2] + v[3]); }

template <int NA> struct AccV {
    static constexpr int kPack = NA * (NA + 1) / 2;
    V4 H[kPack];
    V4 g[NA];
    V4 cost;
    void clear() {
        for (int q = 0; q < kPack; ++q) H[q] = vs(0.0);
        for (int a = 0; a < NA; ++a) g[a] = vs(0.0);
        cost = vs(0.0);
    }
    inline void add(V4 r, const V4 *gf) {
        cost += 0.5 * r * r;
        int q = 0;
        for (int a = 0; a < NA; ++a) {
            g[a] += gf[a] * r;
            const V4 ja = gf[a];
            for (int b = a; b < NA; ++b) H[q++] += ja * gf[b];
        }
    }
    // lane sums into the scalar full-layout accumulator
    void reduce_into(Acc &acc) const {
        acc.cost += hsum(cost);
        int q = 0;
        for (int a = 0; a < kNFull; ++a) {
            if (a < NA) acc.g[a] += hsum(g[a]);
            for (int b = a; b < kNFull; ++b, ++q)
                if (a < NA && b < NA) acc.H[q] += hsum(H[a * NA - a * (a - 1) / 2 + (b - a)]);
        }
    }
};

inline void mv3v(const double *A, const V4 *v, V4 *o) {
    for (int r = 0; r < 3; ++r) o[r] = A[3 * r] * v[0] + A[3 * r + 1] * v[1] + A[3 * r + 2] * v[2];
}
inline void mtv3v(const double *A, const V4 *v, V4 *o) {
    for (int r = 0; r < 3; ++r) o[r] = A[r] * v[0] + A[3 + r] * v[1] + A[6 + r] * v[2];
}

template <int NA>
void evaluate_range_v(const Ctx &C, const Params &p, bool jac, size_t b0, size_t b1, Acc &acc_out) {
    const HostPair &P = *C.P;
    const bool cal = P.variant == kCal;
    const bool sf = P.variant == kSF;
    const double f0 = p.f0, f1 = sf ? p.f0 : p.f1;
    const size_t n0 = C.S.use_reproj ? C.sample[0].size() : 0, n1 = C.S.use_reproj ? C.sample[1].size() : 0;
    const size_t n2 = C.S.use_sampson ? C.sample[2].size() : 0;
    const double *R = p.R, *t = p.t;
    AccV<NA> acc;
    acc.clear();
    V4 gf0[kNFull], gf1[kNFull]; // only the first NA slots are accumulated
    // gathers the lanes of blocks [bi, bi + 4) of list `idx` (clamped), weight 0 past `end`
    auto gather = [&](const std::vector<int> &idx, size_t bi, size_t off, size_t end, int *ii, V4 &w) {
        for (int l = 0; l < 4; ++l) {
            const size_t b = std::min(bi + l, end - 1);
            ii[l] = idx[b - off];
            w[l] = (bi + l < end) ? 1.0 : 0.0;
        }
    };
    if (n0 > 0 && b0 < n0) {
        // LiftProjectionFunctor0 and variants: x1_hat = K1 (R c0 (d0 + o0) + t)
        const size_t end = std::min(b1, n0);
        for (size_t bi = b0; bi < end; bi += 4) {
            int ii[4];
            V4 w;
            gather(C.sample[0], bi, 0, end, ii, w);
            V4 xh[3], x1u, x1v, dd;
            for (int l = 0; l < 4; ++l) {
                xh[0][l] = P.x0[2 * ii[l]];
                xh[1][l] = P.x0[2 * ii[l] + 1];
                x1u[l] = P.x1[2 * ii[l]];
                x1v[l] = P.x1[2 * ii[l] + 1];
                dd[l] = P.d0[ii[l]];
            }
            xh[2] = vs(1.0);
            V4 c[3];
            if (cal)
                mv3v(P.K0i, xh, c);
            else {
                c[0] = xh[0] / f0;
                c[1] = xh[1] / f0;
                c[2] = vs(1.0);
            }
            const V4 a = dd + p.o0;
            const V4 pp[3] = {c[0] * a, c[1] * a, c[2] * a};
            V4 v[3], y[3], h[3];
            mv3v(R, pp, v);
            for (int k = 0; k < 3; ++k) y[k] = v[k] + t[k];
            if (cal)
                mv3v(P.K1, y, h);
            else {
                h[0] = f1 * y[0];
                h[1] = f1 * y[1];
                h[2] = y[2];
            }
            const V4 iz = 1.0 / h[2];
            const V4 r0 = (h[0] * iz - x1u) * w, r1 = (h[1] * iz - x1v) * w;
            if (!jac) {
                acc.cost += 0.5 * r0 * r0;
                acc.cost += 0.5 * r1 * r1;
                continue;
            }
            const V4 Dh[2][3] = {{iz, vs(0.0), -h[0] * iz * iz}, {vs(0.0), iz, -h[1] * iz * iz}};
            V4 G[2][3];
            for (int rr = 0; rr < 2; ++rr)
                for (int k = 0; k < 3; ++k) {
                    if (cal)
                        G[rr][k] = (Dh[rr][0] * P.K1[k] + Dh[rr][1] * P.K1[3 + k] + Dh[rr][2] * P.K1[6 + k]) * w;
                    else
                        G[rr][k] = Dh[rr][k] * (k < 2 ? f1 : 1.0) * w;
                }
            // [v]x columns: Sv[0][k], Sv[1][k], Sv[2][k]
            const V4 Sv[3][3] = {{vs(0.0), -v[2], v[1]}, {v[2], vs(0.0), -v[0]}, {-v[1], v[0], vs(0.0)}};
            V4 Rc[3];
            mv3v(R, c, Rc);
            V4 Rdcf[3] = {vs(0.0), vs(0.0), vs(0.0)};
            if (!cal) {
                const V4 dcf[3] = {-xh[0] / (f0 * f0) * a, -xh[1] / (f0 * f0) * a, vs(0.0)};
                mv3v(R, dcf, Rdcf);
            }
            for (int rr = 0; rr < 2; ++rr) {
                V4 *gf = rr == 0 ? gf0 : gf1;
                for (int k = 0; k < kNFull; ++k) gf[k] = vs(0.0);
                for (int k = 0; k < 3; ++k) {
                    gf[kD0 + k] = -2.0 * (G[rr][0] * Sv[0][k] + G[rr][1] * Sv[1][k] + G[rr][2] * Sv[2][k]);
                    gf[kT0 + k] = G[rr][k];
                }
                gf[kO0] = G[rr][0] * Rc[0] + G[rr][1] * Rc[1] + G[rr][2] * Rc[2];
                if (!cal) {
                    const V4 dyf0 = G[rr][0] * Rdcf[0] + G[rr][1] * Rdcf[1] + G[rr][2] * Rdcf[2];
                    const V4 dhf1 = (Dh[rr][0] * y[0] + Dh[rr][1] * y[1]) * w;
                    if (sf)
                        gf[kF0] = dyf0 + dhf1;
                    else {
                        gf[kF0] = dyf0;
                        gf[kF1] = dhf1;
                    }
                }
            }
            acc.add(r0, gf0);
            acc.add(r1, gf1);
        }
    }
    if (n1 > 0 && b1 > n0 && b0 < n0 + n1) {
        // LiftProjectionFunctor1: x0_hat = K0 R^T (c1 (d1 + o1) s - t)
        const size_t start = std::max(b0, n0), end = std::min(b1, n0 + n1);
        for (size_t bi = start; bi < end; bi += 4) {
            int ii[4];
            V4 w;
            gather(C.sample[1], bi, n0, end, ii, w);
            V4 xh[3], x0u, x0v, dd;
            for (int l = 0; l < 4; ++l) {
                xh[0][l] = P.x1[2 * ii[l]];
                xh[1][l] = P.x1[2 * ii[l] + 1];
                x0u[l] = P.x0[2 * ii[l]];
                x0v[l] = P.x0[2 * ii[l] + 1];
                dd[l] = P.d1[ii[l]];
            }
            xh[2] = vs(1.0);
            V4 c[3];
            if (cal)
                mv3v(P.K1i, xh, c);
            else {
                c[0] = xh[0] / f1;
                c[1] = xh[1] / f1;
                c[2] = vs(1.0);
            }
            const V4 dep = dd + p.o1;
            const V4 a = dep * p.s;
            const V4 u[3] = {c[0] * a - t[0], c[1] * a - t[1], c[2] * a - t[2]};
            V4 y[3], h[3];
            mtv3v(R, u, y);
            if (cal)
                mv3v(P.K0, y, h);
            else {
                h[0] = f0 * y[0];
                h[1] = f0 * y[1];
                h[2] = y[2];
            }
            const V4 iz = 1.0 / h[2];
            const V4 r0 = (h[0] * iz - x0u) * w, r1 = (h[1] * iz - x0v) * w;
            if (!jac) {
                acc.cost += 0.5 * r0 * r0;
                acc.cost += 0.5 * r1 * r1;
                continue;
            }
            const V4 Dh[2][3] = {{iz, vs(0.0), -h[0] * iz * iz}, {vs(0.0), iz, -h[1] * iz * iz}};
            V4 G[2][3];
            for (int rr = 0; rr < 2; ++rr)
                for (int k = 0; k < 3; ++k) {
                    if (cal)
                        G[rr][k] = (Dh[rr][0] * P.K0[k] + Dh[rr][1] * P.K0[3 + k] + Dh[rr][2] * P.K0[6 + k]) * w;
                    else
                        G[rr][k] = Dh[rr][k] * (k < 2 ? f0 : 1.0) * w;
                }
            // dy/ddelta = 2 R^T [u]x
            const V4 Su[3][3] = {{vs(0.0), -u[2], u[1]}, {u[2], vs(0.0), -u[0]}, {-u[1], u[0], vs(0.0)}};
            V4 RtSu[3][3];
            for (int r = 0; r < 3; ++r)
                for (int cc = 0; cc < 3; ++cc) RtSu[r][cc] = R[r] * Su[0][cc] + R[3 + r] * Su[1][cc] + R[6 + r] * Su[2][cc];
            V4 Rtc[3];
            mtv3v(R, c, Rtc);
            V4 Rtdcf[3] = {vs(0.0), vs(0.0), vs(0.0)};
            if (!cal) {
                const V4 dcf[3] = {-xh[0] / (f1 * f1) * a, -xh[1] / (f1 * f1) * a, vs(0.0)};
                mtv3v(R, dcf, Rtdcf);
            }
            for (int rr = 0; rr < 2; ++rr) {
                V4 *gf = rr == 0 ? gf0 : gf1;
                for (int k = 0; k < kNFull; ++k) gf[k] = vs(0.0);
                for (int k = 0; k < 3; ++k) {
                    gf[kD0 + k] = 2.0 * (G[rr][0] * RtSu[0][k] + G[rr][1] * RtSu[1][k] + G[rr][2] * RtSu[2][k]);
                    gf[kT0 + k] = -(G[rr][0] * R[3 * k] + G[rr][1] * R[3 * k + 1] + G[rr][2] * R[3 * k + 2]);
                }
                const V4 gRtc = G[rr][0] * Rtc[0] + G[rr][1] * Rtc[1] + G[rr][2] * Rtc[2];
                gf[kS] = gRtc * dep;
                gf[kO1] = gRtc * p.s;
                if (!cal) {
                    const V4 dyf1 = G[rr][0] * Rtdcf[0] + G[rr][1] * Rtdcf[1] + G[rr][2] * Rtdcf[2];
                    const V4 dhf0 = (Dh[rr][0] * y[0] + Dh[rr][1] * y[1]) * w;
                    if (sf)
                        gf[kF0] = dyf1 + dhf0;
                    else {
                        gf[kF0] = dhf0;
                        gf[kF1] = dyf1;
                    }
                }
            }
            acc.add(r0, gf0);
            acc.add(r1, gf1);
        }
    }
    if (n2 > 0 && b1 > n0 + n1) {
        // SampsonError*Functor: r = w C / |(e0, e1, g0, g1)|
        double Tx[9], E[9];
        skew(t, Tx);
        mm3(Tx, R, E);
        double s0[3] = {1, 1, 1}, s1[3] = {1, 1, 1};
        if (!cal) {
            s0[0] = s0[1] = 1.0 / f0;
            s1[0] = s1[1] = 1.0 / f1;
        }
        double F[9];
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) F[3 * r + c] = E[3 * r + c] * s1[r] * s0[c];
        double dEt[3][9], dEd[3][9];
        for (int k = 0; k < 3; ++k) {
            double ek[3] = {0, 0, 0};
            ek[k] = 1.0;
            double Sk[9];
            skew(ek, Sk);
            mm3(Sk, R, dEt[k]);
            mm3(Tx, dEt[k], dEd[k]);
            for (int e = 0; e < 9; ++e) dEd[k][e] *= 2.0;
        }
        // the f-derivative weights of W (uniform): E_ij s1_i ds0_j and E_ij ds1_i s0_j
        double Ef0[9] = {0}, Ef1[9] = {0};
        if (!cal)
            for (int ii = 0; ii < 3; ++ii)
                for (int jj = 0; jj < 3; ++jj) {
                    Ef0[3 * ii + jj] = E[3 * ii + jj] * s1[ii] * (jj < 2 ? -1.0 / (f0 * f0) : 0.0);
                    Ef1[3 * ii + jj] = E[3 * ii + jj] * (ii < 2 ? -1.0 / (f1 * f1) : 0.0) * s0[jj];
                }
        const double ws = C.S.w_sampson;
        const size_t start = std::max(b0, n0 + n1), end = std::min(b1, n0 + n1 + n2);
        for (size_t bi = start; bi < end; bi += 4) {
            int ii4[4];
            V4 w;
            gather(C.sample[2], bi, n0 + n1, end, ii4, w);
            V4 a[3], b[3];
            {
                V4 xa[3], xb[3];
                for (int l = 0; l < 4; ++l) {
                    xa[0][l] = P.x0[2 * ii4[l]];
                    xa[1][l] = P.x0[2 * ii4[l] + 1];
                    xb[0][l] = P.x1[2 * ii4[l]];
                    xb[1][l] = P.x1[2 * ii4[l] + 1];
                }
                xa[2] = xb[2] = vs(1.0);
                if (cal) {
                    mv3v(P.K0i, xa, a);
                    mv3v(P.K1i, xb, b);
                } else {
                    for (int k = 0; k < 2; ++k) {
                        a[k] = xa[k];
                        b[k] = xb[k];
                    }
                }
                a[2] = b[2] = vs(1.0); // the functor uses the first two coordinates and an implicit 1
            }
            const V4 e0 = F[0] * a[0] + F[1] * a[1] + F[2];
            const V4 e1 = F[3] * a[0] + F[4] * a[1] + F[5];
            const V4 e2 = F[6] * a[0] + F[7] * a[1] + F[8];
            const V4 g0 = F[0] * b[0] + F[3] * b[1] + F[6];
            const V4 g1 = F[1] * b[0] + F[4] * b[1] + F[7];
            const V4 Cc = b[0] * e0 + b[1] * e1 + e2;
            const V4 D = e0 * e0 + e1 * e1 + g0 * g0 + g1 * g1;
            const V4 sD = vsqrt(D);
            const V4 r = ws * Cc / sD * w;
            if (!jac) {
                acc.cost += 0.5 * r * r;
                continue;
            }
            const V4 ev[3] = {e0, e1, e2}, gv[3] = {g0, g1, vs(0.0)};
            const V4 k1 = ws / sD * w, k2 = ws * Cc / (D * sD) * w;
            V4 W[9];
            for (int i3 = 0; i3 < 3; ++i3)
                for (int j3 = 0; j3 < 3; ++j3) {
                    V4 dD = vs(0.0);
                    if (i3 < 2) dD += ev[i3] * a[j3];
                    if (j3 < 2) dD += gv[j3] * b[i3];
                    W[3 * i3 + j3] = k1 * b[i3] * a[j3] - k2 * dD;
                }
            for (int k = 0; k < kNFull; ++k) gf0[k] = vs(0.0);
            for (int k = 0; k < 3; ++k) {
                V4 dt = vs(0.0), ddl = vs(0.0);
                for (int i3 = 0; i3 < 3; ++i3)
                    for (int j3 = 0; j3 < 3; ++j3) {
                        const V4 we = W[3 * i3 + j3] * (s1[i3] * s0[j3]);
                        dt += we * dEt[k][3 * i3 + j3];
                        ddl += we * dEd[k][3 * i3 + j3];
                    }
                gf0[kT0 + k] = dt;
                gf0[kD0 + k] = ddl;
            }
            if (!cal) {
                V4 df0 = vs(0.0), df1 = vs(0.0);
                for (int e = 0; e < 9; ++e) {
                    df0 += W[e] * Ef0[e];
                    df1 += W[e] * Ef1[e];
                }
                if (sf)
                    gf0[kF0] = df0 + df1;
                else {
                    gf0[kF0] = df0;
                    gf0[kF1] = df1;
                }
            }
            acc.add(r, gf0);
        }
    }
    acc.reduce_into(acc_out);
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
    const int variant = C.P->variant;
    auto range = [&](size_t a, size_t b, Acc &acc) {
        if (variant == kTF)
            evaluate_range_v<kNFull>(C, p, jac, a, b, acc);
        else if (variant == kSF)
            evaluate_range_v<kF0 + 1>(C, p, jac, a, b, acc);
        else
            evaluate_range_v<kF0>(C, p, jac, a, b, acc);
    };
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
            lo_pool().run(nchunks, chunk);
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

bool lm_refine(const HostPair &P, const std::vector<int> *sample, const LMSettings &S, Model *m) {
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
