// Batched device Levenberg-Marquardt for the local optimisation (the Ceres solve of
// src/optimizer.h:48-125 and its shared-/two-focal analogues :265-369, :383-499, over
// the cost functors of src/cost_functions.h:16-387) -- SURVEY.md §8(f)1.
//
// One 256-lane workgroup per least-squares problem, any number of problems per launch.
// The problem is a residual-block list over the pair's device-resident correspondences
// (reproj0 blocks, reproj1 blocks, Sampson blocks; index lists in device memory) and a
// start model.  The algorithm is the host LM's (host/lm.cpp, itself the oracle's
// restatement of Ceres' trust-region LM): Jacobi column scaling, LM diagonal clamped to
// [1e-6, 1e32], initial radius 1e4, quaternion manifold Plus, bounds by projection,
// Ceres' non-monotonic step evaluator, function / gradient / parameter tolerances, and
// the parameters of the lowest cost returned.
//
//   * every lane evaluates residual blocks lane, lane + 256, ... with their analytic
//     Jacobians (the expressions of evaluate_range in host/lm.cpp) and accumulates the
//     packed normal equations of the NA parameters the variant can activate (cal 9,
//     sf 10, tf 11) in registers;
//   * the workgroup reduces them in a fixed order (wave butterflies, then the four
//     waves in order), so the result is deterministic;
//   * lane 0 runs the step logic (scaling, Cholesky, Plus, acceptance) on the reduced
//     system in LDS and publishes the next candidate.
#pragma once
#include "../include/mp_math.h"

namespace mp {
namespace {

// workgroup-free wave all-reduce (xor butterfly: every lane gets the same sum)
__device__ inline double lm_wave_sum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

enum LmFull { kLD0 = 0, kLD1, kLD2, kLT0, kLT1, kLT2, kLS, kLO0, kLO1, kLF0, kLF1, kLNFull };

struct LmParams {
    double q[4], R[9], t[3], s, o0, o1, f0, f1;
};

__device__ inline void lm_quat_to_rot(const double *q0, double *R) {
    const double n = sqrt(q0[0] * q0[0] + q0[1] * q0[1] + q0[2] * q0[2] + q0[3] * q0[3]);
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

// Eigen::Quaternion(Matrix3) (host/lm.cpp rot_to_quat)
__device__ inline void lm_rot_to_quat(const double *R, double *q) {
    const double tr = R[0] + R[4] + R[8];
    if (tr > 0) {
        double s = sqrt(tr + 1.0);
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
        double s = sqrt(R[4 * i] - R[4 * j] - R[4 * k] + 1.0);
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

// Packed normal equations over the first NA full-layout parameters.
template <int NA> struct LmAcc {
    static constexpr int kPack = NA * (NA + 1) / 2;
    double H[kPack], g[NA], cost;
    __device__ void clear() {
#pragma unroll
        for (int q = 0; q < kPack; ++q) H[q] = 0.0;
#pragma unroll
        for (int a = 0; a < NA; ++a) g[a] = 0.0;
        cost = 0.0;
    }
    __device__ void add(double r, const double (&gf)[kLNFull]) {
        cost += 0.5 * r * r;
        int q = 0;
#pragma unroll
        for (int a = 0; a < NA; ++a) {
            g[a] += gf[a] * r;
#pragma unroll
            for (int b = a; b < NA; ++b) H[q++] += gf[a] * gf[b];
        }
    }
};

__device__ inline void lm_mv3(const double *A, const double *v, double *o) {
#pragma unroll
    for (int r = 0; r < 3; ++r) o[r] = A[3 * r] * v[0] + A[3 * r + 1] * v[1] + A[3 * r + 2] * v[2];
}
__device__ inline void lm_mtv3(const double *A, const double *v, double *o) {
#pragma unroll
    for (int r = 0; r < 3; ++r) o[r] = A[r] * v[0] + A[3 + r] * v[1] + A[6 + r] * v[2];
}
__device__ inline void lm_mm3(const double *A, const double *B, double *C) {
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) C[3 * r + c] = A[3 * r] * B[c] + A[3 * r + 1] * B[3 + c] + A[3 * r + 2] * B[6 + c];
}
__device__ inline void lm_skew(const double *v, double *S) {
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

// LiftProjectionFunctor0 and variants (host/lm.cpp evaluate_range, first loop)
template <int V, int NA>
__device__ inline void lm_block_reproj0(const PairData &D, const PairConst &C, const LmParams &p, int i, bool jac,
                                        LmAcc<NA> &acc) {
    constexpr bool cal = V == kCal, sf = V == kSF;
    const double f0 = p.f0, f1 = sf ? p.f0 : p.f1;
    const double *R = p.R, *t = p.t;
    double c[3];
    const double xh[3] = {D.x0u[i], D.x0v[i], 1.0};
    if (cal)
        lm_mv3(C.K0i, xh, c);
    else {
        c[0] = xh[0] / f0;
        c[1] = xh[1] / f0;
        c[2] = 1.0;
    }
    const double a = D.d0[i] + p.o0;
    const double pp[3] = {c[0] * a, c[1] * a, c[2] * a};
    double v[3], y[3], h[3];
    lm_mv3(R, pp, v);
#pragma unroll
    for (int k = 0; k < 3; ++k) y[k] = v[k] + t[k];
    if (cal)
        lm_mv3(C.K1, y, h);
    else {
        h[0] = f1 * y[0];
        h[1] = f1 * y[1];
        h[2] = y[2];
    }
    const double iz = 1.0 / h[2];
    const double r0 = h[0] * iz - D.x1u[i], r1 = h[1] * iz - D.x1v[i];
    if (!jac) {
        acc.cost += 0.5 * r0 * r0;
        acc.cost += 0.5 * r1 * r1;
        return;
    }
    const double Dh[2][3] = {{iz, 0, -h[0] * iz * iz}, {0, iz, -h[1] * iz * iz}};
    double G[2][3];
#pragma unroll
    for (int rr = 0; rr < 2; ++rr)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            if (cal)
                G[rr][k] = Dh[rr][0] * C.K1[k] + Dh[rr][1] * C.K1[3 + k] + Dh[rr][2] * C.K1[6 + k];
            else
                G[rr][k] = Dh[rr][k] * (k < 2 ? f1 : 1.0);
        }
    double Sv[9];
    lm_skew(v, Sv);
    double Rc[3];
    lm_mv3(R, c, Rc);
    double Rdcf[3] = {0, 0, 0};
    if (!cal) {
        const double dcf[3] = {-xh[0] / (f0 * f0) * a, -xh[1] / (f0 * f0) * a, 0.0};
        lm_mv3(R, dcf, Rdcf);
    }
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
        double gf[kLNFull];
#pragma unroll
        for (int k = 0; k < kLNFull; ++k) gf[k] = 0.0;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            gf[kLD0 + k] = -2.0 * (G[rr][0] * Sv[k] + G[rr][1] * Sv[3 + k] + G[rr][2] * Sv[6 + k]);
            gf[kLT0 + k] = G[rr][k];
        }
        gf[kLO0] = G[rr][0] * Rc[0] + G[rr][1] * Rc[1] + G[rr][2] * Rc[2];
        if (!cal) {
            const double dyf0 = G[rr][0] * Rdcf[0] + G[rr][1] * Rdcf[1] + G[rr][2] * Rdcf[2];
            const double dhf1 = Dh[rr][0] * y[0] + Dh[rr][1] * y[1];
            if (sf)
                gf[kLF0] = dyf0 + dhf1;
            else {
                gf[kLF0] = dyf0;
                gf[kLF1] = dhf1;
            }
        }
        acc.add(rr == 0 ? r0 : r1, gf);
    }
}

// LiftProjectionFunctor1 (second loop)
template <int V, int NA>
__device__ inline void lm_block_reproj1(const PairData &D, const PairConst &C, const LmParams &p, int i, bool jac,
                                        LmAcc<NA> &acc) {
    constexpr bool cal = V == kCal, sf = V == kSF;
    const double f0 = p.f0, f1 = sf ? p.f0 : p.f1;
    const double *R = p.R, *t = p.t;
    double c[3];
    const double xh[3] = {D.x1u[i], D.x1v[i], 1.0};
    if (cal)
        lm_mv3(C.K1i, xh, c);
    else {
        c[0] = xh[0] / f1;
        c[1] = xh[1] / f1;
        c[2] = 1.0;
    }
    const double dep = D.d1[i] + p.o1;
    const double a = dep * p.s;
    const double u[3] = {c[0] * a - t[0], c[1] * a - t[1], c[2] * a - t[2]};
    double y[3], h[3];
    lm_mtv3(R, u, y);
    if (cal)
        lm_mv3(C.K0, y, h);
    else {
        h[0] = f0 * y[0];
        h[1] = f0 * y[1];
        h[2] = y[2];
    }
    const double iz = 1.0 / h[2];
    const double r0 = h[0] * iz - D.x0u[i], r1 = h[1] * iz - D.x0v[i];
    if (!jac) {
        acc.cost += 0.5 * r0 * r0;
        acc.cost += 0.5 * r1 * r1;
        return;
    }
    const double Dh[2][3] = {{iz, 0, -h[0] * iz * iz}, {0, iz, -h[1] * iz * iz}};
    double G[2][3];
#pragma unroll
    for (int rr = 0; rr < 2; ++rr)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            if (cal)
                G[rr][k] = Dh[rr][0] * C.K0[k] + Dh[rr][1] * C.K0[3 + k] + Dh[rr][2] * C.K0[6 + k];
            else
                G[rr][k] = Dh[rr][k] * (k < 2 ? f0 : 1.0);
        }
    double Su[9], RtSu[9];
    lm_skew(u, Su);
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int cc = 0; cc < 3; ++cc)
            RtSu[3 * r + cc] = R[r] * Su[cc] + R[3 + r] * Su[3 + cc] + R[6 + r] * Su[6 + cc];
    double Rtc[3];
    lm_mtv3(R, c, Rtc);
    double Rtdcf[3] = {0, 0, 0};
    if (!cal) {
        const double dcf[3] = {-xh[0] / (f1 * f1) * a, -xh[1] / (f1 * f1) * a, 0.0};
        lm_mtv3(R, dcf, Rtdcf);
    }
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
        double gf[kLNFull];
#pragma unroll
        for (int k = 0; k < kLNFull; ++k) gf[k] = 0.0;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            gf[kLD0 + k] = 2.0 * (G[rr][0] * RtSu[k] + G[rr][1] * RtSu[3 + k] + G[rr][2] * RtSu[6 + k]);
            gf[kLT0 + k] = -(G[rr][0] * R[3 * k] + G[rr][1] * R[3 * k + 1] + G[rr][2] * R[3 * k + 2]);
        }
        const double gRtc = G[rr][0] * Rtc[0] + G[rr][1] * Rtc[1] + G[rr][2] * Rtc[2];
        gf[kLS] = gRtc * dep;
        gf[kLO1] = gRtc * p.s;
        if (!cal) {
            const double dyf1 = G[rr][0] * Rtdcf[0] + G[rr][1] * Rtdcf[1] + G[rr][2] * Rtdcf[2];
            const double dhf0 = Dh[rr][0] * y[0] + Dh[rr][1] * y[1];
            if (sf)
                gf[kLF0] = dyf1 + dhf0;
            else {
                gf[kLF0] = dhf0;
                gf[kLF1] = dyf1;
            }
        }
        acc.add(rr == 0 ? r0 : r1, gf);
    }
}

// Sampson constants of a parameter set: F = diag(s1) E diag(s0), E = [t]x R, and the
// derivative blocks dE/dt_k = [e_k]x R, dE/ddelta_k = 2 [t]x [e_k]x R
struct LmSampsonConst {
    double E[9], F[9], s0[3], s1[3], dEt[3][9], dEd[3][9];
};
template <int V> __device__ inline void lm_sampson_const(const LmParams &p, LmSampsonConst &K) {
    constexpr bool cal = V == kCal, sf = V == kSF;
    const double f0 = p.f0, f1 = sf ? p.f0 : p.f1;
    double Tx[9];
    lm_skew(p.t, Tx);
    lm_mm3(Tx, p.R, K.E);
#pragma unroll
    for (int k = 0; k < 3; ++k) K.s0[k] = K.s1[k] = 1.0;
    if (!cal) {
        K.s0[0] = K.s0[1] = 1.0 / f0;
        K.s1[0] = K.s1[1] = 1.0 / f1;
    }
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) K.F[3 * r + c] = K.E[3 * r + c] * K.s1[r] * K.s0[c];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        double ek[3] = {0, 0, 0};
        ek[k] = 1.0;
        double Sk[9];
        lm_skew(ek, Sk);
        lm_mm3(Sk, p.R, K.dEt[k]);
        lm_mm3(Tx, K.dEt[k], K.dEd[k]);
#pragma unroll
        for (int e = 0; e < 9; ++e) K.dEd[k][e] *= 2.0;
    }
}

// SampsonError*Functor: r = w C / |(e0, e1, g0, g1)| (third loop)
template <int V, int NA>
__device__ inline void lm_block_sampson(const PairData &D, const PairConst &C, const LmParams &p,
                                        const LmSampsonConst &K, double w_sampson, int i, bool jac, LmAcc<NA> &acc) {
    constexpr bool cal = V == kCal, sf = V == kSF;
    const double f0 = p.f0, f1 = sf ? p.f0 : p.f1;
    double a[3], b[3];
    if (cal) {
        const double xa[3] = {D.x0u[i], D.x0v[i], 1.0}, xb[3] = {D.x1u[i], D.x1v[i], 1.0};
        lm_mv3(C.K0i, xa, a);
        lm_mv3(C.K1i, xb, b);
    } else {
        a[0] = D.x0u[i];
        a[1] = D.x0v[i];
        b[0] = D.x1u[i];
        b[1] = D.x1v[i];
    }
    a[2] = b[2] = 1.0;
    const double *F = K.F;
    const double e0 = F[0] * a[0] + F[1] * a[1] + F[2];
    const double e1 = F[3] * a[0] + F[4] * a[1] + F[5];
    const double e2 = F[6] * a[0] + F[7] * a[1] + F[8];
    const double g0 = F[0] * b[0] + F[3] * b[1] + F[6];
    const double g1 = F[1] * b[0] + F[4] * b[1] + F[7];
    const double Cc = b[0] * e0 + b[1] * e1 + e2;
    const double Dd = e0 * e0 + e1 * e1 + g0 * g0 + g1 * g1;
    const double sD = sqrt(Dd);
    const double r = w_sampson * Cc / sD;
    if (!jac) {
        acc.cost += 0.5 * r * r;
        return;
    }
    const double ev[3] = {e0, e1, e2}, gv[3] = {g0, g1, 0.0};
    double W[9];
    const double k1 = w_sampson / sD, k2 = w_sampson * Cc / (Dd * sD);
#pragma unroll
    for (int ii = 0; ii < 3; ++ii)
#pragma unroll
        for (int jj = 0; jj < 3; ++jj) {
            const double dD = (ii < 2 ? ev[ii] * a[jj] : 0.0) + (jj < 2 ? gv[jj] * b[ii] : 0.0);
            W[3 * ii + jj] = k1 * b[ii] * a[jj] - k2 * dD;
        }
    double WE[9];
#pragma unroll
    for (int ii = 0; ii < 3; ++ii)
#pragma unroll
        for (int jj = 0; jj < 3; ++jj) WE[3 * ii + jj] = W[3 * ii + jj] * K.s1[ii] * K.s0[jj];
    double gf[kLNFull];
#pragma unroll
    for (int k = 0; k < kLNFull; ++k) gf[k] = 0.0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        double dt = 0, dd = 0;
#pragma unroll
        for (int e = 0; e < 9; ++e) {
            dt += WE[e] * K.dEt[k][e];
            dd += WE[e] * K.dEd[k][e];
        }
        gf[kLT0 + k] = dt;
        gf[kLD0 + k] = dd;
    }
    if (!cal) {
        const double ds0[3] = {-1.0 / (f0 * f0), -1.0 / (f0 * f0), 0.0};
        const double ds1[3] = {-1.0 / (f1 * f1), -1.0 / (f1 * f1), 0.0};
        double df0 = 0, df1 = 0;
#pragma unroll
        for (int ii = 0; ii < 3; ++ii)
#pragma unroll
            for (int jj = 0; jj < 3; ++jj) {
                df0 += W[3 * ii + jj] * K.E[3 * ii + jj] * K.s1[ii] * ds0[jj];
                df1 += W[3 * ii + jj] * K.E[3 * ii + jj] * ds1[ii] * K.s0[jj];
            }
        if (sf)
            gf[kLF0] = df0 + df1;
        else {
            gf[kLF0] = df0;
            gf[kLF1] = df1;
        }
    }
    acc.add(r, gf);
}

constexpr int kLmBlock = 256;

// Shared state of one problem (LDS).  The reduced normal equations stay in the full
// NA-parameter layout (packed upper triangle, then g, then the cost); parameters that
// are inactive for the call are masked to an identity row with zero gradient, which
// leaves every operation on the active ones exactly as in the compacted system of
// host/lm.cpp (the extra terms are exact zeros).
template <int NA> struct LmShared {
    static constexpr int kPack = NA * (NA + 1) / 2, kRed = kPack + NA + 1;
    LmParams x, c, best;
    double part[kLmBlock / 64][kRed]; // per-wave reduced accumulators
    double red[2][kRed];              // the systems of x (red[cur]) and of the candidate
    double d[NA];                     // the step (lane 0)
    LmSampsonConst K;                 // Sampson constants of the parameter set being evaluated
    double lo[kLNFull];
    int has_lo[kLNFull];
    int col[kLNFull];
    int cur;
    int action; // decision after an evaluation: 0 stop, 2 propose a step
    int prop;   // proposal: 0 stop, 1 evaluate the candidate sh.c
    // (two words: every wave reads `action` at the top of the loop while lane 0 is
    // already writing the proposal; each word is rewritten only behind a barrier that
    // all of its readers have passed)
};

__device__ inline int lm_up(int a, int b, int na) { return a * na - a * (a - 1) / 2 + (b - a); } // a <= b

// reduce every lane's accumulator over the workgroup into out[kRed] (LDS): the four
// waves' butterflies, then one entry per thread summed over the waves in order
template <int NA> __device__ inline void lm_reduce(LmAcc<NA> &acc, LmShared<NA> &sh, double *out) {
    constexpr int kPack = LmShared<NA>::kPack, kRed = LmShared<NA>::kRed;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int q = 0; q < kPack; ++q) {
        const double v = lm_wave_sum(acc.H[q]);
        if (lane == 0) sh.part[wave][q] = v;
    }
#pragma unroll
    for (int a = 0; a < NA; ++a) {
        const double v = lm_wave_sum(acc.g[a]);
        if (lane == 0) sh.part[wave][kPack + a] = v;
    }
    {
        const double v = lm_wave_sum(acc.cost);
        if (lane == 0) sh.part[wave][kPack + NA] = v;
    }
    __syncthreads();
    if (threadIdx.x < kRed) {
        double v = 0.0;
#pragma unroll
        for (int w = 0; w < kLmBlock / 64; ++w) v += sh.part[w][threadIdx.x];
        out[threadIdx.x] = v;
    }
    __syncthreads();
}

// cost and normal equations of parameter set p over the job's blocks into out
template <int V, int NA>
__device__ inline void lm_evaluate(const PairData &D, const PairConst &C, const LmJob &J, const int *idx,
                                   const LmParams &p, LmShared<NA> &sh, double *out) {
    LmAcc<NA> acc;
    acc.clear();
    const int nb = J.n0 + J.n1 + J.n2;
    if (J.n2 > 0) {
        if (threadIdx.x == 0) lm_sampson_const<V>(p, sh.K);
        __syncthreads();
    }
    // blocks b = lane, lane + 256, ... of the concatenated list, one loop per block type
    int b = threadIdx.x;
    for (; b < J.n0; b += kLmBlock) lm_block_reproj0<V, NA>(D, C, p, idx[J.off0 + b], true, acc);
    for (; b < J.n0 + J.n1; b += kLmBlock) lm_block_reproj1<V, NA>(D, C, p, idx[J.off1 + b - J.n0], true, acc);
    for (; b < nb; b += kLmBlock)
        lm_block_sampson<V, NA>(D, C, p, sh.K, J.w_sampson, idx[J.off2 + b - J.n0 - J.n1], true, acc);
    lm_reduce<NA>(acc, sh, out);
}

// gradient max-norm over the active parameters
template <int NA> __device__ inline double lm_gmax(const double *red, const bool (&act)[NA]) {
    double v = 0.0;
#pragma unroll
    for (int a = 0; a < NA; ++a)
        if (act[a]) v = fmax(v, fabs(red[LmShared<NA>::kPack + a]));
    return v;
}

// The LM step of host/lm.cpp (Jacobi scaling, clamped diagonal / radius, Cholesky) in
// registers with compile-time indices; d = 0 on inactive parameters.  False when the
// damped system is not positive definite.
template <int NA>
__device__ inline bool lm_step(const double *red, const bool (&act)[NA], double radius, double (&d)[NA]) {
    constexpr int kP = NA * (NA + 1) / 2;
    double L[kP]; // lower triangle, row-major packed: (i, j) at i (i + 1) / 2 + j
    double sc[NA], y[NA];
#pragma unroll
    for (int a = 0; a < NA; ++a) {
        const double h = act[a] ? red[lm_up(a, a, NA)] : 1.0;
        sc[a] = 1.0 / (1.0 + sqrt(h));
        y[a] = act[a] ? -red[kP + a] * sc[a] : 0.0;
    }
#pragma unroll
    for (int i = 0; i < NA; ++i)
#pragma unroll
        for (int j = 0; j <= i; ++j) {
            const double h = (act[i] && act[j]) ? red[lm_up(j, i, NA)] : (i == j ? 1.0 : 0.0);
            L[i * (i + 1) / 2 + j] = h * sc[i] * sc[j];
        }
#pragma unroll
    for (int j = 0; j < NA; ++j) {
        double &a = L[j * (j + 1) / 2 + j];
        a += fmin(fmax(a, 1e-6), 1e32) / radius;
    }
    bool ok = true;
#pragma unroll
    for (int j = 0; j < NA; ++j) {
        double dj = L[j * (j + 1) / 2 + j];
#pragma unroll
        for (int k = 0; k < j; ++k) dj -= L[j * (j + 1) / 2 + k] * L[j * (j + 1) / 2 + k];
        ok = ok && (dj > 0);
        dj = sqrt(dj);
        L[j * (j + 1) / 2 + j] = dj;
#pragma unroll
        for (int i = j + 1; i < NA; ++i) {
            double s2 = L[i * (i + 1) / 2 + j];
#pragma unroll
            for (int k = 0; k < j; ++k) s2 -= L[i * (i + 1) / 2 + k] * L[j * (j + 1) / 2 + k];
            L[i * (i + 1) / 2 + j] = s2 / dj;
        }
    }
    if (!ok) return false;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
        double s2 = y[i];
#pragma unroll
        for (int k = 0; k < i; ++k) s2 -= L[i * (i + 1) / 2 + k] * y[k];
        y[i] = s2 / L[i * (i + 1) / 2 + i];
    }
#pragma unroll
    for (int i = NA - 1; i >= 0; --i) {
        double s2 = y[i];
#pragma unroll
        for (int k = i + 1; k < NA; ++k) s2 -= L[k * (k + 1) / 2 + i] * y[k];
        y[i] = s2 / L[i * (i + 1) / 2 + i];
    }
#pragma unroll
    for (int a = 0; a < NA; ++a) d[a] = act[a] ? y[a] * sc[a] : 0.0;
    return true;
}

__device__ inline double lm_amb_norm2(const LmParams &p) {
    return p.q[0] * p.q[0] + p.q[1] * p.q[1] + p.q[2] * p.q[2] + p.q[3] * p.q[3] + p.t[0] * p.t[0] +
           p.t[1] * p.t[1] + p.t[2] * p.t[2] + p.s * p.s + p.o0 * p.o0 + p.o1 * p.o1 + p.f0 * p.f0 + p.f1 * p.f1;
}

// One workgroup per job: out[job] = the refined model, status[job] = 1 (refined),
// 0 (no residuals: unchanged), 2 (a constant bounded block starts infeasible: unchanged)
template <int V>
__global__ void __launch_bounds__(kLmBlock) lm_batch_kernel(PairData D, PairConst C, const LmJob *jobs,
                                                           const int *idx, Model *out, int *status) {
    constexpr int NA = V == kCal ? kLF0 : (V == kSF ? kLF0 + 1 : kLNFull);
    constexpr int kPack = LmShared<NA>::kPack;
    __shared__ LmShared<NA> sh;
    const LmJob &J = jobs[blockIdx.x]; // (read in place: uniform, kept out of registers)
    const bool t0 = threadIdx.x == 0;
    // ---- setup (lm_refine in host/lm.cpp) ----
    if (t0) {
        const bool has_o0 = J.n0 > 0, has_s_o1 = J.n1 > 0;
        for (int k = 0; k < kLNFull; ++k) {
            sh.col[k] = -1;
            sh.has_lo[k] = 0;
            sh.lo[k] = 0.0;
        }
        for (int k = 0; k < 6; ++k) sh.col[k] = k;
        if (has_s_o1) {
            sh.col[kLS] = kLS;
            sh.has_lo[kLS] = 1;
            sh.lo[kLS] = 1e-2;
        }
        if (has_o0 && J.use_shift) sh.col[kLO0] = kLO0;
        if (has_s_o1 && J.use_shift) sh.col[kLO1] = kLO1;
        if (J.min_depth_constraint) {
            sh.has_lo[kLO0] = sh.has_lo[kLO1] = 1;
            sh.lo[kLO0] = -C.min_depth[0] + 1e-2;
            sh.lo[kLO1] = -C.min_depth[1] + 1e-2;
        }
        if (V == kSF) sh.col[kLF0] = kLF0;
        if (V == kTF) {
            sh.col[kLF0] = kLF0;
            sh.col[kLF1] = kLF1;
            sh.has_lo[kLF0] = sh.has_lo[kLF1] = 1;
            sh.lo[kLF0] = sh.lo[kLF1] = 1e-6;
        }
        LmParams &x = sh.x;
        lm_rot_to_quat(J.m.R, x.q);
        lm_quat_to_rot(x.q, x.R);
        for (int k = 0; k < 3; ++k) x.t[k] = J.m.t[k];
        x.s = J.m.scale;
        x.o0 = J.m.offset0;
        x.o1 = J.m.offset1;
        x.f0 = J.m.focal0;
        x.f1 = J.m.focal1;
        sh.best = x;
        sh.cur = 0;
        sh.action = 1;
        if (J.n0 + J.n1 + J.n2 == 0) sh.action = 0;
        // constant bounded blocks must start feasible (Ceres Program::IsFeasible)
        if (!J.use_shift && J.min_depth_constraint) {
            if (has_o0 && x.o0 < sh.lo[kLO0]) sh.action = 0;
            if (has_s_o1 && x.o1 < sh.lo[kLO1]) sh.action = 0;
        }
        if (J.n0 + J.n1 + J.n2 == 0)
            status[blockIdx.x] = 0;
        else
            status[blockIdx.x] = sh.action ? 1 : 2;
    }
    __syncthreads();
    if (sh.action == 0) {
        if (t0) out[blockIdx.x] = J.m;
        return;
    }
    bool act[NA];
#pragma unroll
    for (int a = 0; a < NA; ++a) act[a] = sh.col[a] >= 0;
    lm_evaluate<V, NA>(D, C, J, idx, sh.x, sh, sh.red[0]);
    // ---- trust-region loop (lane 0 decides, every lane evaluates) ----
    double radius = 1e4, decrease = 2.0;
    const int max_nonmono = J.nonmonotonic ? 5 : 0;
    double ref_cost = 0, min_cost = 0, cand_ref = 0, acc_ref = 0.0, acc_cand = 0.0;
    int n_nonmono = 0, iter = 0;
    if (t0) {
        ref_cost = min_cost = cand_ref = sh.red[0][kPack + NA];
        sh.action = (lm_gmax<NA>(sh.red[0], act) <= J.gtol) ? 0 : 2;
    }
    __syncthreads();
    while (sh.action != 0) {
        if (t0) {
            // propose a step from x (repeated while the damped system is not positive definite)
            const double *R = sh.red[sh.cur];
            int prop = 0;
            while (iter < J.max_iter) {
                ++iter;
                double d[NA];
                if (!lm_step<NA>(R, act, radius, d)) {
                    radius /= decrease;
                    decrease *= 2.0;
                    if (radius < 1e-32) break;
                    continue;
                }
#pragma unroll
                for (int a = 0; a < NA; ++a) sh.d[a] = d[a];
                // candidate = Plus(x, d), projected onto the bounds
                const LmParams &x = sh.x;
                LmParams c = x;
                {
                    const double nd = sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
                    if (nd > 0) {
                        const double sn = sin(nd) / nd;
                        const double qd[4] = {cos(nd), sn * d[0], sn * d[1], sn * d[2]};
                        const double *q = x.q;
                        c.q[0] = qd[0] * q[0] - qd[1] * q[1] - qd[2] * q[2] - qd[3] * q[3];
                        c.q[1] = qd[0] * q[1] + qd[1] * q[0] + qd[2] * q[3] - qd[3] * q[2];
                        c.q[2] = qd[0] * q[2] - qd[1] * q[3] + qd[2] * q[0] + qd[3] * q[1];
                        c.q[3] = qd[0] * q[3] + qd[1] * q[2] - qd[2] * q[1] + qd[3] * q[0];
                    }
#pragma unroll
                    for (int k = 0; k < 3; ++k) c.t[k] = x.t[k] + d[3 + k];
                    auto upd = [&](int slot, double v, double dv) {
                        if (sh.col[slot] < 0) return v;
                        v += dv;
                        return (sh.has_lo[slot] && v < sh.lo[slot]) ? sh.lo[slot] : v;
                    };
                    c.s = upd(kLS, c.s, d[kLS]);
                    c.o0 = upd(kLO0, c.o0, d[kLO0]);
                    c.o1 = upd(kLO1, c.o1, d[kLO1]);
                    if (NA > kLF0) c.f0 = upd(kLF0, c.f0, d[NA > kLF0 ? kLF0 : 0]);
                    if (NA > kLF1) c.f1 = upd(kLF1, c.f1, d[NA > kLF1 ? kLF1 : 0]);
                    lm_quat_to_rot(c.q, c.R);
                }
                double step2 = 0;
                {
                    const double dd[12] = {c.q[0] - x.q[0], c.q[1] - x.q[1], c.q[2] - x.q[2], c.q[3] - x.q[3],
                                           c.t[0] - x.t[0], c.t[1] - x.t[1], c.t[2] - x.t[2], c.s - x.s,
                                           c.o0 - x.o0,     c.o1 - x.o1,     c.f0 - x.f0,     c.f1 - x.f1};
#pragma unroll
                    for (int k = 0; k < 12; ++k) step2 += dd[k] * dd[k];
                }
                if (sqrt(step2) <= J.ptol * (sqrt(lm_amb_norm2(x)) + J.ptol)) break; // parameter tolerance
                sh.c = c;
                prop = 1;
                break;
            }
            sh.prop = prop;
        }
        __syncthreads();
        if (sh.prop == 0) break;
        lm_evaluate<V, NA>(D, C, J, idx, sh.c, sh, sh.red[sh.cur ^ 1]);
        if (t0) {
            const double *R = sh.red[sh.cur], *Rc = sh.red[sh.cur ^ 1];
            const double cost = R[kPack + NA], cand_cost = Rc[kPack + NA];
            sh.action = 2;
            if (fabs(cost - cand_cost) <= J.ftol * cost) {
                sh.action = 0; // function tolerance
            } else {
                double d[NA];
#pragma unroll
                for (int a = 0; a < NA; ++a) d[a] = sh.d[a];
                double gd = 0, jd2 = 0;
#pragma unroll
                for (int a = 0; a < NA; ++a) {
                    gd += (act[a] ? R[kPack + a] : 0.0) * d[a];
#pragma unroll
                    for (int b2 = 0; b2 < NA; ++b2) {
                        const double h = (act[a] && act[b2]) ? R[a <= b2 ? lm_up(a, b2, NA) : lm_up(b2, a, NA)] : 0.0;
                        jd2 += d[a] * h * d[b2];
                    }
                }
                const double mcc = -(gd + 0.5 * jd2);
                const double rho = (mcc > 0 && isfinite(cand_cost))
                                       ? fmax((cost - cand_cost) / mcc, (ref_cost - cand_cost) / (acc_ref + mcc))
                                       : -1.0;
                if (rho > 1e-3) {
                    sh.x = sh.c;
                    sh.cur ^= 1;
                    // Ceres TrustRegionStepEvaluator::StepAccepted
                    acc_cand += mcc;
                    acc_ref += mcc;
                    if (cand_cost < min_cost) {
                        min_cost = cand_cost;
                        n_nonmono = 0;
                        cand_ref = cand_cost;
                        acc_cand = 0.0;
                        sh.best = sh.x;
                    } else {
                        ++n_nonmono;
                        if (cand_cost > cand_ref) {
                            cand_ref = cand_cost;
                            acc_cand = 0.0;
                        }
                    }
                    if (n_nonmono == max_nonmono) {
                        ref_cost = cand_ref;
                        acc_ref = acc_cand;
                    }
                    radius = fmin(1e16, radius / fmax(1.0 / 3.0, 1.0 - pow(2.0 * rho - 1.0, 3.0)));
                    decrease = 2.0;
                    if (lm_gmax<NA>(Rc, act) <= J.gtol) sh.action = 0;
                } else {
                    radius /= decrease;
                    decrease *= 2.0;
                    if (radius < 1e-32) sh.action = 0;
                }
            }
            if (iter >= J.max_iter) sh.action = 0;
        }
        __syncthreads();
    }
    if (t0) {
        Model m = J.m;
        const LmParams &b = sh.best;
        lm_quat_to_rot(b.q, m.R);
        for (int k = 0; k < 3; ++k) m.t[k] = b.t[k];
        m.scale = b.s;
        m.offset0 = b.o0;
        m.offset1 = b.o1;
        m.focal0 = b.f0;
        m.focal1 = (V == kSF) ? b.f0 : b.f1;
        out[blockIdx.x] = m;
    }
}

} // namespace
} // namespace mp
