// Test harness (tests/test_md_exact_cpu.py): the device MD solvers of
// madpose_amd/csrc/include/mp_md_exact.h compiled for the host, behind a C ABI, so
// the CPU suite can check them against the oracle bit for bit.
#include <cstring>

#include "mp_md_exact.h"

extern "C" int mdx_check_solve(int variant, const double *x, const double *y, const double *dx, const double *dy,
                               double *sols) {
    double X[4][3], Y[4][3], scr[mp::kMdxScratchSF];
    const int k = variant == 0 ? 3 : 4;
    for (int i = 0; i < 4; ++i)
        for (int c = 0; c < 3; ++c) {
            X[i][c] = i < k ? x[3 * i + c] : 0.0;
            Y[i][c] = i < k ? y[3 * i + c] : 0.0;
        }
    int n = 0;
    auto keep = [&](const double (&sol)[6]) {
        for (int c = 0; c < 6; ++c) sols[6 * n + c] = sol[c];
        ++n;
    };
    const mp::LaneScratch W{scr, 1};
    if (variant == 0) {
        double x3[3][3], y3[3][3];
        for (int i = 0; i < 3; ++i)
            for (int c = 0; c < 3; ++c) {
                x3[i][c] = X[i][c];
                y3[i][c] = Y[i][c];
            }
        mp::mdx_sols_cal(W, x3, y3, dx, dy, keep);
    } else if (variant == 1) {
        mp::mdx_sols_sf(W, X, Y, dx, dy, keep);
    } else {
        mp::mdx_sols_tf(W, X, Y, dx, dy, keep);
    }
    return n;
}

// The pose stage (md_pose_exact) of every solution, as the oracle's md_pose returns
// it: 17 doubles per model (R row-major, t, scale, offset0, offset1, focal0, focal1).
extern "C" int mdx_check_pose(int variant, const double *x, const double *y, const double *dx, const double *dy,
                              double *models) {
    double sols[8][6];
    const int ns = mdx_check_solve(variant, x, y, dx, dy, &sols[0][0]);
    const int k = variant == 0 ? 3 : 4;
    double X[4][3], Y[4][3];
    for (int i = 0; i < 4; ++i)
        for (int c = 0; c < 3; ++c) {
            X[i][c] = i < k ? x[3 * i + c] : 0.0;
            Y[i][c] = i < k ? y[3 * i + c] : 0.0;
        }
    int n = 0;
    for (int q = 0; q < ns; ++q) {
        mp::Model m{};
        const double fa = variant == 0 ? 1.0 : sols[q][4], fb = variant == 0 ? 1.0 : sols[q][5];
        m.focal0 = fa;
        m.focal1 = fb;
        bool ok;
        if (variant == 0) {
            double x3[3][3], y3[3][3];
            for (int i = 0; i < 3; ++i)
                for (int c = 0; c < 3; ++c) {
                    x3[i][c] = X[i][c];
                    y3[i][c] = Y[i][c];
                }
            ok = mp::md_pose_exact<3>(x3, y3, dx, dy, sols[q], fa, fb, m);
        } else {
            ok = mp::md_pose_exact<4>(X, Y, dx, dy, sols[q], fa, fb, m);
        }
        if (!ok) continue;
        std::memcpy(models + 17 * n, &m, sizeof(m));
        ++n;
    }
    return n;
}

// The DLT null vector of a 4x4 matrix by both one-sided Jacobi forms of mp_math.h: the
// exact one (dlt_null4's fallback, the oracle's) and the one with the rotations'
// quotients and square roots rewritten for refined hardware reciprocals
// (smallest_right_sv4_fast, the two-focal recoverPose tests).  On the host both use
// IEEE arithmetic, so this checks the rewrite's algebra (|ga| / sqrt(al be) as
// |ga| rsq(al be), sqrt(1 + zeta^2) as u rsq(u)).
extern "C" void sv4_check(const double *a, double *v_exact, double *v_fast) {
    double A[4][4];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) A[i][j] = a[4 * i + j];
    mp::smallest_right_sv4(A, v_exact);
    mp::smallest_right_sv4_fast(A, v_fast);
}
