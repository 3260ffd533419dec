// Test harness (tests/test_md_exact_cpu.py): the device MD solvers of
// madpose_amd/csrc/include/mp_md_exact.h compiled for the host, behind a C ABI, so
// the CPU suite can check them against the oracle bit for bit.
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
