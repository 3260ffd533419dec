// ORACLE -- test infrastructure only.
//
// Ceres stand-in for the local-optimisation refinement (src/optimizer.h:48-125 and
// the SF/TF analogues at :265-369, :383-499; cost functors src/cost_functions.h).
// Ceres >= 2.0 is not available offline, so its algorithm is restated ("parity
// unpinned"): a Levenberg-Marquardt trust-region loop with Jacobi column scaling,
// LM diagonal clamped to [1e-6, 1e32], initial radius 1e4, step acceptance at
// relative decrease > 1e-3, radius update mu /= max(1/3, 1-(2rho-1)^3), box bounds
// applied by projection after the manifold Plus, QuaternionManifold
// (Plus(q, d) = [cos|d|, sin|d|/|d| d] (x) q), and the function / gradient /
// parameter tolerances of EstimatorConfig.  The product implements the SAME
// algorithm independently (analytic Jacobians); this oracle differentiates with
// forward-mode dual numbers, like Ceres' AutoDiffCostFunction.
#pragma once
#include <cmath>

namespace oracle {

constexpr int kJetN = 12; // q(4) t(3) scale offset0 offset1 focal0 focal1

struct Jet {
    double a;
    double v[kJetN];
    Jet() : a(0) {
        for (int i = 0; i < kJetN; ++i) v[i] = 0;
    }
    Jet(double x) : a(x) {
        for (int i = 0; i < kJetN; ++i) v[i] = 0;
    }
    static Jet var(double x, int k) {
        Jet j(x);
        j.v[k] = 1.0;
        return j;
    }
};
inline Jet operator+(const Jet &x, const Jet &y) {
    Jet r(x.a + y.a);
    for (int i = 0; i < kJetN; ++i) r.v[i] = x.v[i] + y.v[i];
    return r;
}
inline Jet operator-(const Jet &x, const Jet &y) {
    Jet r(x.a - y.a);
    for (int i = 0; i < kJetN; ++i) r.v[i] = x.v[i] - y.v[i];
    return r;
}
inline Jet operator-(const Jet &x) {
    Jet r(-x.a);
    for (int i = 0; i < kJetN; ++i) r.v[i] = -x.v[i];
    return r;
}
inline Jet operator*(const Jet &x, const Jet &y) {
    Jet r(x.a * y.a);
    for (int i = 0; i < kJetN; ++i) r.v[i] = x.a * y.v[i] + x.v[i] * y.a;
    return r;
}
inline Jet operator/(const Jet &x, const Jet &y) {
    Jet r(x.a / y.a);
    const double inv = 1.0 / y.a;
    for (int i = 0; i < kJetN; ++i) r.v[i] = (x.v[i] - r.a * y.v[i]) * inv;
    return r;
}
inline Jet sqrt(const Jet &x) {
    Jet r(std::sqrt(x.a));
    const double d = 0.5 / r.a;
    for (int i = 0; i < kJetN; ++i) r.v[i] = x.v[i] * d;
    return r;
}
inline double value(const Jet &x) { return x.a; }
inline double value(double x) { return x; }

} // namespace oracle
