// ORACLE -- test infrastructure only.
//
// The three estimators' data handling, minimal solvers, residuals and the Ceres
// stand-in (LM) used by LO:
//   src/hybrid_pose_estimator.{h,cpp}               (calibrated)
//   src/hybrid_pose_shared_focal_estimator.{h,cpp}  (shared focal)
//   src/hybrid_pose_two_focal_estimator.{h,cpp}     (two focals)
//   src/optimizer.h, src/cost_functions.h           (LO refinement)
#include <algorithm>
#include <cmath>
#include <limits>

#include "la.h"
#include "lm.h"
#include "oracle.h"

namespace oracle {

namespace {

void inv3(const double *K, double *Ki) {
    double d = det3(K);
    Ki[0] = (K[4] * K[8] - K[5] * K[7]) / d;
    Ki[1] = (K[2] * K[7] - K[1] * K[8]) / d;
    Ki[2] = (K[1] * K[5] - K[2] * K[4]) / d;
    Ki[3] = (K[5] * K[6] - K[3] * K[8]) / d;
    Ki[4] = (K[0] * K[8] - K[2] * K[6]) / d;
    Ki[5] = (K[2] * K[3] - K[0] * K[5]) / d;
    Ki[6] = (K[3] * K[7] - K[4] * K[6]) / d;
    Ki[7] = (K[1] * K[6] - K[0] * K[7]) / d;
    Ki[8] = (K[0] * K[4] - K[1] * K[3]) / d;
}

inline void mv3(const double *M, const double *v, double *o) {
    for (int r = 0; r < 3; ++r) o[r] = M[3 * r] * v[0] + M[3 * r + 1] * v[1] + M[3 * r + 2] * v[2];
}

} // namespace

Problem make_problem(Variant v, int n, const double *x0, const double *x1, const double *d0, const double *d1,
                     const double min_depth[2], const double *cam0, const double *cam1, const EstConfig &cfg,
                     Options *opts) {
    Problem P;
    // the scale-only estimator shares the calibrated geometry (src/hybrid_pose_estimator.h:110-134)
    P.scale_only = (v == SCALE);
    if (v == SCALE) v = CAL;
    P.variant = v;
    P.n = n;
    P.cfg = cfg;
    P.use_ours = opts->use_ours;
    P.use_4p4d = opts->use_4p4d;
    P.min_depth[0] = min_depth[0];
    P.min_depth[1] = min_depth[1];
    P.x0.resize(3 * n);
    P.x1.resize(3 * n);
    P.d0.assign(d0, d0 + n);
    P.d1.assign(d1, d1 + n);
    std::vector<double> thr = opts->squared_inlier_thresholds;
    std::vector<double> w = opts->data_type_weights;
    if (v == CAL) {
        for (int i = 0; i < 9; ++i) {
            P.K0[i] = cam0[i];
            P.K1[i] = cam1[i];
        }
        inv3(P.K0, P.K0inv);
        inv3(P.K1, P.K1inv);
        for (int i = 0; i < n; ++i) {
            P.x0[3 * i] = x0[2 * i];
            P.x0[3 * i + 1] = x0[2 * i + 1];
            P.x0[3 * i + 2] = 1.0;
            P.x1[3 * i] = x1[2 * i];
            P.x1[3 * i + 1] = x1[2 * i + 1];
            P.x1[3 * i + 2] = 1.0;
        }
        // src/hybrid_pose_estimator.h:35-36
        double s = 1.0 / (P.K0[0] + P.K0[4]) + 1.0 / (P.K1[0] + P.K1[4]);
        P.sampson_loss_scale = 1.0 / std::pow(s, 2);
    } else {
        // pp-centring + PoseLib normalize_points(.., true, false, true)
        // (src/hybrid_pose_shared_focal_estimator.cpp:14-22; ..two_focal..:40-48)
        std::vector<double> a(2 * n), b(2 * n);
        for (int i = 0; i < n; ++i) {
            a[2 * i] = x0[2 * i] - cam0[0];
            a[2 * i + 1] = x0[2 * i + 1] - cam0[1];
            b[2 * i] = x1[2 * i] - cam1[0];
            b[2 * i + 1] = x1[2 * i + 1] - cam1[1];
        }
        double scale = 0.0;
        for (int i = 0; i < n; ++i) {
            scale += std::sqrt(a[2 * i] * a[2 * i] + a[2 * i + 1] * a[2 * i + 1]);
            scale += std::sqrt(b[2 * i] * b[2 * i] + b[2 * i + 1] * b[2 * i + 1]);
        }
        scale /= std::sqrt(2.0) * n;
        if (n == 0) scale = 1.0;
        P.norm_scale = scale;
        for (int i = 0; i < n; ++i) {
            P.x0[3 * i] = a[2 * i] / scale;
            P.x0[3 * i + 1] = a[2 * i + 1] / scale;
            P.x0[3 * i + 2] = 1.0;
            P.x1[3 * i] = b[2 * i] / scale;
            P.x1[3 * i + 1] = b[2 * i + 1] / scale;
            P.x1[3 * i + 2] = 1.0;
        }
        thr[0] /= scale * scale;
        thr[1] /= scale * scale;
        for (int i = 0; i < 9; ++i) P.K0[i] = P.K1[i] = P.K0inv[i] = P.K1inv[i] = (i % 4 == 0) ? 1.0 : 0.0;
    }
    // "three data types" (src/hybrid_pose_estimator.cpp:13-23)
    w[1] *= 2 * thr[0] / thr[1];
    P.sampson_squared_weight = w[1];
    opts->data_type_weights = {w[0], w[0], w[1]};
    opts->squared_inlier_thresholds = {thr[0], thr[0], thr[1]};
    P.thr = opts->squared_inlier_thresholds;
    return P;
}

// ---------------------------------------------------------------------------
// residuals (src/hybrid_pose_estimator.cpp:216-261, ..shared..:160-202, ..two..:213-257)
double evaluate_point(const Problem &P, const Model &m, int t, int i, bool is_for_inlier) {
    const double kMax = std::numeric_limits<double>::max();
    if (!is_for_inlier && P.cfg.score_type == EPI_ONLY && t != 2) return kMax;
    if (!is_for_inlier && P.cfg.score_type == MD_ONLY && t == 2) return kMax;
    const double *xa = &P.x0[3 * i], *xb = &P.x1[3 * i];
    double K0[9], K1[9], K0i[9], K1i[9];
    if (P.variant == CAL) {
        std::copy(P.K0, P.K0 + 9, K0);
        std::copy(P.K1, P.K1 + 9, K1);
        std::copy(P.K0inv, P.K0inv + 9, K0i);
        std::copy(P.K1inv, P.K1inv + 9, K1i);
    } else {
        double f0 = m.focal0, f1 = (P.variant == SF) ? m.focal0 : m.focal1;
        double a[9] = {f0, 0, 0, 0, f0, 0, 0, 0, 1}, b[9] = {f1, 0, 0, 0, f1, 0, 0, 0, 1};
        double ai[9] = {1.0 / f0, 0, 0, 0, 1.0 / f0, 0, 0, 0, 1}, bi[9] = {1.0 / f1, 0, 0, 0, 1.0 / f1, 0, 0, 0, 1};
        std::copy(a, a + 9, K0);
        std::copy(b, b + 9, K1);
        std::copy(ai, ai + 9, K0i);
        std::copy(bi, bi + 9, K1i);
    }
    const double *R = m.R, *tt = m.t;
    if (t == 0) {
        double c[3], p[3], q[3], pr[3];
        mv3(K0i, xa, c);
        for (int k = 0; k < 3; ++k) p[k] = c[k] * (P.d0[i] + m.offset0);
        mv3(R, p, q);
        for (int k = 0; k < 3; ++k) q[k] += tt[k];
        mv3(K1, q, pr);
        double z = pr[2];
        double u = pr[0] / z, v = pr[1] / z;
        if (z < 1e-2 || (P.scale_only && P.d0[i] < 1e-2)) return kMax; // scale-only: :395
        return (u - xb[0]) * (u - xb[0]) + (v - xb[1]) * (v - xb[1]);
    } else if (t == 1) {
        double c[3], p[3], q[3], pr[3];
        mv3(K1i, xb, c);
        for (int k = 0; k < 3; ++k) p[k] = c[k] * (P.d1[i] + m.offset1) * m.scale;
        for (int k = 0; k < 3; ++k)
            q[k] = R[k] * (p[0] - tt[0]) + R[3 + k] * (p[1] - tt[1]) + R[6 + k] * (p[2] - tt[2]);
        mv3(K0, q, pr);
        double z = pr[2];
        double u = pr[0] / z, v = pr[1] / z;
        if (z < 1e-2 || (P.scale_only && P.d1[i] < 1e-2)) return kMax; // scale-only: :408
        return (u - xa[0]) * (u - xa[0]) + (v - xa[1]) * (v - xa[1]);
    }
    // t == 2
    double E[9];
    {
        const double tx[9] = {0, -tt[2], tt[1], tt[2], 0, -tt[0], -tt[1], tt[0], 0};
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) E[3 * r + c] = tx[3 * r] * R[c] + tx[3 * r + 1] * R[3 + c] + tx[3 * r + 2] * R[6 + c];
    }
    double ya[3], yb[3];
    double scale_out = 1.0;
    if (P.variant == CAL) {
        double ca[3], cb[3];
        mv3(K0i, xa, ca);
        mv3(K1i, xb, cb);
        double na = std::sqrt(ca[0] * ca[0] + ca[1] * ca[1] + ca[2] * ca[2]);
        double nb = std::sqrt(cb[0] * cb[0] + cb[1] * cb[1] + cb[2] * cb[2]);
        double ua[3] = {ca[0] / na, ca[1] / na, ca[2] / na}, ub[3] = {cb[0] / nb, cb[1] / nb, cb[2] / nb};
        if (!check_cheirality(R, tt, ua, ub, 1e-2)) return kMax;
        ya[0] = ca[0];
        ya[1] = ca[1];
        yb[0] = cb[0];
        yb[1] = cb[1];
        scale_out = P.sampson_loss_scale;
    } else {
        // F = K1^-T E K0^-1 (diagonal K)
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) E[3 * r + c] *= K1i[4 * r] * K0i[4 * c];
        ya[0] = xa[0];
        ya[1] = xa[1];
        yb[0] = xb[0];
        yb[1] = xb[1];
    }
    // src/utils.h:64-83
    double e0 = E[0] * ya[0] + E[1] * ya[1] + E[2];
    double e1 = E[3] * ya[0] + E[4] * ya[1] + E[5];
    double e2 = E[6] * ya[0] + E[7] * ya[1] + E[8];
    double f0 = E[0] * yb[0] + E[3] * yb[1] + E[6];
    double f1 = E[1] * yb[0] + E[4] * yb[1] + E[7];
    double C = yb[0] * e0 + yb[1] * e1 + e2;
    double r2 = C * C / (e0 * e0 + e1 * e1 + f0 * f0 + f1 * f1);
    return r2 * scale_out;
}

// ---------------------------------------------------------------------------
// minimal solvers (src/hybrid_pose_estimator.cpp:65-187, ..shared..:53-130, ..two..:77-185)
namespace {

void ls_affine(const std::vector<double> &d, const std::vector<double> &z, double *a, double *b) {
    // least squares z ~ a d + b via 2x2 normal equations
    double sdd = 0, sd = 0, sz = 0, sdz = 0, n = (double)d.size();
    for (size_t i = 0; i < d.size(); ++i) {
        sdd += d[i] * d[i];
        sd += d[i];
        sz += z[i];
        sdz += d[i] * z[i];
    }
    double det = sdd * n - sd * sd;
    *a = (n * sdz - sd * sz) / det;
    *b = (sdd * sz - sd * sdz) / det;
}

// shared "triangulate + affine depth fit" tail of the point solvers
bool point_model_tail(const Problem &P, const std::vector<int> &idx, const double *R, const double *t, double fa,
                      double fb, Model *out) {
    const int k = (int)idx.size();
    double P0[12] = {fa, 0, 0, 0, 0, fa, 0, 0, 0, 0, 1, 0};
    double P1[12];
    for (int r = 0; r < 3; ++r) {
        double kr = (r < 2) ? fb : 1.0;
        for (int c = 0; c < 3; ++c) P1[4 * r + c] = kr * R[3 * r + c];
        P1[4 * r + 3] = kr * t[r];
    }
    std::vector<double> X(3 * k), z(k), dd0(k), dd1(k);
    for (int j = 0; j < k; ++j) {
        int i = idx[j];
        double p0[2], p1[2];
        if (P.variant == CAL) {
            double c0[3], c1[3];
            mv3(P.K0inv, &P.x0[3 * i], c0);
            mv3(P.K1inv, &P.x1[3 * i], c1);
            p0[0] = c0[0];
            p0[1] = c0[1];
            p1[0] = c1[0];
            p1[1] = c1[1];
        } else {
            p0[0] = P.x0[3 * i];
            p0[1] = P.x0[3 * i + 1];
            p1[0] = P.x1[3 * i];
            p1[1] = P.x1[3 * i + 1];
        }
        triangulate_point_qr(P0, P1, p0, p1, &X[3 * j]);
        dd0[j] = P.d0[i];
        dd1[j] = P.d1[i];
    }
    Model m = *out;
    for (int a = 0; a < 9; ++a) m.R[a] = R[a];
    double tt[3] = {t[0], t[1], t[2]};
    if (!P.cfg.use_shift || P.scale_only) { // scale-only tail: :340-354
        double num = 0, den = 0;
        for (int j = 0; j < k; ++j) {
            num += dd0[j] * X[3 * j + 2];
            den += dd0[j] * dd0[j];
        }
        double s0 = num / den;
        for (int c = 0; c < 3; ++c) tt[c] /= s0;
        num = den = 0;
        for (int j = 0; j < k; ++j) {
            double q[3] = {X[3 * j] / s0, X[3 * j + 1] / s0, X[3 * j + 2] / s0}, o[3];
            mv3(R, q, o);
            double zz = o[2] + tt[2];
            num += dd1[j] * zz;
            den += dd1[j] * dd1[j];
        }
        m.scale = num / den;
        m.offset0 = m.offset1 = 0.0;
    } else {
        for (int j = 0; j < k; ++j) z[j] = X[3 * j + 2];
        double s0, b0;
        ls_affine(dd0, z, &s0, &b0);
        double offset0 = b0 / s0;
        if (P.cfg.min_depth_constraint && offset0 < -P.min_depth[0]) return false;
        for (int c = 0; c < 3; ++c) tt[c] /= s0;
        for (int j = 0; j < k; ++j) {
            double q[3] = {X[3 * j] / s0, X[3 * j + 1] / s0, X[3 * j + 2] / s0}, o[3];
            mv3(R, q, o);
            z[j] = o[2] + tt[2];
        }
        double sc, b1;
        ls_affine(dd1, z, &sc, &b1);
        double offset1 = b1 / sc;
        if (P.cfg.min_depth_constraint && offset1 < -P.min_depth[1]) return false;
        m.scale = sc;
        m.offset0 = offset0;
        m.offset1 = offset1;
    }
    for (int c = 0; c < 3; ++c) m.t[c] = tt[c];
    *out = m;
    return true;
}

} // namespace

int minimal_solver(const Problem &P, const std::vector<std::vector<int>> &sample, int solver_idx,
                   std::vector<Model> *models) {
    models->clear();
    if (solver_idx == 0) {
        const std::vector<int> &idx = sample[0];
        const int k = (int)idx.size();
        double x[12], y[12], dx[4], dy[4];
        for (int j = 0; j < k; ++j) {
            int i = idx[j];
            if (P.variant == CAL) {
                mv3(P.K0inv, &P.x0[3 * i], &x[3 * j]);
                mv3(P.K1inv, &P.x1[3 * i], &y[3 * j]);
            } else {
                for (int c = 0; c < 3; ++c) {
                    x[3 * j + c] = P.x0[3 * i + c];
                    y[3 * j + c] = P.x1[3 * i + c];
                }
            }
            dx[j] = P.d0[i];
            dy[j] = P.d1[i];
        }
        if (P.scale_only) {
            // src/hybrid_pose_estimator.cpp:319-327: Procrustes of the (unlifted)
            // calibrated points, scale moved onto the second camera
            const double W[3] = {1.0, 1.0, 1.0};
            Model m = estimate_scale_and_pose(x, y, W, 3);
            m.scale = 1.0 / m.scale;
            models->push_back(m);
            return 1;
        }
        if (P.variant == CAL && !P.cfg.use_shift) {
            models->push_back(md_pose_noshift_cal(x, y, dx, dy));
            return (int)models->size();
        }
        std::vector<Model> sols;
        if (P.variant == CAL && P.use_ours)
            sols = md_pose_cal_ours(x, y, dx, dy);
        else if (P.variant == SF && P.use_ours)
            sols = md_pose_sf_ours(x, y, dx, dy);
        else if (P.variant == TF && P.use_ours)
            sols = md_pose_tf_ours(x, y, dx, dy);
        else if (P.variant == TF && P.use_4p4d)
            sols = md_pose_tf_4p4d(x, y, dx, dy);
        else
            sols = md_pose(P.variant, x, y, dx, dy);
        for (Model m : sols) {
            // src/hybrid_pose_estimator.cpp:80-85
            if (!P.cfg.min_depth_constraint ||
                (m.offset0 > -P.min_depth[0] && m.offset1 > -P.min_depth[1] * m.scale)) {
                m.offset1 /= m.scale;
                models->push_back(m);
            }
        }
        return (int)models->size();
    }
    // point solvers
    const std::vector<int> &idx = sample[2];
    const int k = (int)idx.size();
    std::vector<double> b0(3 * k), b1(3 * k);
    for (int j = 0; j < k; ++j) {
        int i = idx[j];
        double c0[3], c1[3];
        if (P.variant == CAL) {
            mv3(P.K0inv, &P.x0[3 * i], c0);
            mv3(P.K1inv, &P.x1[3 * i], c1);
        } else {
            for (int c = 0; c < 3; ++c) {
                c0[c] = P.x0[3 * i + c];
                c1[c] = P.x1[3 * i + c];
            }
        }
        double n0 = std::sqrt(c0[0] * c0[0] + c0[1] * c0[1] + c0[2] * c0[2]);
        double n1 = std::sqrt(c1[0] * c1[0] + c1[1] * c1[1] + c1[2] * c1[2]);
        for (int c = 0; c < 3; ++c) {
            b0[3 * j + c] = c0[c] / n0;
            b1[3 * j + c] = c1[c] / n1;
        }
    }
    if (P.variant == CAL) {
        for (const Model &pose : relpose_5pt(b0.data(), b1.data())) {
            Model m;
            if (point_model_tail(P, idx, pose.R, pose.t, 1.0, 1.0, &m)) models->push_back(m);
        }
    }
    std::vector<double> p0(2 * k), p1(2 * k);
    for (int j = 0; j < k; ++j) {
        p0[2 * j] = P.x0[3 * idx[j]];
        p0[2 * j + 1] = P.x0[3 * idx[j] + 1];
        p1[2 * j] = P.x1[3 * idx[j]];
        p1[2 * j + 1] = P.x1[3 * idx[j] + 1];
    }
    if (P.variant == SF) {
        // src/hybrid_pose_shared_focal_estimator.cpp:74-128
        for (const Model &ip : relpose_6pt_shared_focal(b0.data(), b1.data())) {
            Model m;
            m.focal0 = m.focal1 = ip.focal0;
            if (point_model_tail(P, idx, ip.R, ip.t, ip.focal0, ip.focal0, &m)) models->push_back(m);
        }
    } else if (P.variant == TF) {
        // src/hybrid_pose_two_focal_estimator.cpp:103-182
        for (const auto &F : relpose_7pt(b0.data(), b1.data())) {
            double f0, f1;
            bougnoux_focals(F.data(), &f0, &f1);
            f0 = std::sqrt(std::fabs(f0));
            f1 = std::sqrt(std::fabs(f1));
            double E[9];
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 3; ++c) E[3 * r + c] = (r < 2 ? f1 : 1.0) * F[3 * r + c] * (c < 2 ? f0 : 1.0);
            double R[9], t[3];
            recover_pose(E, p0.data(), p1.data(), k, 1e9, R, t);
            Model m;
            m.focal0 = f0;
            m.focal1 = f1;
            if (point_model_tail(P, idx, R, t, f0, f1, &m)) models->push_back(m);
        }
    }
    return (int)models->size();
}

// ---------------------------------------------------------------------------
// LM (Ceres stand-in)
namespace {

enum Slot { QW = 0, QX, QY, QZ, TX, TY, TZ, SC, O0, O1, F0, F1 };

template <class T> void quat_to_R(const T q[4], T R[9]) {
    using std::sqrt;
    T n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    T w = q[0] / n, x = q[1] / n, y = q[2] / n, z = q[3] / n;
    R[0] = T(1.0) - T(2.0) * (y * y + z * z);
    R[1] = T(2.0) * (x * y - w * z);
    R[2] = T(2.0) * (x * z + w * y);
    R[3] = T(2.0) * (x * y + w * z);
    R[4] = T(1.0) - T(2.0) * (x * x + z * z);
    R[5] = T(2.0) * (y * z - w * x);
    R[6] = T(2.0) * (x * z - w * y);
    R[7] = T(2.0) * (y * z + w * x);
    R[8] = T(1.0) - T(2.0) * (x * x + y * y);
}

void R_to_quat(const double R[9], double q[4]) {
    // Eigen::Quaternion(const Matrix3&) algorithm (Shepperd)
    double tr = R[0] + R[4] + R[8];
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
        if (R[8] > R[3 * i + i]) i = 2;
        int j = (i + 1) % 3, k = (j + 1) % 3;
        double s = std::sqrt(R[3 * i + i] - R[3 * j + j] - R[3 * k + k] + 1.0);
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

struct LMProblem {
    const Problem *P;
    const std::vector<int> *i0, *i1, *i2;
    bool use_reproj, use_sampson, use_shift, min_depth_constraint;
    double w_sampson;
    bool has_o0, has_s_o1, has_focal;
};

// residual blocks evaluated with T = Jet (derivatives) or double
template <class T> void residuals(const LMProblem &L, const T *x, std::vector<T> *res) {
    using std::sqrt;
    const Problem &P = *L.P;
    res->clear();
    T R[9];
    quat_to_R(x + QW, R);
    const T *t = x + TX;
    T f0 = T(1.0), f1 = T(1.0);
    if (P.variant == SF) {
        f0 = x[F0];
        f1 = x[F0];
    } else if (P.variant == TF) {
        f0 = x[F0];
        f1 = x[F1];
    }
    if (L.use_reproj) {
        for (int i : *L.i0) {
            // LiftProjection*Functor0 (src/cost_functions.h:16-49, 193-227, 303-337)
            T c[3];
            if (P.variant == CAL) {
                double cc[3];
                mv3(P.K0inv, &P.x0[3 * i], cc);
                c[0] = T(cc[0]);
                c[1] = T(cc[1]);
                c[2] = T(cc[2]);
            } else {
                c[0] = T(P.x0[3 * i]) / f0;
                c[1] = T(P.x0[3 * i + 1]) / f0;
                c[2] = T(1.0);
            }
            T dep = T(P.d0[i]) + x[O0];
            T p[3] = {c[0] * dep, c[1] * dep, c[2] * dep};
            T q[3];
            for (int r = 0; r < 3; ++r) q[r] = R[3 * r] * p[0] + R[3 * r + 1] * p[1] + R[3 * r + 2] * p[2] + t[r];
            T h[3];
            if (P.variant == CAL) {
                for (int r = 0; r < 3; ++r) h[r] = T(P.K1[3 * r]) * q[0] + T(P.K1[3 * r + 1]) * q[1] + T(P.K1[3 * r + 2]) * q[2];
            } else {
                h[0] = f1 * q[0];
                h[1] = f1 * q[1];
                h[2] = q[2];
            }
            res->push_back(h[0] / h[2] - T(P.x1[3 * i]));
            res->push_back(h[1] / h[2] - T(P.x1[3 * i + 1]));
        }
        for (int i : *L.i1) {
            // LiftProjection*Functor1 (src/cost_functions.h:51-90, 229-268, 339-379)
            T c[3];
            if (P.variant == CAL) {
                double cc[3];
                mv3(P.K1inv, &P.x1[3 * i], cc);
                c[0] = T(cc[0]);
                c[1] = T(cc[1]);
                c[2] = T(cc[2]);
            } else {
                c[0] = T(P.x1[3 * i]) / f1;
                c[1] = T(P.x1[3 * i + 1]) / f1;
                c[2] = T(1.0);
            }
            T dep = (T(P.d1[i]) + x[O1]) * x[SC];
            T p[3] = {c[0] * dep - t[0], c[1] * dep - t[1], c[2] * dep - t[2]};
            T q[3];
            for (int r = 0; r < 3; ++r) q[r] = R[r] * p[0] + R[3 + r] * p[1] + R[6 + r] * p[2];
            T h[3];
            if (P.variant == CAL) {
                for (int r = 0; r < 3; ++r) h[r] = T(P.K0[3 * r]) * q[0] + T(P.K0[3 * r + 1]) * q[1] + T(P.K0[3 * r + 2]) * q[2];
            } else {
                h[0] = f0 * q[0];
                h[1] = f0 * q[1];
                h[2] = q[2];
            }
            res->push_back(h[0] / h[2] - T(P.x0[3 * i]));
            res->push_back(h[1] / h[2] - T(P.x0[3 * i + 1]));
        }
    }
    if (L.use_sampson) {
        // SampsonError*Functor (src/cost_functions.h:92-141, 270-301, 381-387)
        T E[9];
        const T tx[9] = {T(0.0), -t[2], t[1], t[2], T(0.0), -t[0], -t[1], t[0], T(0.0)};
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) E[3 * r + c] = tx[3 * r] * R[c] + tx[3 * r + 1] * R[3 + c] + tx[3 * r + 2] * R[6 + c];
        if (P.variant != CAL) {
            T i0 = T(1.0) / f0, i1 = T(1.0) / f1;
            T s0[3] = {i0, i0, T(1.0)}, s1[3] = {i1, i1, T(1.0)};
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 3; ++c) E[3 * r + c] = E[3 * r + c] * s1[r] * s0[c];
        }
        for (int i : *L.i2) {
            double a[3], b[3];
            if (P.variant == CAL) {
                mv3(P.K0inv, &P.x0[3 * i], a);
                mv3(P.K1inv, &P.x1[3 * i], b);
            } else {
                for (int c = 0; c < 3; ++c) {
                    a[c] = P.x0[3 * i + c];
                    b[c] = P.x1[3 * i + c];
                }
            }
            T e0 = E[0] * T(a[0]) + E[1] * T(a[1]) + E[2];
            T e1 = E[3] * T(a[0]) + E[4] * T(a[1]) + E[5];
            T e2 = E[6] * T(a[0]) + E[7] * T(a[1]) + E[8];
            T g0 = E[0] * T(b[0]) + E[3] * T(b[1]) + E[6];
            T g1 = E[1] * T(b[0]) + E[4] * T(b[1]) + E[7];
            T C = T(b[0]) * e0 + T(b[1]) * e1 + e2;
            T nrm = sqrt(e0 * e0 + e1 * e1 + g0 * g0 + g1 * g1);
            res->push_back(C / nrm * T(L.w_sampson));
        }
    }
}

bool cholesky_solve(std::vector<double> A, int n, std::vector<double> b, std::vector<double> *x) {
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
    *x = b;
    return true;
}

struct Bounds {
    bool has_lo[12] = {false};
    double lo[12] = {0};
};

// tangent coordinates: list of (kind, ambient slot): kind 0 = quaternion (3 cols), 1 = scalar/t
struct Tangent {
    std::vector<int> slots; // ambient slot for each scalar tangent column; QW marks the 3 rotation columns
    int dim = 0;
};

void evaluate(const LMProblem &L, const double *x, const Tangent &T, std::vector<double> *r, std::vector<double> *J,
              int *nres) {
    Jet xj[kJetN];
    for (int k = 0; k < kJetN; ++k) xj[k] = Jet::var(x[k], k);
    std::vector<Jet> res;
    residuals<Jet>(L, xj, &res);
    const int m = (int)res.size();
    *nres = m;
    r->resize(m);
    J->assign((size_t)m * T.dim, 0.0);
    // QuaternionManifold::PlusJacobian at x
    const double *q = x + QW;
    const double PJ[4][3] = {{-q[1], -q[2], -q[3]}, {q[0], q[3], -q[2]}, {-q[3], q[0], q[1]}, {q[2], -q[1], q[0]}};
    for (int i = 0; i < m; ++i) {
        (*r)[i] = res[i].a;
        int col = 0;
        for (size_t s = 0; s < T.slots.size(); ++s) {
            int sl = T.slots[s];
            if (sl == QW) {
                for (int c = 0; c < 3; ++c) {
                    double v = 0;
                    for (int a = 0; a < 4; ++a) v += res[i].v[QW + a] * PJ[a][c];
                    (*J)[(size_t)i * T.dim + col + c] = v;
                }
                col += 3;
            } else {
                (*J)[(size_t)i * T.dim + col] = res[i].v[sl];
                col += 1;
            }
        }
    }
}

double cost_at(const LMProblem &L, const double *x) {
    std::vector<double> res;
    residuals<double>(L, x, &res);
    double c = 0;
    for (double v : res) c += v * v;
    return 0.5 * c;
}

void plus(const double *x, const Tangent &T, const std::vector<double> &d, const Bounds &B, double *out) {
    for (int k = 0; k < kJetN; ++k) out[k] = x[k];
    int col = 0;
    for (int sl : T.slots) {
        if (sl == QW) {
            double dv[3] = {d[col], d[col + 1], d[col + 2]};
            double nd = std::sqrt(dv[0] * dv[0] + dv[1] * dv[1] + dv[2] * dv[2]);
            if (nd > 0) {
                double s = std::sin(nd) / nd;
                double qd[4] = {std::cos(nd), s * dv[0], s * dv[1], s * dv[2]};
                const double *q = x + QW;
                out[QW] = qd[0] * q[0] - qd[1] * q[1] - qd[2] * q[2] - qd[3] * q[3];
                out[QX] = qd[0] * q[1] + qd[1] * q[0] + qd[2] * q[3] - qd[3] * q[2];
                out[QY] = qd[0] * q[2] - qd[1] * q[3] + qd[2] * q[0] + qd[3] * q[1];
                out[QZ] = qd[0] * q[3] + qd[1] * q[2] - qd[2] * q[1] + qd[3] * q[0];
            }
            col += 3;
        } else {
            out[sl] = x[sl] + d[col];
            if (B.has_lo[sl] && out[sl] < B.lo[sl]) out[sl] = B.lo[sl];
            col += 1;
        }
    }
}

// returns false when there are no residuals (Solve() returning false)
bool run_lm(const LMProblem &L, const EstConfig &cfg, Model *m) {
    const Problem &P = *L.P;
    double x[kJetN] = {0};
    R_to_quat(m->R, x + QW);
    for (int c = 0; c < 3; ++c) x[TX + c] = m->t[c];
    x[SC] = m->scale;
    x[O0] = m->offset0;
    x[O1] = m->offset1;
    x[F0] = m->focal0;
    x[F1] = m->focal1;

    int nres_total = 0;
    if (L.use_reproj) nres_total += (int)(L.i0->size() + L.i1->size());
    if (L.use_sampson) nres_total += (int)L.i2->size();
    if (nres_total == 0) return false;

    Tangent T;
    Bounds B;
    T.slots.push_back(QW);
    T.slots.push_back(TX);
    T.slots.push_back(TY);
    T.slots.push_back(TZ);
    T.dim = 6;
    const bool has_o0 = L.use_reproj && !L.i0->empty();
    const bool has_s_o1 = L.use_reproj && !L.i1->empty();
    if (has_s_o1) {
        T.slots.push_back(SC);
        T.dim++;
        B.has_lo[SC] = true;
        B.lo[SC] = 1e-2;
    }
    if (has_o0 && L.use_shift) {
        T.slots.push_back(O0);
        T.dim++;
    }
    if (has_s_o1 && L.use_shift) {
        T.slots.push_back(O1);
        T.dim++;
    }
    if (L.min_depth_constraint) {
        B.has_lo[O0] = true;
        B.lo[O0] = -P.min_depth[0] + 1e-2;
        B.has_lo[O1] = true;
        B.lo[O1] = -P.min_depth[1] + 1e-2;
    }
    if (P.variant == SF) {
        T.slots.push_back(F0);
        T.dim++;
    } else if (P.variant == TF) {
        T.slots.push_back(F0);
        T.slots.push_back(F1);
        T.dim += 2;
        B.has_lo[F0] = B.has_lo[F1] = true;
        B.lo[F0] = B.lo[F1] = 1e-6;
    }
    // Ceres Program::IsFeasible: constant blocks must start inside their bounds,
    // otherwise Solve() fails and the parameters are left untouched.
    if (!L.use_shift && L.min_depth_constraint) {
        if (has_o0 && x[O0] < B.lo[O0]) return true;
        if (has_s_o1 && x[O1] < B.lo[O1]) return true;
    }
    const int n = T.dim;
    const int max_iter = (int)cfg.ceres_max_num_iterations;
    const double ftol = cfg.ceres_function_tolerance, gtol = cfg.ceres_gradient_tolerance,
                 ptol = cfg.ceres_parameter_tolerance;

    std::vector<double> r, J;
    int m_res = 0;
    evaluate(L, x, T, &r, &J, &m_res);
    double cost = 0;
    for (double v : r) cost += v * v;
    cost *= 0.5;
    auto gradient = [&](std::vector<double> *g) {
        g->assign(n, 0.0);
        for (int i = 0; i < m_res; ++i)
            for (int j = 0; j < n; ++j) (*g)[j] += J[(size_t)i * n + j] * r[i];
    };
    std::vector<double> g;
    gradient(&g);
    auto gmax = [&]() {
        double v = 0;
        for (double e : g) v = std::max(v, std::fabs(e));
        return v;
    };
    double radius = 1e4, decrease = 2.0;
    // Ceres TrustRegionStepEvaluator (use_nonmonotonic_steps, at most 5 consecutive
    // non-monotonic steps; 0 when off) and TrustRegionMinimizer's rule that the user's
    // parameters are written only on a new minimum cost
    const int max_nonmono = cfg.ceres_use_nonmonotonic_steps ? 5 : 0;
    double ref_cost = cost, min_cost = cost, cand_ref = cost, acc_ref = 0.0, acc_cand = 0.0;
    int n_nonmono = 0;
    double best[kJetN];
    for (int k = 0; k < kJetN; ++k) best[k] = x[k];
    if (gmax() <= gtol) goto done;
    for (int iter = 0; iter < max_iter; ++iter) {
        // Jacobi scaling + LM step
        std::vector<double> sc(n), H((size_t)n * n, 0.0), rhs(n, 0.0), y;
        for (int j = 0; j < n; ++j) {
            double s = 0;
            for (int i = 0; i < m_res; ++i) s += J[(size_t)i * n + j] * J[(size_t)i * n + j];
            sc[j] = 1.0 / (1.0 + std::sqrt(s));
        }
        for (int i = 0; i < m_res; ++i)
            for (int a = 0; a < n; ++a) {
                double ja = J[(size_t)i * n + a] * sc[a];
                rhs[a] -= ja * r[i];
                for (int b = 0; b < n; ++b) H[a * n + b] += ja * J[(size_t)i * n + b] * sc[b];
            }
        for (int j = 0; j < n; ++j) {
            double dgl = std::min(std::max(H[j * n + j], 1e-6), 1e32);
            H[j * n + j] += dgl / radius;
        }
        if (!cholesky_solve(H, n, rhs, &y)) {
            radius /= decrease;
            decrease *= 2.0;
            if (radius < 1e-32) break;
            continue;
        }
        std::vector<double> d(n);
        for (int j = 0; j < n; ++j) d[j] = y[j] * sc[j];
        double cand[kJetN];
        plus(x, T, d, B, cand);
        double step_norm = 0, xnorm = 0;
        for (int k = 0; k < kJetN; ++k) {
            step_norm += (cand[k] - x[k]) * (cand[k] - x[k]);
            xnorm += x[k] * x[k];
        }
        step_norm = std::sqrt(step_norm);
        xnorm = std::sqrt(xnorm);
        double cand_cost = cost_at(L, cand);
        if (step_norm <= ptol * (xnorm + ptol)) break;
        if (std::fabs(cost - cand_cost) <= ftol * cost) break;
        // linearised model decrease
        double gd = 0, jd2 = 0;
        for (int j = 0; j < n; ++j) gd += g[j] * d[j];
        for (int i = 0; i < m_res; ++i) {
            double s = 0;
            for (int j = 0; j < n; ++j) s += J[(size_t)i * n + j] * d[j];
            jd2 += s * s;
        }
        double mcc = -(gd + 0.5 * jd2);
        double rho = -1.0;
        if (mcc > 0 && std::isfinite(cand_cost)) {
            const double relative = (cost - cand_cost) / mcc;
            const double historical = (ref_cost - cand_cost) / (acc_ref + mcc);
            rho = std::max(relative, historical);
        }
        if (rho > 1e-3) {
            for (int k = 0; k < kJetN; ++k) x[k] = cand[k];
            evaluate(L, x, T, &r, &J, &m_res);
            cost = cand_cost;
            gradient(&g);
            acc_cand += mcc;
            acc_ref += mcc;
            if (cost < min_cost) {
                min_cost = cost;
                n_nonmono = 0;
                cand_ref = cost;
                acc_cand = 0.0;
                for (int k = 0; k < kJetN; ++k) best[k] = x[k];
            } else {
                ++n_nonmono;
                if (cost > cand_ref) {
                    cand_ref = cost;
                    acc_cand = 0.0;
                }
            }
            if (n_nonmono == max_nonmono) {
                ref_cost = cand_ref;
                acc_ref = acc_cand;
            }
            radius = std::min(1e16, radius / std::max(1.0 / 3.0, 1.0 - std::pow(2.0 * rho - 1.0, 3)));
            decrease = 2.0;
            if (gmax() <= gtol) break;
        } else {
            radius /= decrease;
            decrease *= 2.0;
            if (radius < 1e-32) break;
        }
    }
done:
    double qn[4] = {best[QW], best[QX], best[QY], best[QZ]};
    quat_to_R<double>(qn, m->R);
    for (int c = 0; c < 3; ++c) m->t[c] = best[TX + c];
    m->scale = best[SC];
    m->offset0 = best[O0];
    m->offset1 = best[O1];
    m->focal0 = best[F0];
    m->focal1 = best[F1];
    if (P.variant == SF) m->focal1 = best[F0];
    return true;
}

bool lm_call(const Problem &P, const std::vector<std::vector<int>> &sample, Model *m, bool use_shift) {
    LMProblem L;
    L.P = &P;
    L.i0 = &sample[0];
    L.i1 = &sample[1];
    L.i2 = &sample[2];
    L.use_reproj = P.cfg.lo_type != EPI_ONLY;
    L.use_sampson = P.cfg.lo_type != MD_ONLY;
    // HybridPoseOptimizerScaleOnly: offsets constant and unbounded (src/optimizer.h:202-209)
    L.use_shift = use_shift && !P.scale_only;
    L.min_depth_constraint = P.cfg.min_depth_constraint && !P.scale_only;
    if (P.variant == CAL)
        L.w_sampson = std::sqrt(P.sampson_squared_weight) / (1.0 / (P.K0[0] + P.K0[4]) + 1.0 / (P.K1[0] + P.K1[4]));
    else
        L.w_sampson = std::sqrt(P.sampson_squared_weight);
    return run_lm(L, P.cfg, m);
}

bool too_small(const Problem &P, const std::vector<std::vector<int>> &s) {
    int kmd = (P.variant == CAL) ? 3 : 4;
    int kpt = (P.variant == CAL) ? 5 : (P.variant == SF ? 6 : 7);
    return ((int)s[0].size() < kmd && (int)s[1].size() < kmd) || (int)s[2].size() < kpt;
}

} // namespace

bool non_minimal_solver(const Problem &P, const std::vector<std::vector<int>> &sample, int, Model *m) {
    if (too_small(P, sample)) return false;
    // NonMinimalSolver passes est_config.use_shift (cal :203, sf :146); tf leaves the default (true)
    bool use_shift = (P.variant == TF) ? true : P.cfg.use_shift;
    return lm_call(P, sample, m, use_shift);
}

Model estimate_scale_and_pose(const double *X, const double *Y, const double *W, int k) {
    double wsum = 0.0, cX[3] = {0, 0, 0}, cY[3] = {0, 0, 0};
    for (int i = 0; i < k; ++i) {
        wsum += W[i];
        for (int c = 0; c < 3; ++c) {
            cX[c] += X[3 * i + c] * W[i];
            cY[c] += Y[3 * i + c] * W[i];
        }
    }
    for (int c = 0; c < 3; ++c) {
        cX[c] /= wsum;
        cY[c] /= wsum;
    }
    Mat S(3, 3);
    for (int i = 0; i < k; ++i)
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) S(a, b) += (Y[3 * i + a] - cY[a]) * W[i] * (X[3 * i + b] - cX[b]);
    Mat U, V;
    std::vector<double> sv;
    jacobi_svd(S, &U, &sv, &V);
    double Um[9], Vm[9];
    for (int a = 0; a < 9; ++a) {
        Um[a] = U(a / 3, a % 3);
        Vm[a] = V(a / 3, a % 3);
    }
    if (det3(Um) * det3(Vm) < 0)
        for (int r = 0; r < 3; ++r) Um[3 * r + 2] = -Um[3 * r + 2];
    Model m;
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) m.R[3 * r + c] = Um[3 * r] * Vm[3 * c] + Um[3 * r + 1] * Vm[3 * c + 1] + Um[3 * r + 2] * Vm[3 * c + 2];
    double num = 0.0, den = 0.0;
    for (int i = 0; i < k; ++i) {
        double xc[3], rx[3];
        for (int c = 0; c < 3; ++c) xc[c] = X[3 * i + c] - cX[c];
        mv3(m.R, xc, rx);
        for (int c = 0; c < 3; ++c) {
            num += (Y[3 * i + c] - cY[c]) * rx[c];
            den += rx[c] * rx[c];
        }
    }
    m.scale = num / den;
    double rc[3];
    mv3(m.R, cX, rc);
    for (int c = 0; c < 3; ++c) m.t[c] = cY[c] - m.scale * rc[c];
    m.offset0 = m.offset1 = 0.0;
    return m;
}

void least_squares(const Problem &P, const std::vector<std::vector<int>> &sample, int, Model *m) {
    if (too_small(P, sample)) return;
    // LeastSquares passes use_shift only in the calibrated estimator (:281)
    bool use_shift = (P.variant == CAL) ? P.cfg.use_shift : true;
    lm_call(P, sample, m, use_shift);
}

} // namespace oracle
