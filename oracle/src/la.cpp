// ORACLE -- test infrastructure only.  See la.h.
#include "la.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <limits>

namespace oracle {

bool qr_solve(const Mat &A0, const Mat &B0, Mat *X) {
    const int n = A0.r, m = B0.c;
    Mat A = A0, B = B0;
    std::vector<int> perm(n);
    std::vector<double> cn(n);
    for (int j = 0; j < n; ++j) {
        perm[j] = j;
        double s = 0;
        for (int i = 0; i < n; ++i) s += A(i, j) * A(i, j);
        cn[j] = s;
    }
    double maxpiv = 0;
    for (int k = 0; k < n; ++k) {
        // column pivot: largest remaining column norm (recomputed for accuracy)
        int p = k;
        double best = -1;
        for (int j = k; j < n; ++j) {
            double s = 0;
            for (int i = k; i < n; ++i) s += A(i, j) * A(i, j);
            cn[j] = s;
            if (s > best) {
                best = s;
                p = j;
            }
        }
        if (p != k) {
            for (int i = 0; i < n; ++i) std::swap(A(i, k), A(i, p));
            std::swap(perm[k], perm[p]);
        }
        double alpha = std::sqrt(best);
        if (k == 0) maxpiv = alpha;
        if (alpha <= maxpiv * 1e-15 || alpha == 0.0) return false;
        if (A(k, k) > 0) alpha = -alpha;
        // v = x - alpha e1
        std::vector<double> v(n - k);
        for (int i = k; i < n; ++i) v[i - k] = A(i, k);
        v[0] -= alpha;
        double vn = 0;
        for (double e : v) vn += e * e;
        if (vn > 0) {
            for (int j = k; j < n; ++j) {
                double d = 0;
                for (int i = k; i < n; ++i) d += v[i - k] * A(i, j);
                d = 2 * d / vn;
                for (int i = k; i < n; ++i) A(i, j) -= d * v[i - k];
            }
            for (int j = 0; j < m; ++j) {
                double d = 0;
                for (int i = k; i < n; ++i) d += v[i - k] * B(i, j);
                d = 2 * d / vn;
                for (int i = k; i < n; ++i) B(i, j) -= d * v[i - k];
            }
        }
    }
    // back substitution R z = Q^T B, then X = P z
    Mat Z(n, m);
    for (int j = 0; j < m; ++j)
        for (int i = n - 1; i >= 0; --i) {
            double s = B(i, j);
            for (int k = i + 1; k < n; ++k) s -= A(i, k) * Z(k, j);
            Z(i, j) = s / A(i, i);
        }
    *X = Mat(n, m);
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < m; ++j) (*X)(perm[i], j) = Z(i, j);
    return true;
}

static void lu_full(Mat &A, std::vector<int> &rp, std::vector<int> &cp) {
    const int n = A.r;
    rp.resize(n);
    cp.resize(n);
    for (int i = 0; i < n; ++i) rp[i] = cp[i] = i;
    for (int k = 0; k < n; ++k) {
        int pi = k, pj = k;
        double best = -1;
        for (int i = k; i < n; ++i)
            for (int j = k; j < n; ++j)
                if (std::fabs(A(i, j)) > best) {
                    best = std::fabs(A(i, j));
                    pi = i;
                    pj = j;
                }
        if (pi != k) {
            for (int j = 0; j < n; ++j) std::swap(A(k, j), A(pi, j));
            std::swap(rp[k], rp[pi]);
        }
        if (pj != k) {
            for (int i = 0; i < n; ++i) std::swap(A(i, k), A(i, pj));
            std::swap(cp[k], cp[pj]);
        }
        if (A(k, k) == 0.0) continue;
        for (int i = k + 1; i < n; ++i) {
            double l = A(i, k) / A(k, k);
            A(i, k) = l;
            for (int j = k + 1; j < n; ++j) A(i, j) -= l * A(k, j);
        }
    }
}

void lu_full_steps(Mat &A, std::vector<int> &rp, std::vector<int> &cp, int steps) {
    const int n = A.r, m = A.c;
    rp.resize(n);
    cp.resize(m);
    for (int i = 0; i < n; ++i) rp[i] = i;
    for (int j = 0; j < m; ++j) cp[j] = j;
    for (int k = 0; k < steps; ++k) {
        int pi = k, pj = k;
        double best = -1;
        for (int i = k; i < n; ++i)
            for (int j = k; j < m; ++j)
                if (std::fabs(A(i, j)) > best) {
                    best = std::fabs(A(i, j));
                    pi = i;
                    pj = j;
                }
        if (pi != k) {
            for (int j = 0; j < m; ++j) std::swap(A(k, j), A(pi, j));
            std::swap(rp[k], rp[pi]);
        }
        if (pj != k) {
            for (int i = 0; i < n; ++i) std::swap(A(i, k), A(i, pj));
            std::swap(cp[k], cp[pj]);
        }
        if (A(k, k) == 0.0) continue;
        for (int i = k + 1; i < n; ++i) {
            double l = A(i, k) / A(k, k);
            A(i, k) = l;
            for (int j = k + 1; j < m; ++j) A(i, j) -= l * A(k, j);
        }
    }
}

Mat right_null_rank(const Mat &A0, int rank) {
    const int m = A0.c;
    Mat A = A0;
    std::vector<int> rp, cp;
    lu_full_steps(A, rp, cp, rank);
    Mat Z(m, m - rank);
    for (int f = 0; f < m - rank; ++f) {
        std::vector<double> y(m, 0.0);
        y[rank + f] = 1.0;
        for (int i = rank - 1; i >= 0; --i) {
            double s = 0.0;
            for (int k = i + 1; k < m; ++k) s -= A(i, k) * y[k];
            y[i] = (A(i, i) != 0.0) ? s / A(i, i) : 0.0;
        }
        for (int i = 0; i < m; ++i) Z(cp[i], f) = y[i];
    }
    return Z;
}

std::vector<double> particular_solution(const Mat &A0, const std::vector<double> &b, int rank) {
    const int n = A0.r, m = A0.c;
    Mat A = A0;
    std::vector<int> rp, cp;
    lu_full_steps(A, rp, cp, rank);
    std::vector<double> y(n);
    for (int i = 0; i < n; ++i) {
        double s = b[rp[i]];
        for (int k = 0; k < std::min(i, rank); ++k) s -= A(i, k) * y[k];
        y[i] = s;
    }
    std::vector<double> z(m, 0.0);
    for (int i = rank - 1; i >= 0; --i) {
        double s = y[i];
        for (int k = i + 1; k < rank; ++k) s -= A(i, k) * z[k];
        z[i] = (A(i, i) != 0.0) ? s / A(i, i) : 0.0;
    }
    std::vector<double> x(m, 0.0);
    for (int i = 0; i < m; ++i) x[cp[i]] = z[i];
    return x;
}

void householder_deflate(Mat &C, Mat Z) {
    const int n = Z.r, kz = Z.c;
    for (int k = 0; k < kz; ++k) {
        double nx = 0.0;
        for (int i = k; i < n; ++i) nx += Z(i, k) * Z(i, k);
        double alpha = std::sqrt(nx);
        if (alpha == 0.0) continue;
        if (Z(k, k) > 0) alpha = -alpha;
        std::vector<double> v(n - k);
        for (int i = k; i < n; ++i) v[i - k] = Z(i, k);
        v[0] -= alpha;
        double vn = 0.0;
        for (double e : v) vn += e * e;
        if (!(vn > 0.0)) continue;
        // the rest of Z
        for (int j = k; j < kz; ++j) {
            double d = 0.0;
            for (int i = k; i < n; ++i) d += v[i - k] * Z(i, j);
            d = 2.0 * d / vn;
            for (int i = k; i < n; ++i) Z(i, j) -= d * v[i - k];
        }
        // C <- H C (rows k..n-1), then C <- C H (columns k..n-1)
        for (int j = 0; j < C.c; ++j) {
            double d = 0.0;
            for (int i = k; i < n; ++i) d += v[i - k] * C(i, j);
            d = 2.0 * d / vn;
            for (int i = k; i < n; ++i) C(i, j) -= d * v[i - k];
        }
        for (int i = 0; i < C.r; ++i) {
            double d = 0.0;
            for (int j = k; j < n; ++j) d += C(i, j) * v[j - k];
            d = 2.0 * d / vn;
            for (int j = k; j < n; ++j) C(i, j) -= d * v[j - k];
        }
    }
}

bool lu_full_solve(const Mat &A0, const Mat &B, Mat *X) {
    const int n = A0.r, m = B.c;
    Mat A = A0;
    std::vector<int> rp, cp;
    lu_full(A, rp, cp);
    for (int k = 0; k < n; ++k)
        if (A(k, k) == 0.0) return false;
    *X = Mat(n, m);
    for (int j = 0; j < m; ++j) {
        std::vector<double> y(n);
        for (int i = 0; i < n; ++i) {
            double s = B(rp[i], j);
            for (int k = 0; k < i; ++k) s -= A(i, k) * y[k];
            y[i] = s;
        }
        for (int i = n - 1; i >= 0; --i) {
            double s = y[i];
            for (int k = i + 1; k < n; ++k) s -= A(i, k) * y[k];
            y[i] = s / A(i, i);
        }
        for (int i = 0; i < n; ++i) (*X)(cp[i], j) = y[i];
    }
    return true;
}

std::vector<double> null_vector(const Mat &A0) {
    const int n = A0.r;
    Mat A = A0;
    std::vector<int> rp, cp;
    lu_full(A, rp, cp);
    // the last pivot is the smallest: set that variable to 1 and back substitute
    std::vector<double> z(n, 0.0);
    z[n - 1] = 1.0;
    for (int i = n - 2; i >= 0; --i) {
        double s = 0;
        for (int k = i + 1; k < n; ++k) s -= A(i, k) * z[k];
        z[i] = (A(i, i) != 0.0) ? s / A(i, i) : 0.0;
    }
    std::vector<double> v(n);
    double nn = 0;
    for (int i = 0; i < n; ++i) {
        v[cp[i]] = z[i];
        nn += z[i] * z[i];
    }
    nn = std::sqrt(nn);
    for (double &e : v) e /= nn;
    return v;
}

static inline double sign_of(double a, double b) { return b >= 0 ? std::fabs(a) : -std::fabs(a); }

static void balance(Mat &a) {
    const int n = a.r;
    const double radix = 2.0, sqrdx = 4.0;
    bool done = false;
    while (!done) {
        done = true;
        for (int i = 0; i < n; ++i) {
            double r = 0, c = 0;
            for (int j = 0; j < n; ++j)
                if (j != i) {
                    c += std::fabs(a(j, i));
                    r += std::fabs(a(i, j));
                }
            if (c != 0.0 && r != 0.0) {
                double g = r / radix, f = 1.0, s = c + r;
                while (c < g) {
                    f *= radix;
                    c *= sqrdx;
                }
                g = r * radix;
                while (c > g) {
                    f /= radix;
                    c /= sqrdx;
                }
                if ((c + r) / f < 0.95 * s) {
                    done = false;
                    g = 1.0 / f;
                    for (int j = 0; j < n; ++j) a(i, j) *= g;
                    for (int j = 0; j < n; ++j) a(j, i) *= f;
                }
            }
        }
    }
}

static void to_hessenberg(Mat &a) {
    // Gaussian elimination with pivoting (EISPACK elmhes)
    const int n = a.r;
    for (int m = 1; m < n - 1; ++m) {
        double x = 0.0;
        int i = m;
        for (int j = m; j < n; ++j)
            if (std::fabs(a(j, m - 1)) > std::fabs(x)) {
                x = a(j, m - 1);
                i = j;
            }
        if (i != m) {
            for (int j = m - 1; j < n; ++j) std::swap(a(i, j), a(m, j));
            for (int j = 0; j < n; ++j) std::swap(a(j, i), a(j, m));
        }
        if (x != 0.0) {
            for (i = m + 1; i < n; ++i) {
                double y = a(i, m - 1);
                if (y != 0.0) {
                    y /= x;
                    a(i, m - 1) = y;
                    for (int j = m; j < n; ++j) a(i, j) -= y * a(m, j);
                    for (int j = 0; j < n; ++j) a(j, m) += y * a(j, i);
                }
            }
        }
    }
    for (int i = 2; i < n; ++i)
        for (int j = 0; j < i - 1; ++j) a(i, j) = 0.0;
}

static bool hqr(Mat &a, std::vector<double> &wr, std::vector<double> &wi) {
    const int n = a.r;
    wr.assign(n, 0.0);
    wi.assign(n, 0.0);
    double anorm = 0.0;
    for (int i = 0; i < n; ++i)
        for (int j = std::max(i - 1, 0); j < n; ++j) anorm += std::fabs(a(i, j));
    int nn = n - 1;
    double t = 0.0;
    double p = 0, q = 0, r = 0, s = 0, w = 0, x = 0, y = 0, z = 0;
    while (nn >= 0) {
        int its = 0, l;
        do {
            for (l = nn; l >= 1; --l) {
                s = std::fabs(a(l - 1, l - 1)) + std::fabs(a(l, l));
                if (s == 0.0) s = anorm;
                if (std::fabs(a(l, l - 1)) + s == s) {
                    a(l, l - 1) = 0.0;
                    break;
                }
            }
            x = a(nn, nn);
            if (l == nn) {
                wr[nn] = x + t;
                wi[nn--] = 0.0;
            } else {
                y = a(nn - 1, nn - 1);
                w = a(nn, nn - 1) * a(nn - 1, nn);
                if (l == nn - 1) {
                    p = 0.5 * (y - x);
                    q = p * p + w;
                    z = std::sqrt(std::fabs(q));
                    x += t;
                    if (q >= 0.0) {
                        z = p + sign_of(z, p);
                        wr[nn - 1] = wr[nn] = x + z;
                        if (z != 0.0) wr[nn] = x - w / z;
                        wi[nn - 1] = wi[nn] = 0.0;
                    } else {
                        wr[nn - 1] = wr[nn] = x + p;
                        wi[nn - 1] = -(wi[nn] = z);
                    }
                    nn -= 2;
                } else {
                    if (its == 60) return false;
                    if (its == 10 || its == 20 || its == 40) {
                        t += x;
                        for (int i = 0; i <= nn; ++i) a(i, i) -= x;
                        s = std::fabs(a(nn, nn - 1)) + std::fabs(a(nn - 1, nn - 2));
                        y = x = 0.75 * s;
                        w = -0.4375 * s * s;
                    }
                    ++its;
                    int m;
                    for (m = nn - 2; m >= l; --m) {
                        z = a(m, m);
                        r = x - z;
                        s = y - z;
                        p = (r * s - w) / a(m + 1, m) + a(m, m + 1);
                        q = a(m + 1, m + 1) - z - r - s;
                        r = a(m + 2, m + 1);
                        s = std::fabs(p) + std::fabs(q) + std::fabs(r);
                        p /= s;
                        q /= s;
                        r /= s;
                        if (m == l) break;
                        double u = std::fabs(a(m, m - 1)) * (std::fabs(q) + std::fabs(r));
                        double v = std::fabs(p) * (std::fabs(a(m - 1, m - 1)) + std::fabs(z) + std::fabs(a(m + 1, m + 1)));
                        if (u + v == v) break;
                    }
                    for (int i = m + 2; i <= nn; ++i) {
                        a(i, i - 2) = 0.0;
                        if (i != m + 2) a(i, i - 3) = 0.0;
                    }
                    for (int k = m; k <= nn - 1; ++k) {
                        if (k != m) {
                            p = a(k, k - 1);
                            q = a(k + 1, k - 1);
                            r = 0.0;
                            if (k != nn - 1) r = a(k + 2, k - 1);
                            if ((x = std::fabs(p) + std::fabs(q) + std::fabs(r)) != 0.0) {
                                p /= x;
                                q /= x;
                                r /= x;
                            }
                        }
                        if ((s = sign_of(std::sqrt(p * p + q * q + r * r), p)) != 0.0) {
                            if (k == m) {
                                if (l != m) a(k, k - 1) = -a(k, k - 1);
                            } else
                                a(k, k - 1) = -s * x;
                            p += s;
                            x = p / s;
                            y = q / s;
                            z = r / s;
                            q /= p;
                            r /= p;
                            for (int j = k; j <= nn; ++j) {
                                p = a(k, j) + q * a(k + 1, j);
                                if (k != nn - 1) {
                                    p += r * a(k + 2, j);
                                    a(k + 2, j) -= p * z;
                                }
                                a(k + 1, j) -= p * y;
                                a(k, j) -= p * x;
                            }
                            int mmin = nn < k + 3 ? nn : k + 3;
                            for (int i = l; i <= mmin; ++i) {
                                p = x * a(i, k) + y * a(i, k + 1);
                                if (k != nn - 1) {
                                    p += z * a(i, k + 2);
                                    a(i, k + 2) -= p * r;
                                }
                                a(i, k + 1) -= p * q;
                                a(i, k) -= p;
                            }
                        }
                    }
                }
            }
        } while (l < nn - 1);
    }
    return true;
}

bool eig_real(Mat A, std::vector<double> *wr, std::vector<double> *wi) {
    if (A.r == 1) {
        wr->assign(1, A(0, 0));
        wi->assign(1, 0.0);
        return true;
    }
    balance(A);
    to_hessenberg(A);
    return hqr(A, *wr, *wi);
}

std::vector<double> poly_real_roots(std::vector<double> c) {
    while (!c.empty() && c.back() == 0.0) c.pop_back();
    std::vector<double> out;
    const int n = (int)c.size() - 1;
    if (n < 1) return out;
    if (n == 1) {
        out.push_back(-c[0] / c[1]);
        return out;
    }
    Mat C(n, n);
    for (int j = 0; j < n; ++j) C(0, j) = -c[n - 1 - j] / c[n];
    for (int i = 1; i < n; ++i) C(i, i - 1) = 1.0;
    std::vector<double> wr, wi;
    if (!eig_real(C, &wr, &wi)) return out;
    for (int i = 0; i < n; ++i)
        if (wi[i] == 0.0) out.push_back(wr[i]);
    return out;
}

void jacobi_svd(const Mat &A0, Mat *U, std::vector<double> *s, Mat *V) {
    // one-sided (Hestenes) Jacobi: orthogonalise the columns of A V
    const int n = A0.c, m = A0.r;
    Mat A = A0;
    Mat W(n, n);
    for (int i = 0; i < n; ++i) W(i, i) = 1.0;
    for (int sweep = 0; sweep < 60; ++sweep) {
        double off = 0.0;
        for (int p = 0; p < n - 1; ++p)
            for (int q = p + 1; q < n; ++q) {
                double al = 0, be = 0, ga = 0;
                for (int i = 0; i < m; ++i) {
                    al += A(i, p) * A(i, p);
                    be += A(i, q) * A(i, q);
                    ga += A(i, p) * A(i, q);
                }
                if (ga == 0.0) continue;
                double rel = std::fabs(ga) / std::sqrt(al * be);
                if (!(rel > 1e-17)) continue;
                off = std::max(off, rel);
                double zeta = (be - al) / (2.0 * ga);
                double t = (zeta >= 0 ? 1.0 : -1.0) / (std::fabs(zeta) + std::sqrt(1.0 + zeta * zeta));
                double c = 1.0 / std::sqrt(1.0 + t * t), sn = c * t;
                for (int i = 0; i < m; ++i) {
                    double ap = A(i, p), aq = A(i, q);
                    A(i, p) = c * ap - sn * aq;
                    A(i, q) = sn * ap + c * aq;
                }
                for (int i = 0; i < n; ++i) {
                    double wp = W(i, p), wq = W(i, q);
                    W(i, p) = c * wp - sn * wq;
                    W(i, q) = sn * wp + c * wq;
                }
            }
        if (off < 1e-16) break;
    }
    std::vector<double> sv(n);
    for (int j = 0; j < n; ++j) {
        double t = 0;
        for (int i = 0; i < m; ++i) t += A(i, j) * A(i, j);
        sv[j] = std::sqrt(t);
    }
    std::vector<int> ord(n);
    for (int j = 0; j < n; ++j) ord[j] = j;
    std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return sv[a] > sv[b]; });
    *s = std::vector<double>(n);
    *U = Mat(m, n);
    *V = Mat(n, n);
    const double tol = (sv[ord[0]] > 0 ? sv[ord[0]] : 1.0) * 1e-13;
    for (int k = 0; k < n; ++k) {
        int j = ord[k];
        (*s)[k] = sv[j];
        for (int i = 0; i < n; ++i) (*V)(i, k) = W(i, j);
        if (sv[j] > tol)
            for (int i = 0; i < m; ++i) (*U)(i, k) = A(i, j) / sv[j];
        else {
            // complete U with an orthonormal vector (Gram-Schmidt on unit vectors)
            for (int e = 0; e < m; ++e) {
                std::vector<double> u(m, 0.0);
                u[e] = 1.0;
                for (int kk = 0; kk < k; ++kk) {
                    double d = 0;
                    for (int i = 0; i < m; ++i) d += (*U)(i, kk) * u[i];
                    for (int i = 0; i < m; ++i) u[i] -= d * (*U)(i, kk);
                }
                double nn = 0;
                for (double x : u) nn += x * x;
                if (nn > 0.1) {
                    nn = std::sqrt(nn);
                    for (int i = 0; i < m; ++i) (*U)(i, k) = u[i] / nn;
                    break;
                }
            }
        }
    }
}

// Eigen 3.4's two-sided Jacobi SVD as the reference calls it for the MD poses
// (Eigen::JacobiSVD<Eigen::MatrixXd>(S, ComputeFullU | ComputeFullV), src/solver.cpp:517,
// :722, :1026; Eigen is not vendored in /root/reference: restated from Eigen 3.4.0
// JacobiSVD.h compute(), RealSvd2x2.h real_2x2_jacobi_svd and Jacobi.h makeJacobi /
// apply_rotation_in_the_plane, square real input, no QR preconditioner).  Parity with
// Eigen itself is unpinned; the device restates this function operation for operation
// (madpose_amd/csrc/include/mp_md_exact.h mdx::svd3).
namespace {
struct Rot {
    double c, s;
};
// rows p, q of the row-major 3 x 3 M: x' = c x + s y, y' = -s x + c y (the identity is a no-op)
void rot_rows(double *M, int p, int q, Rot j) {
    if (j.c == 1.0 && j.s == 0.0) return;
    for (int i = 0; i < 3; ++i) {
        const double xi = M[3 * p + i], yi = M[3 * q + i];
        M[3 * p + i] = j.c * xi + j.s * yi;
        M[3 * q + i] = -j.s * xi + j.c * yi;
    }
}
// columns p, q: MatrixBase::applyOnTheRight(p, q, j) applies j^T = (c, -s) to the columns
void rot_cols(double *M, int p, int q, Rot j) {
    const Rot t{j.c, -j.s};
    if (t.c == 1.0 && t.s == 0.0) return;
    for (int i = 0; i < 3; ++i) {
        const double xi = M[3 * i + p], yi = M[3 * i + q];
        M[3 * i + p] = t.c * xi + t.s * yi;
        M[3 * i + q] = -t.s * xi + t.c * yi;
    }
}
Rot make_jacobi(double x, double y, double z) {
    const double deno = 2.0 * std::fabs(y);
    if (deno < DBL_MIN) return Rot{1.0, 0.0};
    const double tau = (x - z) / deno;
    const double w = std::sqrt(tau * tau + 1.0);
    const double t = tau > 0.0 ? 1.0 / (tau + w) : 1.0 / (tau - w);
    const double sign_t = t > 0.0 ? 1.0 : -1.0;
    const double n = 1.0 / std::sqrt(t * t + 1.0);
    return Rot{n, -sign_t * (y / std::fabs(y)) * std::fabs(t) * n};
}
} // namespace

void eigen_jacobi_svd3(const double A[9], double U[9], double V[9]) {
    const double precision = 2.0 * DBL_EPSILON, consider_zero = DBL_MIN;
    double scale = 0.0;
    for (int i = 0; i < 9; ++i) {
        const double a = std::fabs(A[i]);
        if (std::isnan(a)) scale = a;
        else if (!std::isnan(scale)) scale = scale < a ? a : scale;
    }
    double W[9];
    for (int i = 0; i < 9; ++i) U[i] = V[i] = (i % 4 == 0) ? 1.0 : 0.0;
    if (!std::isfinite(scale)) { // Eigen: InvalidInput, U and V left as they are
        return;
    }
    if (scale == 0.0) scale = 1.0;
    for (int i = 0; i < 9; ++i) W[i] = A[i] / scale;
    double max_diag = std::fabs(W[0]);
    for (int i = 1; i < 3; ++i) max_diag = max_diag < std::fabs(W[4 * i]) ? std::fabs(W[4 * i]) : max_diag;
    bool finished = false;
    while (!finished) {
        finished = true;
        for (int p = 1; p < 3; ++p)
            for (int q = 0; q < p; ++q) {
                const double pm = precision * max_diag;
                const double threshold = consider_zero < pm ? pm : consider_zero;
                if (std::fabs(W[3 * p + q]) > threshold || std::fabs(W[3 * q + p]) > threshold) {
                    finished = false;
                    // real_2x2_jacobi_svd on [W(p,p) W(p,q); W(q,p) W(q,q)]
                    double m00 = W[3 * p + p], m01 = W[3 * p + q], m10 = W[3 * q + p], m11 = W[3 * q + q];
                    Rot rot1;
                    const double t = m00 + m11, d = m10 - m01;
                    if (std::fabs(d) < DBL_MIN) {
                        rot1 = Rot{1.0, 0.0};
                    } else {
                        const double u = t / d;
                        const double tmp = std::sqrt(1.0 + u * u);
                        rot1 = Rot{u / tmp, 1.0 / tmp};
                    }
                    if (!(rot1.c == 1.0 && rot1.s == 0.0)) { // m.applyOnTheLeft(0, 1, rot1)
                        const double x0 = m00, y0 = m10, x1 = m01, y1 = m11;
                        m00 = rot1.c * x0 + rot1.s * y0;
                        m10 = -rot1.s * x0 + rot1.c * y0;
                        m01 = rot1.c * x1 + rot1.s * y1;
                        m11 = -rot1.s * x1 + rot1.c * y1;
                    }
                    (void)m10;
                    const Rot jr = make_jacobi(m00, m01, m11);
                    // j_left = rot1 * j_right^T, (c1, s1) * (c2, s2) = (c1 c2 - s1 s2, c1 s2 + s1 c2)
                    const double c2 = jr.c, s2 = -jr.s;
                    const Rot jl{rot1.c * c2 - rot1.s * s2, rot1.c * s2 + rot1.s * c2};
                    rot_rows(W, p, q, jl);
                    rot_cols(U, p, q, Rot{jl.c, -jl.s}); // U.applyOnTheRight(p, q, j_left^T)
                    rot_cols(W, p, q, jr);
                    rot_cols(V, p, q, jr);
                    const double dp = std::fabs(W[3 * p + p]), dq = std::fabs(W[3 * q + q]);
                    const double m = dp < dq ? dq : dp;
                    max_diag = max_diag < m ? m : max_diag;
                }
            }
    }
    double sv[3];
    for (int i = 0; i < 3; ++i) {
        const double a = W[4 * i];
        sv[i] = std::fabs(a);
        if (a < 0.0)
            for (int r = 0; r < 3; ++r) U[3 * r + i] = -U[3 * r + i];
    }
    for (int i = 0; i < 3; ++i) sv[i] *= scale;
    for (int i = 0; i < 3; ++i) {
        int pos = i; // maxCoeff(&pos) over the tail: the first maximum
        for (int j = i + 1; j < 3; ++j)
            if (sv[j] > sv[pos]) pos = j;
        if (sv[pos] == 0.0) break;
        if (pos != i) {
            std::swap(sv[i], sv[pos]);
            for (int r = 0; r < 3; ++r) {
                std::swap(U[3 * r + i], U[3 * r + pos]);
                std::swap(V[3 * r + i], V[3 * r + pos]);
            }
        }
    }
}

double det3(const double M[9]) {
    return M[0] * (M[4] * M[8] - M[5] * M[7]) - M[1] * (M[3] * M[8] - M[5] * M[6]) + M[2] * (M[3] * M[7] - M[4] * M[6]);
}

} // namespace oracle
