// ORACLE -- test infrastructure only (see oracle/README.md).  Never linked into the
// product library; only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
// leg load it, and only as the checker.
//
// Small dense linear algebra used by the CPU restatement.  The reference relies on
// Eigen (colPivHouseholderQr, fullPivHouseholderQr, EigenSolver, JacobiSVD:
// src/solver.cpp:100,263,450,104,517; src/utils.h:34).  Eigen is not available
// offline, so these are written from the textbook algorithms:
//   * Householder QR with column pivoting            (Golub & Van Loan 5.4.1)
//   * LU with complete pivoting + null vectors        (GvL 3.4.8)
//   * balancing + Hessenberg + Francis double-shift QR (EISPACK balanc/elmhes/hqr)
//   * one-sided (Hestenes) cyclic Jacobi SVD for small matrices (Eigen's JacobiSVD
//     is a two-sided Jacobi scheme; both converge to the same factorisation)
#pragma once
#include <cmath>
#include <cstring>
#include <vector>

namespace oracle {

struct Mat {
    int r = 0, c = 0;
    std::vector<double> a;
    Mat() {}
    Mat(int r_, int c_) : r(r_), c(c_), a((size_t)r_ * c_, 0.0) {}
    double &operator()(int i, int j) { return a[(size_t)i * c + j]; }
    double operator()(int i, int j) const { return a[(size_t)i * c + j]; }
};

inline Mat matmul(const Mat &A, const Mat &B) {
    Mat C(A.r, B.c);
    for (int i = 0; i < A.r; ++i)
        for (int k = 0; k < A.c; ++k) {
            double v = A(i, k);
            if (v == 0.0) continue;
            for (int j = 0; j < B.c; ++j) C(i, j) += v * B(k, j);
        }
    return C;
}

inline Mat transpose(const Mat &A) {
    Mat T(A.c, A.r);
    for (int i = 0; i < A.r; ++i)
        for (int j = 0; j < A.c; ++j) T(j, i) = A(i, j);
    return T;
}

// Solve A X = B (A square n x n) with Householder QR + column pivoting.
// Returns false when A is numerically rank deficient.
bool qr_solve(const Mat &A, const Mat &B, Mat *X);

// Solve A X = B with LU + complete pivoting.
bool lu_full_solve(const Mat &A, const Mat &B, Mat *X);

// Unit null vector of a square, (numerically) singular matrix via complete-pivot LU:
// the column with the smallest final pivot is the free variable.
std::vector<double> null_vector(const Mat &A);

// Eigenvalues of a general real matrix (balance + Hessenberg + Francis QR).
// wi[k] == 0.0 exactly for eigenvalues that the real Schur form returns as real
// (1x1 blocks, or 2x2 blocks whose eigenvalues are real), the same convention as
// Eigen::EigenSolver.  Returns false if QR did not converge.
bool eig_real(Mat A, std::vector<double> *wr, std::vector<double> *wi);

// Real roots of sum_k c[k] x^k (c ascending, degree = c.size()-1) via the companion
// matrix.  Leading zero coefficients are trimmed.  Roots are those with wi == 0.
std::vector<double> poly_real_roots(std::vector<double> c);

// One-sided Jacobi SVD of a small square matrix: A = U diag(s) V^T, s descending.
void jacobi_svd(const Mat &A, Mat *U, std::vector<double> *s, Mat *V);
// Eigen 3.4 JacobiSVD<MatrixXd>(A, ComputeFullU | ComputeFullV) of a real 3 x 3 matrix
// (row-major A, U, V; A = U diag(s) V^T, s descending); see la.cpp
void eigen_jacobi_svd3(const double A[9], double U[9], double V[9]);

double det3(const double M[9]);

// LU with complete pivoting stopped after `steps` pivots (rank-revealing for a matrix
// of known rank `steps`): A is overwritten by P A Q = L U (unit L below the diagonal
// in the first `steps` columns; the trailing block is the rounding residue).
void lu_full_steps(Mat &A, std::vector<int> &rp, std::vector<int> &cp, int steps);
// Right null space (n - rank columns) of A of known rank, from lu_full_steps:
// U11 y1 + U12 y2 = 0 with y2 = e_k, x = Q y.
Mat right_null_rank(const Mat &A, int rank);
// A particular solution of A x = b for A of known rank (b in the range of A): the
// first `rank` variables of Q^T x from the LU, the others zero.
std::vector<double> particular_solution(const Mat &A, const std::vector<double> &b, int rank);
// C <- Q^T C Q with Q = H_0 ... H_{k-1} the Householder reflectors of the QR of the
// n x k matrix Z (GvL 5.2.1, v = x - alpha e1, alpha = -sign(x_0) |x|): the first k
// columns of Q span the columns of Z.
void householder_deflate(Mat &C, Mat Z);

} // namespace oracle
