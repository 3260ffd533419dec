// Residual-block evaluation of the host LM (lm.cpp), built twice: for x86-64-v4
// (AVX-512) and x86-64-v3 (AVX2).  The two builds share one source (lm_eval.inc) and
// give identical results; lm.cpp calls the AVX-512 one when the CPU has it.
#pragma once
#include <cstddef>

namespace mp {

// full parameter layout of the LO problems: rotation tangent, t, s, o0, o1, focals
enum LmFull { kD0 = 0, kD1, kD2, kT0, kT1, kT2, kS, kO0, kO1, kF0, kF1, kNFull };
constexpr int kNPack = kNFull * (kNFull + 1) / 2;

// one problem: the pair's host arrays (x0, x1 interleaved 2n; d0, d1 n; pixels for
// the calibrated variant, normalized pixels otherwise) and the block index lists in
// use (n0 / n1 = 0 without reprojection terms, n2 = 0 without Sampson terms)
struct LmEvalIn {
    int variant;
    const double *x0, *x1, *d0, *d1;
    const double *K0, *K1, *K0i, *K1i;
    const int *s0, *s1, *s2;
    size_t n0, n1, n2;
    double w_sampson;
};
struct LmEvalParams {
    double R[9], t[3], s, o0, o1, f0, f1;
};

// adds the cost 0.5 r^2 of blocks [b0, b1) of the concatenated list (s0, s1, s2) to
// *cost and, with jac, the packed upper triangle of J^T J to H (kNPack) and J^T r to g
// (kNFull), in the full layout
void lm_eval_range_w4(const LmEvalIn &E, const LmEvalParams &p, bool jac, size_t b0, size_t b1, double *H, double *g,
                      double *cost);
void lm_eval_range_w8(const LmEvalIn &E, const LmEvalParams &p, bool jac, size_t b0, size_t b1, double *H, double *g,
                      double *cost);

} // namespace mp
