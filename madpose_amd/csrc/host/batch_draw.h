// Minimal-sample batches of the estimator loop (host side, no HIP): the solver types
// and samples of B speculative iterations drawn from the reference's two random
// streams (rng.h).  A header of its own so that tests/test_sampler_cpu.py can check
// the batch drawing against the draw-by-draw loop with the host compiler alone.
#pragma once
#include <atomic>
#include <cstdint>
#include <vector>

#include "rng.h"

namespace mp {

// ---------------------------------------------------------------------------
// Minimal-sample batches (host).  One batch holds its iterations' solver types and
// samples (in a pinned host slot), plus snapshots of both random streams every
// kSnap iterations so a rewind to iteration j replays fewer than kSnap iterations.
constexpr uint32_t kSnap = 512;
struct Batch {
    uint32_t B = 0;
    int nmd = 0, npt = 0, slot = 0;
    std::vector<uint8_t> types;
    std::vector<IterationStream> snaps;
};

// Draws B iterations from rs into g and the slot memory at `smp`: the samples
// (8 ints per iteration), then right behind them the iteration lists -- MD iterations
// ascending from the front, point iterations from the back (descending) -- so the
// batch is one contiguous block of 9B ints (one upload).  Returns false if *abort was
// raised first (checked every 256 iterations; every kSnap in the two-pass path).
//
// Both solvers live with the standard sample sizes (the hybrid case): the draws of
// the two streams are independent given the solver types, so the batch is drawn in
// two passes -- the selection stream's types of all B iterations, then the sampler
// stream with the types known -- each pass a tight loop over one generator.  An
// iteration's sample comes from one window of max(A + Bg, C) buffered outputs formed
// for either solver (both "would be redrawn" tests computed, the type's one used);
// any redraw takes the draw-by-draw code.  The MD iteration keeps v[0..A), the point
// iteration v[0..C); slots A..C of an MD iteration are never read.  Same draws,
// types, lists and snapshots as the one-pass loop (tests/test_engine_gpu.py, the
// fixed-seed parity suite); 29 -> 23 ns per calibrated iteration on the build host.
// simd: both passes 8 / 16 iterations at a time on AVX-512 (batch_draw_simd.h) where
// the host has it, the same draws (tests/test_sampler_cpu.py).

// pass 2, one iteration (type st) at the sampler stream's position
template <int A, int Bg, int C>
inline void hybrid_sample_one(IterationStream &rs, int st, uint32_t j, uint32_t B, int *smp, int *lists, int &nmd,
                              int &npt) {
    constexpr int W = A + Bg > C ? A + Bg : C, K = A > C ? A : C;
    Mt19937 &samp = rs.samp;
    const uint64_t range = rs.pick.range;
    const uint32_t thr = rs.pick.threshold;
    int *idx = smp + 8 * (size_t)j;
    lists[st ? B - 1 - npt : nmd] = (int)j;
    nmd += st ^ 1;
    npt += st;
    if (const uint32_t *w = samp.window(W)) {
        int v[W];
        uint32_t lo_md = 0xffffffffu, lo_pt = 0xffffffffu;
#pragma unroll
        for (int k = 0; k < W; ++k) {
            const uint64_t pr = (uint64_t)w[k] * range;
            const uint32_t lo = (uint32_t)pr;
            if (k < A + Bg) lo_md = lo < lo_md ? lo : lo_md;
            if (k < C) lo_pt = lo < lo_pt ? lo : lo_pt;
            v[k] = (int)(uint32_t)(pr >> 32);
        }
        int dmd = 0, dpt = 0;
#pragma unroll
        for (int i = 1; i < A; ++i)
#pragma unroll
            for (int k = 0; k < i; ++k) dmd |= v[i] == v[k];
#pragma unroll
        for (int i = A + 1; i < A + Bg; ++i)
#pragma unroll
            for (int k = A; k < i; ++k) dmd |= v[i] == v[k];
#pragma unroll
        for (int i = 1; i < C; ++i)
#pragma unroll
            for (int k = 0; k < i; ++k) dpt |= v[i] == v[k];
        const uint32_t lo = st ? lo_pt : lo_md;
        const int dup = st ? dpt : dmd;
        if (!((lo < thr) | dup)) {
#pragma unroll
            for (int k = 0; k < K; ++k) idx[k] = v[k];
            samp.skip(A + Bg + st * (C - A - Bg));
            return;
        }
    }
    int tmp[8];
    for (int t = 0; t < 3; ++t) {
        const int k = rs.ss[st][t];
        if (k == 0) continue;
        const bool keep = (st == 0 && t == 0) || (st == 1 && t == 2);
        rs.distinct(k, keep ? idx : tmp);
    }
}

} // namespace mp
#include "batch_draw_simd.h"
namespace mp {

template <int A, int Bg, int C>
inline bool draw_batch_hybrid(IterationStream &rs, Batch &g, uint32_t B, int *smp, const std::atomic<bool> *abort,
                              bool simd) {
    int *lists = smp + 8 * (size_t)B;
    g.snaps.assign((B + kSnap - 1) / kSnap, rs);
    uint8_t *ty = g.types.data();
    if (rs.pick.range != (uint32_t)rs.n) rs.pick.set((uint32_t)rs.n);
    int nmd = 0, npt = 0;
#if MP_DRAW_SIMD
    if (simd && draw_simd_available()) {
        draw_types_simd(rs, g, B);
        if (!draw_samples_simd<A, Bg, C>(rs, g, B, smp, lists, abort, nmd, npt)) return false;
        g.nmd = nmd;
        g.npt = npt;
        return true;
    }
#else
    (void)simd;
#endif
    const double p0 = rs.prior[0], ps = rs.prior[0] + rs.prior[1];
    Mt19937 &sel = rs.sel;
    for (uint32_t j = 0; j < B; ++j) {
        if (j % kSnap == 0) g.snaps[j / kSnap].sel = sel;
        // SelectMinimalSolver with both priors > 0: u <= prior[0] picks solver 0
        ty[j] = uniform_real(sel, 0.0, ps) <= p0 ? 0 : 1;
    }
    for (uint32_t j = 0; j < B; ++j) {
        if (j % kSnap == 0) {
            if (abort && abort->load(std::memory_order_relaxed)) return false;
            g.snaps[j / kSnap].samp = rs.samp;
        }
        hybrid_sample_one<A, Bg, C>(rs, ty[j], j, B, smp, lists, nmd, npt);
    }
    g.nmd = nmd;
    g.npt = npt;
    return true;
}

// mode: 0 = the draw-by-draw loop (MADPOSE_SAMPLER_TWO_PASS=0, tests), 1 = two passes,
// 2 = two passes on AVX-512 where available (default)
inline bool draw_batch(IterationStream &rs, Batch &g, uint32_t B, int slot, int *smp, const std::atomic<bool> *abort,
                       int mode = 2) {
    int *lists = smp + 8 * (size_t)B;
    g.B = B;
    g.slot = slot;
    g.nmd = g.npt = 0;
    g.types.resize(B);
    g.snaps.clear();
    {
        const double *p = rs.prior;
        const int(*s)[3] = rs.ss;
        if (mode > 0 && p[0] > 0.0 && p[1] > 0.0 && s[0][2] == 0 && s[1][0] == 0 && s[1][1] == 0 && s[0][0] == s[0][1]) {
            const int a = s[0][0], c = s[1][2];
            if (a == 3 && c == 5) return draw_batch_hybrid<3, 3, 5>(rs, g, B, smp, abort, mode > 1);
            if (a == 4 && c == 6) return draw_batch_hybrid<4, 4, 6>(rs, g, B, smp, abort, mode > 1);
            if (a == 4 && c == 7) return draw_batch_hybrid<4, 4, 7>(rs, g, B, smp, abort, mode > 1);
        }
    }
    for (uint32_t j = 0; j < B; ++j) {
        if (j % kSnap == 0) g.snaps.push_back(rs);
        if (abort && (j & 255) == 0 && abort->load(std::memory_order_relaxed)) return false;
        const int st = rs.next(smp + 8 * j);
        g.types[j] = (uint8_t)st;
        if (st == 0)
            lists[g.nmd++] = (int)j;
        else
            lists[B - 1 - g.npt++] = (int)j;
    }
    return true;
}

} // namespace mp
