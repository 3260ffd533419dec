// The two passes of the hybrid batch drawing (batch_draw.h) on AVX-512, for hosts
// that have it (the MI355X boxes' EPYC 9575F does; checked at run time, the scalar
// passes otherwise).  The same outputs of the same generators, consumed in the same
// order, tested the same way -- every type, kept index, list entry, snapshot and end
// state equals the scalar passes' (tests/sampler_check.cpp):
//
//   types (pass 1): 8 iterations per vector.  Each takes exactly two selection-stream
//     outputs (uniform_real never redraws), so iteration i reads outputs 2i and 2i + 1
//     of the block; the double arithmetic is uniform_real's operation for operation
//     (the 2^32 product is exact, one rounding in the sum, the scaling by 2^-64 exact,
//     the clamp below 1, one rounding in (b - a) * c, + a = + 0 exact).
//   samples (pass 2): up to 16 iterations per vector.  Without redraws iteration i
//     starts at the prefix sum of its predecessors' consumption (A + Bg for MD, C for
//     point), so its W outputs are gathered from there; Lemire products, rejection
//     and duplicate tests as hybrid_sample_one.  The lanes before the first one that
//     would redraw are committed; that iteration runs the scalar code (which redraws
//     draw by draw), and the next vector starts behind it.  A vector never crosses a
//     snapshot point (kSnap) or the end of the generator's block (the iteration that
//     does runs scalar, which refills the block).
#pragma once
#if defined(__x86_64__) && (defined(__clang__) || defined(__GNUC__))
#define MP_DRAW_SIMD 1
#include <immintrin.h>
#include <algorithm>
#include <cstring>

namespace mp {

#define MP_AVX512 __attribute__((target("avx512f,avx512bw,avx512vl,avx512dq")))

inline bool draw_simd_available() {
    static const bool ok = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
                           __builtin_cpu_supports("avx512vl") && __builtin_cpu_supports("avx512dq");
    return ok;
}

MP_AVX512 inline void draw_types_simd(IterationStream &rs, Batch &g, uint32_t B) {
    uint8_t *ty = g.types.data();
    const double p0 = rs.prior[0], ps = rs.prior[0] + rs.prior[1];
    Mt19937 &sel = rs.sel;
    const __m512d two32 = _mm512_set1_pd(4294967296.0), inv64 = _mm512_set1_pd(0x1p-64), one = _mm512_set1_pd(1.0);
    double below_one;
    {
        const uint64_t b = 0x3fefffffffffffffull; // nextafter(1.0, 0.0)
        std::memcpy(&below_one, &b, sizeof b);
    }
    const __m512d vb1 = _mm512_set1_pd(below_one), vps = _mm512_set1_pd(ps), vp0 = _mm512_set1_pd(p0),
                  zero = _mm512_setzero_pd();
    uint32_t j = 0;
    while (j < B) {
        if (j % kSnap == 0) g.snaps[j / kSnap].sel = sel;
        int room;
        const uint32_t *w = sel.rest(&room);
        uint32_t L = std::min<uint32_t>(8, std::min<uint32_t>(kSnap - j % kSnap, B - j));
        L = std::min<uint32_t>(L, (uint32_t)room / 2);
        if (L == 0) { // the iteration straddles the block end
            ty[j] = uniform_real(sel, 0.0, ps) <= p0 ? 0 : 1;
            ++j;
            continue;
        }
        const __mmask16 m16 = (__mmask16)((1u << (2 * L)) - 1);
        const __m512i raw = _mm512_maskz_loadu_epi32(m16, w);
        // outputs 2i (low) and 2i + 1 (high) of each 64-bit lane
        const __m256i g1 = _mm512_cvtepi64_epi32(raw);
        const __m256i g2 = _mm512_cvtepi64_epi32(_mm512_srli_epi64(raw, 32));
        const __m512d d1 = _mm512_cvtepu32_pd(g1), d2 = _mm512_cvtepu32_pd(g2);
        const __m512d sum = _mm512_add_pd(d1, _mm512_mul_pd(d2, two32));
        __m512d c = _mm512_mul_pd(sum, inv64);
        c = _mm512_mask_blend_pd(_mm512_cmp_pd_mask(c, one, _CMP_GE_OQ), c, vb1);
        const __m512d u = _mm512_add_pd(_mm512_mul_pd(vps, c), zero);
        const __mmask8 pt = (__mmask8)(~_mm512_cmp_pd_mask(u, vp0, _CMP_LE_OQ)); // u <= p0 picks solver 0
        _mm_mask_storeu_epi8(ty + j, (__mmask16)((1u << L) - 1), _mm_maskz_set1_epi8((__mmask16)pt, 1));
        sel.skip(2 * (int)L);
        j += L;
    }
}

// (hi, lo) halves of the 64-bit products v * range, per 32-bit lane
MP_AVX512 inline void draw_mul_hi_lo(__m512i v, __m512i range, __m512i &hi, __m512i &lo) {
    const __m512i ev = _mm512_mul_epu32(v, range);                        // lanes 0, 2, ...
    const __m512i od = _mm512_mul_epu32(_mm512_srli_epi64(v, 32), range); // lanes 1, 3, ...
    const __m512i himask = _mm512_set1_epi64((long long)0xffffffff00000000ull);
    hi = _mm512_or_si512(_mm512_srli_epi64(ev, 32), _mm512_and_si512(od, himask));
    lo = _mm512_or_si512(_mm512_andnot_si512(himask, ev), _mm512_slli_epi64(od, 32));
}

template <int A, int Bg, int C>
MP_AVX512 inline bool draw_samples_simd(IterationStream &rs, Batch &g, uint32_t B, int *smp, int *lists,
                                        const std::atomic<bool> *abort, int &nmd, int &npt) {
    constexpr int W = A + Bg > C ? A + Bg : C, K = A > C ? A : C;
    static_assert(W <= 8 && K <= 8, "sample sizes");
    const uint8_t *ty = g.types.data();
    Mt19937 &samp = rs.samp;
    const __m512i vrange = _mm512_set1_epi64((long long)rs.pick.range);
    const __m512i vthr = _mm512_set1_epi32((int)rs.pick.threshold);
    const __m512i lane = _mm512_setr_epi32(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
    const __m512i lane8 = _mm512_slli_epi32(lane, 3);
    alignas(64) int off[16];
    uint32_t j = 0;
    while (j < B) {
        if (j % kSnap == 0) {
            if (abort && abort->load(std::memory_order_relaxed)) return false;
            g.snaps[j / kSnap].samp = samp;
        }
        int room;
        const uint32_t *w = samp.rest(&room);
        uint32_t L = std::min<uint32_t>(16, std::min<uint32_t>(kSnap - j % kSnap, B - j));
        L = std::min<uint32_t>(L, (uint32_t)room / W);
        if (L == 0) { // the iteration may cross the block end: scalar
            hybrid_sample_one<A, Bg, C>(rs, ty[j], j, B, smp, lists, nmd, npt);
            ++j;
            continue;
        }
        unsigned stm = 0;
        {
            int o = 0;
            for (uint32_t i = 0; i < L; ++i) {
                const int st = ty[j + i];
                off[i] = o;
                o += st ? C : A + Bg;
                stm |= (unsigned)st << i;
            }
            for (uint32_t i = L; i < 16; ++i) off[i] = 0;
        }
        const __mmask16 lm = (__mmask16)((1u << L) - 1);
        const __mmask16 ptm = (__mmask16)stm, mdm = (__mmask16)(~stm & lm);
        const __m512i voff = _mm512_load_si512(off);
        __m512i hi[W];
        __mmask16 rej_md = 0, rej_pt = 0;
#pragma unroll
        for (int k = 0; k < W; ++k) {
            const __m512i v =
                _mm512_mask_i32gather_epi32(_mm512_setzero_si512(), lm, _mm512_add_epi32(voff, _mm512_set1_epi32(k)),
                                            (const int *)w, 4);
            __m512i lo;
            draw_mul_hi_lo(v, vrange, hi[k], lo);
            const __mmask16 r = _mm512_cmplt_epu32_mask(lo, vthr);
            if (k < A + Bg) rej_md |= r;
            if (k < C) rej_pt |= r;
        }
        __mmask16 dmd = 0, dpt = 0;
#pragma unroll
        for (int i = 1; i < A; ++i)
#pragma unroll
            for (int k = 0; k < i; ++k) dmd |= _mm512_cmpeq_epi32_mask(hi[i], hi[k]);
#pragma unroll
        for (int i = A + 1; i < A + Bg; ++i)
#pragma unroll
            for (int k = A; k < i; ++k) dmd |= _mm512_cmpeq_epi32_mask(hi[i], hi[k]);
#pragma unroll
        for (int i = 1; i < C; ++i)
#pragma unroll
            for (int k = 0; k < i; ++k) dpt |= _mm512_cmpeq_epi32_mask(hi[i], hi[k]);
        const unsigned bad = (unsigned)(((rej_md | dmd) & mdm) | ((rej_pt | dpt) & ptm));
        const uint32_t p = bad ? (uint32_t)__builtin_ctz(bad) : L; // lanes [0, p) need no redraw
        if (p > 0) {
            const __mmask16 cm = (__mmask16)((1u << p) - 1);
            // the kept indices, 8 slots per iteration: the K vectors transposed in
            // registers (two iterations per 512-bit row), stored for lanes [0, p) only
            {
                __m512i c[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) c[k] = k < K ? hi[k < K ? k : 0] : _mm512_setzero_si512();
                const __m512i t0 = _mm512_unpacklo_epi32(c[0], c[1]), t1 = _mm512_unpackhi_epi32(c[0], c[1]);
                const __m512i t2 = _mm512_unpacklo_epi32(c[2], c[3]), t3 = _mm512_unpackhi_epi32(c[2], c[3]);
                const __m512i t4 = _mm512_unpacklo_epi32(c[4], c[5]), t5 = _mm512_unpackhi_epi32(c[4], c[5]);
                const __m512i t6 = _mm512_unpacklo_epi32(c[6], c[7]), t7 = _mm512_unpackhi_epi32(c[6], c[7]);
                // per 128-bit block b: u0 = lanes 4b (k 0-3 | 4-7 halves follow), ...
                const __m512i u0 = _mm512_unpacklo_epi64(t0, t2), u1 = _mm512_unpackhi_epi64(t0, t2);
                const __m512i u2 = _mm512_unpacklo_epi64(t1, t3), u3 = _mm512_unpackhi_epi64(t1, t3);
                const __m512i u4 = _mm512_unpacklo_epi64(t4, t6), u5 = _mm512_unpackhi_epi64(t4, t6);
                const __m512i u6 = _mm512_unpacklo_epi64(t5, t7), u7 = _mm512_unpackhi_epi64(t5, t7);
                // u0 / u4: k 0-3 / 4-7 of lanes 4b; u1 / u5: lanes 4b + 1; u2 / u6: 4b + 2;
                // u3 / u7: 4b + 3 (b = 128-bit block).  Row r (iterations 2r, 2r + 1):
                const __m512i lo01 = _mm512_shuffle_i32x4(u0, u4, 0x44), hi01 = _mm512_shuffle_i32x4(u0, u4, 0xee);
                const __m512i lo11 = _mm512_shuffle_i32x4(u1, u5, 0x44), hi11 = _mm512_shuffle_i32x4(u1, u5, 0xee);
                const __m512i lo21 = _mm512_shuffle_i32x4(u2, u6, 0x44), hi21 = _mm512_shuffle_i32x4(u2, u6, 0xee);
                const __m512i lo31 = _mm512_shuffle_i32x4(u3, u7, 0x44), hi31 = _mm512_shuffle_i32x4(u3, u7, 0xee);
                // loXX holds blocks (b0: k0-3, b1: k0-3, b0: k4-7, b1: k4-7) -> reorder to
                // (b0: k0-3, b0: k4-7, b1: k0-3, b1: k4-7)
                const __m512i r[8] = {
                    _mm512_shuffle_i32x4(lo01, lo11, 0x88), _mm512_shuffle_i32x4(lo21, lo31, 0x88),
                    _mm512_shuffle_i32x4(lo01, lo11, 0xdd), _mm512_shuffle_i32x4(lo21, lo31, 0xdd),
                    _mm512_shuffle_i32x4(hi01, hi11, 0x88), _mm512_shuffle_i32x4(hi21, hi31, 0x88),
                    _mm512_shuffle_i32x4(hi01, hi11, 0xdd), _mm512_shuffle_i32x4(hi21, hi31, 0xdd)};
                int *base = smp + 8 * (size_t)j;
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const unsigned pair = ((unsigned)cm >> (2 * q)) & 3u;
                    const __mmask16 sm = (__mmask16)((pair & 1u ? 0x00ffu : 0u) | (pair & 2u ? 0xff00u : 0u));
                    if (sm) _mm512_mask_storeu_epi32(base + 16 * q, sm, r[q]);
                }
            }
            const __m512i it = _mm512_add_epi32(lane, _mm512_set1_epi32((int)j));
            const __mmask16 cmd = mdm & cm, cpt = ptm & cm;
            const int nm = __builtin_popcount((unsigned)cmd);
            _mm512_mask_storeu_epi32(lists + nmd, (__mmask16)((1u << nm) - 1), _mm512_maskz_compress_epi32(cmd, it));
            nmd += nm;
            // point iterations from the back, descending: the reversed lanes compressed
            const __m512i rev = _mm512_permutexvar_epi32(_mm512_sub_epi32(_mm512_set1_epi32(15), lane), it);
            unsigned rpt = 0;
            for (int i = 0; i < 16; ++i) rpt |= (((unsigned)cpt >> i) & 1u) << (15 - i);
            const int np = __builtin_popcount((unsigned)cpt);
            _mm512_mask_storeu_epi32(lists + (B - (uint32_t)npt - (uint32_t)np), (__mmask16)((1u << np) - 1),
                                     _mm512_maskz_compress_epi32((__mmask16)rpt, rev));
            npt += np;
            samp.skip(p == L ? off[L - 1] + (((stm >> (L - 1)) & 1u) ? C : A + Bg)
                             : off[p]); // the consumption of lanes [0, p)
            j += p;
        }
        if (p < L) { // the first lane that redraws: draw by draw
            hybrid_sample_one<A, Bg, C>(rs, ty[j], j, B, smp, lists, nmd, npt);
            ++j;
        }
    }
    return true;
}

#undef MP_AVX512

} // namespace mp
#else
#define MP_DRAW_SIMD 0
#endif
