// Random streams of the reference's RANSAC loop, restated so they do not depend on
// the host toolchain's libstdc++ version:
//   * MT19937 (Matsumoto & Nishimura 1998), default seeding of std::mt19937;
//   * uniform_int_distribution<int>(a, b) as implemented by GCC >= 11 for a 32-bit
//     engine: Lemire's nearly-divisionless downscaling ("_S_nd");
//   * uniform_real_distribution<double>(a, b) = a + (b - a) * generate_canonical<double,53>
//     with two 32-bit draws: (g1 + g2 * 2^32) / 2^64, clamped below 1.
// tests/test_rng.py pins all three against tests/golden/rng_gcc11.json, which was
// produced with this container's g++ 11.4 (std::mt19937 + std distributions), i.e.
// the streams the reference consumes in src/hybrid_ransac.h:64,79-80,226-229.
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#if defined(__x86_64__) && (defined(__clang__) || defined(__GNUC__))
#include <immintrin.h>
#endif

namespace mp {

class Mt19937 {
  public:
    explicit Mt19937(uint32_t seed = 5489u) { seed_with(seed); }
    void seed_with(uint32_t seed) {
        mt_[0] = seed;
        for (int i = 1; i < 624; ++i) mt_[i] = 1812433253u * (mt_[i - 1] ^ (mt_[i - 1] >> 30)) + (uint32_t)i;
        idx_ = 624;
        draws_ = 0;
    }
    uint32_t operator()() {
        if (idx_ >= 624) twist();
        ++draws_;
        return out_[idx_++];
    }
    // outputs consumed since seeding: two copies of one stream are at the same
    // position iff their counts agree
    uint64_t draws() const { return draws_; }
    void discard(uint64_t k) { // block by block: the same state as k calls
        while (k > 0) {
            if (idx_ >= 624) twist();
            const uint64_t take = std::min<uint64_t>(k, (uint64_t)(624 - idx_));
            idx_ += (int)take;
            draws_ += take;
            k -= take;
        }
    }
    // the next k outputs without consuming them, or nullptr if they cross a block
    const uint32_t *window(int k) {
        if (idx_ >= 624) twist();
        return idx_ + k <= 624 ? out_ + idx_ : nullptr;
    }
    // the buffered outputs from the current position to the end of the block (at
    // least one: an exhausted block is refilled first); *n = how many
    const uint32_t *rest(int *n) {
        if (idx_ >= 624) twist();
        *n = 624 - idx_;
        return out_ + idx_;
    }
    void skip(int k) {
        idx_ += k;
        draws_ += (uint64_t)k;
    }

  private:
    // the recurrence split at the two wrap points so the inner loops carry no modulo
    // and vectorize; the 624 outputs of a block are tempered in one pass
    static inline uint32_t step(uint32_t cur, uint32_t nxt, uint32_t far) {
        const uint32_t y = (cur & 0x80000000u) | (nxt & 0x7fffffffu);
        return far ^ (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
    }
    void twist() {
#if defined(__x86_64__) && (defined(__clang__) || defined(__GNUC__))
        static const bool avx512 = __builtin_cpu_supports("avx512f");
        if (avx512) {
            twist_avx512();
            return;
        }
#endif
        int i = 0;
        for (; i < 624 - 397; ++i) mt_[i] = step(mt_[i], mt_[i + 1], mt_[i + 397]);
        for (; i < 623; ++i) mt_[i] = step(mt_[i], mt_[i + 1], mt_[i + 397 - 624]);
        mt_[623] = step(mt_[623], mt_[0], mt_[396]);
        for (i = 0; i < 624; ++i) {
            uint32_t y = mt_[i];
            y ^= y >> 11;
            y ^= (y << 7) & 0x9d2c5680u;
            y ^= (y << 15) & 0xefc60000u;
            y ^= y >> 18;
            out_[i] = y;
        }
        idx_ = 0;
    }
#if defined(__x86_64__) && (defined(__clang__) || defined(__GNUC__))
    // the same recurrence and tempering, 16 words per AVX-512 vector (integer
    // operations: the same words); the wrap points as in twist()
    __attribute__((target("avx512f"))) static inline __m512i step16(__m512i cur, __m512i nxt, __m512i far) {
        const __m512i y = _mm512_or_si512(_mm512_and_si512(cur, _mm512_set1_epi32((int)0x80000000u)),
                                          _mm512_and_si512(nxt, _mm512_set1_epi32(0x7fffffff)));
        const __m512i mag = _mm512_and_si512(_mm512_sub_epi32(_mm512_setzero_si512(),
                                                              _mm512_and_si512(y, _mm512_set1_epi32(1))),
                                             _mm512_set1_epi32((int)0x9908b0dfu));
        return _mm512_xor_si512(_mm512_xor_si512(far, _mm512_srli_epi32(y, 1)), mag);
    }
    __attribute__((target("avx512f"))) void twist_avx512() {
        int i = 0;
        for (; i + 16 <= 624 - 397; i += 16)
            _mm512_storeu_si512(mt_ + i, step16(_mm512_loadu_si512(mt_ + i), _mm512_loadu_si512(mt_ + i + 1),
                                                _mm512_loadu_si512(mt_ + i + 397)));
        for (; i < 624 - 397; ++i) mt_[i] = step(mt_[i], mt_[i + 1], mt_[i + 397]);
        for (; i + 16 <= 623; i += 16)
            _mm512_storeu_si512(mt_ + i, step16(_mm512_loadu_si512(mt_ + i), _mm512_loadu_si512(mt_ + i + 1),
                                                _mm512_loadu_si512(mt_ + i + 397 - 624)));
        for (; i < 623; ++i) mt_[i] = step(mt_[i], mt_[i + 1], mt_[i + 397 - 624]);
        mt_[623] = step(mt_[623], mt_[0], mt_[396]);
        for (i = 0; i < 624; i += 16) { // 624 = 39 x 16
            __m512i y = _mm512_loadu_si512(mt_ + i);
            y = _mm512_xor_si512(y, _mm512_srli_epi32(y, 11));
            y = _mm512_xor_si512(y, _mm512_and_si512(_mm512_slli_epi32(y, 7), _mm512_set1_epi32((int)0x9d2c5680u)));
            y = _mm512_xor_si512(y, _mm512_and_si512(_mm512_slli_epi32(y, 15), _mm512_set1_epi32((int)0xefc60000u)));
            y = _mm512_xor_si512(y, _mm512_srli_epi32(y, 18));
            _mm512_storeu_si512(out_ + i, y);
        }
        idx_ = 0;
    }
#endif
    uint32_t mt_[624];
    uint32_t out_[624];
    int idx_;
    uint64_t draws_ = 0;
};

// uniform integer in [a, b]
inline int uniform_int(Mt19937 &g, int a, int b) {
    const uint32_t urange = (uint32_t)b - (uint32_t)a;
    if (urange == 0xffffffffu) return (int)((uint32_t)a + g());
    const uint32_t range = urange + 1u;
    uint64_t product = (uint64_t)g() * (uint64_t)range;
    uint32_t low = (uint32_t)product;
    if (low < range) {
        const uint32_t threshold = (uint32_t)(-range) % range;
        while (low < threshold) {
            product = (uint64_t)g() * (uint64_t)range;
            low = (uint32_t)product;
        }
    }
    return (int)((uint32_t)a + (uint32_t)(product >> 32));
}

// uniform_int(g, 0, range - 1) with the rejection threshold precomputed: identical
// draws (low < threshold implies low < range, so the two-step test above reduces
// to this one)
struct UniformIndex {
    uint32_t range = 1, threshold = 0;
    void set(uint32_t r) {
        range = r;
        threshold = (uint32_t)(-r) % r;
    }
    inline int operator()(Mt19937 &g) const {
        uint64_t product = (uint64_t)g() * (uint64_t)range;
        while ((uint32_t)product < threshold) product = (uint64_t)g() * (uint64_t)range;
        return (int)(uint32_t)(product >> 32);
    }
};

// uniform real in [a, b)
inline double uniform_real(Mt19937 &g, double a, double b) {
    const double r = 4294967296.0; // 2^32
    double sum = (double)g();
    sum += (double)g() * r;
    double c = sum * 0x1p-64; // == sum / 2^64 exactly
    if (c >= 1.0) c = std::nextafter(1.0, 0.0);
    return (b - a) * c + a;
}

// The per-iteration random decisions of HybridLOMSAC::EstimateModel:
// SelectMinimalSolver (src/hybrid_ransac.h:210-243, selection/LO stream `sel`) then
// HybridUniformSampling::Sample (RansacLib, sampler stream `samp`): for each data
// type t, ss[s][t] distinct draws of uniform_int(0, n-1), redrawing duplicates.
// Only the indices of the type the solver consumes are kept (type 0 for the MD
// solver, type 2 for the point solver); the type-1 draws of an MD iteration are
// consumed and discarded exactly as in the reference.
struct IterationStream {
    Mt19937 sel, samp;
    double prior[2] = {1.0, 1.0};
    int ss[2][3] = {{3, 3, 0}, {0, 0, 5}};
    int n = 0;
    UniformIndex pick;

    void seed(uint32_t s) {
        sel.seed_with(s);
        samp.seed_with(s);
    }
    // K distinct draws into out (redrawing duplicates)
    template <int K> inline void distinct(int *out) {
        for (int i = 0; i < K; ++i) {
            int v;
            bool dup;
            do {
                v = pick(samp);
                dup = false;
                for (int j = 0; j < i; ++j) dup |= out[j] == v;
            } while (dup);
            out[i] = v;
        }
    }
    inline void distinct(int k, int *out) {
        switch (k) {
        case 3: distinct<3>(out); break;
        case 4: distinct<4>(out); break;
        case 5: distinct<5>(out); break;
        case 6: distinct<6>(out); break;
        case 7: distinct<7>(out); break;
        default:
            for (int i = 0; i < k; ++i) {
                int v;
                bool dup;
                do {
                    v = pick(samp);
                    dup = false;
                    for (int j = 0; j < i; ++j) dup |= out[j] == v;
                } while (dup);
                out[i] = v;
            }
        }
    }
    // Fast path of one iteration's sample: the next A + B (MD: two groups) or A
    // (point: one group) buffered outputs, taken when none of them would be
    // redrawn -- no Lemire rejection, no duplicate within a group -- which is what
    // the draw-by-draw code does in that case.  False: nothing consumed.
    template <int A, int B> inline bool fast_groups(int *idx) {
        const uint32_t *w = samp.window(A + B);
        if (!w) return false;
        int v[A + B];
        bool bad = false;
#pragma unroll
        for (int k = 0; k < A + B; ++k) {
            const uint64_t prod = (uint64_t)w[k] * (uint64_t)pick.range;
            bad |= (uint32_t)prod < pick.threshold;
            v[k] = (int)(uint32_t)(prod >> 32);
        }
#pragma unroll
        for (int i = 1; i < A; ++i)
#pragma unroll
            for (int j = 0; j < i; ++j) bad |= v[i] == v[j];
#pragma unroll
        for (int i = A + 1; i < A + B; ++i)
#pragma unroll
            for (int j = A; j < i; ++j) bad |= v[i] == v[j];
        if (bad) return false;
#pragma unroll
        for (int k = 0; k < A; ++k) idx[k] = v[k];
        samp.skip(A + B);
        return true;
    }
    inline bool fast_sample(int st, int *idx) {
        const int *g = ss[st];
        if (st == 0 && g[2] == 0) {
            if (g[0] == 3 && g[1] == 3) return fast_groups<3, 3>(idx);
            if (g[0] == 4 && g[1] == 4) return fast_groups<4, 4>(idx);
        } else if (st == 1 && g[0] == 0 && g[1] == 0) {
            if (g[2] == 5) return fast_groups<5, 0>(idx);
            if (g[2] == 6) return fast_groups<6, 0>(idx);
            if (g[2] == 7) return fast_groups<7, 0>(idx);
        }
        return false;
    }
    int next(int *idx) {
        const double u = uniform_real(sel, 0.0, prior[0] + prior[1]);
        int st = -1;
        double acc = 0.0;
        for (int s = 0; s < 2; ++s) {
            if (prior[s] == 0.0) continue;
            acc += prior[s];
            if (u <= acc) {
                st = s;
                break;
            }
        }
        if (st < 0) st = prior[1] > 0 ? 1 : 0; // unreachable: u < prior sum
        if (pick.range != (uint32_t)n) pick.set((uint32_t)n);
        if (fast_sample(st, idx)) return st;
        int tmp[8];
        for (int t = 0; t < 3; ++t) {
            const int k = ss[st][t];
            if (k == 0) continue;
            const bool keep = (st == 0 && t == 0) || (st == 1 && t == 2);
            distinct(k, keep ? idx : tmp);
        }
        return st;
    }
};

} // namespace mp
