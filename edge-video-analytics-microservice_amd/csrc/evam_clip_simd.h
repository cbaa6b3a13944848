// evam_clip_simd.h — host-only: pass 1 of evam_pp_run (ROI clipping, evam_geom.h's roi_clip) eight ROIs at a
// time on AVX2. Shared by libevam_pp.so and the ASan/UBSan harness tests/native/planner_check.cpp, which checks
// it against roi_clip on random and edge-case ROI sets.
#pragma once
#include <immintrin.h>
#include <stdint.h>

#include <algorithm>

#include "../../include/evam_pp.h"
#include "evam_geom.h"

namespace evam {

// Pass 1 of a call whose ROIs all index sources of one size (the common case: one decoder), eight ROIs per
// step: roi_clip's arithmetic on AVX2 lanes, the (x0, y0, cw, ch) heads of geo[] written by a 4 x 8
// transpose, and the group's max crop size, origin mask and uniformity reduced on the way. Items it does not
// cover exactly — full-frame (w or h <= 0), |x|, |y|, w or h beyond 2^20, an out-of-range source, an empty
// clip — return false, and the caller runs the scalar pass (which reports the error or takes the full frame).
// C3's 1,600 ROIs: ~7 -> ~3 us of host time per call.
__attribute__((target("avx2"))) inline bool clip_rois_avx2(const evam_roi* items, int n, int n_srcs, int W, int H, bool even,
                                                  Geom* geo, int& mcw, int& mch, uint32_t& xm, bool& uni) {
    const __m256i idx = _mm256_setr_epi32(0, 5, 10, 15, 20, 25, 30, 35);
    const __m256i vW = _mm256_set1_epi32(W), vH = _mm256_set1_epi32(H), zero = _mm256_setzero_si256();
    const __m256i one = _mm256_set1_epi32(1), v31 = _mm256_set1_epi32(31);
    const __m256i lim = _mm256_set1_epi32(1 << 20), nlim = _mm256_set1_epi32(-(1 << 20)), last = _mm256_set1_epi32(n_srcs - 1);
    const __m256i msk = _mm256_set1_epi32(even ? ~1 : ~0), up = even ? one : zero;
    __m256i bad = zero, a = zero, b = zero, m = zero;
    int i = 0;
    for (; i + 8 <= n; i += 8) {
        const int* base = reinterpret_cast<const int*>(items + i);
        const __m256i si = _mm256_i32gather_epi32(base, idx, 4);
        const __m256i x = _mm256_i32gather_epi32(base + 1, idx, 4);
        const __m256i y = _mm256_i32gather_epi32(base + 2, idx, 4);
        const __m256i w = _mm256_i32gather_epi32(base + 3, idx, 4);
        const __m256i h = _mm256_i32gather_epi32(base + 4, idx, 4);
        bad = _mm256_or_si256(bad, _mm256_or_si256(_mm256_cmpgt_epi32(zero, si), _mm256_cmpgt_epi32(si, last)));
        bad = _mm256_or_si256(bad, _mm256_or_si256(_mm256_cmpgt_epi32(one, w), _mm256_cmpgt_epi32(one, h)));
        bad = _mm256_or_si256(bad, _mm256_or_si256(_mm256_cmpgt_epi32(w, lim), _mm256_cmpgt_epi32(h, lim)));
        bad = _mm256_or_si256(bad, _mm256_or_si256(_mm256_cmpgt_epi32(x, lim), _mm256_cmpgt_epi32(nlim, x)));
        bad = _mm256_or_si256(bad, _mm256_or_si256(_mm256_cmpgt_epi32(y, lim), _mm256_cmpgt_epi32(nlim, y)));
        // within those bounds x + w and y + h are exact in 32 bits
        const __m256i x0 = _mm256_and_si256(_mm256_min_epi32(_mm256_max_epi32(x, zero), vW), msk);
        const __m256i y0 = _mm256_and_si256(_mm256_min_epi32(_mm256_max_epi32(y, zero), vH), msk);
        __m256i x1 = _mm256_min_epi32(_mm256_max_epi32(_mm256_add_epi32(x, w), zero), vW);
        __m256i y1 = _mm256_min_epi32(_mm256_max_epi32(_mm256_add_epi32(y, h), zero), vH);
        x1 = _mm256_min_epi32(_mm256_and_si256(_mm256_add_epi32(x1, up), msk), vW);
        y1 = _mm256_min_epi32(_mm256_and_si256(_mm256_add_epi32(y1, up), msk), vH);
        const __m256i cw = _mm256_sub_epi32(x1, x0), ch = _mm256_sub_epi32(y1, y0);
        bad = _mm256_or_si256(bad, _mm256_or_si256(_mm256_cmpgt_epi32(one, cw), _mm256_cmpgt_epi32(one, ch)));
        a = _mm256_max_epi32(a, cw);
        b = _mm256_max_epi32(b, ch);
        m = _mm256_or_si256(m, _mm256_sllv_epi32(one, _mm256_and_si256(x0, v31)));
        const __m256i t0 = _mm256_unpacklo_epi32(x0, y0), t1 = _mm256_unpackhi_epi32(x0, y0);
        const __m256i t2 = _mm256_unpacklo_epi32(cw, ch), t3 = _mm256_unpackhi_epi32(cw, ch);
        const __m256i g0 = _mm256_unpacklo_epi64(t0, t2), g1 = _mm256_unpackhi_epi64(t0, t2);
        const __m256i g2 = _mm256_unpacklo_epi64(t1, t3), g3 = _mm256_unpackhi_epi64(t1, t3);
        Geom* g = geo + i;
        _mm_storeu_si128(reinterpret_cast<__m128i*>(&g[0]), _mm256_castsi256_si128(g0));
        _mm_storeu_si128(reinterpret_cast<__m128i*>(&g[1]), _mm256_castsi256_si128(g1));
        _mm_storeu_si128(reinterpret_cast<__m128i*>(&g[2]), _mm256_castsi256_si128(g2));
        _mm_storeu_si128(reinterpret_cast<__m128i*>(&g[3]), _mm256_castsi256_si128(g3));
        _mm_storeu_si128(reinterpret_cast<__m128i*>(&g[4]), _mm256_extracti128_si256(g0, 1));
        _mm_storeu_si128(reinterpret_cast<__m128i*>(&g[5]), _mm256_extracti128_si256(g1, 1));
        _mm_storeu_si128(reinterpret_cast<__m128i*>(&g[6]), _mm256_extracti128_si256(g2, 1));
        _mm_storeu_si128(reinterpret_cast<__m128i*>(&g[7]), _mm256_extracti128_si256(g3, 1));
    }
    if (!_mm256_testz_si256(bad, bad)) return false;
    alignas(32) int A[8], B[8], M[8];
    _mm256_store_si256(reinterpret_cast<__m256i*>(A), a);
    _mm256_store_si256(reinterpret_cast<__m256i*>(B), b);
    _mm256_store_si256(reinterpret_cast<__m256i*>(M), m);
    int ra = 0, rb = 0;
    uint32_t rm = 0;
    for (int k = 0; k < 8; k++) { ra = std::max(ra, A[k]); rb = std::max(rb, B[k]); rm |= (uint32_t)M[k]; }
    const int f = even ? kNV12 : kBGRX;  // roi_clip widens 4:2:0 formats only
    for (; i < n; i++) {  // the last n % 8 items
        const evam_roi& r = items[i];
        if ((unsigned)r.src_index >= (unsigned)n_srcs || r.w <= 0 || r.h <= 0) return false;
        if (roi_clip(f, W, H, true, r.x, r.y, r.w, r.h, geo[i])) return false;
        ra = std::max(ra, geo[i].cw); rb = std::max(rb, geo[i].ch); rm |= 1u << (geo[i].x0 & 31);
    }
    uint32_t neq = 0;
    const int cw0 = geo[0].cw, ch0 = geo[0].ch;
    for (int k = 0; k < n; k++) neq |= (uint32_t)(geo[k].cw ^ cw0) | (uint32_t)(geo[k].ch ^ ch0);
    mcw = ra; mch = rb; xm = rm; uni = neq == 0;
    return true;
}

}  // namespace evam
