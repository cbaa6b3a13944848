// planner_check.cpp — host-only checks of the planner arithmetic libevam_pp.so shares with its kernels
// (edge-video-analytics-microservice_amd/csrc/evam_geom.h), built and run under AddressSanitizer +
// UBSan by tests/test_native_asan.py, together with the C oracle (oracle/evam_oracle.c) exercised on
// tightly allocated frames so any out-of-bounds read in it is caught too.
//
// TEST INFRASTRUCTURE ONLY: links the oracle as the checker of the geometry rules.
//
// Every check draws its cases from a fixed-seed generator; a failure prints the case and exits 1.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <vector>

#include "../../edge-video-analytics-microservice_amd/csrc/evam_geom.h"
#include "../../edge-video-analytics-microservice_amd/csrc/evam_clip_simd.h"

extern "C" {
typedef struct { int x0, y0, cw, ch, rw, rh, ox, oy; } orc_geom;
int orc_item_geometry(int fourcc, int W, int H, int x, int y, int w, int h, int mode, int placement, int DW,
                      int DH, orc_geom* g);
void orc_linear_table(int ssize, int dsize, int is_x, int32_t* ofs, int16_t* c0, int16_t* c1);
int orc_preprocess_item(int fourcc, const uint8_t* const planes[3], const int pitch[3], int W, int H, int x, int y,
                        int w, int h, int mode, int placement, int color_rgb, int out_f32, const float* lut,
                        const uint8_t fill[3], void* dst, int slot, int DW, int DH, int32_t* geom_out);
void orc_norm_lut(int norm_flags, const float range[2], const float mean[3], const float std_[3], float* lut);
}

using namespace evam;

static const int kFourcc[4] = {EVAM_FOURCC_NV12, EVAM_FOURCC_I420, EVAM_FOURCC_BGRX, EVAM_FOURCC_BGR};
static std::mt19937_64 rng(20261016);
static int uni(int lo, int hi) { return std::uniform_int_distribution<int>(lo, hi)(rng); }
static int failures = 0;

#define CHECK(cond, ...)                                                       \
    do {                                                                       \
        if (!(cond)) {                                                         \
            fprintf(stderr, "FAIL %s:%d: %s | ", __FILE__, __LINE__, #cond);   \
            fprintf(stderr, __VA_ARGS__);                                      \
            fprintf(stderr, "\n");                                             \
            if (++failures > 20) exit(1);                                      \
        }                                                                      \
    } while (0)

// A rect drawn from the interesting classes: inside, straddling, outside, degenerate, int32 extremes.
static void random_rect(int W, int H, int& x, int& y, int& w, int& h) {
    switch (uni(0, 9)) {
    case 0: x = uni(INT32_MIN / 2, INT32_MAX); y = uni(INT32_MIN / 2, INT32_MAX); w = uni(-5, INT32_MAX); h = uni(-5, INT32_MAX); break;
    case 1: x = INT32_MAX - uni(0, 3); y = uni(0, H); w = INT32_MAX; h = uni(1, 50); break;
    case 2: x = uni(-3 * W, 3 * W); y = uni(-3 * H, 3 * H); w = uni(-2, 4 * W); h = uni(-2, 4 * H); break;
    case 3: x = uni(0, W); y = uni(0, H); w = 0; h = uni(-3, 3); break;
    default: x = uni(-20, W); y = uni(-20, H); w = uni(1, W + 40); h = uni(1, H + 40); break;
    }
}

static void check_geometry() {
    int n = 0, empty = 0;
    for (int it = 0; it < 200000; it++) {
        const int f = uni(0, 3);
        const bool yuv = f == kNV12 || f == kI420;
        int W = uni(1, 5000), H = uni(1, 3000);
        if (yuv) { W = (W + 1) & ~1; H = (H + 1) & ~1; }
        int x, y, w, h;
        random_rect(W, H, x, y, w, h);
        const int mode = uni(0, 2), placement = uni(0, 1), DW = uni(1, 1024), DH = uni(1, 1024);
        const bool has = uni(0, 7) != 0;
        Geom g{};
        orc_geom o{};
        const int rc = roi_geometry(f, W, H, has, x, y, w, h, mode, placement, DW, DH, g);
        const int ro = orc_item_geometry(kFourcc[f], W, H, has ? x : 0, has ? y : 0, has ? w : 0, has ? h : 0, mode,
                                         placement, DW, DH, &o);
        CHECK((rc != 0) == (ro != 0), "f=%d %dx%d rect(%d,%d,%d,%d) rc %d oracle %d", f, W, H, x, y, w, h, rc, ro);
        if (rc || ro) { empty++; continue; }
        n++;
        CHECK(memcmp(&g, &o, sizeof(g)) == 0, "f=%d %dx%d rect(%d,%d,%d,%d) mode %d: (%d %d %d %d %d %d %d %d) vs oracle "
              "(%d %d %d %d %d %d %d %d)", f, W, H, x, y, w, h, mode, g.x0, g.y0, g.cw, g.ch, g.rw, g.rh, g.ox, g.oy,
              o.x0, o.y0, o.cw, o.ch, o.rw, o.rh, o.ox, o.oy);
        CHECK(g.x0 >= 0 && g.y0 >= 0 && g.x0 + g.cw <= W && g.y0 + g.ch <= H && g.cw > 0 && g.ch > 0,
              "crop outside the frame");
        if (yuv) CHECK(!((g.x0 | g.y0) & 1), "4:2:0 crop origin odd");
    }
    printf("geometry: %d clipped rects equal to the oracle's, %d empty agreed\n", n, empty);
}

static void check_linear_tables() {
    std::vector<int32_t> ofs;
    std::vector<int16_t> c0, c1;
    for (int it = 0; it < 3000; it++) {
        const int ss = uni(1, 4000), ds = uni(1, 2000), is_x = uni(0, 1);
        ofs.resize(ds); c0.resize(ds); c1.resize(ds);
        orc_linear_table(ss, ds, is_x, ofs.data(), c0.data(), c1.data());
        const double scale = 1. / ((double)ds / ss);
        for (int d = 0; d < ds; d++) {
            int s, a, b;
            linear_coef(d, scale, ss, is_x != 0, s, a, b);
            CHECK(s == ofs[d] && a == c0[d] && b == c1[d], "%d->%d x=%d d=%d: (%d,%d,%d) vs (%d,%d,%d)", ss, ds, is_x, d,
                  s, a, b, ofs[d], c0[d], c1[d]);
            if (is_x) CHECK(s >= 0 && s <= ss - 1, "x tap outside the row");
        }
    }
    printf("linear tables: 3000 axes equal to the oracle's\n");
}

// The ROI kernel stages, per output row, the footprint item_footprint gives; it must cover every tap of
// every visible column and be the minimal 16-byte-aligned window; the host sizes its LDS buffer with
// row_bytes_bound, which must bound the staged bytes.
static void check_footprints() {
    for (int it = 0; it < 20000; it++) {
        const int f = uni(0, 3), bpp = fmt_bpp(f);
        const bool yuv = f == kNV12 || f == kI420;
        int W = uni(2, 2000) & ~1, H = uni(2, 1200) & ~1;
        int x, y, w, h;
        random_rect(W, H, x, y, w, h);
        const int mode = uni(0, 2), DW = uni(1, 600), DH = uni(1, 400);
        Geom g{};
        if (roi_geometry(f, W, H, true, x, y, w, h, mode, uni(0, 1), DW, DH, g)) continue;
        const double scx = 1. / ((double)g.rw / g.cw);
        int fsY, nY, fsC, nC;
        item_footprint(f, bpp, g.x0, g.cw, g.rw, g.ox, scx, DW, fsY, nY, fsC, nC);
        int lo = INT32_MAX, hi = -1;
        for (int X = std::max(0, g.ox); X < std::min(DW, g.ox + g.rw); X++) {
            int s, a, b;
            linear_coef(X - g.ox, scx, g.cw, true, s, a, b);
            lo = std::min(lo, g.x0 + s);
            hi = std::max(hi, g.x0 + std::min(s + 1, g.cw - 1));
        }
        if (hi < 0) { CHECK(nY == 0, "no visible column but a footprint"); continue; }
        CHECK(fsY == ((lo * bpp) & ~15) && fsY + 16 * nY == ((hi * bpp + bpp + 15) & ~15), "luma window");
        CHECK(fsY + 16 * nY <= ((W * bpp + 15) & ~15), "luma window past the 16-B-rounded row");
        if (yuv) {
            const int clo = f == kNV12 ? 2 * (lo >> 1) : lo >> 1, chi = f == kNV12 ? 2 * (hi >> 1) + 2 : (hi >> 1) + 1;
            CHECK(fsC <= clo && fsC + 16 * nC >= chi && fsC + 16 > clo && fsC + 16 * (nC - 1) < chi, "chroma window");
        }
        const int NP = fmt_nplanes(f);
        CHECK(2 * 16 * nY + 2 * (NP - 1) * 16 * nC <= row_bytes_bound(f, g.cw), "row_bytes_bound f=%d cw=%d", f, g.cw);
    }
    printf("footprints: 20000 ROI windows minimal, covering, and within row_bytes_bound\n");
}

// a uniform group's wave-kernel segments must hold every item's footprint, whatever the
// item's crop origin. Check wave_segments against each item's own per-tile chunk counts.
static void check_wave_segments() {
    int groups = 0, misaligned_needs_more = 0;
    std::vector<XTab> xt;
    std::vector<YTab> yt;
    for (int it = 0; it < 3000; it++) {
        const int f = uni(0, 3), bpp = fmt_bpp(f);
        const bool yuv = f == kNV12 || f == kI420;
        const int W = 1920, H = 1080;
        int cw = uni(2, 900), ch = uni(2, 600);
        if (yuv) { cw &= ~1; ch &= ~1; cw = std::max(cw, 2); ch = std::max(ch, 2); }
        const int DW = uni(1, 700), DH = uni(1, 300), mode = uni(0, 2), placement = uni(0, 1);
        const int n = uni(1, 40);
        std::vector<int> x0(n);
        uint32_t mask = 0;
        for (int k = 0; k < n; k++) {
            x0[k] = uni(0, W - cw);
            if (yuv) x0[k] &= ~1;
            mask |= 1u << (x0[k] & 31);
        }
        Geom g{};
        if (roi_geometry(f, W, H, true, x0[0], 0, cw, ch, mode, placement, DW, DH, g)) continue;
        xt.resize(DW); yt.resize(DH);
        build_tables_into(g, DW, DH, xt.data(), yt.data());
        for (int tw : {64, 128, 256}) {
            int mY, mC, rY, rC;
            wave_segments(f, g.ox, g.rw, DW, xt.data(), mask, tw, mY, mC);
            wave_segments(f, g.ox, g.rw, DW, xt.data(), 1u << (x0[0] & 31), tw, rY, rC);
            bool more = false;
            for (int k = 0; k < n; k++)
                for (int X0 = 0; X0 < DW; X0 += tw) {
                    const int Xv0 = std::max(X0, g.ox), Xv1 = std::min(std::min(X0 + tw, DW), g.ox + g.rw) - 1;
                    if (Xv0 > Xv1) continue;
                    int fsY, nY, fsC, nC;
                    footprint_chunks(f, bpp, x0[k] + xt[Xv0].s0, x0[k] + xt[Xv1].s1, fsY, nY, fsC, nC);
                    CHECK(nY <= mY && nC <= mC, "f=%d cw=%d x0=%d tile %d: (%d,%d) > segments (%d,%d)", f, cw, x0[k], X0,
                          nY, nC, mY, mC);
                    more |= nY > rY || nC > rC;
                }
            misaligned_needs_more += more;
        }
        groups++;
    }
    printf("wave segments: %d uniform groups covered; %d tile widths where the first item's origin alone would "
           "under-size the staging (the r1 bug)\n", groups, misaligned_needs_more);
    CHECK(misaligned_needs_more > 0, "the generator never produced the misaligned case");
}

static void check_bytes_and_order() {
    Geom g{};
    CHECK(roi_geometry(kNV12, 1920, 1080, false, 0, 0, 0, 0, EVAM_RESIZE_NO_ASPECT, 0, 512, 512, g) == 0, "C2 geometry");
    CHECK(item_src_bytes(kNV12, g, 512, 512) == 3002880, "C2 algorithmic source bytes %lld",
          (long long)item_src_bytes(kNV12, g, 512, 512));
    CHECK(roi_geometry(kNV12, 3840, 2160, false, 0, 0, 0, 0, EVAM_RESIZE_ASPECT, 0, 640, 640, g) == 0, "C4 geometry");
    CHECK(g.rw == 640 && g.rh == 360, "C4 letterbox size");
    for (int it = 0; it < 500; it++) {
        const int n = uni(1, 2000), DH = uni(1, 300);
        std::vector<Geom> geo(n);
        std::vector<int> idx(n), bucket(n);
        for (int i = 0; i < n; i++) {
            geo[i] = Geom{0, 0, uni(1, 4000), uni(1, 3000), 1, 1, 0, 0};
            idx[i] = n - 1 - i;
        }
        std::vector<int> ord;
        roi_largest_first(idx.data(), n, geo.data(), DH, it % 5 != 0, bucket.data(), ord);
        std::vector<int> seen(n, 0);
        CHECK((int)ord.size() == n, "order size");
        for (int p = 0; p < n; p++) {
            seen[ord[p]]++;
            if (p) CHECK(bucket[ord[p - 1]] <= bucket[ord[p]], "not largest first");
        }
        for (int i = 0; i < n; i++) CHECK(seen[i] == 1, "not a permutation");
    }
    printf("algorithmic bytes KAT (C2 3,002,880) and ROI launch order checked\n");
}

// The oracle under ASan: frames allocated to exactly rows x pitch bytes, random crops / modes / formats.
static void check_oracle_bounds() {
    float lut[768];
    const float range[2] = {0.f, 1.f}, mean[3] = {0.1f, 0.2f, 0.3f}, sd[3] = {0.3f, 0.2f, 0.1f};
    orc_norm_lut(3, range, mean, sd, lut);
    int runs = 0;
    for (int it = 0; it < 400; it++) {
        const int f = uni(0, 3), bpp = fmt_bpp(f);
        const bool yuv = f == kNV12 || f == kI420;
        int W = uni(2, 200), H = uni(2, 120);
        if (yuv) { W &= ~1; H &= ~1; }
        const int np = fmt_nplanes(f);
        std::vector<std::vector<uint8_t>> pl(np);
        const uint8_t* planes[3] = {nullptr, nullptr, nullptr};
        int pitch[3] = {0, 0, 0};
        for (int p = 0; p < np; p++) {
            const int rb = p == 0 ? W * bpp : (f == kNV12 ? W : W / 2);
            const int rows = p == 0 ? H : H / 2;
            pitch[p] = rb + uni(0, 1) * 16;
            pl[p].resize((size_t)pitch[p] * rows);
            for (auto& b : pl[p]) b = (uint8_t)uni(0, 255);
            planes[p] = pl[p].data();
        }
        int x, y, w, h;
        random_rect(W, H, x, y, w, h);
        const int mode = uni(0, 2), DW = uni(1, 96), DH = uni(1, 96), f32 = uni(0, 1);
        std::vector<uint8_t> out((size_t)3 * DW * DH * (f32 ? 4 : 1));
        const uint8_t fill[3] = {1, 2, 3};
        int32_t geom[8];
        const int rc = orc_preprocess_item(kFourcc[f], planes, pitch, W, H, x, y, w, h, mode, uni(0, 1), uni(0, 1),
                                           f32, f32 ? lut : nullptr, fill, out.data(), 0, DW, DH, geom);
        runs += rc == 0;
    }
    printf("oracle: %d random items pre-processed on tight allocations\n", runs);
}

// ROI tail split: the C3 case, fewer ROIs than CUs, an even split, and for random sizes: the units never exceed the
// resident slots, the split ROIs are the tail beyond a whole number per CU, and the row tiles cover [0, DH) exactly.
static void check_roi_tail() {
    int ns = -1;
    CHECK(roi_tail_tiles(1600, 256, 1792, 4, 72, ns) == 4 && ns == 64, "tail split n=%d", ns);
    CHECK(roi_tail_tiles(1536, 256, 1792, 4, 72, ns) == 1 && ns == 0, "tail split n=%d", ns);
    CHECK(roi_tail_tiles(40, 256, 1792, 4, 72, ns) == 4 && ns == 40, "tail split n=%d", ns);
    CHECK(roi_tail_tiles(1600, 256, 1792, 1, 72, ns) == 1 && ns == 0, "tail split n=%d", ns);
    CHECK(roi_tail_tiles(1700, 256, 1792, 4, 72, ns) == 1 && ns == 0, "tail split n=%d", ns);  // 1536 + 164 x 2 > 1792: no room
    CHECK(roi_tail_tiles(10, 256, 1792, 7, 3, ns) == 3 && ns == 10, "tail split n=%d", ns);      // at most DH tiles
    for (int it = 0; it < 20000; it++) {
        const int n_cu = uni(1, 300), per = uni(1, 8), n = uni(1, 3000);
        const int64_t slots = (int64_t)n_cu * per;
        const int DH = uni(1, 100), rt = uni(0, 8);
        const int ts = roi_tail_tiles(n, n_cu, slots, rt, DH, ns);
        CHECK(ts >= 1 && ts <= std::max(1, std::min(rt, DH)), "tail split n=%d", ns);
        CHECK(ns == (ts > 1 ? n % n_cu : 0), "tail split n=%d", ns);
        if (ts > 1) CHECK((int64_t)n + (int64_t)ns * (ts - 1) <= slots, "tail split n=%d", ns);
        int covered = 0, prev = 0;
        for (int t = 0; t < ts; t++) {
            const int y0 = DH * t / ts, y1 = DH * (t + 1) / ts;
            CHECK(y0 == prev && y1 > y0, "tail split n=%d", ns);
            covered += y1 - y0;
            prev = y1;
        }
        CHECK(covered == DH, "tail split n=%d", ns);
    }
}

// Pass 1 on AVX2 (csrc/evam_clip_simd.h) against roi_clip item by item: the same (x0, y0, cw, ch) and reductions
// when it accepts a set, and a refusal (the scalar pass then runs) whenever any item is one it does not cover:
// full-frame, out-of-range source, empty clip, or a coordinate beyond 2^20.
static void check_clip_simd() {
    if (!__builtin_cpu_supports("avx2")) {
        printf("clip_simd: no AVX2 on this CPU, skipped\n");
        return;
    }
    int accepted = 0, refused = 0;
    for (int it = 0; it < 4000; it++) {
        const int f = uni(0, 3);
        const bool even = f == kNV12 || f == kI420;
        int W = uni(1, 5000), H = uni(1, 3000);
        if (even) { W = (W + 1) & ~1; H = (H + 1) & ~1; }
        const int n = uni(8, 300), n_srcs = uni(1, 40);
        const int mix = uni(0, 3);  // 0: plain ROIs only; else a few drawn from every class
        std::vector<evam_roi> r(n);
        bool cover = true;
        for (int i = 0; i < n; i++) {
            int x, y, w, h;
            if (mix == 0 || uni(0, 40) != 0) { w = uni(1, W); h = uni(1, H); x = uni(-8, W - 1); y = uni(-8, H - 1); }
            else random_rect(W, H, x, y, w, h);
            if (uni(0, 2) == 0 && i == 0) { w = W; h = H; x = 0; y = 0; }  // uniform sets too
            r[i] = {uni(0, 200) == 0 && mix ? n_srcs : uni(0, n_srcs - 1), x, y, w, h};
            if (it % 7 == 0) r[i] = r[0];
        }
        std::vector<Geom> a(n), b(n);
        int mcw = -1, mch = -1;
        uint32_t xm = 0;
        bool un = false;
        const bool ok = clip_rois_avx2(r.data(), n, n_srcs, W, H, even, a.data(), mcw, mch, xm, un);
        int emcw = 0, emch = 0;
        uint32_t exm = 0;
        bool eun = true;
        for (int i = 0; i < n; i++) {
            const evam_roi& q = r[i];
            const bool in = (unsigned)q.src_index < (unsigned)n_srcs && q.w > 0 && q.h > 0 && q.w <= (1 << 20) &&
                            q.h <= (1 << 20) && q.x >= -(1 << 20) && q.x <= (1 << 20) && q.y >= -(1 << 20) &&
                            q.y <= (1 << 20);
            if (!in || roi_clip(f, W, H, true, q.x, q.y, q.w, q.h, b[i])) { cover = false; continue; }
            emcw = std::max(emcw, b[i].cw); emch = std::max(emch, b[i].ch); exm |= 1u << (b[i].x0 & 31);
            eun &= b[i].cw == b[0].cw && b[i].ch == b[0].ch;
        }
        CHECK(ok == cover, "clip_simd it %d: accepted %d, scalar coverage %d", it, ok, cover);
        if (!ok || !cover) { refused++; continue; }
        accepted++;
        for (int i = 0; i < n; i++)
            CHECK(a[i].x0 == b[i].x0 && a[i].y0 == b[i].y0 && a[i].cw == b[i].cw && a[i].ch == b[i].ch,
                  "clip_simd it %d item %d rect(%d,%d,%d,%d) in %dx%d: (%d %d %d %d) vs (%d %d %d %d)", it, i, r[i].x,
                  r[i].y, r[i].w, r[i].h, W, H, a[i].x0, a[i].y0, a[i].cw, a[i].ch, b[i].x0, b[i].y0, b[i].cw, b[i].ch);
        CHECK(mcw == emcw && mch == emch && xm == exm && un == eun, "clip_simd it %d reductions", it);
    }
    printf("clip_simd: %d ROI sets equal to roi_clip, %d refused as the scalar pass would handle them\n", accepted,
           refused);
}



// band_six_columns admits a column table only if the band kernel's six-column lanes (DD) read, for every visible
// pixel, the luma and chroma columns the per-pixel taps name: px 0 (c0, c1), 1 (c1, c2), 2 (c3, c4), 3 (c4, c5),
// chroma of c0 / c1 from c0, of c2 / c3 from c2, of c4 / c5 from c4, for every even crop origin.
static void check_six_columns() {
    int admitted = 0, c1_ok = 0;
    for (int it = 0; it < 4000; it++) {
        Geom g{};
        const int DW = it == 0 ? 512 : 4 * uni(1, 200);
        g.cw = it == 0 ? 768 : (it % 3 == 0 ? 3 * uni(1, 300) : uni(2, 2000));
        g.rw = it == 0 ? DW : (it % 3 == 0 ? std::min(DW, 2 * (g.cw / 3)) : uni(1, DW));
        if (g.rw < 1) g.rw = 1;
        g.ox = it % 5 == 0 ? 4 * uni(0, (DW - g.rw) / 4) : uni(0, DW - g.rw);
        g.ch = g.rh = 8;
        std::vector<XTab> xt(DW);
        std::vector<YTab> yt(8);
        build_tables_into(g, DW, 8, xt.data(), yt.data());
        const uint32_t x0_mask = it % 7 == 1 ? 0x6u : 0x1u;  // origins 1, 2 (odd: never admitted) or 0
        const bool ok = band_six_columns(xt.data(), DW, x0_mask);
        if (x0_mask & 0xAAAAAAAAu) CHECK(!ok, "odd crop origin admitted");
        if (it == 0) c1_ok = ok;
        if (!ok) continue;
        admitted++;
        for (int X = 0; X < DW; X += 4) {
            const XTab* e = &xt[X];
            if (!((e[0].a0 | e[0].a1) || (e[1].a0 | e[1].a1) || (e[2].a0 | e[2].a1) || (e[3].a0 | e[3].a1))) continue;
            const int c[6] = {e[0].s0, e[0].s1, e[1].s1, e[2].s0, e[2].s1, e[3].s1};
            const int tap[4][2] = {{0, 1}, {1, 2}, {3, 4}, {4, 5}};
            for (int x0 : {0, 2, 6, 30}) {
                auto chroma = [&](int s) { return (x0 + s) >> 1; };
                for (int j = 0; j < 4; j++) {
                    CHECK((e[j].a0 | e[j].a1) != 0, "partly visible lane admitted (X=%d)", X + j);
                    CHECK(c[tap[j][0]] == e[j].s0 && c[tap[j][1]] == e[j].s1, "cw %d rw %d ox %d DW %d X %d: luma taps",
                          g.cw, g.rw, g.ox, DW, X + j);
                    for (int t = 0; t < 2; t++) {
                        const int k = tap[j][t];
                        CHECK(chroma(c[k & ~1]) == chroma(t ? e[j].s1 : e[j].s0), "cw %d rw %d X %d: chroma tap",
                              g.cw, g.rw, X + j);
                    }
                }
            }
        }
    }
    CHECK(c1_ok, "C1 (768 -> 512) not admitted");
    printf("six-column lanes: %d of 4000 tables admitted, every admitted lane exact\n", admitted);
}

// The fused four-pass ROI launch order (roi_launch_order, evam_pp_run since round 6) against the multi-pass plan it
// replaced, restated here: roi_largest_first, one unit per ROI in that order with the tail split's row tiles for the
// last nsplit, a stable counting sort of the units by row groups (largest first), then the snake deal. Same units at
// the same positions, for the C3 shape and random groups (sorted or call order, snake on or off, odd CU counts).
static void check_roi_launch_order() {
    struct U { int item, r0, r1; bool operator==(const U& o) const { return item == o.item && r0 == o.r0 && r1 == o.r1; } };
    int cases = 0;
    for (int it = 0; it < 3000; it++) {
        const bool c3 = it < 50;
        const int f = c3 ? kNV12 : uni(0, 3);
        const int n = c3 ? 1600 : uni(1, 2500), DH = c3 ? 72 : uni(1, 200);
        const int n_cu = c3 ? 256 : (it % 3 ? 256 : uni(1, 300));
        const int64_t slots = c3 ? 1792 : (int64_t)n_cu * uni(1, 8);
        const int roi_tail = c3 ? 4 : uni(0, 8), buf = c3 ? 12 * 1024 : uni(1, 32) * 512;
        const int rcap = c3 ? 42 : uni(1, 64);
        const bool sort = c3 || it % 7 != 0, snake = c3 || it % 5 != 0;
        std::vector<Geom> geo(n);
        std::vector<int> idx(n);
        for (int i = 0; i < n; i++) {
            geo[i] = Geom{0, 0, c3 ? uni(24, 400) & ~1 : uni(1, 3000), c3 ? uni(24, 300) & ~1 : uni(1, 2000), 1, 1, 0, 0};
            idx[i] = i;
        }
        auto rg = [&](int cw) {
            const int R = std::max(1, std::min(std::min(buf / row_bytes_bound(f, cw), rcap), DH));
            return (uint32_t)R | ((uint32_t)((DH + R - 1) / R) << 16);
        };
        // the multi-pass reference
        std::vector<int> bucket(n), ord;
        roi_largest_first(idx.data(), n, geo.data(), DH, sort, bucket.data(), ord);
        int nsplit = 0;
        const int ts = roi_tail_tiles(n, n_cu, slots, roi_tail, DH, nsplit);
        std::vector<U> un;
        std::vector<int> cost;
        for (int p = 0; p < n; p++) {
            const int i = ord[p];
            const uint32_t e = rg(geo[i].cw);
            if (p < n - nsplit) {
                un.push_back({i, 0, DH});
                cost.push_back((int)(e >> 16));
                continue;
            }
            const int R = (int)(e & 0xFFFF);
            for (int t = 0; t < ts; t++) {
                const int y0 = DH * t / ts, y1 = DH * (t + 1) / ts;
                un.push_back({i, y0, y1});
                cost.push_back((y1 - y0 + R - 1) / R);
            }
        }
        std::vector<int> order(un.size());
        for (size_t u = 0; u < un.size(); u++) order[u] = (int)u;
        std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return cost[a] > cost[b]; });
        const int nu = (int)order.size(), band = std::max(1, n_cu);
        if (snake)
            for (int b0 = band; b0 < nu; b0 += 2 * band) std::reverse(order.begin() + b0, order.begin() + std::min(nu, b0 + band));
        // the fused planner
        std::vector<uint32_t> sc;
        std::vector<U> got(nu, U{-1, -1, -1});
        std::vector<int> hits(nu, 0);
        const int nu2 = roi_launch_order(idx.data(), n, geo.data(), DH, n_cu, slots, roi_tail, sort, snake, rg, sc,
                                         [&](int q, int item, int r0, int r1) {
                                             if (q >= 0 && q < nu) { got[q] = U{item, r0, r1}; hits[q]++; }
                                         });
        CHECK(nu2 == nu, "launch order: %d units, expected %d (case %d)", nu2, nu, it);
        for (int q = 0; q < nu && failures < 20; q++) {
            CHECK(hits[q] == 1, "launch order: position %d written %d times (case %d)", q, hits[q], it);
            const U& w = un[order[q]];
            CHECK(got[q] == w, "launch order case %d pos %d: (%d,%d,%d) expected (%d,%d,%d)", it, q, got[q].item,
                  got[q].r0, got[q].r1, w.item, w.r0, w.r1);
        }
        cases++;
    }
    printf("ROI launch order: fused planner equals the multi-pass plan on %d groups\n", cases);
}

// The frame-to-XCD deal (EVAM_PP_ROI_XCD=1): a permutation of the launch positions; every unit inside the interleave
// (positions below 8 x the smallest XCD's unit count) sits on its frame's XCD (position % 8); the XCDs' summed costs
// differ by at most the largest frame's cost (LPT).
static void check_roi_xcd_deal() {
    int cases = 0;
    for (int it = 0; it < 2000; it++) {
        const int n_frames = uni(1, 64), nu = uni(1, 3000), n_cu = it % 3 ? 256 : 8 * uni(1, 40);
        std::vector<int> frame(nu), cost(nu), pos, scr;
        for (int q = 0; q < nu; q++) { frame[q] = uni(0, n_frames - 1); cost[q] = uni(1, 16); }
        std::sort(cost.begin(), cost.end(), [](int a, int b) { return a > b; });
        roi_xcd_deal(frame.data(), cost.data(), nu, n_frames, n_cu, 8, pos, scr);
        std::vector<int> hit(nu, 0);
        for (int q = 0; q < nu; q++) {
            CHECK(pos[q] >= 0 && pos[q] < nu, "xcd deal: position %d of %d (case %d)", pos[q], nu, it);
            if (pos[q] >= 0 && pos[q] < nu) hit[pos[q]]++;
        }
        for (int p = 0; p < nu; p++) CHECK(hit[p] == 1, "xcd deal: position %d used %d times (case %d)", p, hit[p], it);
        const int* fxcd = scr.data() + n_frames;  // the frame -> XCD map the deal leaves in its scratch
        std::vector<int64_t> cnt(8, 0), load(8, 0), fcost(n_frames, 0);
        for (int q = 0; q < nu; q++) { cnt[fxcd[frame[q]]]++; load[fxcd[frame[q]]] += cost[q]; fcost[frame[q]] += cost[q]; }
        const int64_t n_min = *std::min_element(cnt.begin(), cnt.end());
        for (int q = 0; q < nu; q++)
            if (pos[q] < 8 * n_min) CHECK(pos[q] % 8 == fxcd[frame[q]], "xcd deal: unit %d off its frame's XCD (case %d)", q, it);
        const int64_t spread = *std::max_element(load.begin(), load.end()) - *std::min_element(load.begin(), load.end());
        CHECK(spread <= *std::max_element(fcost.begin(), fcost.end()), "xcd deal: XCD loads spread %lld (case %d)",
              (long long)spread, it);
        cases++;
    }
    printf("ROI XCD deal: %d random unit lists, permutations, frames on their XCDs, LPT-balanced\n", cases);
}

int main() {
    check_six_columns();
    check_clip_simd();
    check_roi_tail();
    check_roi_launch_order();
    check_roi_xcd_deal();
    check_geometry();
    check_linear_tables();
    check_footprints();
    check_wave_segments();
    check_bytes_and_order();
    check_oracle_bounds();
    if (failures) {
        fprintf(stderr, "%d check(s) failed\n", failures);
        return 1;
    }
    printf("planner_check: all checks passed\n");
    return 0;
}
