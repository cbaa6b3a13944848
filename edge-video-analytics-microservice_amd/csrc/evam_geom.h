// evam_geom.h — the integer / IEEE arithmetic shared by the HIP kernels and the host planner of
// libevam_pp.so: OpenCV INTER_LINEAR coefficient entries, ROI clipping and aspect-ratio geometry,
// staged source footprints, LDS staging bounds and the algorithmic byte count (SURVEY.md §8 a2, a5,
// a6, d). Everything here is plain C++ on integers and IEEE doubles/floats, so the device and the
// host compute bit-identical values; tests/native/planner_check.cpp compiles this header for the host
// alone under AddressSanitizer / UBSan (tests/test_native_asan.py).
//
// EVAM_HD marks functions the kernels call too: evam_pp.hip defines it as __host__ __device__ before
// including this header; a host-only build leaves it empty. Translation units that include this
// header must be compiled with -ffp-contract=off (linear_coef is OpenCV's exact float sequence).
#ifndef EVAM_GEOM_H
#define EVAM_GEOM_H

#include <stdint.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include "../../include/evam_pp.h"

#ifndef EVAM_HD
#define EVAM_HD
#endif

namespace evam {

enum FmtId { kNV12 = 0, kI420 = 1, kBGRX = 2, kBGR = 3 };

inline int fmt_bpp(int f) { return f == kBGRX ? 4 : (f == kBGR ? 3 : 1); }
inline int fmt_nplanes(int f) { return f == kNV12 ? 2 : (f == kI420 ? 3 : 1); }

// Row-kernel (uniform geometry) tables, built on the host once per geometry and cached in the
// descriptor block. Indexed by output column X / output row Y of the DW x DH plane.
struct alignas(16) XTab {  // 16 B
    int32_t s0, s1;      // source columns of the two taps, relative to the crop (s1 = min(s0+1, cw-1))
    uint16_t a0, a1;     // 11-bit weights << 4; both 0: column shows padding
    int32_t pad;
};
struct alignas(16) YTab {  // 16 B
    int32_t r0, r1;      // source rows of the two taps, relative to the crop (clamped)
    int32_t b0, b1;      // 11-bit weights << 8; both 0: row shows padding
};

// hal::resize INTER_LINEAR table entry (OpenCV resize.cpp). Every operation is a single IEEE
// rounding; the translation unit is compiled with -ffp-contract=off so (d+0.5)*scale-0.5 never
// becomes an FMA.
EVAM_HD inline void linear_coef(int d, double scale, int ssize, bool is_x, int& s, int& c0, int& c1) {
    double t = ((double)d + 0.5) * scale;
    t = t - 0.5;
    float f = (float)t;
    float fl = floorf(f);
    int si = (int)fl;
    f = f - fl;
    if (is_x) {
        if (si < 0) { f = 0.f; si = 0; }
        if (si >= ssize - 1) { f = 0.f; si = ssize - 1; }
    }
    s = si;
    float w0 = (1.f - f) * 2048.f;
    float w1 = f * 2048.f;
    c0 = (int)rintf(w0);
    c1 = (int)rintf(w1);
}

struct Geom {
    int x0, y0, cw, ch, rw, rh, ox, oy;
};

// ROI clipping / 4:2:0 even alignment (rules documented in include/evam_pp.h). Shared by the host
// planner and the ROI kernel, which derives every item's geometry from the raw evam_roi on the device.
// Returns 0 or EVAM_PP_ERR_EMPTY_ROI.
EVAM_HD inline int roi_clip(int f, int W, int H, bool has_roi, int rx, int ry, int rwid, int rhei, Geom& g) {
    int x0 = 0, y0 = 0, x1 = W, y1 = H;
    if (has_roi && rwid > 0 && rhei > 0) {
        // 64-bit: x + w of caller-supplied int32 rects may exceed INT32_MAX
        auto cl = [](long long v, int hi) { return v < 0 ? 0 : (v > hi ? hi : (int)v); };
        x0 = cl(rx, W); y0 = cl(ry, H);
        x1 = cl((long long)rx + rwid, W); y1 = cl((long long)ry + rhei, H);
        if (f == kNV12 || f == kI420) {
            x0 &= ~1; y0 &= ~1;
            x1 = (x1 + 1) & ~1; x1 = x1 < W ? x1 : W;
            y1 = (y1 + 1) & ~1; y1 = y1 < H ? y1 : H;
        }
    }
    if (x1 - x0 <= 0 || y1 - y0 <= 0) return EVAM_PP_ERR_EMPTY_ROI;
    g.x0 = x0; g.y0 = y0; g.cw = x1 - x0; g.ch = y1 - y0;
    return 0;
}

// Crop + resize + placement of one item (DL Streamer model-proc resize / crop).
EVAM_HD inline int roi_geometry(int f, int W, int H, bool has_roi, int rx, int ry, int rwid, int rhei, int mode,
                                int placement, int DW, int DH, Geom& g) {
    if (roi_clip(f, W, H, has_roi, rx, ry, rwid, rhei, g)) return EVAM_PP_ERR_EMPTY_ROI;
    g.ox = 0; g.oy = 0;
    if (mode == EVAM_RESIZE_NO_ASPECT) {
        g.rw = DW; g.rh = DH;
        return 0;
    }
    const double sx = (double)DW / g.cw, sy = (double)DH / g.ch;
    const bool x_dom = mode == EVAM_RESIZE_ASPECT ? (sx <= sy) : (sx >= sy);
    if (x_dom) { g.rw = DW; g.rh = (int)(g.ch * sx); }
    else { g.rh = DH; g.rw = (int)(g.cw * sy); }
    g.rw = g.rw > 1 ? g.rw : 1;
    g.rh = g.rh > 1 ? g.rh : 1;
    if (mode == EVAM_RESIZE_ASPECT) {
        g.rw = g.rw < DW ? g.rw : DW;
        g.rh = g.rh < DH ? g.rh : DH;
        if (placement == EVAM_PLACE_CENTER) { g.ox = (DW - g.rw) / 2; g.oy = (DH - g.rh) / 2; }
    } else {
        g.rw = g.rw > DW ? g.rw : DW;
        g.rh = g.rh > DH ? g.rh : DH;
        g.ox = -((g.rw - DW) / 2);
        g.oy = -((g.rh - DH) / 2);
    }
    return 0;
}

// 16-byte-aligned byte windows [fs, fs + 16 n) of a luma / packed row (Y) and of a chroma row (C) that
// the taps of source columns [xa, xb] (absolute) read.
EVAM_HD inline void footprint_chunks(int FMT, int bpp, int xa, int xb, int& fsY, int& nY, int& fsC, int& nC) {
    fsY = (xa * bpp) & ~15;
    nY = (((xb * bpp + bpp + 15) & ~15) - fsY) >> 4;
    fsC = nC = 0;
    if (FMT == kNV12) {
        fsC = (2 * (xa >> 1)) & ~15;
        nC = (((2 * (xb >> 1) + 2 + 15) & ~15) - fsC) >> 4;
    } else if (FMT == kI420) {
        fsC = (xa >> 1) & ~15;
        nC = ((((xb >> 1) + 1 + 15) & ~15) - fsC) >> 4;
    }
}

// Source footprint of one item's visible output columns (ROI kernel).
EVAM_HD inline void item_footprint(int FMT, int bpp, int x0, int cw, int rw, int ox, double scx, int DW, int& fsY,
                                   int& nY, int& fsC, int& nC) {
    fsY = nY = fsC = nC = 0;
    const int Xv0 = ox > 0 ? ox : 0;
    const int Xv1 = (ox + rw < DW ? ox + rw : DW) - 1;
    if (Xv0 > Xv1) return;
    int sa, sb, c0, c1;
    linear_coef(Xv0 - ox, scx, cw, true, sa, c0, c1);
    linear_coef(Xv1 - ox, scx, cw, true, sb, c0, c1);
    const int xa = x0 + sa, xb = x0 + (sb + 1 < cw - 1 ? sb + 1 : cw - 1);
    footprint_chunks(FMT, bpp, xa, xb, fsY, nY, fsC, nC);
}

// Upper bound of the staged bytes of one output row of an item whose crop is cw pixels wide (both
// luma / packed taps plus both chroma taps of every chroma plane), for the host's buffer sizing.
inline int row_bytes_bound(int f, int cw) {
    const int bpp = fmt_bpp(f);
    const int segY = ((cw * bpp + 15) / 16 + 1) * 16;
    const int segC = f == kNV12 ? ((cw + 1 + 15) / 16 + 1) * 16 : (f == kI420 ? ((cw / 2 + 1 + 15) / 16 + 1) * 16 : 0);
    const int npc = f == kI420 ? 2 : (f == kNV12 ? 1 : 0);
    return 2 * segY + 2 * npc * segC;
}

// Widest 16-byte chunk counts (mY luma/packed, mC chroma) of the per-tile footprints of a uniform
// group, over every tile of tw output columns and every crop-origin residue x0 mod 32 present
// (x0_mask bit r). The chunk count of a footprint depends on x0 only through x0 mod 32 (the 16-byte
// phase of every plane: luma / packed at bpp 1, 3, 4; NV12 chroma 2 (x >> 1); I420 chroma x >> 1).
// xt: the group's column table; ox / rw: its placement and resized width.
inline void wave_segments(int f, int ox, int rw, int DW, const XTab* xt, uint32_t x0_mask, int tw, int& mY,
                          int& mC) {
    const int bpp = fmt_bpp(f);
    mY = mC = 0;
    for (int r = 0; r < 32; r++) {
        if (!((x0_mask >> r) & 1u)) continue;
        for (int X0 = 0; X0 < DW; X0 += tw) {
            const int Xv0 = std::max(X0, ox), Xv1 = std::min(std::min(X0 + tw, DW), ox + rw) - 1;
            if (Xv0 > Xv1) continue;
            int fsY, nY, fsC, nC;
            footprint_chunks(f, bpp, r + xt[Xv0].s0, r + xt[Xv1].s1, fsY, nY, fsC, nC);
            mY = std::max(mY, nY);
            mC = std::max(mC, nC);
        }
    }
}

// Algorithmic bytes of one item: distinct touched source rows x the byte width of
// the source window feeding the visible output, per plane; plus output bytes.
inline int64_t item_src_bytes(int f, const Geom& g, int DW, int DH) {
    const int dx_lo = std::max(-g.ox, 0), dx_hi = std::min(DW - g.ox, g.rw) - 1;
    const int dy_lo = std::max(-g.oy, 0), dy_hi = std::min(DH - g.oy, g.rh) - 1;
    if (dx_lo > dx_hi || dy_lo > dy_hi) return 0;
    const double scx = 1. / ((double)g.rw / g.cw), scy = 1. / ((double)g.rh / g.ch);
    int s, c0, c1, sxa, sxb;
    linear_coef(dx_lo, scx, g.cw, true, sxa, c0, c1);
    linear_coef(dx_hi, scx, g.cw, true, sxb, c0, c1);
    int xa = g.x0 + sxa, xb = g.x0 + std::min(sxb + 1, g.cw - 1);
    if (dx_lo == 0 && dx_hi == g.rw - 1) { xa = g.x0; xb = g.x0 + g.cw - 1; }  // whole crop window
    int64_t rows = 0, crow = 0;
    int last = -1, lastc = -1;
    for (int dy = dy_lo; dy <= dy_hi; dy++) {
        linear_coef(dy, scy, g.ch, false, s, c0, c1);
        const int r0 = g.y0 + std::min(std::max(s, 0), g.ch - 1);
        const int r1 = g.y0 + std::min(std::max(s + 1, 0), g.ch - 1);
        for (int r : {r0, r1}) {  // rows are non-decreasing in dy
            if (r > last) { rows++; last = r; }
            if ((r >> 1) > lastc) { crow++; lastc = r >> 1; }
        }
    }
    const int bpp = fmt_bpp(f);
    int64_t bytes = rows * (int64_t)(xb - xa + 1) * bpp;
    if (f == kNV12) bytes += crow * (int64_t)(2 * (xb >> 1) + 2 - 2 * (xa >> 1));
    if (f == kI420) bytes += 2 * crow * (int64_t)((xb >> 1) - (xa >> 1) + 1);
    return bytes;
}

// OpenCV coefficient tables of one uniform geometry, indexed by output column / row of the DW x DH plane
// (padding columns / rows get zero weights).
inline void build_tables_into(const Geom& g, int DW, int DH, XTab* x, YTab* y) {
    const double scx = 1. / ((double)g.rw / g.cw), scy = 1. / ((double)g.rh / g.ch);
    for (int X = 0; X < DW; X++) {
        x[X] = XTab{};
        const int dx = X - g.ox;
        if (dx < 0 || dx >= g.rw) continue;  // padding: s0 = s1 = 0, weights 0
        int sx, a0, a1;
        linear_coef(dx, scx, g.cw, true, sx, a0, a1);
        x[X].s0 = sx;
        x[X].s1 = std::min(sx + 1, g.cw - 1);
        x[X].a0 = (uint16_t)(a0 << 4);
        x[X].a1 = (uint16_t)(a1 << 4);
    }
    for (int Y = 0; Y < DH; Y++) {
        y[Y] = YTab{};
        const int dy = Y - g.oy;
        if (dy < 0 || dy >= g.rh) continue;
        int sy, b0, b1;
        linear_coef(dy, scy, g.ch, false, sy, b0, b1);
        y[Y].r0 = std::min(std::max(sy, 0), g.ch - 1);
        y[Y].r1 = std::min(std::max(sy + 1, 0), g.ch - 1);
        y[Y].b0 = b0 << 8;
        y[Y].b1 = b1 << 8;
    }
}

// Six-column lanes (band kernel, 4 pixels per lane): every lane with a visible pixel has four, and their taps read
// six source columns c0..c5 as pixel 0 (c0, c1), 1 (c1, c2), 2 (c3, c4), 3 (c4, c5), with c0 / c1, c2 / c3 and
// c4 / c5 in one chroma column each. A 3:2 horizontal scale (C1: 768 -> 512) has this shape on every lane, so a lane
// converts 6 luma samples and 3 chroma samples per source row instead of 8 and 8. Crop origins are even for 4:2:0
// (roi_clip), so the chroma column of crop-relative column s is x0 / 2 + s / 2 on every item.
inline bool band_six_columns(const XTab* xt, int DW, uint32_t x0_mask) {
    if (DW % 4 || (x0_mask & 0xAAAAAAAAu)) return false;
    for (int X = 0; X < DW; X += 4) {
        const XTab* e = xt + X;
        bool vis[4], any = false, all = true;
        for (int j = 0; j < 4; j++) {
            vis[j] = (e[j].a0 | e[j].a1) != 0;
            any |= vis[j];
            all &= vis[j];
        }
        if (!any) continue;
        if (!all) return false;
        if (e[0].s1 != e[1].s0 || e[2].s1 != e[3].s0) return false;
        if ((e[0].s0 >> 1) != (e[0].s1 >> 1) || (e[1].s1 >> 1) != (e[2].s0 >> 1) || (e[2].s1 >> 1) != (e[3].s1 >> 1))
            return false;
    }
    return true;
}

// ROI launch order: largest estimated work first (counting sort on 64 buckets of crop width x touched
// rows, stable within a bucket). idx: the group's item indices; bucket: scratch indexed by item index.
inline void roi_largest_first(const int* idx, int n, const Geom* geo, int DH, bool sort, int* bucket,
                              std::vector<int>& ord) {
    if (!sort) {  // call order (the default: the units are ordered by row groups afterwards); bucket is not written
        ord.assign(idx, idx + n);
        return;
    }
    int64_t maxw = 1;
    if (sort)
        for (int m = 0; m < n; m++) {
            const int i = idx[m];
            maxw = std::max(maxw, (int64_t)geo[i].cw * std::min(geo[i].ch, 2 * DH));
        }
    int start[65] = {0};
    const double to_bucket = 63.0 / (double)maxw;  // a multiply per ROI, not a 64-bit division
    for (int m = 0; m < n; m++) {
        const int i = idx[m];
        const int64_t w = (int64_t)geo[i].cw * std::min(geo[i].ch, 2 * DH);
        bucket[i] = sort ? 63 - std::min(63, (int)((double)w * to_bucket)) : 0;  // 0 = largest
        start[bucket[i] + 1]++;
    }
    for (int b = 0; b < 64; b++) start[b + 1] += start[b];
    ord.assign(start[64], 0);
    for (int m = 0; m < n; m++) ord[start[bucket[idx[m]]]++] = idx[m];
}


}  // namespace evam

// ROI tail split (evam_pp_run's one-unit-per-ROI plan): every ROI does the same DW x DH pixel work, so when n ROIs
// do not divide evenly over n_cu CUs, the last n % n_cu in launch order are cut into row tiles — up to roi_tail
// each, at most DH, and only as many as keep all units within the resident slots. Returns the tiles per split ROI
// (1: no split) and sets nsplit to the number of ROIs split (the last nsplit of the launch order).
inline int roi_tail_tiles(int n, int n_cu, int64_t slots, int roi_tail, int DH, int& nsplit) {
    nsplit = 0;
    if (n <= 0 || n_cu <= 0) return 1;
    const int tail = n % n_cu;
    if (roi_tail <= 1 || tail == 0 || DH < 2) return 1;
    const int64_t fit = (slots - (int64_t)(n - tail)) / tail;
    const int ts = (int)std::max<int64_t>(1, std::min<int64_t>({(int64_t)roi_tail, (int64_t)DH, fit}));
    nsplit = ts > 1 ? tail : 0;
    return ts;
}

// The ROI kernel's launch order of one format group in one-unit-per-ROI plans, in four passes over the ROIs with no
// intermediate unit list (round 6; the host call was 30+ us at 1,600 ROIs, half of it in the multi-pass planning):
//   1. row-group cost per ROI (rg(cw): R | groups << 16, memoised by the caller) and the largest work estimate;
//   2. the bytes bucket of every ROI (roi_largest_first's 64 buckets; all 0 without `sort`) and its histogram;
//   3. the tail split (roi_tail_tiles: the last nsplit ROIs of the bytes order, i.e. the highest buckets, the last
//      ones of the threshold bucket) and one histogram over (cost descending, split, bucket);
//   4. every unit's position from that histogram, then the snake deal (every other band of n_cu positions reversed),
//      handed to emit(position, item, row0, row1) — the caller writes the record straight into its slot.
// The order equals the multi-pass plan it replaced (roi_largest_first, units in that order with the tail split, a stable
// counting sort by row groups, the snake deal): tests/native/planner_check.cpp compares both on random groups.
// sc: scratch. Returns the number of units.
template <class RgFn, class EmitFn>
inline int roi_launch_order(const int* idx, int n, const evam::Geom* geo, int DH, int n_cu, int64_t slots, int roi_tail,
                            bool sort, bool snake, RgFn&& rg, std::vector<uint32_t>& sc, EmitFn&& emit) {
    if (n <= 0) return 0;
    sc.resize(2 * (size_t)n);
    uint32_t* e_of = sc.data();       // per ROI: R | groups << 16
    uint32_t* b_of = sc.data() + n;   // per ROI: work estimate (pass 1), then bytes bucket | split flag << 8
    int maxcost = 1;
    uint32_t maxw = 1;
    const int dh2 = 2 * DH;
    for (int m = 0; m < n; m++) {
        const evam::Geom& g = geo[idx[m]];
        const uint32_t e = rg(g.cw);
        e_of[m] = e;
        maxcost = std::max(maxcost, (int)(e >> 16));
        // crop width x touched rows: < 2^30 (frames are at most 32,768 on a side, validated by the caller)
        const uint32_t w = (uint32_t)g.cw * (uint32_t)std::min(g.ch, dh2);
        b_of[m] = w;
        maxw = std::max(maxw, w);
    }
    int hist64[64] = {0};
    if (sort) {
        // roi_largest_first's buckets from the stored estimates: a sequential pass the compiler vectorises, then the
        // histogram (the geometry is not gathered twice)
        const double to_bucket = 63.0 / (double)maxw;
        for (int m = 0; m < n; m++)
            b_of[m] = 63u - (uint32_t)std::min(63, (int)((double)b_of[m] * to_bucket));  // 0 = largest
        for (int m = 0; m < n; m++) hist64[b_of[m]]++;
    } else {
        std::fill(b_of, b_of + n, 0u);
        hist64[0] = n;
    }
    int nsplit = 0;
    const int ts = roi_tail_tiles(n, n_cu, slots, roi_tail, DH, nsplit);
    // the split ROIs: every ROI of the buckets above bt, and the last kt (in call order) of bucket bt
    int bt = 64, kt = 0;
    for (int left = nsplit, b = 63; left > 0 && b >= 0; b--) {
        bt = b;
        kt = std::min(left, hist64[b]);
        left -= kt;
    }
    const int nb = (maxcost + 1) * 128;  // bin = (maxcost - cost) * 128 + split * 64 + bucket
    sc.resize(2 * (size_t)n + (size_t)nb + 1);
    e_of = sc.data();
    b_of = sc.data() + n;
    uint32_t* start = sc.data() + 2 * (size_t)n;
    std::fill(start, start + nb + 1, 0u);
    int seen_bt = 0;
    for (int m = 0; m < n; m++) {
        const uint32_t b = b_of[m];
        bool split = (int)b > bt;
        if ((int)b == bt && ts > 1) split = seen_bt++ >= hist64[bt] - kt;
        if (!split || ts <= 1) {
            start[(size_t)(maxcost - (int)(e_of[m] >> 16)) * 128 + b + 1]++;
            continue;
        }
        b_of[m] = b | 0x100u;
        const int R = (int)(e_of[m] & 0xFFFF);
        for (int t = 0; t < ts; t++) {
            const int y0 = DH * t / ts, y1 = DH * (t + 1) / ts;
            start[(size_t)(maxcost - (y1 - y0 + R - 1) / R) * 128 + 64 + b + 1]++;
        }
    }
    for (int k = 0; k < nb; k++) start[k + 1] += start[k];
    const int nu = (int)start[nb];
    const int band = std::max(1, n_cu);
    const int band_shift = (band & (band - 1)) == 0 ? __builtin_ctz((unsigned)band) : -1;  // 256 CUs: a shift
    auto deal = [&](int p) {  // snake: positions of odd bands reversed within their band
        if (!snake) return p;
        const int b = band_shift >= 0 ? p >> band_shift : p / band;
        if (!(b & 1)) return p;
        const int lo = b * band, hi = std::min(nu, lo + band);
        return lo + hi - 1 - p;
    };
    for (int m = 0; m < n; m++) {
        const uint32_t b = b_of[m];
        if (!(b & 0x100u)) {
            emit(deal((int)start[(size_t)(maxcost - (int)(e_of[m] >> 16)) * 128 + b]++), idx[m], 0, DH);
            continue;
        }
        const int R = (int)(e_of[m] & 0xFFFF);
        const uint32_t bb = b & 0xFFu;
        for (int t = 0; t < ts; t++) {
            const int y0 = DH * t / ts, y1 = DH * (t + 1) / ts;
            emit(deal((int)start[(size_t)(maxcost - (y1 - y0 + R - 1) / R) * 128 + 64 + bb]++), idx[m], y0, y1);
        }
    }
    return nu;
}

// Frame-to-XCD deal of a sorted unit list (EVAM_PP_ROI_XCD=1, round 6 experiment for C3's 1.5x read over-fetch):
// workgroup p of a launch starts on XCD p % n_xcd and, within it, on CU (p / n_xcd) % (n_cu / n_xcd). Frames go to XCDs
// largest total cost first onto the least loaded XCD, so the overlapping crops of one frame share one L2; each XCD keeps
// its units in the sorted (largest-first) order, dealt over its CUs snake-wise (every other band of its CUs reversed);
// position n_xcd * j + x holds XCD x's j-th unit. Units beyond the smallest XCD's count (the smallest units) fill the
// positions after the interleave, in sorted order. unit[q] = (frame, cost) of sorted position q; pos[q] = its slot.
inline void roi_xcd_deal(const int* frame, const int* cost, int nu, int n_frames, int n_cu, int n_xcd,
                         std::vector<int>& pos, std::vector<int>& scratch) {
    pos.assign((size_t)nu, 0);
    if (nu <= 0) return;
    n_xcd = std::max(1, n_xcd);
    const int cus = std::max(1, n_cu / n_xcd);
    scratch.assign((size_t)n_frames * 2 + (size_t)nu + 2 * (size_t)n_xcd, 0);
    int* fcost = scratch.data();                       // per frame: summed unit cost
    int* fxcd = fcost + n_frames;                      // per frame: its XCD
    int* local = fxcd + n_frames;                      // per unit: index within its XCD
    int* cnt = local + nu;                             // per XCD: units
    int* load = cnt + n_xcd;                           // per XCD: summed cost
    for (int q = 0; q < nu; q++) fcost[frame[q]] += cost[q];
    std::vector<int> order((size_t)n_frames);
    for (int f = 0; f < n_frames; f++) order[f] = f;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return fcost[a] > fcost[b]; });
    for (int f : order) {
        int best = 0;
        for (int x = 1; x < n_xcd; x++)
            if (load[x] < load[best]) best = x;
        fxcd[f] = best;
        load[best] += fcost[f];
    }
    for (int q = 0; q < nu; q++) local[q] = cnt[fxcd[frame[q]]]++;
    int n_min = cnt[0];
    for (int x = 1; x < n_xcd; x++) n_min = std::min(n_min, cnt[x]);
    int rest = n_xcd * n_min;
    for (int q = 0; q < nu; q++) {
        const int x = fxcd[frame[q]], j = local[q];
        if (j >= n_min) {
            pos[q] = rest++;
            continue;
        }
        const int b = j / cus;
        const int lo = b * cus, hi = std::min(n_min, lo + cus);
        const int jj = (b & 1) ? lo + hi - 1 - j : j;
        pos[q] = n_xcd * jj + x;
    }
}

#endif  // EVAM_GEOM_H
