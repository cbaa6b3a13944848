// evam_pp.hip — MI355X (gfx950) frame pre-processing backend: fused colour-convert + OpenCV-exact
// INTER_LINEAR resize + letterbox/central-crop placement + normalisation + NCHW batch packing.
//
// Drop-in for DL Streamer 2022.1's `opencv` pre-proc backend (ImagePreprocessor::Convert, third
// party) that EVAM selects through pipelines/*/pipeline.json element properties
// (pipelines/object_detection/vehicle/pipeline.json:5,13-18; pipelines/object_classification/
// vehicle_attributes/pipeline.json:4-5,12-23; pipelines/action_recognition/general/pipeline.json:3-4).
// The C ABI is declared in include/evam_pp.h; SURVEY.md §8 is the scope table.
//
// Design (DESIGN.md has the full write-up):
//  * One launch per (source format, call). One 256-thread workgroup per (item, output tile of TW x TH
//    pixels). The workgroup
//      1. computes the OpenCV coefficient tables for its tile columns/rows on the device, in the exact
//         double/float operation sequence of hal::resize (no FMA contraction: built -ffp-contract=off);
//      2. stages the source footprint of the tile — two luma rows and two chroma rows per output row,
//         duplicated rows skipped, columns [first tap, last tap] aligned out to 16 B — from HBM into LDS
//         with 128-bit coalesced loads;
//      3. for every output pixel converts its four taps to BGR (BT.601 20-bit fixed point), runs the
//         11-bit horizontal pass and the VResizeLinear 32s->8u vertical pass, maps the u8 result
//         through the per-channel normalisation LUT (fp32 out) and stores planar NCHW.
//  * Letterbox padding tiles never touch the source. Nothing is MFMA-shaped: the path is HBM-bound
//    integer gather work (roofline: HBM, 8 TB/s).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/evam_pp.h"

namespace {

// ------------------------------------------------------------------------------------------------
// constants
// ------------------------------------------------------------------------------------------------
constexpr int kThreads = 256;
constexpr int kLutBytes = 3 * 256 * 4;
constexpr int kLdsBudget = 48 * 1024;

// OpenCV color_yuv.simd.hpp ITUR_BT_601_*; the -128 chroma bias is folded into the constants.
constexpr int kCY = 1220542, kCUB = 2116026, kCUG = -409993, kCVG = -852492, kCVR = 1673527;
constexpr int kHalf = 1 << 19;
constexpr int kKR = kHalf - 128 * kCVR;
constexpr int kKG = kHalf - 128 * kCVG - 128 * kCUG;
constexpr int kKB = kHalf - 128 * kCUB;

enum FmtId { kNV12 = 0, kI420 = 1, kBGRX = 2, kBGR = 3 };

// ------------------------------------------------------------------------------------------------
// device-side descriptors
// ------------------------------------------------------------------------------------------------
struct alignas(16) ItemDesc {
    const uint8_t* plane[3];
    int32_t pitch[3];
    int32_t x0, y0, cw, ch;  // effective crop in source pixels
    int32_t rw, rh, ox, oy;  // resized size, placement in the DW x DH plane
    int32_t slot;
    int32_t pad_;
    double scale_x, scale_y; // OpenCV: 1. / ((double)rw / cw)
};
static_assert(sizeof(ItemDesc) == 96, "ItemDesc layout");

struct KParams {
    const ItemDesc* items;
    const float* lut;  // [3][256]
    void* dst;
    int DW, DH;
    int TW, TH, tiles_x, tiles_per_item;
    uint32_t tw_magic;  // ceil(2^32 / TW)
    int strideY, strideC;  // LDS bytes per staged row
    int offRow, offSlot, offLut, offY, offC, offV;  // LDS carve (coltab at 0)
    int color_rgb;
    uint32_t fill;  // packed u8 fill, output channel order
};

struct ColEntry {  // 16 B, one per tile column
    int16_t oY0, oY1;  // LDS byte offset of the two taps in a staged luma/packed row (-1: column not in image)
    int16_t oC0, oC1;  // LDS byte offset in a staged chroma row (NV12: U of the UV pair)
    int16_t a0, a1;    // 11-bit horizontal weights
    int16_t pad0, pad1;
};

struct RowEntry {  // 32 B, one per tile row
    int32_t y0, y1;   // LDS byte offsets of the two staged luma rows (-1: row not in image)
    int32_t c0, c1;   // LDS byte offsets of the two staged chroma rows
    int32_t b0, b1;   // 11-bit vertical weights
    int32_t pad0, pad1;
};

// ------------------------------------------------------------------------------------------------
// exact OpenCV arithmetic (shared host/device)
// ------------------------------------------------------------------------------------------------
// hal::resize INTER_LINEAR table entry. Every operation is a single IEEE rounding; the translation
// unit is compiled with -ffp-contract=off so (d+0.5)*scale-0.5 never becomes an FMA.
__host__ __device__ inline void linear_coef(int d, double scale, int ssize, bool is_x, int& s, int& c0,
                                            int& c1) {
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

__device__ __forceinline__ uint32_t umulhi(uint32_t a, uint32_t b) { return __umulhi(a, b); }

__device__ __forceinline__ int clamp255(int v) { return min(max(v, 0), 255); }

// BT.601 20-bit fixed point (OpenCV uvToRGBuv + yRGBuvToRGBA). Arguments are raw bytes.
__device__ __forceinline__ void yuv_to_bgr(int Y, int U, int V, int& b, int& g, int& r) {
    const int y = max(Y - 16, 0) * kCY;
    const int ruv = kCVR * V + kKR;
    const int guv = kCVG * V + kCUG * U + kKG;
    const int buv = kCUB * U + kKB;
    b = clamp255((y + buv) >> 20);
    g = clamp255((y + guv) >> 20);
    r = clamp255((y + ruv) >> 20);
}

template <int FMT>
__device__ __forceinline__ void tap(const uint8_t* __restrict__ lds, int yrow, int crow, int vrow, int oy,
                                    int oc, int& b, int& g, int& r) {
    if constexpr (FMT == kNV12) {
        const int Y = lds[yrow + oy];
        const uint32_t uv = *reinterpret_cast<const uint16_t*>(lds + crow + oc);
        yuv_to_bgr(Y, uv & 0xFF, uv >> 8, b, g, r);
    } else if constexpr (FMT == kI420) {
        const int Y = lds[yrow + oy];
        yuv_to_bgr(Y, lds[crow + oc], lds[vrow + oc], b, g, r);
    } else if constexpr (FMT == kBGRX) {
        const uint32_t p = *reinterpret_cast<const uint32_t*>(lds + yrow + oy);
        b = p & 0xFF; g = (p >> 8) & 0xFF; r = (p >> 16) & 0xFF;
    } else {
        b = lds[yrow + oy]; g = lds[yrow + oy + 1]; r = lds[yrow + oy + 2];
    }
}

// VResizeLinear<uchar,int,short,FixedPtCast<int,uchar,22>,VResizeLinearVec_32s8u>
__device__ __forceinline__ int vresize(int D0, int D1, int b0, int b1) {
    return (((b0 * (D0 >> 4)) >> 16) + ((b1 * (D1 >> 4)) >> 16) + 2) >> 2;
}

template <int FMT>
struct FmtTraits {
    static constexpr int bpp = FMT == kBGRX ? 4 : (FMT == kBGR ? 3 : 1);
    static constexpr int nchroma = FMT == kNV12 ? 1 : (FMT == kI420 ? 2 : 0);
};

// 128-bit row staging: n_slots rows of `bytes` bytes (multiple of 16) from global to LDS.
__device__ __forceinline__ void stage_plane(uint8_t* __restrict__ lds, int lds_off, int stride,
                                            const int32_t* __restrict__ slot_rows, int n_slots,
                                            const uint8_t* __restrict__ plane, int pitch, int fs, int bytes,
                                            int tid) {
    const int cpr = bytes >> 4;
    if (cpr <= 0) return;
    const uint32_t magic = 0xFFFFFFFFu / (uint32_t)cpr + 1u;
    const int total = n_slots * cpr;
#pragma unroll 4
    for (int c = tid; c < total; c += kThreads) {
        const int slot = (cpr & (cpr - 1)) == 0 ? (c >> __builtin_ctz(cpr)) : (int)umulhi((uint32_t)c, magic);
        const int col = c - slot * cpr;
        const int row = slot_rows[slot];
        if (row >= 0) {
            const uint4 v = *reinterpret_cast<const uint4*>(plane + (size_t)row * pitch + fs + col * 16);
            *reinterpret_cast<uint4*>(lds + lds_off + slot * stride + col * 16) = v;
        }
    }
}

template <int OUT>
__device__ __forceinline__ void store_px(const KParams& P, const float* __restrict__ lut, size_t base,
                                         size_t plane, int v0, int v1, int v2) {
    if constexpr (OUT == 0) {
        uint8_t* d = reinterpret_cast<uint8_t*>(P.dst);
        d[base] = (uint8_t)v0;
        d[base + plane] = (uint8_t)v1;
        d[base + 2 * plane] = (uint8_t)v2;
    } else {
        float* d = reinterpret_cast<float*>(P.dst);
        d[base] = lut[v0];
        d[base + plane] = lut[256 + v1];
        d[base + 2 * plane] = lut[512 + v2];
    }
}

template <int FMT, int OUT>
__global__ __launch_bounds__(kThreads) void evam_pp_kernel(const KParams P) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    using T = FmtTraits<FMT>;
    const int tid = threadIdx.x;
    const int item_idx = blockIdx.x / P.tiles_per_item;
    const int tile = blockIdx.x - item_idx * P.tiles_per_item;
    const int ty = tile / P.tiles_x;
    const int tx = tile - ty * P.tiles_x;
    const ItemDesc& it = P.items[item_idx];

    const int X0 = tx * P.TW, Y0 = ty * P.TH;
    const int X1 = min(X0 + P.TW, P.DW), Y1 = min(Y0 + P.TH, P.DH);
    const size_t plane = (size_t)P.DW * P.DH;
    const size_t slot_base = (size_t)it.slot * 3 * plane;
    const int npx = P.TW * P.TH;

    float* lut_s = reinterpret_cast<float*>(smem + P.offLut);
    if constexpr (OUT == 1) {
        for (int i = tid; i < 768; i += kThreads) lut_s[i] = P.lut[i];
    }

    // visible resized-image range inside this tile
    const int dx_lo = max(X0 - it.ox, 0), dx_hi = min(X1 - it.ox, it.rw) - 1;
    const int dy_lo = max(Y0 - it.oy, 0), dy_hi = min(Y1 - it.oy, it.rh) - 1;
    const int f0 = P.fill & 0xFF, f1 = (P.fill >> 8) & 0xFF, f2 = (P.fill >> 16) & 0xFF;

    if (dx_lo > dx_hi || dy_lo > dy_hi) {  // pure padding tile: no source traffic
        if constexpr (OUT == 1) __syncthreads();
        for (int p = tid; p < npx; p += kThreads) {
            const int ly = (int)umulhi((uint32_t)p, P.tw_magic);
            const int lx = p - ly * P.TW;
            const int X = X0 + lx, Y = Y0 + ly;
            if (X < X1 && Y < Y1) store_px<OUT>(P, lut_s, slot_base + (size_t)Y * P.DW + X, plane, f0, f1, f2);
        }
        return;
    }

    // ---- 1. coefficient tables for this tile, LDS offsets relative to the 16-B aligned footprint ----
    int sxa, sxb, cdummy0, cdummy1;
    linear_coef(dx_lo, it.scale_x, it.cw, true, sxa, cdummy0, cdummy1);
    linear_coef(dx_hi, it.scale_x, it.cw, true, sxb, cdummy0, cdummy1);
    const int xa = it.x0 + sxa;                        // first source column touched
    const int xb = it.x0 + min(sxb + 1, it.cw - 1);    // last source column touched
    const int fsY = (xa * T::bpp) & ~15;
    const int feY = (xb * T::bpp + T::bpp + 15) & ~15;
    int fsC = 0, feC = 0;
    if constexpr (FMT == kNV12) {
        fsC = (2 * (xa >> 1)) & ~15;
        feC = (2 * (xb >> 1) + 2 + 15) & ~15;
    } else if constexpr (FMT == kI420) {
        fsC = (xa >> 1) & ~15;
        feC = ((xb >> 1) + 1 + 15) & ~15;
    }

    ColEntry* coltab = reinterpret_cast<ColEntry*>(smem);
    RowEntry* rowtab = reinterpret_cast<RowEntry*>(smem + P.offRow);
    int32_t* slotY = reinterpret_cast<int32_t*>(smem + P.offSlot);
    int32_t* slotC = slotY + 2 * P.TH;

    for (int lx = tid; lx < P.TW; lx += kThreads) {
        ColEntry e;
        const int dx = X0 + lx - it.ox;
        if (X0 + lx < X1 && dx >= 0 && dx < it.rw) {
            int sx, a0, a1;
            linear_coef(dx, it.scale_x, it.cw, true, sx, a0, a1);
            const int ca = it.x0 + sx, cb = it.x0 + min(sx + 1, it.cw - 1);
            e.oY0 = (int16_t)(ca * T::bpp - fsY);
            e.oY1 = (int16_t)(cb * T::bpp - fsY);
            if constexpr (FMT == kNV12) {
                e.oC0 = (int16_t)(2 * (ca >> 1) - fsC);
                e.oC1 = (int16_t)(2 * (cb >> 1) - fsC);
            } else {
                e.oC0 = (int16_t)((ca >> 1) - fsC);
                e.oC1 = (int16_t)((cb >> 1) - fsC);
            }
            e.a0 = (int16_t)a0;
            e.a1 = (int16_t)a1;
        } else {
            e.oY0 = -1; e.oY1 = -1; e.oC0 = 0; e.oC1 = 0; e.a0 = 0; e.a1 = 0;
        }
        e.pad0 = 0; e.pad1 = 0;
        coltab[lx] = e;
    }
    for (int ly = tid; ly < P.TH; ly += kThreads) {
        RowEntry e;
        const int dy = Y0 + ly - it.oy;
        int ya = -1, yb = -1, ca = -1, cb = -1;
        if (Y0 + ly < Y1 && dy >= 0 && dy < it.rh) {
            int sy, b0, b1;
            linear_coef(dy, it.scale_y, it.ch, false, sy, b0, b1);
            ya = it.y0 + min(max(sy, 0), it.ch - 1);
            yb = it.y0 + min(max(sy + 1, 0), it.ch - 1);
            e.y0 = P.offY + (2 * ly) * P.strideY;
            e.y1 = yb == ya ? e.y0 : P.offY + (2 * ly + 1) * P.strideY;
            if constexpr (T::nchroma > 0) {
                ca = ya >> 1;
                cb = yb >> 1;
                e.c0 = (2 * ly) * P.strideC;
                e.c1 = cb == ca ? e.c0 : (2 * ly + 1) * P.strideC;
                if (cb == ca) cb = -1;
            } else {
                e.c0 = 0; e.c1 = 0;
            }
            if (yb == ya) yb = -1;
            e.b0 = b0;
            e.b1 = b1;
        } else {
            e.y0 = -1; e.y1 = -1; e.c0 = 0; e.c1 = 0; e.b0 = 0; e.b1 = 0;
        }
        e.pad0 = 0; e.pad1 = 0;
        rowtab[ly] = e;
        slotY[2 * ly] = ya;
        slotY[2 * ly + 1] = yb;
        slotC[2 * ly] = ca;
        slotC[2 * ly + 1] = cb;
    }
    __syncthreads();

    // ---- 2. stage the source footprint (HBM -> LDS, 16 B per lane) ----
    stage_plane(smem, P.offY, P.strideY, slotY, 2 * P.TH, it.plane[0], it.pitch[0], fsY, feY - fsY, tid);
    if constexpr (T::nchroma >= 1)
        stage_plane(smem, P.offC, P.strideC, slotC, 2 * P.TH, it.plane[1], it.pitch[1], fsC, feC - fsC, tid);
    if constexpr (T::nchroma == 2)
        stage_plane(smem, P.offV, P.strideC, slotC, 2 * P.TH, it.plane[2], it.pitch[2], fsC, feC - fsC, tid);
    __syncthreads();

    // ---- 3. convert + resize + normalise + planar store ----
    const int cbase = P.offC;
    const int vdelta = P.offV - P.offC;
    for (int p = tid; p < npx; p += kThreads) {
        const int ly = (int)umulhi((uint32_t)p, P.tw_magic);
        const int lx = p - ly * P.TW;
        const int X = X0 + lx, Y = Y0 + ly;
        if (X >= X1 || Y >= Y1) continue;
        const size_t base = slot_base + (size_t)Y * P.DW + X;
        const ColEntry ce = coltab[lx];
        const RowEntry re = rowtab[ly];
        if (ce.oY0 < 0 || re.y0 < 0) {
            store_px<OUT>(P, lut_s, base, plane, f0, f1, f2);
            continue;
        }
        int bA, gA, rA, bB, gB, rB;
        // row 0
        tap<FMT>(smem, re.y0, cbase + re.c0, cbase + re.c0 + vdelta, ce.oY0, ce.oC0, bA, gA, rA);
        tap<FMT>(smem, re.y0, cbase + re.c0, cbase + re.c0 + vdelta, ce.oY1, ce.oC1, bB, gB, rB);
        const int Db0 = bA * ce.a0 + bB * ce.a1;
        const int Dg0 = gA * ce.a0 + gB * ce.a1;
        const int Dr0 = rA * ce.a0 + rB * ce.a1;
        // row 1
        tap<FMT>(smem, re.y1, cbase + re.c1, cbase + re.c1 + vdelta, ce.oY0, ce.oC0, bA, gA, rA);
        tap<FMT>(smem, re.y1, cbase + re.c1, cbase + re.c1 + vdelta, ce.oY1, ce.oC1, bB, gB, rB);
        const int Db1 = bA * ce.a0 + bB * ce.a1;
        const int Dg1 = gA * ce.a0 + gB * ce.a1;
        const int Dr1 = rA * ce.a0 + rB * ce.a1;
        const int vb = vresize(Db0, Db1, re.b0, re.b1);
        const int vg = vresize(Dg0, Dg1, re.b0, re.b1);
        const int vr = vresize(Dr0, Dr1, re.b0, re.b1);
        if (P.color_rgb)
            store_px<OUT>(P, lut_s, base, plane, vr, vg, vb);
        else
            store_px<OUT>(P, lut_s, base, plane, vb, vg, vr);
    }
}

// ------------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------------
thread_local std::string g_last_error;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

#define HIP_TRY(expr)                                                                       \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess)                                                               \
            return fail(EVAM_PP_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(e_));   \
    } while (0)

int fmt_id(int fourcc) {
    switch (fourcc) {
    case EVAM_FOURCC_NV12: return kNV12;
    case EVAM_FOURCC_I420: return kI420;
    case EVAM_FOURCC_BGRX:
    case EVAM_FOURCC_BGRA: return kBGRX;
    case EVAM_FOURCC_BGR: return kBGR;
    default: return -1;
    }
}

int fmt_bpp(int f) { return f == kBGRX ? 4 : (f == kBGR ? 3 : 1); }
int fmt_nplanes(int f) { return f == kNV12 ? 2 : (f == kI420 ? 3 : 1); }

struct Geom {
    int x0, y0, cw, ch, rw, rh, ox, oy;
};

// ROI clipping / 4:2:0 even alignment / aspect-ratio geometry. Rules documented in include/evam_pp.h.
int item_geometry(int f, int W, int H, const evam_roi* roi, const evam_preproc& cfg, int DW, int DH, Geom& g) {
    int x0 = 0, y0 = 0, x1 = W, y1 = H;
    if (roi && roi->w > 0 && roi->h > 0) {
        auto cl = [](int v, int hi) { return v < 0 ? 0 : (v > hi ? hi : v); };
        x0 = cl(roi->x, W); y0 = cl(roi->y, H);
        x1 = cl(roi->x + roi->w, W); y1 = cl(roi->y + roi->h, H);
        if (f == kNV12 || f == kI420) {
            x0 &= ~1; y0 &= ~1;
            x1 = std::min(W, (x1 + 1) & ~1);
            y1 = std::min(H, (y1 + 1) & ~1);
        }
    }
    if (x1 - x0 <= 0 || y1 - y0 <= 0) return EVAM_PP_ERR_EMPTY_ROI;
    g.x0 = x0; g.y0 = y0; g.cw = x1 - x0; g.ch = y1 - y0; g.ox = 0; g.oy = 0;
    if (cfg.resize_mode == EVAM_RESIZE_NO_ASPECT) {
        g.rw = DW; g.rh = DH;
        return 0;
    }
    const double sx = (double)DW / g.cw, sy = (double)DH / g.ch;
    const bool x_dom = cfg.resize_mode == EVAM_RESIZE_ASPECT ? (sx <= sy) : (sx >= sy);
    if (x_dom) { g.rw = DW; g.rh = (int)(g.ch * sx); }
    else { g.rh = DH; g.rw = (int)(g.cw * sy); }
    g.rw = std::max(g.rw, 1);
    g.rh = std::max(g.rh, 1);
    if (cfg.resize_mode == EVAM_RESIZE_ASPECT) {
        g.rw = std::min(g.rw, DW);
        g.rh = std::min(g.rh, DH);
        if (cfg.placement == EVAM_PLACE_CENTER) { g.ox = (DW - g.rw) / 2; g.oy = (DH - g.rh) / 2; }
    } else {
        g.rw = std::max(g.rw, DW);
        g.rh = std::max(g.rh, DH);
        g.ox = -((g.rw - DW) / 2);
        g.oy = -((g.rh - DH) / 2);
    }
    return 0;
}

void build_lut(const evam_preproc& cfg, float* lut) {
    const volatile float alpha = (float)(((double)cfg.range[1] - (double)cfg.range[0]) / 255.0);
    const volatile float beta = cfg.range[0];
    for (int c = 0; c < 3; c++)
        for (int u = 0; u < 256; u++) {
            volatile float v = (float)u;
            if (cfg.norm_flags & EVAM_NORM_RANGE) {
                volatile float m = v * alpha;
                v = m + beta;
            }
            if (cfg.norm_flags & EVAM_NORM_MEAN_STD) {
                volatile float s = v - cfg.mean[c];
                v = s / cfg.std[c];
            }
            lut[c * 256 + u] = v;
        }
}

// Algorithmic bytes of one item: distinct touched source rows x the byte width of
// the source window feeding the visible output, per plane; plus output bytes.
int64_t item_src_bytes(int f, const Geom& g, int DW, int DH) {
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

struct TileCfg {
    int TW, TH, strideY, strideC, lds, offRow, offSlot, offLut, offY, offC, offV;
};

// Tile shape: ~1024 output pixels per 256-thread workgroup, shrunk until the staged footprint fits.
TileCfg choose_tiles(int f, int DW, int DH, double max_ratio_x, int out_dtype) {
    TileCfg t{};
    if (DW <= 256) t.TW = DW;
    else if (DW % 128 == 0) t.TW = 128;
    else if (DW % 64 == 0) t.TW = 64;
    else t.TW = 128;
    t.TH = std::max(1, std::min(DH, 1024 / t.TW));
    const int bpp = fmt_bpp(f);
    for (;;) {
        const int span = (int)std::ceil((t.TW - 1) * max_ratio_x) + 4;  // source columns
        t.strideY = ((span * bpp + 32) + 15) & ~15;
        t.strideC = f == kNV12 ? ((span + 2 + 32 + 15) & ~15) : (f == kI420 ? ((span / 2 + 2 + 32 + 15) & ~15) : 0);
        const int nC = f == kNV12 ? 1 : (f == kI420 ? 2 : 0);
        int off = ((int)sizeof(ColEntry) * t.TW + 15) & ~15;
        t.offRow = off;
        off += (int)sizeof(RowEntry) * t.TH;
        t.offSlot = off;
        off += 4 * 4 * t.TH;
        off = (off + 15) & ~15;
        t.offLut = off;
        if (out_dtype == EVAM_DTYPE_F32) off += kLutBytes;
        t.offY = off;
        off += 2 * t.TH * t.strideY;
        t.offC = off;
        off += 2 * t.TH * t.strideC;
        t.offV = off;
        if (nC == 2) off += 2 * t.TH * t.strideC;
        t.lds = off;
        if (t.lds <= kLdsBudget) break;
        if (t.TH > 1) t.TH = std::max(1, t.TH / 2);
        else if (t.TW > 16) t.TW = std::max(16, t.TW / 2);
        else break;
    }
    return t;
}

template <int FMT, int OUT>
hipError_t launch_t(const KParams& p, int grid, int lds, hipStream_t s) {
    hipLaunchKernelGGL((evam_pp_kernel<FMT, OUT>), dim3(grid), dim3(kThreads), lds, s, p);
    return hipGetLastError();
}

hipError_t launch(int f, int out, const KParams& p, int grid, int lds, hipStream_t s) {
    switch (f * 2 + out) {
    case kNV12 * 2 + 0: return launch_t<kNV12, 0>(p, grid, lds, s);
    case kNV12 * 2 + 1: return launch_t<kNV12, 1>(p, grid, lds, s);
    case kI420 * 2 + 0: return launch_t<kI420, 0>(p, grid, lds, s);
    case kI420 * 2 + 1: return launch_t<kI420, 1>(p, grid, lds, s);
    case kBGRX * 2 + 0: return launch_t<kBGRX, 0>(p, grid, lds, s);
    case kBGRX * 2 + 1: return launch_t<kBGRX, 1>(p, grid, lds, s);
    case kBGR * 2 + 0: return launch_t<kBGR, 0>(p, grid, lds, s);
    default: return launch_t<kBGR, 1>(p, grid, lds, s);
    }
}

}  // namespace

struct evam_pp {
    int device = 0;
    hipStream_t stream = nullptr;
    int opt_stats = 0, opt_timing = 0;
    evam_pp_stats stats{};
    // descriptor block: [LUT 3 KB][ItemDesc x n] in device memory; re-uploaded only when it changes.
    uint8_t* d_block = nullptr;
    size_t d_block_cap = 0;
    std::vector<uint8_t> h_block, h_last;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    bool timed = false;
};

extern "C" {

int evam_pp_abi_version(void) { return EVAM_PP_ABI_VERSION; }

const char* evam_pp_last_error(void) { return g_last_error.c_str(); }

int evam_pp_create(int hip_device, void* hip_stream, evam_pp** out) {
    if (!out) return fail(EVAM_PP_ERR_INVALID_ARG, "evam_pp_create: out is NULL");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
        return fail(EVAM_PP_ERR_NO_DEVICE, "evam_pp_create: no HIP device");
    if (hip_device < 0 || hip_device >= n)
        return fail(EVAM_PP_ERR_NO_DEVICE, "evam_pp_create: device %d out of range [0,%d)", hip_device, n);
    HIP_TRY(hipSetDevice(hip_device));
    evam_pp* h = new (std::nothrow) evam_pp();
    if (!h) return fail(EVAM_PP_ERR_OOM, "evam_pp_create: out of host memory");
    h->device = hip_device;
    h->stream = reinterpret_cast<hipStream_t>(hip_stream);
    if (hipEventCreate(&h->ev0) != hipSuccess || hipEventCreate(&h->ev1) != hipSuccess) {
        delete h;
        return fail(EVAM_PP_ERR_HIP, "evam_pp_create: hipEventCreate failed");
    }
    *out = h;
    return EVAM_PP_OK;
}

void evam_pp_destroy(evam_pp* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    if (h->d_block) {
        (void)hipStreamSynchronize(h->stream);
        (void)hipFree(h->d_block);
    }
    if (h->ev0) (void)hipEventDestroy(h->ev0);
    if (h->ev1) (void)hipEventDestroy(h->ev1);
    delete h;
}

int evam_pp_set_stream(evam_pp* h, void* hip_stream) {
    if (!h) return fail(EVAM_PP_ERR_INVALID_ARG, "evam_pp_set_stream: NULL handle");
    h->stream = reinterpret_cast<hipStream_t>(hip_stream);
    return EVAM_PP_OK;
}

int evam_pp_set_option(evam_pp* h, int option, int value) {
    if (!h) return fail(EVAM_PP_ERR_INVALID_ARG, "evam_pp_set_option: NULL handle");
    if (option == EVAM_OPT_STATS) h->opt_stats = value != 0;
    else if (option == EVAM_OPT_TIMING) h->opt_timing = value != 0;
    else return fail(EVAM_PP_ERR_INVALID_ARG, "evam_pp_set_option: unknown option %d", option);
    return EVAM_PP_OK;
}

int evam_pp_sync(evam_pp* h) {
    if (!h) return fail(EVAM_PP_ERR_INVALID_ARG, "evam_pp_sync: NULL handle");
    HIP_TRY(hipSetDevice(h->device));
    HIP_TRY(hipStreamSynchronize(h->stream));
    return EVAM_PP_OK;
}

int evam_pp_get_stats(evam_pp* h, evam_pp_stats* out) {
    if (!h || !out) return fail(EVAM_PP_ERR_INVALID_ARG, "evam_pp_get_stats: NULL argument");
    if (h->timed) {
        HIP_TRY(hipEventSynchronize(h->ev1));
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, h->ev0, h->ev1));
        h->stats.last_kernel_ms = ms;
    }
    *out = h->stats;
    return EVAM_PP_OK;
}

int evam_pp_linear_table(int src_size, int dst_size, int is_x, int32_t* ofs, int16_t* c0, int16_t* c1) {
    if (src_size <= 0 || dst_size <= 0 || !ofs || !c0 || !c1)
        return fail(EVAM_PP_ERR_INVALID_ARG, "evam_pp_linear_table: bad arguments");
    const double scale = 1. / ((double)dst_size / src_size);
    for (int d = 0; d < dst_size; d++) {
        int s, a, b;
        linear_coef(d, scale, src_size, is_x != 0, s, a, b);
        ofs[d] = s;
        c0[d] = (int16_t)a;
        c1[d] = (int16_t)b;
    }
    return EVAM_PP_OK;
}

int evam_pp_run(evam_pp* h, const evam_image* srcs, int n_srcs, const evam_roi* items, int n_items,
                const evam_preproc* cfg, const evam_tensor* dst, evam_transform* out_xform) {
    if (!h || !srcs || !cfg || !dst) return fail(EVAM_PP_ERR_INVALID_ARG, "evam_pp_run: NULL argument");
    if (n_srcs <= 0) return fail(EVAM_PP_ERR_INVALID_ARG, "evam_pp_run: n_srcs must be > 0");
    if (!items) n_items = n_srcs;
    if (n_items <= 0) return fail(EVAM_PP_ERR_INVALID_ARG, "evam_pp_run: n_items must be > 0");
    if (!dst->data) return fail(EVAM_PP_ERR_INVALID_ARG, "evam_pp_run: dst->data is NULL");
    if (dst->c != 3) return fail(EVAM_PP_ERR_UNSUPPORTED, "evam_pp_run: dst must have 3 channels (got %d)", dst->c);
    if (dst->n <= 0 || dst->h <= 0 || dst->w <= 0)
        return fail(EVAM_PP_ERR_INVALID_ARG, "evam_pp_run: bad dst shape %dx%dx%dx%d", dst->n, dst->c, dst->h, dst->w);
    if (cfg->out_dtype != EVAM_DTYPE_U8 && cfg->out_dtype != EVAM_DTYPE_F32)
        return fail(EVAM_PP_ERR_UNSUPPORTED, "evam_pp_run: unknown out_dtype %d", cfg->out_dtype);
    if (cfg->resize_mode < 0 || cfg->resize_mode > 2)
        return fail(EVAM_PP_ERR_INVALID_ARG, "evam_pp_run: unknown resize_mode %d", cfg->resize_mode);
    if ((cfg->norm_flags & EVAM_NORM_MEAN_STD) && cfg->out_dtype == EVAM_DTYPE_F32)
        for (int c = 0; c < 3; c++)
            if (cfg->std[c] == 0.f) return fail(EVAM_PP_ERR_INVALID_ARG, "evam_pp_run: std[%d] == 0", c);
    const int DW = dst->w, DH = dst->h;
    const int64_t plane = (int64_t)DW * DH;
    if (plane * 3 * (int64_t)dst->n > ((int64_t)1 << 40))
        return fail(EVAM_PP_ERR_INVALID_ARG, "evam_pp_run: dst too large");

    // ---- validate sources ----
    for (int i = 0; i < n_srcs; i++) {
        const evam_image& s = srcs[i];
        const int f = fmt_id(s.fourcc);
        if (f < 0) return fail(EVAM_PP_ERR_UNSUPPORTED, "evam_pp_run: srcs[%d] fourcc 0x%08x unsupported", i, s.fourcc);
        if (s.width <= 0 || s.height <= 0 || s.width > 32768 || s.height > 32768)
            return fail(EVAM_PP_ERR_INVALID_ARG, "evam_pp_run: srcs[%d] bad size %dx%d", i, s.width, s.height);
        if ((f == kNV12 || f == kI420) && ((s.width | s.height) & 1))
            return fail(EVAM_PP_ERR_INVALID_ARG, "evam_pp_run: srcs[%d] 4:2:0 frame must have even size (%dx%d)", i, s.width, s.height);
        for (int p = 0; p < fmt_nplanes(f); p++) {
            const int row_bytes = p == 0 ? s.width * fmt_bpp(f) : (f == kNV12 ? s.width : s.width / 2);
            if (!s.planes[p]) return fail(EVAM_PP_ERR_INVALID_ARG, "evam_pp_run: srcs[%d].planes[%d] is NULL", i, p);
            if (((uintptr_t)s.planes[p] & 15) || (s.pitch[p] & 15))
                return fail(EVAM_PP_ERR_ALIGNMENT, "evam_pp_run: srcs[%d] plane %d pointer/pitch (%d) not 16-byte aligned", i, p, s.pitch[p]);
            if (s.pitch[p] < row_bytes)
                return fail(EVAM_PP_ERR_INVALID_ARG, "evam_pp_run: srcs[%d] plane %d pitch %d < row bytes %d", i, p, s.pitch[p], row_bytes);
        }
    }

    // ---- plan: geometry per item, grouped by source format ----
    std::vector<Geom> geo(n_items);
    std::vector<int> fmt(n_items);
    double max_ratio[4] = {0, 0, 0, 0};
    int count[4] = {0, 0, 0, 0};
    int64_t src_bytes = 0;
    for (int i = 0; i < n_items; i++) {
        const evam_roi* r = items ? &items[i] : nullptr;
        const int si = items ? r->src_index : i;
        if (si < 0 || si >= n_srcs)
            return fail(EVAM_PP_ERR_INVALID_ARG, "evam_pp_run: items[%d].src_index %d out of range", i, si);
        const int slot = dst->slot_offset + i * dst->slot_stride;
        if (slot < 0 || slot >= dst->n)
            return fail(EVAM_PP_ERR_INVALID_ARG, "evam_pp_run: item %d -> slot %d outside tensor batch %d", i, slot, dst->n);
        const evam_image& s = srcs[si];
        fmt[i] = fmt_id(s.fourcc);
        int rc = item_geometry(fmt[i], s.width, s.height, r, *cfg, DW, DH, geo[i]);
        if (rc) return fail(rc, "evam_pp_run: items[%d] ROI (%d,%d,%d,%d) is empty after clipping to %dx%d", i,
                            r ? r->x : 0, r ? r->y : 0, r ? r->w : 0, r ? r->h : 0, s.width, s.height);
        max_ratio[fmt[i]] = std::max(max_ratio[fmt[i]], (double)geo[i].cw / geo[i].rw);
        count[fmt[i]]++;
        if (out_xform) {
            evam_transform& t = out_xform[i];
            t.scale_x = (float)((double)geo[i].rw / geo[i].cw);
            t.scale_y = (float)((double)geo[i].rh / geo[i].ch);
            t.crop_x = geo[i].x0; t.crop_y = geo[i].y0; t.crop_w = geo[i].cw; t.crop_h = geo[i].ch;
            t.pad_x = geo[i].ox; t.pad_y = geo[i].oy;
            t.resized_w = geo[i].rw; t.resized_h = geo[i].rh;
        }
        if (h->opt_stats) src_bytes += item_src_bytes(fmt[i], geo[i], DW, DH);
    }

    // ---- descriptor block ----
    const size_t nbytes = kLutBytes + sizeof(ItemDesc) * (size_t)n_items;
    h->h_block.assign(nbytes, 0);
    if (cfg->out_dtype == EVAM_DTYPE_F32) build_lut(*cfg, reinterpret_cast<float*>(h->h_block.data()));
    ItemDesc* desc = reinterpret_cast<ItemDesc*>(h->h_block.data() + kLutBytes);
    int order = 0;
    int first[4] = {0, 0, 0, 0};
    for (int f = 0; f < 4; f++) {
        first[f] = order;
        for (int i = 0; i < n_items; i++) {
            if (fmt[i] != f) continue;
            const evam_image& s = srcs[items ? items[i].src_index : i];
            ItemDesc& d = desc[order++];
            for (int p = 0; p < 3; p++) { d.plane[p] = s.planes[p]; d.pitch[p] = s.pitch[p]; }
            const Geom& g = geo[i];
            d.x0 = g.x0; d.y0 = g.y0; d.cw = g.cw; d.ch = g.ch;
            d.rw = g.rw; d.rh = g.rh; d.ox = g.ox; d.oy = g.oy;
            d.slot = dst->slot_offset + i * dst->slot_stride;
            d.pad_ = 0;
            d.scale_x = 1. / ((double)g.rw / g.cw);
            d.scale_y = 1. / ((double)g.rh / g.ch);
        }
    }

    HIP_TRY(hipSetDevice(h->device));
    if (h->h_last.size() != nbytes || memcmp(h->h_last.data(), h->h_block.data(), nbytes) != 0) {
        if (nbytes > h->d_block_cap) {
            if (h->d_block) {
                HIP_TRY(hipStreamSynchronize(h->stream));
                HIP_TRY(hipFree(h->d_block));
                h->d_block = nullptr;
                h->d_block_cap = 0;
            }
            const size_t cap = std::max<size_t>(nbytes * 2, 64 * 1024);
            if (hipMalloc(&h->d_block, cap) != hipSuccess)
                return fail(EVAM_PP_ERR_OOM, "evam_pp_run: hipMalloc(%zu) failed", cap);
            h->d_block_cap = cap;
        }
        // Stream-ordered after every earlier launch that read the block, so it is safe to overwrite.
        HIP_TRY(hipMemcpyAsync(h->d_block, h->h_block.data(), nbytes, hipMemcpyHostToDevice, h->stream));
        h->h_last = h->h_block;
    }

    // ---- launches ----
    if (h->opt_timing) HIP_TRY(hipEventRecord(h->ev0, h->stream));
    int launches = 0;
    for (int f = 0; f < 4; f++) {
        if (!count[f]) continue;
        const TileCfg t = choose_tiles(f, DW, DH, max_ratio[f], cfg->out_dtype);
        if (t.lds > 160 * 1024 || t.strideY >= 32768 || t.strideC >= 32768)
            return fail(EVAM_PP_ERR_UNSUPPORTED, "evam_pp_run: source footprint too wide (%.1fx downscale)", max_ratio[f]);
        KParams p{};
        p.items = reinterpret_cast<const ItemDesc*>(h->d_block + kLutBytes) + first[f];
        p.lut = reinterpret_cast<const float*>(h->d_block);
        p.dst = dst->data;
        p.DW = DW; p.DH = DH;
        p.TW = t.TW; p.TH = t.TH;
        p.tiles_x = (DW + t.TW - 1) / t.TW;
        const int tiles_y = (DH + t.TH - 1) / t.TH;
        p.tiles_per_item = p.tiles_x * tiles_y;
        p.tw_magic = (uint32_t)(0xFFFFFFFFu / (uint32_t)t.TW) + 1u;
        p.strideY = t.strideY; p.strideC = t.strideC;
        p.offRow = t.offRow; p.offSlot = t.offSlot; p.offLut = t.offLut;
        p.offY = t.offY; p.offC = t.offC; p.offV = t.offV;
        p.color_rgb = cfg->color_order == EVAM_COLOR_RGB;
        p.fill = (uint32_t)cfg->fill[0] | ((uint32_t)cfg->fill[1] << 8) | ((uint32_t)cfg->fill[2] << 16);
        const int64_t grid = (int64_t)count[f] * p.tiles_per_item;
        if (grid > 0x7FFFFFFF) return fail(EVAM_PP_ERR_INVALID_ARG, "evam_pp_run: grid too large");
        if (t.lds > 64 * 1024) {
            hipError_t e = hipSuccess;
            switch (f * 2 + cfg->out_dtype) {
#define SETATTR(F, O) case F * 2 + O: e = hipFuncSetAttribute((const void*)evam_pp_kernel<F, O>, hipFuncAttributeMaxDynamicSharedMemorySize, t.lds); break;
                SETATTR(kNV12, 0) SETATTR(kNV12, 1) SETATTR(kI420, 0) SETATTR(kI420, 1)
                SETATTR(kBGRX, 0) SETATTR(kBGRX, 1) SETATTR(kBGR, 0) SETATTR(kBGR, 1)
#undef SETATTR
            }
            if (e != hipSuccess) return fail(EVAM_PP_ERR_HIP, "hipFuncSetAttribute: %s", hipGetErrorString(e));
        }
        hipError_t e = launch(f, cfg->out_dtype, p, (int)grid, t.lds, h->stream);
        if (e != hipSuccess) return fail(EVAM_PP_ERR_HIP, "kernel launch failed: %s", hipGetErrorString(e));
        launches++;
    }
    if (h->opt_timing) HIP_TRY(hipEventRecord(h->ev1, h->stream));
    h->timed = h->opt_timing != 0;

    h->stats.n_items = n_items;
    h->stats.n_launches = launches;
    h->stats.src_bytes = h->opt_stats ? src_bytes : 0;
    h->stats.dst_bytes = (int64_t)n_items * plane * 3 * (cfg->out_dtype == EVAM_DTYPE_F32 ? 4 : 1);
    return EVAM_PP_OK;
}

}  // extern "C"
