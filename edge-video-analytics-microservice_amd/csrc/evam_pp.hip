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
constexpr int kLoaderThreads = 64;   // wave 0: tables + LDS-DMA
constexpr int kConsumers = 256;      // waves 1..4: convert + store
constexpr int kBlock = kLoaderThreads + kConsumers;
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
    int TW, TH, tiles_x, tiles_per_item, n_tiles;
    uint32_t tw_magic;  // ceil(2^32 / TW)
    int tab_bytes;      // one table set: coltab | rowtab | slotY | slotC
    int buf_bytes;      // one staging buffer (upper bound of a tile's packed footprint)
    int offTab, offBuf; // LDS carve: LUT at 0 (fp32 out), 2 table sets at offTab, 2 buffers at offBuf
    int color_rgb;
    uint32_t fill;      // packed u8 fill, output channel order
    int ablate;         // diagnostics only (EVAM_PP_ABLATE bits): 1 no DMA, 2 no pixel math, 4 no stores
};

struct ColEntry {  // 16 B, one per tile column
    int16_t oY0, oY1;  // byte offset of the two taps inside a staged luma/packed row (-1: not in image)
    int16_t oC0, oC1;  // byte offset inside a staged chroma row (NV12: U of the UV pair)
    int16_t a0, a1;    // 11-bit horizontal weights
    int16_t pad0, pad1;
};

struct RowEntry {  // 32 B, one per tile row
    int32_t y0, y1;   // buffer byte offsets of the two staged luma rows (-1: row not in image)
    int32_t c0, c1;   // buffer byte offsets of the two staged chroma rows
    int32_t b0, b1;   // 11-bit vertical weights
    int32_t pad0, pad1;
};

// Per-tile values every lane holds (wave-uniform).
struct TileInfo {
    const uint8_t* plane[3];  // copied out of the descriptor during setup: no descriptor load may sit
    int pitch[3];             // between the DMA issue and the compute (its vmcnt wait would drain the DMA)
    int slot;
    int X0, Y0, X1, Y1;
    int active;        // the tile shows part of the resized image (else pure padding)
    int fsY, cprY;     // luma/packed footprint: 16-B aligned start byte, 16-B chunks per row
    int fsC, cprC;     // chroma footprint
    int offC, offV;    // chroma / V plane offsets inside the staging buffer
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

// BT.601 20-bit fixed point (OpenCV uvToRGBuv + yRGBuvToRGBA). Arguments are raw bytes; every
// product fits the full-rate 24-bit multiplier.
__device__ __forceinline__ void yuv_to_bgr(int Y, int U, int V, int& b, int& g, int& r) {
    const int y = __mul24(max(Y - 16, 0), kCY);
    const int ruv = __mul24(kCVR, V) + kKR;
    const int guv = __mul24(kCVG, V) + __mul24(kCUG, U) + kKG;
    const int buv = __mul24(kCUB, U) + kKB;
    b = clamp255((y + buv) >> 20);
    g = clamp255((y + guv) >> 20);
    r = clamp255((y + ruv) >> 20);
}

template <int FMT>
__device__ __forceinline__ void tap(const uint8_t* __restrict__ buf, int yrow, int crow, int vrow, int oy,
                                    int oc, int& b, int& g, int& r) {
    if constexpr (FMT == kNV12) {
        const int Y = buf[yrow + oy];
        const uint32_t uv = *reinterpret_cast<const uint16_t*>(buf + crow + oc);
        yuv_to_bgr(Y, uv & 0xFF, uv >> 8, b, g, r);
    } else if constexpr (FMT == kI420) {
        const int Y = buf[yrow + oy];
        yuv_to_bgr(Y, buf[crow + oc], buf[vrow + oc], b, g, r);
    } else if constexpr (FMT == kBGRX) {
        const uint32_t p = *reinterpret_cast<const uint32_t*>(buf + yrow + oy);
        b = p & 0xFF; g = (p >> 8) & 0xFF; r = (p >> 16) & 0xFF;
    } else {
        b = buf[yrow + oy]; g = buf[yrow + oy + 1]; r = buf[yrow + oy + 2];
    }
}

// VResizeLinear<uchar,int,short,FixedPtCast<int,uchar,22>,VResizeLinearVec_32s8u>.
// D >> 4 <= 32655 and |b| <= 2048, so both products are exact on the 24-bit multiplier.
__device__ __forceinline__ int vresize(int D0, int D1, int b0, int b1) {
    return ((__mul24(b0, D0 >> 4) >> 16) + (__mul24(b1, D1 >> 4) >> 16) + 2) >> 2;
}

template <int FMT>
struct FmtTraits {
    static constexpr int bpp = FMT == kBGRX ? 4 : (FMT == kBGR ? 3 : 1);
    static constexpr int nchroma = FMT == kNV12 ? 1 : (FMT == kI420 ? 2 : 0);
};

// One 16-byte LDS-DMA load: global -> LDS at (wave-uniform lds_base + lane * 16).
__device__ __forceinline__ void glds16(const uint8_t* g, uint8_t* lds_wave_base) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                     (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

// Issue the LDS-DMA loads of one plane's staged rows. Rows are packed back to back in the buffer
// (row slot s at s * cpr * 16), so chunk c of the flattened (slot, column) space lands at c * 16 and a
// wave's 64 chunks form one contiguous 1 KiB LDS run, as LDS-DMA requires. Skipped slots (row < 0:
// duplicate or invisible rows) issue nothing.
__device__ __forceinline__ void issue_plane(uint8_t* lds_plane, const int32_t* __restrict__ slot_rows, int n_slots,
                                            const uint8_t* __restrict__ plane, int pitch, int fs, int cpr, int tid,
                                            int nthr) {
    if (cpr <= 0) return;
    // c / cpr: shift for powers of two (cpr == 1 included: its magic number would overflow to 0),
    // else the round-up reciprocal (exact for c * cpr < 2^32).
    const bool pow2 = (cpr & (cpr - 1)) == 0;
    const int sh = __builtin_ctz((unsigned)cpr);
    const uint32_t magic = pow2 ? 0u : 0xFFFFFFFFu / (uint32_t)cpr + 1u;
    const int total = n_slots * cpr;
    const int wave_off = tid & ~63;
    for (int c0 = 0; c0 < total; c0 += nthr) {
        const int c = c0 + tid;
        if (c < total) {
            const int slot = pow2 ? (c >> sh) : (int)umulhi((uint32_t)c, magic);
            const int col = c - slot * cpr;
            const int row = slot_rows[slot];
            if (row >= 0)
                glds16(plane + (uint32_t)row * (uint32_t)pitch + fs + col * 16, lds_plane + (c0 + wave_off) * 16);
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

// Per-tile values the consumer waves read from the table set header (written by the loader).
struct TileHdr {
    int X0, Y0, X1, Y1;
    int active, offC, offV, slot;
};
constexpr int kHdrBytes = (int)sizeof(TileHdr);

__device__ __forceinline__ ColEntry* tab_cols(uint8_t* tab) { return reinterpret_cast<ColEntry*>(tab + kHdrBytes); }
__device__ __forceinline__ RowEntry* tab_rows(uint8_t* tab, const KParams& P) {
    return reinterpret_cast<RowEntry*>(tab + kHdrBytes + P.TW * (int)sizeof(ColEntry));
}
__device__ __forceinline__ int32_t* tab_slots(uint8_t* tab, const KParams& P) {
    return reinterpret_cast<int32_t*>(tab + kHdrBytes + P.TW * (int)sizeof(ColEntry) + P.TH * (int)sizeof(RowEntry));
}

// Tile geometry, footprint and coefficient tables, written to the table set `tab` by `nthr` threads.
template <int FMT>
__device__ __forceinline__ void setup_tile(const KParams& P, int t, uint8_t* tab, TileInfo& ti, int tid, int nthr) {
    using T = FmtTraits<FMT>;
    const int item = t / P.tiles_per_item;
    const int tile = t - item * P.tiles_per_item;
    const int ty = tile / P.tiles_x;
    const int tx = tile - ty * P.tiles_x;
    // Descriptors are read-only for the launch: read them through the constant address space so they
    // become scalar (s_load, lgkmcnt) loads, which never wait behind the LDS-DMA on vmcnt.
    const __attribute__((address_space(4))) ItemDesc* it =
        (const __attribute__((address_space(4))) ItemDesc*)(P.items) + item;
    for (int i = 0; i < 3; i++) {
        ti.plane[i] = it->plane[i];
        ti.pitch[i] = it->pitch[i];
    }
    ti.slot = it->slot;
    ti.X0 = tx * P.TW;
    ti.Y0 = ty * P.TH;
    ti.X1 = min(ti.X0 + P.TW, P.DW);
    ti.Y1 = min(ti.Y0 + P.TH, P.DH);
    const int ox = it->ox, oy = it->oy, rw = it->rw, rh = it->rh, cw = it->cw, ch = it->ch;
    const int x0 = it->x0, y0 = it->y0;
    const double scx = it->scale_x, scy = it->scale_y;
    const int dx_lo = max(ti.X0 - ox, 0), dx_hi = min(ti.X1 - ox, rw) - 1;
    const int dy_lo = max(ti.Y0 - oy, 0), dy_hi = min(ti.Y1 - oy, rh) - 1;
    ti.active = dx_lo <= dx_hi && dy_lo <= dy_hi;
    ti.fsY = ti.cprY = ti.fsC = ti.cprC = ti.offC = ti.offV = 0;
    if (ti.active) {
        int sxa, sxb, cd0, cd1;
        linear_coef(dx_lo, scx, cw, true, sxa, cd0, cd1);
        linear_coef(dx_hi, scx, cw, true, sxb, cd0, cd1);
        const int xa = x0 + sxa;                      // first source column touched
        const int xb = x0 + min(sxb + 1, cw - 1);     // last source column touched
        ti.fsY = (xa * T::bpp) & ~15;
        ti.cprY = (((xb * T::bpp + T::bpp + 15) & ~15) - ti.fsY) >> 4;
        if constexpr (FMT == kNV12) {
            ti.fsC = (2 * (xa >> 1)) & ~15;
            ti.cprC = (((2 * (xb >> 1) + 2 + 15) & ~15) - ti.fsC) >> 4;
        } else if constexpr (FMT == kI420) {
            ti.fsC = (xa >> 1) & ~15;
            ti.cprC = ((((xb >> 1) + 1 + 15) & ~15) - ti.fsC) >> 4;
        }
        ti.offC = 2 * P.TH * ti.cprY * 16;
        ti.offV = ti.offC + 2 * P.TH * ti.cprC * 16;
    }
    if (tid == 0) {
        TileHdr h;
        h.X0 = ti.X0; h.Y0 = ti.Y0; h.X1 = ti.X1; h.Y1 = ti.Y1;
        h.active = ti.active; h.offC = ti.offC; h.offV = ti.offV; h.slot = ti.slot;
        *reinterpret_cast<TileHdr*>(tab) = h;
    }
    if (!ti.active) return;
    const int fwY = ti.cprY * 16, fwC = ti.cprC * 16;
    ColEntry* coltab = tab_cols(tab);
    RowEntry* rowtab = tab_rows(tab, P);
    int32_t* slotY = tab_slots(tab, P);
    int32_t* slotC = slotY + 2 * P.TH;
    for (int lx = tid; lx < P.TW; lx += nthr) {
        ColEntry e;
        const int dx = ti.X0 + lx - ox;
        if (ti.X0 + lx < ti.X1 && dx >= 0 && dx < rw) {
            int sx, a0, a1;
            linear_coef(dx, scx, cw, true, sx, a0, a1);
            const int ca = x0 + sx, cb = x0 + min(sx + 1, cw - 1);
            e.oY0 = (int16_t)(ca * T::bpp - ti.fsY);
            e.oY1 = (int16_t)(cb * T::bpp - ti.fsY);
            if constexpr (FMT == kNV12) {
                e.oC0 = (int16_t)(2 * (ca >> 1) - ti.fsC);
                e.oC1 = (int16_t)(2 * (cb >> 1) - ti.fsC);
            } else {
                e.oC0 = (int16_t)((ca >> 1) - ti.fsC);
                e.oC1 = (int16_t)((cb >> 1) - ti.fsC);
            }
            e.a0 = (int16_t)a0;
            e.a1 = (int16_t)a1;
        } else {
            e.oY0 = -1; e.oY1 = -1; e.oC0 = 0; e.oC1 = 0; e.a0 = 0; e.a1 = 0;
        }
        e.pad0 = 0; e.pad1 = 0;
        coltab[lx] = e;
    }
    for (int ly = tid; ly < P.TH; ly += nthr) {
        RowEntry e;
        const int dy = ti.Y0 + ly - oy;
        int ya = -1, yb = -1, ca = -1, cb = -1;
        if (ti.Y0 + ly < ti.Y1 && dy >= 0 && dy < rh) {
            int sy, b0, b1;
            linear_coef(dy, scy, ch, false, sy, b0, b1);
            ya = y0 + min(max(sy, 0), ch - 1);
            yb = y0 + min(max(sy + 1, 0), ch - 1);
            e.y0 = (2 * ly) * fwY;
            e.y1 = yb == ya ? e.y0 : (2 * ly + 1) * fwY;
            if (yb == ya) yb = -1;
            if constexpr (T::nchroma > 0) {
                ca = ya >> 1;
                cb = (yb < 0 ? ya : yb) >> 1;
                e.c0 = ti.offC + (2 * ly) * fwC;
                e.c1 = cb == ca ? e.c0 : ti.offC + (2 * ly + 1) * fwC;
                if (cb == ca) cb = -1;
            } else {
                e.c0 = 0; e.c1 = 0;
            }
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
}

template <int FMT>
__device__ __forceinline__ void issue_tile(const KParams& P, const TileInfo& ti, uint8_t* tab, uint8_t* buf,
                                           int tid, int nthr) {
    using T = FmtTraits<FMT>;
    const int32_t* slotY = tab_slots(tab, P);
    const int32_t* slotC = slotY + 2 * P.TH;
    issue_plane(buf, slotY, 2 * P.TH, ti.plane[0], ti.pitch[0], ti.fsY, ti.cprY, tid, nthr);
    if constexpr (T::nchroma >= 1)
        issue_plane(buf + ti.offC, slotC, 2 * P.TH, ti.plane[1], ti.pitch[1], ti.fsC, ti.cprC, tid, nthr);
    if constexpr (T::nchroma == 2)
        issue_plane(buf + ti.offV, slotC, 2 * P.TH, ti.plane[2], ti.pitch[2], ti.fsC, ti.cprC, tid, nthr);
}

// Convert + resize + normalise + planar store of one tile from its staged footprint (kConsumers threads).
template <int FMT, int OUT>
__device__ __forceinline__ void compute_tile(const KParams& P, uint8_t* tab, const uint8_t* buf,
                                             const float* lut_s, int tid) {
    const TileHdr hd = *reinterpret_cast<const TileHdr*>(tab);
    const size_t plane = (size_t)P.DW * P.DH;
    const size_t slot_base = (size_t)hd.slot * 3 * plane;
    const int npx = P.TW * P.TH;
    const int f0 = P.fill & 0xFF, f1 = (P.fill >> 8) & 0xFF, f2 = (P.fill >> 16) & 0xFF;
    const ColEntry* coltab = tab_cols(tab);
    const RowEntry* rowtab = tab_rows(tab, P);
    const int vdelta = hd.offV - hd.offC;
    for (int p = tid; p < npx; p += kConsumers) {
        const int ly = P.TW == 1 ? p : (int)umulhi((uint32_t)p, P.tw_magic);  // p / TW
        const int lx = p - ly * P.TW;
        const int X = hd.X0 + lx, Y = hd.Y0 + ly;
        if (X >= hd.X1 || Y >= hd.Y1) continue;
        const size_t base = slot_base + (size_t)Y * P.DW + X;
        if (!hd.active || (P.ablate & 2)) {
            if (!(P.ablate & 4)) store_px<OUT>(P, lut_s, base, plane, f0, f1, f2);
            continue;
        }
        const ColEntry ce = coltab[lx];
        const RowEntry re = rowtab[ly];
        if (ce.oY0 < 0 || re.y0 < 0) {
            store_px<OUT>(P, lut_s, base, plane, f0, f1, f2);
            continue;
        }
        int bA, gA, rA, bB, gB, rB;
        tap<FMT>(buf, re.y0, re.c0, re.c0 + vdelta, ce.oY0, ce.oC0, bA, gA, rA);
        tap<FMT>(buf, re.y0, re.c0, re.c0 + vdelta, ce.oY1, ce.oC1, bB, gB, rB);
        const int Db0 = __mul24(bA, ce.a0) + __mul24(bB, ce.a1);
        const int Dg0 = __mul24(gA, ce.a0) + __mul24(gB, ce.a1);
        const int Dr0 = __mul24(rA, ce.a0) + __mul24(rB, ce.a1);
        tap<FMT>(buf, re.y1, re.c1, re.c1 + vdelta, ce.oY0, ce.oC0, bA, gA, rA);
        tap<FMT>(buf, re.y1, re.c1, re.c1 + vdelta, ce.oY1, ce.oC1, bB, gB, rB);
        const int Db1 = __mul24(bA, ce.a0) + __mul24(bB, ce.a1);
        const int Dg1 = __mul24(gA, ce.a0) + __mul24(gB, ce.a1);
        const int Dr1 = __mul24(rA, ce.a0) + __mul24(rB, ce.a1);
        const int vb = vresize(Db0, Db1, re.b0, re.b1);
        const int vg = vresize(Dg0, Dg1, re.b0, re.b1);
        const int vr = vresize(Dr0, Dr1, re.b0, re.b1);
        if (P.ablate & 4) {
            asm volatile("" :: "v"(vb), "v"(vg), "v"(vr));  // keep the math alive
            continue;
        }
        if (P.color_rgb)
            store_px<OUT>(P, lut_s, base, plane, vr, vg, vb);
        else
            store_px<OUT>(P, lut_s, base, plane, vb, vg, vr);
    }
}

// Persistent loader/consumer kernel. Wave 0 is the loader: it builds the tables of tile t + G and
// streams its source footprint into the other staging buffer by LDS-DMA, then waits only for its own
// DMA (it never stores). Waves 1..4 are consumers: they convert tile t and store it, and never wait for
// their stores. One raw s_barrier per tile hands buffer and tables over. Workgroup g processes tiles
// g, g + G, g + 2G, ...; a grid of one workgroup per tile degenerates to load -> barrier -> compute.
template <int FMT, int OUT>
__global__ __launch_bounds__(kBlock) void evam_pp_kernel(const KParams P) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int tid = threadIdx.x;
    const bool loader = __builtin_amdgcn_readfirstlane(tid >> 6) == 0;  // wave 0, provably wave-uniform
    const float* lut_s = reinterpret_cast<const float*>(smem);
    int t = blockIdx.x;
    if (t >= P.n_tiles) return;
    uint8_t* const tab0 = smem + P.offTab;
    uint8_t* const tab1 = tab0 + P.tab_bytes;
    uint8_t* const buf0 = smem + P.offBuf;
    uint8_t* const buf1 = buf0 + P.buf_bytes;
    if (loader) {
        TileInfo ti;
        setup_tile<FMT>(P, t, tab0, ti, tid, kLoaderThreads);
        if (ti.active && !(P.ablate & 1)) issue_tile<FMT>(P, ti, tab0, buf0, tid, kLoaderThreads);
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    } else {
        if constexpr (OUT == 1) {
            float* l = reinterpret_cast<float*>(smem);
            for (int i = tid - kLoaderThreads; i < 768; i += kConsumers) l[i] = P.lut[i];
        }
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    int b = 0;
    for (;;) {
        const int tn = t + (int)gridDim.x;
        const bool has_next = tn < P.n_tiles;
        if (loader) {
            if (has_next) {
                uint8_t* tab_n = b ? tab0 : tab1;
                uint8_t* buf_n = b ? buf0 : buf1;
                TileInfo ti;
                setup_tile<FMT>(P, tn, tab_n, ti, tid, kLoaderThreads);
                if (ti.active && !(P.ablate & 1)) issue_tile<FMT>(P, ti, tab_n, buf_n, tid, kLoaderThreads);
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // own DMA + table writes
            }
        } else {
            compute_tile<FMT, OUT>(P, b ? tab1 : tab0, b ? buf1 : buf0, lut_s, tid - kLoaderThreads);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads of tab/buf done; stores stay in flight
        }
        if (!has_next) break;
        __builtin_amdgcn_s_barrier();
        t = tn;
        b ^= 1;
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
    int TW, TH, strideY, strideC, tab_bytes, buf_bytes, offTab, offBuf, lds;
};

int env_int(const char* name, int dflt) {
    const char* v = getenv(name);
    return (v && *v) ? atoi(v) : dflt;
}

// Tile shape: TW x TH output pixels per 256-thread workgroup iteration (~512 by default), shrunk until
// two table sets + two staging buffers fit the LDS budget. EVAM_PP_TW / EVAM_PP_TH override (tuning).
TileCfg choose_tiles(int f, int DW, int DH, double max_ratio_x, int out_dtype) {
    TileCfg t{};
    if (DW <= 256) t.TW = DW;
    else if (DW % 128 == 0) t.TW = 128;
    else if (DW % 64 == 0) t.TW = 64;
    else t.TW = 128;
    t.TH = std::max(1, std::min(DH, 512 / t.TW));
    t.TW = std::max(1, std::min(DW, env_int("EVAM_PP_TW", t.TW)));
    t.TH = std::max(1, std::min(DH, env_int("EVAM_PP_TH", t.TH)));
    const int bpp = fmt_bpp(f);
    const int nC = f == kNV12 ? 1 : (f == kI420 ? 2 : 0);
    for (;;) {
        const int span = (int)std::ceil((t.TW - 1) * max_ratio_x) + 4;  // source columns touched, upper bound
        t.strideY = ((span * bpp + 32) + 15) & ~15;
        t.strideC = f == kNV12 ? ((span + 2 + 32 + 15) & ~15) : (f == kI420 ? ((span / 2 + 2 + 32 + 15) & ~15) : 0);
        t.tab_bytes = (32 + (int)sizeof(ColEntry) * t.TW + (int)sizeof(RowEntry) * t.TH + 16 * t.TH + 15) & ~15;
        t.buf_bytes = 2 * t.TH * (t.strideY + nC * t.strideC);
        t.offTab = out_dtype == EVAM_DTYPE_F32 ? kLutBytes : 0;
        t.offBuf = t.offTab + 2 * t.tab_bytes;
        t.lds = t.offBuf + 2 * t.buf_bytes;
        if (t.lds <= kLdsBudget) break;
        if (t.TH > 1) t.TH = std::max(1, t.TH / 2);
        else if (t.TW > 16) t.TW = std::max(16, t.TW / 2);
        else break;
    }
    return t;
}

template <int FMT, int OUT>
hipError_t launch_t(const KParams& p, int grid, int lds, hipStream_t s) {
    hipLaunchKernelGGL((evam_pp_kernel<FMT, OUT>), dim3(grid), dim3(kBlock), lds, s, p);
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
    int n_cu = 256;
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
    if (hipDeviceGetAttribute(&h->n_cu, hipDeviceAttributeMultiprocessorCount, hip_device) != hipSuccess || h->n_cu <= 0)
        h->n_cu = 256;
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
        const int64_t n_tiles = (int64_t)count[f] * p.tiles_per_item;
        if (n_tiles > 0x7FFFFFFF) return fail(EVAM_PP_ERR_INVALID_ARG, "evam_pp_run: too many tiles");
        p.n_tiles = (int)n_tiles;
        p.tw_magic = t.TW > 1 ? (uint32_t)(0xFFFFFFFFu / (uint32_t)t.TW) + 1u : 0u;
        p.tab_bytes = t.tab_bytes; p.buf_bytes = t.buf_bytes;
        p.offTab = t.offTab; p.offBuf = t.offBuf;
        p.color_rgb = cfg->color_order == EVAM_COLOR_RGB;
        p.ablate = env_int("EVAM_PP_ABLATE", 0);
        p.fill = (uint32_t)cfg->fill[0] | ((uint32_t)cfg->fill[1] << 8) | ((uint32_t)cfg->fill[2] << 16);
        // Persistent grid: every resident workgroup slot gets a strided share of the tiles.
        // EVAM_PP_WGS_PER_CU=0 launches one workgroup per tile instead (no cross-tile prefetch).
        // Default: persistent, as many workgroups per CU as LDS and the 32-wave limit allow.
        const int per_cu = env_int("EVAM_PP_WGS_PER_CU",
                                   std::max(1, std::min(32 / (kBlock / 64), (160 * 1024) / std::max(t.lds, 1))));
        int64_t grid = per_cu > 0 ? std::min<int64_t>(n_tiles, (int64_t)h->n_cu * per_cu) : n_tiles;
        int lds = t.lds;
        if (grid == n_tiles) {
            // One tile per workgroup: no prefetch, so one table set + one buffer; the smaller LDS
            // footprint buys occupancy (latency hiding across workgroups instead of inside one).
            p.offBuf = t.offTab + t.tab_bytes;
            lds = p.offBuf + t.buf_bytes;
        }
        if (lds > 64 * 1024) {
            hipError_t e = hipSuccess;
            switch (f * 2 + cfg->out_dtype) {
#define SETATTR(F, O) case F * 2 + O: e = hipFuncSetAttribute((const void*)evam_pp_kernel<F, O>, hipFuncAttributeMaxDynamicSharedMemorySize, lds); break;
                SETATTR(kNV12, 0) SETATTR(kNV12, 1) SETATTR(kI420, 0) SETATTR(kI420, 1)
                SETATTR(kBGRX, 0) SETATTR(kBGRX, 1) SETATTR(kBGR, 0) SETATTR(kBGR, 1)
#undef SETATTR
            }
            if (e != hipSuccess) return fail(EVAM_PP_ERR_HIP, "hipFuncSetAttribute: %s", hipGetErrorString(e));
        }
        hipError_t e = launch(f, cfg->out_dtype, p, (int)grid, lds, h->stream);
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
