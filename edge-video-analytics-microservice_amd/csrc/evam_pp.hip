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
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <tuple>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>
#include <immintrin.h>

#include "../../include/evam_pp.h"

#define EVAM_HD __host__ __device__
#include "evam_geom.h"
#include "evam_rings.h"
#include "evam_clip_simd.h"

namespace {

using namespace evam;

// ------------------------------------------------------------------------------------------------
// constants
// ------------------------------------------------------------------------------------------------
constexpr int kThreads = 256;

constexpr int kLutBytes = 3 * 256 * 4;
// Stage-removal diagnostics (bits: 2 no pixel math, 4 no stores, 8 loads only, 16 no loads, 32/64/128 stop
// early). Compile-time only: a product build is 0, every diagnostic branch folds away, and no environment
// setting can change results. A build with -DEVAM_PP_ABLATE=bits computes INVALID tensors; evam_pp_create
// refuses it unless EVAM_PP_DIAGNOSTIC_BUILD_OK=1 (tools/prof_ablate.sh).
#ifndef EVAM_PP_ABLATE
#define EVAM_PP_ABLATE 0
#endif
constexpr int kAblate = EVAM_PP_ABLATE;
// Cache-policy bits of the output stores: 2 = nt (non-temporal). The outputs are written once and
// read by nobody in the launch; streaming them past the caches measured 1.5-3 % faster on C2/C3/C4
// and 10 % on C5 (profiles/r02r_store_policy.txt). EVAM_PP_LOAD_AUX: the same bits for the LDS-DMA
// source reads (A/B builds).
#ifndef EVAM_PP_STORE_AUX
#define EVAM_PP_STORE_AUX 2
#endif
#ifndef EVAM_PP_LOAD_AUX
#define EVAM_PP_LOAD_AUX 0
#endif

// OpenCV color_yuv.simd.hpp ITUR_BT_601_*; the -128 chroma bias is folded into the constants.
constexpr int kCY = 1220542, kCUB = 2116026, kCUG = -409993, kCVG = -852492, kCVR = 1673527;
constexpr int kHalf = 1 << 19;
constexpr int kKR = kHalf - 128 * kCVR - 16 * kCY;  // the luma term is max(Y,16)*CY (see yuv_to_bgr)
constexpr int kKG = kHalf - 128 * kCVG - 128 * kCUG - 16 * kCY;
constexpr int kKB = kHalf - 128 * kCUB - 16 * kCY;

// ------------------------------------------------------------------------------------------------
// device-side descriptors
// ------------------------------------------------------------------------------------------------
struct alignas(16) ItemDesc {
    const uint8_t* plane[3];
    int32_t pitch[3];
    int32_t x0, y0, cw, ch;  // effective crop in source pixels
    int32_t rw, rh, ox, oy;  // resized size, placement in the DW x DH plane
    int32_t index;    // item index in the call: output slot = slot_offset + index * slot_stride
    int32_t pad_;
    double scale_x, scale_y; // OpenCV: 1. / ((double)rw / cw)
};
static_assert(sizeof(ItemDesc) == 96, "ItemDesc layout");

struct KParams {
    const ItemDesc* items;
    const float* lut;  // [3][256]
    void* dst;
    int slot_offset, slot_stride;  // output slot of item i = slot_offset + i * slot_stride
    int DW, DH;
    int TW, TH, tiles_x, tiles_per_item, n_tiles;
    uint32_t tw_magic;  // ceil(2^32 / TW) (TW > 1)
    int offCol, offRow; // LDS carve: LUT at 0 (fp32 out), column table, row table
    int color_rgb;
    uint32_t fill;      // packed u8 fill, output channel order
};

// Per output column of a tile: absolute byte offsets of the two horizontal taps inside a source row.
struct alignas(16) ColEntry {  // 16 B
    int32_t oY0, oY1;  // luma / packed-pixel byte offsets of tap 0 / tap 1 (always valid addresses)
    int32_t oC0;       // chroma byte offset of tap 0 (NV12: U of the UV pair; I420: U/V plane column)
    uint16_t a0, a1;   // 11-bit horizontal weights << 4 (see vresize); both 0: the column shows padding
};
// Per output row of a tile: byte offsets of the two vertical taps' rows inside the planes.
struct alignas(16) RowEntry {  // 32 B
    int32_t y0, y1;   // row offsets in the luma / packed plane (always valid addresses)
    int32_t c0, c1;   // row offsets in the chroma plane(s) (I420: same offset for U and V)
    int32_t b0, b1;   // 11-bit vertical weights << 8 (see vresize); both 0: the row shows padding
    int32_t pad0, pad1;
};

// Per-item arguments of the uniform-geometry kernels (staged / wave / rows), carried in the launch's
// kernel arguments: every item of such a launch shares crop size, resized size and placement, so an
// item differs only in its frame (planes, pitches), its crop origin and its output slot. Passing them
// in the kernarg segment means a new set of frames (a decoder's next surfaces, a rotating frame pool)
// costs no descriptor upload and no cross-stream wait; launches take up to kArgItems items each.
struct ItemArg {  // 48 B
    const uint8_t* plane[3];
    int32_t pitch[3];
    int32_t x0, y0;   // crop origin in source pixels
    int32_t index;    // item index in the call: output slot = slot_offset + index * slot_stride
};
static_assert(sizeof(ItemArg) == 48, "ItemArg layout");
constexpr int kArgItems = 64;  // 3 KB of items per launch; the whole parameter block stays < 4 KB


struct RParams {
    ItemArg items[kArgItems];
    int ox, rw;          // uniform placement / resized width
    const float* lut;    // [3][256]
    const XTab* xtab;    // [DW]
    const YTab* ytab;    // [DH]
    void* dst;
    int slot_offset, slot_stride;  // output slot of item i = slot_offset + i * slot_stride
    int DW, DH;
    int TW, TH, tiles_x, tiles_per_item;
    int nsegx;           // TW / 64 column segments per tile row
    int color_rgb;
    uint32_t fill;
};

constexpr int kSlot = 1024;  // bytes of one staged source-row segment = one wave-wide 16 B/lane LDS-DMA

struct SParams {
    ItemArg items[kArgItems];
    int ox, rw;          // uniform placement / resized width
    const float* lut;    // [3][256]
    const XTab* xtab;    // [DW]
    const YTab* ytab;    // [DH]
    void* dst;
    int slot_offset, slot_stride;  // output slot of item i = slot_offset + i * slot_stride
    int DW, DH;
    int TH, tiles_x, tiles_per_item;
    int offBuf;          // LDS offset of staging buffer 0 (after the LUT)
    int buf_bytes;       // one staging buffer: 2 R planes x slot_bytes
    int slot_bytes;      // one staged row segment: the widest 16-byte-aligned footprint of the launch
    int color_rgb;
    uint32_t fill;
    int xcd_remap;       // 1: consecutive tiles land on one XCD (shared halo rows stay in one L2)
    int ntcol;           // tiles_x when <= kTCols (tcol valid), else 0 (the kernel reads xtab)
    int2 tcol[16];       // per tile column: crop-relative source columns of its first / last visible
                         // output column's taps, or (-1, -1) for a tile of padding columns only
};
constexpr int kTCols = 16;

// Workgroups are dispatched round-robin over the 8 XCDs (block b runs on XCD b % 8). Remap so each
// XCD walks a contiguous run of tiles: neighbouring tiles of one frame share source rows at their
// edges, and those rows then hit the same L2. Bijective for any grid size.
__device__ inline int xcd_tile(int b, int grid) {
    const int q = grid >> 3, r = grid & 7, x = b & 7, i = b >> 3;
    return x < r ? x * (q + 1) + i : r * (q + 1) + (x - r) * q + i;
}

// ------------------------------------------------------------------------------------------------
// exact OpenCV arithmetic (shared host/device)
// ------------------------------------------------------------------------------------------------

__device__ __forceinline__ uint32_t umulhi(uint32_t a, uint32_t b) { return __umulhi(a, b); }

__device__ __forceinline__ int clamp255(int v) { return min(max(v, 0), 255); }

// BT.601 20-bit fixed point (OpenCV uvToRGBuv + yRGBuvToRGBA). Arguments are raw bytes; every
// product fits the full-rate 24-bit multiplier.
__device__ __forceinline__ void yuv_to_bgr(int Y, int U, int V, int& b, int& g, int& r) {
    const int y = __mul24(max(Y, 16), kCY);  // max(Y-16,0)*CY + 16*CY; the 16*CY is folded into kK*
    const int ruv = __mul24(kCVR, V) + kKR;
    const int guv = __mul24(kCVG, V) + __mul24(kCUG, U) + kKG;
    const int buv = __mul24(kCUB, U) + kKB;
    b = clamp255((y + buv) >> 20);
    g = clamp255((y + guv) >> 20);
    r = clamp255((y + ruv) >> 20);
}

// VResizeLinear<uchar,int,short,FixedPtCast<int,uchar,22>,VResizeLinearVec_32s8u>:
//   dst = (((b0 * (D0 >> 4)) >> 16) + ((b1 * (D1 >> 4)) >> 16) + 2) >> 2
// evaluated on the full-rate 24-bit multiplier. The column table holds a' = a << 4 and the row table
// b' = b << 8, so the horizontal pass yields D' = D << 4 (< 2^23) and
//   (b * (D >> 4)) >> 16 == mulhi_u24(b', D' & ~0xFF)
// exactly (b' * ((D >> 4) << 8) = b * (D >> 4) * 2^16).
__device__ __forceinline__ uint32_t mulhi_u24(uint32_t a, uint32_t b) {
    return (uint32_t)(((uint64_t)(a & 0xFFFFFFu) * (uint64_t)(b & 0xFFFFFFu)) >> 32);
}
__device__ __forceinline__ int vresize(uint32_t D0s, uint32_t D1s, uint32_t b0s, uint32_t b1s) {
    return (int)((mulhi_u24(b0s, D0s & 0xFFFF00u) + mulhi_u24(b1s, D1s & 0xFFFF00u) + 2u) >> 2);
}
// Same, for OUT == 1 returned as 4 * result (the byte offset into a float LUT section).
template <int OUT>
__device__ __forceinline__ uint32_t vfinal(uint32_t D0s, uint32_t D1s, uint32_t b0s, uint32_t b1s) {
    const uint32_t x = mulhi_u24(b0s, D0s & 0xFFFF00u) + mulhi_u24(b1s, D1s & 0xFFFF00u) + 2u;
    return OUT == 1 ? (x & ~3u) : (x >> 2);
}
// Same, for horizontal results already masked with kVMask (a kernel that reuses a source row's results).
constexpr uint32_t kVMask = 0xFFFF00u;
template <int OUT>
__device__ __forceinline__ uint32_t vfinal_masked(uint32_t D0m, uint32_t D1m, uint32_t b0s, uint32_t b1s) {
    const uint32_t x = mulhi_u24(b0s, D0m) + mulhi_u24(b1s, D1m) + 2u;
    return OUT == 1 ? (x & ~3u) : (x >> 2);
}

template <int FMT>
struct FmtTraits {
    static constexpr int bpp = FMT == kBGRX ? 4 : (FMT == kBGR ? 3 : 1);
    static constexpr int nchroma = FMT == kNV12 ? 1 : (FMT == kI420 ? 2 : 0);
};

// Raw bytes of one source pixel, read straight from the frame (global memory, through L1/L2).
// Plane bases are wave-uniform (SGPR) and offsets 32-bit, so each load is one saddr-form instruction.
template <int FMT>
__device__ __forceinline__ void load_tap(const uint8_t* __restrict__ p0, const uint8_t* __restrict__ p1,
                                         const uint8_t* __restrict__ p2, uint32_t oy, uint32_t oc, uint32_t (&v)[3]) {
    if constexpr (FMT == kNV12) {
        v[0] = p0[oy];
        v[1] = *reinterpret_cast<const uint16_t*>(p1 + oc);
    } else if constexpr (FMT == kI420) {
        v[0] = p0[oy];
        v[1] = p1[oc];
        v[2] = p2[oc];
    } else if constexpr (FMT == kBGRX) {
        v[0] = *reinterpret_cast<const uint32_t*>(p0 + oy);
    } else {
        v[0] = p0[oy];
        v[1] = p0[oy + 1];
        v[2] = p0[oy + 2];
    }
}

template <int FMT>
__device__ __forceinline__ void to_bgr(const uint32_t (&v)[3], int& b, int& g, int& r) {
    if constexpr (FMT == kNV12) {
        yuv_to_bgr((int)v[0], (int)(v[1] & 0xFF), (int)(v[1] >> 8), b, g, r);
    } else if constexpr (FMT == kI420) {
        yuv_to_bgr((int)v[0], (int)v[1], (int)v[2], b, g, r);
    } else if constexpr (FMT == kBGRX) {
        b = v[0] & 0xFF; g = (v[0] >> 8) & 0xFF; r = (v[0] >> 16) & 0xFF;
    } else {
        b = (int)v[0]; g = (int)v[1]; r = (int)v[2];
    }
}

// Planar stores of one pixel. Plane bases are wave-uniform (SGPR) and the offset is a 32-bit byte
// offset, so every store is one saddr-form instruction with no 64-bit address arithmetic.
template <int OUT>
__device__ __forceinline__ void store_px(uint8_t* d0, uint8_t* d1, uint8_t* d2, const float* __restrict__ lut,
                                         uint32_t o, int v0, int v1, int v2) {
    if constexpr (OUT == 0) {
        d0[o] = (uint8_t)v0;
        d1[o] = (uint8_t)v1;
        d2[o] = (uint8_t)v2;
    } else {
        const uint32_t ob = o << 2;
        *reinterpret_cast<float*>(d0 + ob) = lut[v0];
        *reinterpret_cast<float*>(d1 + ob) = lut[256 + v1];
        *reinterpret_cast<float*>(d2 + ob) = lut[512 + v2];
    }
}

// One workgroup per output tile (TW x TH pixels of one item). The workgroup builds the OpenCV
// coefficient tables of its columns and rows in LDS (device-side, exact double/float sequence), then
// every lane gathers the four taps of its pixels directly from the frame in HBM — luma and chroma
// bytes through L1, adjacent lanes sharing cache lines — converts them to BGR, runs both resize passes,
// maps the u8 result through the normalisation LUT and stores the three planes. No staging, no barrier
// after the tables: the memory pipeline overlaps loads of many pixels and many waves.
template <int FMT, int OUT>
__global__ __launch_bounds__(kThreads) void evam_pp_kernel(const KParams P) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    using T = FmtTraits<FMT>;
    const int tid = threadIdx.x;
    const int t = blockIdx.x;
    const int item = t / P.tiles_per_item;
    const int tile = t - item * P.tiles_per_item;
    const int ty = tile / P.tiles_x;
    const int tx = tile - ty * P.tiles_x;
    // Descriptors are read-only for the launch: the constant address space makes them scalar loads.
    const __attribute__((address_space(4))) ItemDesc* it =
        (const __attribute__((address_space(4))) ItemDesc*)(P.items) + item;
    const uint8_t* __restrict__ p0 = it->plane[0];
    const uint8_t* __restrict__ p1 = it->plane[1];
    const uint8_t* __restrict__ p2 = it->plane[2];
    const int pitch0 = it->pitch[0], pitch1 = it->pitch[1];
    const int x0 = it->x0, y0 = it->y0, cw = it->cw, ch = it->ch;
    const int rw = it->rw, rh = it->rh, ox = it->ox, oy = it->oy;
    const double scx = it->scale_x, scy = it->scale_y;
    const int X0 = tx * P.TW, Y0 = ty * P.TH;
    const int X1 = min(X0 + P.TW, P.DW), Y1 = min(Y0 + P.TH, P.DH);
    const size_t plane = (size_t)P.DW * P.DH;
    const size_t esz = OUT == 1 ? 4 : 1;
    uint8_t* const d0 = reinterpret_cast<uint8_t*>(P.dst) + (size_t)(P.slot_offset + it->index * P.slot_stride) * 3 * plane * esz;
    uint8_t* const d1 = d0 + plane * esz;
    uint8_t* const d2 = d1 + plane * esz;

    float* lut_s = reinterpret_cast<float*>(smem);
    if constexpr (OUT == 1) {
        for (int i = tid; i < 768; i += kThreads) lut_s[i] = P.lut[i];
    }
    ColEntry* coltab = reinterpret_cast<ColEntry*>(smem + P.offCol);
    RowEntry* rowtab = reinterpret_cast<RowEntry*>(smem + P.offRow);
    for (int lx = tid; lx < P.TW; lx += kThreads) {
        ColEntry e;
        const int dx = X0 + lx - ox;
        if (X0 + lx < X1 && dx >= 0 && dx < rw) {
            int sx, a0, a1;
            linear_coef(dx, scx, cw, true, sx, a0, a1);
            const int ca = x0 + sx, cb = x0 + min(sx + 1, cw - 1);
            e.oY0 = ca * T::bpp;
            e.oY1 = cb * T::bpp;
            e.oC0 = FMT == kNV12 ? 2 * (ca >> 1) : (ca >> 1);
            e.a0 = (uint16_t)(a0 << 4);
            e.a1 = (uint16_t)(a1 << 4);
        } else {
            e.oY0 = 0; e.oY1 = 0; e.oC0 = 0; e.a0 = 0; e.a1 = 0;
        }
        coltab[lx] = e;
    }
    for (int ly = tid; ly < P.TH; ly += kThreads) {
        RowEntry e;
        const int dy = Y0 + ly - oy;
        if (Y0 + ly < Y1 && dy >= 0 && dy < rh) {
            int sy, b0, b1;
            linear_coef(dy, scy, ch, false, sy, b0, b1);
            const int ya = y0 + min(max(sy, 0), ch - 1);
            const int yb = y0 + min(max(sy + 1, 0), ch - 1);
            e.y0 = ya * pitch0;
            e.y1 = yb * pitch0;
            e.c0 = (ya >> 1) * pitch1;
            e.c1 = (yb >> 1) * pitch1;
            e.b0 = b0 << 8;
            e.b1 = b1 << 8;
        } else {
            e.y0 = 0; e.y1 = 0; e.c0 = 0; e.c1 = 0; e.b0 = 0; e.b1 = 0;
        }
        e.pad0 = 0; e.pad1 = 0;
        rowtab[ly] = e;
    }
    __syncthreads();

    const int f0 = P.fill & 0xFF, f1 = (P.fill >> 8) & 0xFF, f2 = (P.fill >> 16) & 0xFF;
    const int npx = P.TW * P.TH;
    // (lx, ly) of pixel p = tid + k * 256, advanced incrementally (no per-pixel division).
    const int qstep = kThreads / P.TW, rstep = kThreads - qstep * P.TW;
    int ly = tid / P.TW;
    int lx = tid - ly * P.TW;
    const uint32_t o_tile = (uint32_t)(Y0 * P.DW + X0);

    // Software pipeline, one pixel deep: the tap loads of pixel k+1 are issued before pixel k is
    // converted, so every wave always has a pixel's loads in flight while it computes.
    struct Px {
        uint32_t raw[4][3];
        uint32_t o, wa, wb0, wb1;
        int mode;  // 0: outside the tile, 1: padding / fill, 2: image pixel
    };
    auto gather = [&](int p, Px& x) {
        const int cx = lx, cy = ly;
        lx += rstep;
        ly += qstep;
        if (lx >= P.TW) { lx -= P.TW; ly++; }
        const bool in_tile = p < npx && X0 + cx < X1 && Y0 + cy < Y1;
        const ColEntry ce = coltab[in_tile ? cx : 0];
        const RowEntry re = rowtab[in_tile ? cy : 0];
        x.wa = (uint32_t)ce.a0 | ((uint32_t)ce.a1 << 16);
        x.wb0 = (uint32_t)re.b0;
        x.wb1 = (uint32_t)re.b1;
        const bool img = in_tile && x.wa != 0 && (x.wb0 | x.wb1) != 0 && !(kAblate & 2);
        x.mode = !in_tile ? 0 : (img ? 2 : 1);
        x.o = o_tile + __umul24((uint32_t)cy, (uint32_t)P.DW) + (uint32_t)cx;
        if (kAblate & 16) {  // diagnostics: no loads, math on synthetic bytes
            for (int k = 0; k < 4; k++) { x.raw[k][0] = (ce.oY0 + k) & 255; x.raw[k][1] = (re.y0 + ce.oC0 * k) & 0xFFFF; x.raw[k][2] = k; }
            return;
        }
        // Table offsets are valid addresses even for padding / out-of-tile lanes: no selects here.
        const uint32_t oc1 = FMT == kNV12 ? ((uint32_t)ce.oY1 & ~1u) : ((uint32_t)ce.oY1 >> 1);  // tap-1 chroma
        load_tap<FMT>(p0, p1, p2, (uint32_t)(re.y0 + ce.oY0), (uint32_t)(re.c0 + ce.oC0), x.raw[0]);
        load_tap<FMT>(p0, p1, p2, (uint32_t)(re.y0 + ce.oY1), (uint32_t)re.c0 + oc1, x.raw[1]);
        load_tap<FMT>(p0, p1, p2, (uint32_t)(re.y1 + ce.oY0), (uint32_t)(re.c1 + ce.oC0), x.raw[2]);
        load_tap<FMT>(p0, p1, p2, (uint32_t)(re.y1 + ce.oY1), (uint32_t)re.c1 + oc1, x.raw[3]);
    };
    auto finish = [&](const Px& x) {
        if (x.mode == 0) return;
        if (x.mode == 1) {
            if (!(kAblate & 4)) store_px<OUT>(d0, d1, d2, lut_s, x.o, f0, f1, f2);
            return;
        }
        if (kAblate & 8) {  // diagnostics: loads only, trivial math
            uint32_t acc = 0;
            for (int k = 0; k < 4; k++) acc += x.raw[k][0] + x.raw[k][1] + x.raw[k][2];
            asm volatile("" :: "v"(acc));
            return;
        }
        const uint32_t a0 = x.wa & 0xFFFF, a1 = x.wa >> 16;  // 15-bit
        int bA, gA, rA, bB, gB, rB;
        to_bgr<FMT>(x.raw[0], bA, gA, rA);
        to_bgr<FMT>(x.raw[1], bB, gB, rB);
        const uint32_t Db0 = __umul24(bA, a0) + __umul24(bB, a1);
        const uint32_t Dg0 = __umul24(gA, a0) + __umul24(gB, a1);
        const uint32_t Dr0 = __umul24(rA, a0) + __umul24(rB, a1);
        to_bgr<FMT>(x.raw[2], bA, gA, rA);
        to_bgr<FMT>(x.raw[3], bB, gB, rB);
        const uint32_t Db1 = __umul24(bA, a0) + __umul24(bB, a1);
        const uint32_t Dg1 = __umul24(gA, a0) + __umul24(gB, a1);
        const uint32_t Dr1 = __umul24(rA, a0) + __umul24(rB, a1);
        const int vb = vresize(Db0, Db1, x.wb0, x.wb1);
        const int vg = vresize(Dg0, Dg1, x.wb0, x.wb1);
        const int vr = vresize(Dr0, Dr1, x.wb0, x.wb1);
        if (kAblate & 4) {
            asm volatile("" :: "v"(vb), "v"(vg), "v"(vr));  // keep the math alive
            return;
        }
        if (P.color_rgb)
            store_px<OUT>(d0, d1, d2, lut_s, x.o, vr, vg, vb);
        else
            store_px<OUT>(d0, d1, d2, lut_s, x.o, vb, vg, vr);
    };
    if (tid >= npx) return;
    Px cur, nxt;
    gather(tid, cur);
    for (int p = tid + kThreads; p < npx; p += kThreads) {
        gather(p, nxt);
        finish(cur);
        cur = nxt;
    }
    finish(cur);
}

// BT.601 split into the chroma part (per chroma sample) and the per-luma part, so a chroma sample
// shared by two taps is converted once. Same integers as yuv_to_bgr.
struct UV3 { int b, g, r; };
__device__ __forceinline__ UV3 uv_terms(int U, int V) {
    return UV3{__mul24(kCUB, U) + kKB, __mul24(kCVG, V) + __mul24(kCUG, U) + kKG, __mul24(kCVR, V) + kKR};
}
__device__ __forceinline__ void y_plus_uv(int Y, const UV3& t, int& b, int& g, int& r) {
    const int y = __mul24(max(Y, 16), kCY);
    b = clamp255((y + t.b) >> 20);
    g = clamp255((y + t.g) >> 20);
    r = clamp255((y + t.r) >> 20);
}

// Saturating form of the same integers, two taps per register. The chroma terms carry the bias
// 2^32 - 2^28 on top of kK*, so for S = y + term (the BT.601 sum before >> 20) the unsigned
// saturating add y + term' is S + 2^32 - 2^28 when S < 2^28 and 0xFFFFFFFF otherwise; every term'
// lies in [0, 2^32) (no wrap). Its high half is then floor(S / 2^16) + 61440, and one u16
// saturating subtract of 61440 clamps it to [0, 4095], i.e. to 16 * clamp255(S >> 20) plus four
// low bits that a mask drops. Two taps' high halves share one register (v_perm), so the clamp costs
// a packed subtract and a mask per tap pair, and the horizontal pass D = c0*a0 + c1*a1 is one
// v_dot2_u32_u16 that yields 16 * D, the D' vresize takes. tools/check_sat_clamp.py checks the
// clamp against clamp255((y + term) >> 20) over all 2^24 (Y, U, V).
typedef unsigned short evam_u16x2 __attribute__((ext_vector_type(2)));
constexpr uint32_t kSatBias = 0xF0000000u;  // 2^32 - 2^28
constexpr uint32_t kKBs = (uint32_t)kKB + kSatBias, kKGs = (uint32_t)kKG + kSatBias, kKRs = (uint32_t)kKR + kSatBias;
struct UVs { uint32_t b, g, r; };
__device__ __forceinline__ UVs uv_terms_sat(uint32_t U, uint32_t V) {
    // G as two chained v_mad_i32_i24 (the opaque middle value keeps the compiler from re-forming two products and
    // an add3): 4 VALU per chroma sample instead of 5
    int gu = __mul24((int)U, kCUG) + (int)kKGs;
    asm("" : "+v"(gu));
    return UVs{__umul24(U, (uint32_t)kCUB) + kKBs, (uint32_t)(__mul24((int)V, kCVG) + gu), __umul24(V, (uint32_t)kCVR) + kKRs};
}
__device__ __forceinline__ uint32_t luma_term(uint32_t Y) { return __umul24(max(Y, 16u), (uint32_t)kCY); }
// One source row, one channel: taps' sums s0 (column x0) and s1 (column x1), packed weights w = a0 | a1 << 16
// (plain 11-bit) -> 16 * (c0 * a0 + c1 * a1).
// hpass_sums: the same from the taps' saturated sums (pixels whose taps meet at one column share a sum).
__device__ __forceinline__ uint32_t hpass_sums(uint32_t s0, uint32_t s1, uint32_t w) {
    const evam_u16x2 h = __builtin_bit_cast(evam_u16x2, __builtin_amdgcn_perm(s1, s0, 0x07060302u));
    const evam_u16x2 c = __builtin_elementwise_sub_sat(h, (evam_u16x2){61440, 61440});
    const uint32_t c16 = __builtin_bit_cast(uint32_t, c) & 0xFFF0FFF0u;
    return __builtin_amdgcn_udot2(__builtin_bit_cast(evam_u16x2, c16), __builtin_bit_cast(evam_u16x2, w), 0u, false);
}
__device__ __forceinline__ uint32_t hpass_sat(uint32_t y0, uint32_t t0, uint32_t y1, uint32_t t1, uint32_t w) {
    return hpass_sums(__builtin_elementwise_add_sat(y0, t0), __builtin_elementwise_add_sat(y1, t1), w);
}
// u8 bytes (x >> 2) of four vertical-pass sums x = mulhi + mulhi + 2 < 2^16 (each result <= 255), packed little-endian: two u16 pairs, one packed
// shift each, one byte permute (5 VALU for 4 pixels instead of 4 shifts and 4 shift / or steps)
__device__ __forceinline__ uint32_t pack4_u8_sums(uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3) {
    const evam_u16x2 p01 = __builtin_bit_cast(evam_u16x2, x0 | (x1 << 16)) >> (evam_u16x2){2, 2};
    const evam_u16x2 p23 = __builtin_bit_cast(evam_u16x2, x2 | (x3 << 16)) >> (evam_u16x2){2, 2};
    return __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, p23), __builtin_bit_cast(uint32_t, p01), 0x06040200u);
}

// Horizontal pass of one source row, three channels, from the two taps' luma bytes and chroma terms.
__device__ __forceinline__ void hrow_sat(uint32_t Y0, uint32_t Y1, const UVs& tA, const UVs& tB, uint32_t w,
                                         uint32_t (&H)[3]) {
    const uint32_t yA = luma_term(Y0), yB = luma_term(Y1);
    H[0] = hpass_sat(yA, tA.b, yB, tB.b, w);
    H[1] = hpass_sat(yA, tA.g, yB, tB.g, w);
    H[2] = hpass_sat(yA, tA.r, yB, tB.r, w);
}

template <int FMT>
struct Chroma {  // raw chroma of one tap: NV12 packed UV (u16), I420 U and V bytes
    uint32_t u, v;
};
template <int FMT>
__device__ __forceinline__ UV3 chroma_terms(const Chroma<FMT>& c) {
    if constexpr (FMT == kNV12) return uv_terms((int)(c.u & 0xFF), (int)(c.u >> 8));
    else return uv_terms((int)c.u, (int)c.v);
}

// Uniform-geometry kernel: every item of the launch has the same crop size, resized size and
// placement, so the coefficient tables come precomputed from the host (XTab / YTab, L2-resident) and
// each wave walks whole 64-pixel row segments. Row pointers, vertical weights and the destination row
// are wave-uniform SGPR values; column offsets and horizontal weights are per-lane registers loaded
// once per workgroup. The inner loop therefore spends its VALU slots on the arithmetic alone. When
// both vertical taps read the same chroma row (4:2:0, ~half the rows) their chroma is loaded and
// converted once.
template <int FMT, int OUT>
__global__ __launch_bounds__(kThreads) void evam_pp_rows(const RParams P) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    using T = FmtTraits<FMT>;
    constexpr bool kYUV = FMT == kNV12 || FMT == kI420;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int t = blockIdx.x;
    const int item = t / P.tiles_per_item;
    const int tile = t - item * P.tiles_per_item;
    const int ty = tile / P.tiles_x;
    const int tx = tile - ty * P.tiles_x;
    const ItemArg& it = P.items[item];
    const __attribute__((address_space(4))) YTab* ytab = (const __attribute__((address_space(4))) YTab*)(P.ytab);
    const uint8_t* __restrict__ p0 = it.plane[0];
    const uint8_t* __restrict__ p1 = it.plane[1];
    const uint8_t* __restrict__ p2 = it.plane[2];
    const int pitch0 = it.pitch[0], pitch1 = it.pitch[1], pitch2 = it.pitch[2];
    const int x0 = it.x0, y0 = it.y0;
    const size_t plane = (size_t)P.DW * P.DH;
    const size_t esz = OUT == 1 ? 4 : 1;
    uint8_t* const d0 = reinterpret_cast<uint8_t*>(P.dst) + (size_t)(P.slot_offset + it.index * P.slot_stride) * 3 * plane * esz;
    uint8_t* const d1 = d0 + plane * esz;
    uint8_t* const d2 = d1 + plane * esz;
    // Buffer resources (wave-uniform). Offsets are always in range by construction, so the range
    // check is set wide open.
    const __amdgpu_buffer_rsrc_t rsY = __builtin_amdgcn_make_buffer_rsrc((void*)p0, (short)0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsC = __builtin_amdgcn_make_buffer_rsrc((void*)(p1 ? p1 : p0), (short)0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsV = __builtin_amdgcn_make_buffer_rsrc((void*)(p2 ? p2 : p0), (short)0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsD0 = __builtin_amdgcn_make_buffer_rsrc((void*)d0, (short)0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsD1 = __builtin_amdgcn_make_buffer_rsrc((void*)d1, (short)0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsD2 = __builtin_amdgcn_make_buffer_rsrc((void*)d2, (short)0, 0x7FFFFFFF, 0x00020000);

    float* lut_s = reinterpret_cast<float*>(smem);
    if constexpr (OUT == 1) {
        for (int i = tid; i < 768; i += kThreads) lut_s[i] = P.lut[i];
        __syncthreads();
    }
    const int f0 = P.fill & 0xFF, f1 = (P.fill >> 8) & 0xFF, f2 = (P.fill >> 16) & 0xFF;

    // Which 64-pixel column segments and which rows of the tile this wave owns.
    const int X0 = tx * P.TW, Y0 = ty * P.TH, Y1 = min(Y0 + P.TH, P.DH);
    int seg0, seg_step, nseg, row0, row_step;
    if (P.nsegx >= 4) { seg0 = wave; seg_step = 4; nseg = P.nsegx >> 2; row0 = 0; row_step = 1; }
    else { seg0 = wave % P.nsegx; seg_step = 0; nseg = 1; row0 = wave / P.nsegx; row_step = 4 / P.nsegx; }

    // Per-lane column state, up to two segments per wave.
    uint32_t oY0[2], oY1[2], oC0[2], oC1[2], wa[2], xo[2];
    bool xin[2];
#pragma unroll
    for (int j = 0; j < 2; j++) {
        const int X = X0 + (seg0 + j * seg_step) * 64 + lane;
        xin[j] = j < nseg && X < P.DW;
        const XTab xt = P.xtab[xin[j] ? X : 0];
        const int ca = x0 + xt.s0, cb = x0 + xt.s1;
        oY0[j] = (uint32_t)(ca * T::bpp);
        oY1[j] = (uint32_t)(cb * T::bpp);
        oC0[j] = FMT == kNV12 ? (uint32_t)(2 * (ca >> 1)) : (uint32_t)(ca >> 1);
        oC1[j] = FMT == kNV12 ? (uint32_t)(2 * (cb >> 1)) : (uint32_t)(cb >> 1);
        wa[j] = (uint32_t)xt.a0 | ((uint32_t)xt.a1 << 16);
        xo[j] = (uint32_t)(xin[j] ? X : 0);
    }

    for (int Y = Y0 + row0; Y < Y1; Y += row_step) {
        const int yr0 = ytab[Y].r0, yr1 = ytab[Y].r1, yb0 = ytab[Y].b0, yb1 = ytab[Y].b1;  // scalar loads
        const uint32_t orow = (uint32_t)(Y * P.DW);
        if ((yb0 | yb1) == 0 || (kAblate & 2)) {  // padding row (letterbox)
#pragma unroll
            for (int j = 0; j < 2; j++)
                if (xin[j] && !(kAblate & 4)) store_px<OUT>(d0, d1, d2, lut_s, orow + xo[j], f0, f1, f2);
            continue;
        }
        const int ya = y0 + yr0, yb = y0 + yr1;
        // Wave-uniform row offsets go in the buffer instructions' SGPR offset; the per-lane column
        // offsets are the VGPR offsets: no per-tap address arithmetic at all.
        const int sY0 = ya * pitch0, sY1 = yb * pitch0;
        const int sC0 = (ya >> 1) * pitch1, sC1 = (yb >> 1) * pitch1;
        const int sV0 = (ya >> 1) * pitch2, sV1 = (yb >> 1) * pitch2;
        const uint32_t wb0 = (uint32_t)yb0, wb1 = (uint32_t)yb1;
        const int sO = (int)(orow * (uint32_t)esz);

        auto run = [&](auto share_tag) {
            constexpr bool kShare = decltype(share_tag)::value;
            // ---- gather: every tap of every owned segment, before any arithmetic ----
            uint32_t q[2][4][3];
            Chroma<FMT> ch[2][4];
            if (kAblate & 16) {  // diagnostics: no loads, arithmetic on synthetic bytes
#pragma unroll
                for (int j = 0; j < 2; j++)
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        q[j][k][0] = (oY0[j] + 37 * k) & 255; q[j][k][1] = (oY1[j] + k) & 255; q[j][k][2] = (oC0[j] + k) & 255;
                        ch[j][k].u = (oC1[j] * (k + 1)) & 0xFFFF; ch[j][k].v = (oC0[j] ^ k) & 255;
                    }
            } else
#pragma unroll
            for (int j = 0; j < 2; j++) {
                if constexpr (kYUV) {
                    q[j][0][0] = __builtin_amdgcn_raw_buffer_load_b8(rsY, oY0[j], sY0, 0);
                    q[j][1][0] = __builtin_amdgcn_raw_buffer_load_b8(rsY, oY1[j], sY0, 0);
                    q[j][2][0] = __builtin_amdgcn_raw_buffer_load_b8(rsY, oY0[j], sY1, 0);
                    q[j][3][0] = __builtin_amdgcn_raw_buffer_load_b8(rsY, oY1[j], sY1, 0);
                    if constexpr (FMT == kNV12) {
                        ch[j][0].u = __builtin_amdgcn_raw_buffer_load_b16(rsC, oC0[j], sC0, 0);
                        ch[j][1].u = __builtin_amdgcn_raw_buffer_load_b16(rsC, oC1[j], sC0, 0);
                        if constexpr (!kShare) {
                            ch[j][2].u = __builtin_amdgcn_raw_buffer_load_b16(rsC, oC0[j], sC1, 0);
                            ch[j][3].u = __builtin_amdgcn_raw_buffer_load_b16(rsC, oC1[j], sC1, 0);
                        }
                    } else {
                        ch[j][0].u = __builtin_amdgcn_raw_buffer_load_b8(rsC, oC0[j], sC0, 0);
                        ch[j][0].v = __builtin_amdgcn_raw_buffer_load_b8(rsV, oC0[j], sV0, 0);
                        ch[j][1].u = __builtin_amdgcn_raw_buffer_load_b8(rsC, oC1[j], sC0, 0);
                        ch[j][1].v = __builtin_amdgcn_raw_buffer_load_b8(rsV, oC1[j], sV0, 0);
                        if constexpr (!kShare) {
                            ch[j][2].u = __builtin_amdgcn_raw_buffer_load_b8(rsC, oC0[j], sC1, 0);
                            ch[j][2].v = __builtin_amdgcn_raw_buffer_load_b8(rsV, oC0[j], sV1, 0);
                            ch[j][3].u = __builtin_amdgcn_raw_buffer_load_b8(rsC, oC1[j], sC1, 0);
                            ch[j][3].v = __builtin_amdgcn_raw_buffer_load_b8(rsV, oC1[j], sV1, 0);
                        }
                    }
                } else {
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        const int sr = (k >> 1) ? sY1 : sY0;
                        const uint32_t o = (k & 1) ? oY1[j] : oY0[j];
                        if constexpr (FMT == kBGRX) {
                            q[j][k][0] = __builtin_amdgcn_raw_buffer_load_b32(rsY, o, sr, 0);
                        } else {
                            q[j][k][0] = __builtin_amdgcn_raw_buffer_load_b8(rsY, o, sr, 0);
                            q[j][k][1] = __builtin_amdgcn_raw_buffer_load_b8(rsY, o + 1, sr, 0);
                            q[j][k][2] = __builtin_amdgcn_raw_buffer_load_b8(rsY, o + 2, sr, 0);
                        }
                    }
                }
                if (j + 1 >= nseg) break;
            }
            // ---- arithmetic + stores ----
#pragma unroll
            for (int j = 0; j < 2; j++) {
                if (j < nseg && xin[j]) {
                    if (kAblate & 8) {  // diagnostics: loads only
                        uint32_t acc = ch[j][0].u + ch[j][1].u + (kShare ? 0u : ch[j][2].u + ch[j][3].u);
#pragma unroll
                        for (int k = 0; k < 4; k++) acc += q[j][k][0];
                        asm volatile("" :: "v"(acc));
                        continue;
                    }
                    const uint32_t a0 = wa[j] & 0xFFFF, a1 = wa[j] >> 16;  // 15-bit
                    int c[4][3];
                    if constexpr (kYUV) {
                        const UV3 tA = chroma_terms<FMT>(ch[j][0]);
                        const UV3 tB = chroma_terms<FMT>(ch[j][1]);
                        const UV3 tC = kShare ? tA : chroma_terms<FMT>(ch[j][2]);
                        const UV3 tD = kShare ? tB : chroma_terms<FMT>(ch[j][3]);
                        y_plus_uv((int)q[j][0][0], tA, c[0][0], c[0][1], c[0][2]);
                        y_plus_uv((int)q[j][1][0], tB, c[1][0], c[1][1], c[1][2]);
                        y_plus_uv((int)q[j][2][0], tC, c[2][0], c[2][1], c[2][2]);
                        y_plus_uv((int)q[j][3][0], tD, c[3][0], c[3][1], c[3][2]);
                    } else {
#pragma unroll
                        for (int k = 0; k < 4; k++) {
                            if constexpr (FMT == kBGRX) {
                                c[k][0] = q[j][k][0] & 0xFF; c[k][1] = (q[j][k][0] >> 8) & 0xFF; c[k][2] = (q[j][k][0] >> 16) & 0xFF;
                            } else {
                                c[k][0] = (int)q[j][k][0]; c[k][1] = (int)q[j][k][1]; c[k][2] = (int)q[j][k][2];
                            }
                        }
                    }
                    int v[3];
#pragma unroll
                    for (int ch3 = 0; ch3 < 3; ch3++) {
                        const uint32_t D0 = __umul24(c[0][ch3], a0) + __umul24(c[1][ch3], a1);
                        const uint32_t D1 = __umul24(c[2][ch3], a0) + __umul24(c[3][ch3], a1);
                        v[ch3] = vresize(D0, D1, wb0, wb1);
                    }
                    if (kAblate & 4) {
                        asm volatile("" :: "v"(v[0]), "v"(v[1]), "v"(v[2]));
                    } else {
                        if (P.color_rgb) { const int tmp = v[0]; v[0] = v[2]; v[2] = tmp; }
                        if (wa[j] == 0) {  // letterbox padding column (zero weights): the fill, in output plane order
                            v[0] = f0; v[1] = f1; v[2] = f2;
                        }
                        const uint32_t vo = xo[j] * (uint32_t)esz;
                        if constexpr (OUT == 1) {
                            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(lut_s[v[0]]), rsD0, vo, sO, EVAM_PP_STORE_AUX);
                            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(lut_s[256 + v[1]]), rsD1, vo, sO, EVAM_PP_STORE_AUX);
                            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(lut_s[512 + v[2]]), rsD2, vo, sO, EVAM_PP_STORE_AUX);
                        } else {
                            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)v[0], rsD0, vo, sO, EVAM_PP_STORE_AUX);
                            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)v[1], rsD1, vo, sO, EVAM_PP_STORE_AUX);
                            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)v[2], rsD2, vo, sO, EVAM_PP_STORE_AUX);
                        }
                    }
                }
            }
        };
        if constexpr (kYUV) {
            if ((ya >> 1) == (yb >> 1)) run(std::true_type{});
            else run(std::false_type{});
        } else {
            run(std::false_type{});
        }
    }
}

// Row table of up to 64 consecutive output rows held one row per lane (r0, r1, b0, b1 in four VGPRs),
// read back as wave-uniform values with v_readlane: the per-row lookups of the staging loops then cost
// no scalar-memory round trip (a dependent s_load per row serialised the DMA issue).
struct LaneRows {
    int r0, r1, b0, b1;
    __device__ __forceinline__ void load(const YTab* ytab, int Ybase, int n, int lane) {
        const int Y = Ybase + (lane < n ? lane : 0);
        const YTab e = ytab[Y];
        r0 = e.r0; r1 = e.r1; b0 = e.b0; b1 = e.b1;
    }
    __device__ __forceinline__ int R0(int i) const { return __builtin_amdgcn_readlane(r0, i); }
    __device__ __forceinline__ int R1(int i) const { return __builtin_amdgcn_readlane(r1, i); }
    __device__ __forceinline__ int B0(int i) const { return __builtin_amdgcn_readlane(b0, i); }
    __device__ __forceinline__ int B1(int i) const { return __builtin_amdgcn_readlane(b1, i); }
};

// Workgroup barrier for data written to LDS by ds_write only: lgkmcnt(0) and a raw s_barrier. __syncthreads()
// also waits vmcnt(0), which drains every LDS-DMA in flight (cdna_hip_programming.md, Pipelining across barriers).
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ void vmcnt_at_most(int n) {
    n = __builtin_amdgcn_readfirstlane(n);
    if (n >= 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    else if (n >= 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if (n >= 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if (n >= 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Same, exact for n <= 24 (a jump over immediates; larger n waits for 24).
__device__ __forceinline__ void vmcnt_exact(int n) {
    n = __builtin_amdgcn_readfirstlane(n);
#define EVAM_VMC(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    switch (n) {
        EVAM_VMC(0) EVAM_VMC(1) EVAM_VMC(2) EVAM_VMC(3) EVAM_VMC(4) EVAM_VMC(5) EVAM_VMC(6) EVAM_VMC(7) EVAM_VMC(8)
        EVAM_VMC(9) EVAM_VMC(10) EVAM_VMC(11) EVAM_VMC(12) EVAM_VMC(13) EVAM_VMC(14) EVAM_VMC(15) EVAM_VMC(16)
        EVAM_VMC(17) EVAM_VMC(18) EVAM_VMC(19) EVAM_VMC(20) EVAM_VMC(21) EVAM_VMC(22) EVAM_VMC(23)
        default: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
    }
#undef EVAM_VMC
}

// Staged uniform-geometry kernel. A workgroup owns a TW x TH tile (TW = 64 x NSEGX) and walks it in
// groups of R output rows. For each group the source row segments its taps need (two luma rows and
// two chroma rows per output row, each at most kSlot bytes wide) are brought into LDS by LDS-DMA —
// one 16 B/lane buffer_load ... lds per row segment, the row offset in the SGPR offset — into one of
// NBUF staging buffers, NBUF - 1 groups ahead of the group being converted: the DMA of several groups
// is in flight while the workgroup converts, which is what hides HBM latency when the frames stream
// from HBM rather than from the Infinity Cache. Taps are then LDS byte reads with immediate slot
// offsets, so neither the staging nor the gather costs VALU address arithmetic, and VMEM carries only
// wide loads and the planar stores. The DMA and the stores share vmcnt, which retires in issue order:
// every wave counts the VMEM operations it issues (all its branches are wave-uniform, so the count is
// exact) and waits for group g with vmcnt(operations issued after group g's DMA), so stores and later
// groups' DMA stay in flight.
template <int FMT, int OUT, int R, int NSEGX, int NBUF>
__global__ __launch_bounds__(kThreads) void evam_pp_staged(const SParams P) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    using T = FmtTraits<FMT>;
    constexpr bool kYUV = FMT == kNV12 || FMT == kI420;
    constexpr int NP = FMT == kI420 ? 3 : (FMT == kNV12 ? 2 : 1);  // staged planes
    constexpr int NS = 2 * R * NP;                                   // slots per staging buffer
    constexpr int SPW = NSEGX > 4 ? NSEGX / 4 : 1;                   // column segments per wave
    constexpr int RSTEP = NSEGX >= 4 ? 1 : 4 / NSEGX;                // waves sharing a column segment
    constexpr int RPW = R / RSTEP;                                   // rows per wave per group
    static_assert(NSEGX <= 4 && NBUF == 2, "retired shapes (round 5): full-width tiles, 2 KB slots, 3 buffers");
    constexpr int SLOT_MAX = kSlot;                                  // largest staged row segment
    const int SLOT = P.slot_bytes;                                   // this launch's segment (<= SLOT_MAX)
    static_assert(R % RSTEP == 0, "R must be a multiple of 4 / NSEGX");
    static_assert(NSEGX <= 4 || R == 1, "full-width (2 KB slot) tiles stage one row per group");
    static_assert(NBUF >= 2 && NBUF <= 3, "2 or 3 staging buffers");
    constexpr int TW = 64 * NSEGX;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // Prologue critical path: the launch parameters, then (in parallel) the item's arguments, the tile's
    // row table and its column footprint (from the parameters when tiles_x <= kTCols), then the first
    // DMA. Two batches of scalar loads, one wait each: (1) the launch parameters, (2) the item's
    // arguments and the tile column's footprint (the row table's vector load goes out between them).
    // Without the empty asm uses, branches on parameters split the loads into ~6 dependent round trips
    // before the first DMA (C2 +0.5 to +3 %, C5 +0.4 to +1.4 %: profiles/r02zz_prologue_batch_ab.txt).
    const int p_xcd = P.xcd_remap, p_tpi = P.tiles_per_item, p_tx = P.tiles_x, p_TH = P.TH, p_DH = P.DH;
    const int p_grid = gridDim.x;
    asm volatile("" ::"s"(p_xcd), "s"(p_tpi), "s"(p_tx), "s"(p_TH), "s"(p_DH), "s"(p_grid), "s"(P.ytab), "s"(P.ox),
                 "s"(P.rw), "s"(P.slot_bytes), "s"(P.offBuf), "s"(P.color_rgb), "s"(P.DW),
                 "s"(P.ntcol));
    const int t_x = xcd_tile(blockIdx.x, p_grid);
    const int t = p_xcd ? t_x : (int)blockIdx.x;
    const int item = t / p_tpi;
    const int tile = t - item * p_tpi;
    const int ty = tile / p_tx;
    const int tx = tile - ty * p_tx;
    const int Y0 = ty * p_TH, Y1 = min(Y0 + p_TH, p_DH);
    const int rows = Y1 - Y0;
    // The tile's row table (<= 64 rows, host-checked), one row per lane in every wave: per-group lookups
    // are v_readlane instead of dependent scalar loads from L2 (~1 us per group in the loop's critical
    // path when the frames stream from HBM, profiles/r02_skeleton.txt).
    LaneRows lr;
    lr.load(P.ytab, Y0, rows, lane);
    const ItemArg& it = P.items[item];
    const __attribute__((address_space(4))) XTab* xtab_s = (const __attribute__((address_space(4))) XTab*)(P.xtab);
    const uint8_t* p0 = it.plane[0];
    const uint8_t* p1 = it.plane[1];
    const uint8_t* p2 = it.plane[2];
    const int pitch0 = it.pitch[0], pitch1 = it.pitch[1], pitch2 = it.pitch[2];
    const int x0 = it.x0, y0 = it.y0, ox = P.ox, rw = P.rw;
    const int2 tc = P.tcol[min(tx, kTCols - 1)];
    const int p_ntcol = P.ntcol, p_index = it.index;
    asm volatile("" ::"s"(p0), "s"(p1), "s"(p2), "s"(pitch0), "s"(pitch1), "s"(pitch2), "s"(x0), "s"(y0),
                 "s"(p_index), "s"(tc.x), "s"(tc.y), "s"(P.dst), "s"(P.slot_offset), "s"(P.slot_stride));
    const size_t plane = (size_t)P.DW * P.DH;
    const size_t esz = OUT == 1 ? 4 : 1;
    uint8_t* const d0 = reinterpret_cast<uint8_t*>(P.dst) + (size_t)(P.slot_offset + it.index * P.slot_stride) * 3 * plane * esz;
    uint8_t* const d1 = d0 + plane * esz;
    uint8_t* const d2 = d1 + plane * esz;
    const __amdgpu_buffer_rsrc_t rsY = __builtin_amdgcn_make_buffer_rsrc((void*)p0, (short)0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsC = __builtin_amdgcn_make_buffer_rsrc((void*)(p1 ? p1 : p0), (short)0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsV = __builtin_amdgcn_make_buffer_rsrc((void*)(p2 ? p2 : p0), (short)0, 0x7FFFFFFF, 0x00020000);
    // plane of source channel 0 / 2 (B / R): swapped for RGB order
    const __amdgpu_buffer_rsrc_t rsD0 = __builtin_amdgcn_make_buffer_rsrc((void*)(P.color_rgb ? d2 : d0), (short)0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsD1 = __builtin_amdgcn_make_buffer_rsrc((void*)d1, (short)0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsD2 = __builtin_amdgcn_make_buffer_rsrc((void*)(P.color_rgb ? d0 : d2), (short)0, 0x7FFFFFFF, 0x00020000);

    float* lut_s = reinterpret_cast<float*>(smem);
    // fill in source channel order (P.fill is in output plane order); fp32: LUT byte offsets
    const uint32_t fq0 = P.fill & 0xFF, fq1 = (P.fill >> 8) & 0xFF, fq2 = (P.fill >> 16) & 0xFF;
    const uint32_t fsh = OUT == 1 ? 2 : 0;
    const uint32_t fillv[3] = {(P.color_rgb ? fq2 : fq0) << fsh, fq1 << fsh, (P.color_rgb ? fq0 : fq2) << fsh};

    const int X0 = tx * TW;
    const int rph = NSEGX >= 4 ? 0 : wave / NSEGX;
    // visible (non-padding) columns of the tile -> source footprint (wave-uniform)
    const int Xv0 = max(X0, ox), Xv1 = min(min(X0 + TW, P.DW), ox + rw) - 1;
    const bool cols = Xv0 <= Xv1;
    int fsY = 0, nY = 0, fsC = 0, nC = 0;
    if (cols) {
        int s0, s1;
        if (tx < p_ntcol) { s0 = tc.x; s1 = tc.y; }
        else { s0 = xtab_s[Xv0].s0; s1 = xtab_s[Xv1].s1; }
        footprint_chunks(FMT, T::bpp, x0 + s0, x0 + s1, fsY, nY, fsC, nC);
    }
    if (kAblate & 128) return;  // diagnostics: prologue parameters only
    // per-lane column state for each of this wave's SPW 64-column segments (seg = wave + 4 j, or
    // wave % NSEGX for narrow tiles), filled once the first DMA is in flight: LDS byte offsets of the taps
    // inside a slot, weights
    int X[SPW];
    bool xin[SPW], wave_stores[SPW];  // wave_stores: lane 0 of this wave stores segment j (wave-uniform)
    uint32_t lY0[SPW], lY1[SPW], lC0[SPW], lC1[SPW], wa[SPW], wp[SPW], xo[SPW];  // wp: a0 | a1 << 16, plain
#pragma unroll
    for (int j = 0; j < SPW; j++) {
        const int seg = NSEGX >= 4 ? wave + 4 * j : wave % NSEGX;
        X[j] = X0 + seg * 64 + lane;
        xin[j] = X[j] < P.DW;
        wave_stores[j] = X0 + seg * 64 < P.DW;
        xo[j] = (uint32_t)(xin[j] ? X[j] : 0) * (uint32_t)esz;
        lY0[j] = lY1[j] = lC0[j] = lC1[j] = wa[j] = wp[j] = 0;
    }
    const int ngroups = (rows + R - 1) / R;
    // letterbox padding columns anywhere in this tile (the per-pixel fill select is skipped otherwise)
    const bool anypadc = Xv0 > X0 || Xv1 < min(X0 + TW, P.DW) - 1;

    // ---- LDS-DMA of group g into buffer `buf` (slot s = plane * 2R + 2 * row + tap) ----
    // Returns the number of VMEM instructions this wave issued (wave-uniform; nY, nC >= 1 whenever
    // `cols`, so lane 0 is active in every issued instruction).
    // Static DMA roles: with 2R = 4 the (row, tap) pairs of a group are exactly the four waves, so wave
    // w stages row w >> 1, tap w & 1 of every plane. Otherwise the slots are dealt round-robin.
    const int dr = wave >> 1, dtap = wave & 1;
    auto issue = [&](int g, uint8_t* buf) -> int {
        if (!cols || (kAblate & 16)) return 0;
        if constexpr (2 * R == 4) {
            const int Y = Y0 + g * R + dr;
            if (Y >= Y1) return 0;
            const int b0 = lr.B0(Y - Y0), b1 = lr.B1(Y - Y0);
            if ((b0 | b1) == 0) return 0;  // padding row: nothing to stage
            const int ya = y0 + lr.R0(Y - Y0), yb = y0 + lr.R1(Y - Y0);
            const int yr = dtap ? yb : ya;
            int n = 0;
#pragma unroll
            for (int c0 = 0; c0 < SLOT_MAX / 16; c0 += 64) {  // one wave-wide 1 KB DMA per 64 chunks
                if (c0 >= nY) break;
                if (lane + c0 < nY)
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(
                        rsY, (__attribute__((address_space(3))) void*)(buf + wave * SLOT + c0 * 16), 16, (lane + c0) * 16,
                        yr * pitch0 + fsY, EVAM_PP_LOAD_AUX, 0);
                n++;
            }
            if constexpr (NP >= 2) {
                if (dtap && (ya >> 1) == (yb >> 1)) return n;  // chroma row shared by both taps
#pragma unroll
                for (int c0 = 0; c0 < SLOT_MAX / 16; c0 += 64) {
                    if (c0 >= nC) break;
                    if (lane + c0 < nC) {
                        __builtin_amdgcn_raw_ptr_buffer_load_lds(
                            rsC, (__attribute__((address_space(3))) void*)(buf + (2 * R + wave) * SLOT + c0 * 16), 16,
                            (lane + c0) * 16, (yr >> 1) * pitch1 + fsC, EVAM_PP_LOAD_AUX, 0);
                        if constexpr (NP >= 3)
                            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                                rsV, (__attribute__((address_space(3))) void*)(buf + (4 * R + wave) * SLOT + c0 * 16), 16,
                                (lane + c0) * 16, (yr >> 1) * pitch2 + fsC, EVAM_PP_LOAD_AUX, 0);
                    }
                    n += NP - 1;
                }
            }
            return n;
        } else {
            int n = 0;
#pragma unroll
            for (int s0 = 0; s0 < NS; s0 += 4) {
                const int s = s0 + wave;
                if (s >= NS) continue;
                const int pl = s / (2 * R), loc = s - pl * 2 * R, r = loc >> 1, tap = loc & 1;
                const int Y = Y0 + g * R + r;
                if (Y >= Y1) continue;
                const int b0 = lr.B0(Y - Y0), b1 = lr.B1(Y - Y0);
                if ((b0 | b1) == 0) continue;  // padding row: nothing to stage
                const int ya = y0 + lr.R0(Y - Y0), yb = y0 + lr.R1(Y - Y0);
                const int yr = tap ? yb : ya;
                if (pl > 0 && tap && (ya >> 1) == (yb >> 1)) continue;  // chroma row shared by both taps
                const int nck = pl == 0 ? nY : nC;
#pragma unroll
                for (int c0 = 0; c0 < SLOT_MAX / 16; c0 += 64) {  // one wave-wide 1 KB DMA per 64 chunks
                    if (c0 >= nck) break;
                    __attribute__((address_space(3))) void* dstl =
                        (__attribute__((address_space(3))) void*)(buf + s * SLOT + c0 * 16);
                    if (lane + c0 < nck) {
                        const int co = (lane + c0) * 16;
                        if (pl == 0)
                            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsY, dstl, 16, co, yr * pitch0 + fsY, EVAM_PP_LOAD_AUX, 0);
                        else if (pl == 1)
                            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsC, dstl, 16, co, (yr >> 1) * pitch1 + fsC, EVAM_PP_LOAD_AUX, 0);
                        else
                            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsV, dstl, 16, co, (yr >> 1) * pitch2 + fsC, EVAM_PP_LOAD_AUX, 0);
                    }
                    n++;
                }
            }
            return n;
        }
    };

    // ---- convert + resize + normalise + store the rows of group g owned by this wave ----
    // Channel routing: v[c] holds source channel c (B, G, R). It is stored to output plane c, or 2 - c for
    // RGB order, through swapped plane resources; the LDS LUT is loaded with its sections in source
    // channel order (prologue), so the per-pixel path carries no swap. For fp32 output the vertical
    // pass yields 4 * v, the LUT byte offset, directly ((x + 2) & ~3 instead of (x + 2) >> 2).
    // Returns the number of stores this wave issued: 3 per owned row when the wave stores at all (the
    // padding-column select is branchless, so every storing row issues exactly three).
    auto compute = [&](int g, const uint8_t* buf) -> int {
        int n = 0;
#pragma unroll
        for (int kj = 0; kj < RPW * SPW; kj++) {
            const int k = kj / SPW, j = kj % SPW;
            const int r = rph + k * RSTEP;
            const int Y = Y0 + g * R + r;
            if (Y >= Y1 || !wave_stores[j]) continue;
            const int b0 = lr.B0(Y - Y0), b1 = lr.B1(Y - Y0);
            const int sO = (int)((uint32_t)(Y * P.DW) * (uint32_t)esz);
            n += 3;
            auto put = [&](const uint32_t (&v)[3]) {
                if (kAblate & 4) {
                    asm volatile("" :: "v"(v[0]), "v"(v[1]), "v"(v[2]));
                    return;
                }
                if (!xin[j]) return;  // lane 0 is in: the wave still issues all three stores
                if constexpr (OUT == 1) {
                    const uint8_t* lb = reinterpret_cast<const uint8_t*>(lut_s);
                    __builtin_amdgcn_raw_buffer_store_b32(*reinterpret_cast<const uint32_t*>(lb + v[0]), rsD0, xo[j], sO, EVAM_PP_STORE_AUX);
                    __builtin_amdgcn_raw_buffer_store_b32(*reinterpret_cast<const uint32_t*>(lb + 1024 + v[1]), rsD1, xo[j], sO, EVAM_PP_STORE_AUX);
                    __builtin_amdgcn_raw_buffer_store_b32(*reinterpret_cast<const uint32_t*>(lb + 2048 + v[2]), rsD2, xo[j], sO, EVAM_PP_STORE_AUX);
                } else {
                    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)v[0], rsD0, xo[j], sO, EVAM_PP_STORE_AUX);
                    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)v[1], rsD1, xo[j], sO, EVAM_PP_STORE_AUX);
                    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)v[2], rsD2, xo[j], sO, EVAM_PP_STORE_AUX);
                }
            };
            if ((b0 | b1) == 0 || (kAblate & 2)) {  // padding row (wave-uniform)
                put(fillv);
                continue;
            }
            const bool padc = wa[j] == 0;  // letterbox padding column: taps at valid offsets, value replaced
            const uint32_t wb0 = (uint32_t)b0, wb1 = (uint32_t)b1;
            const uint8_t* sy0 = buf + (2 * r) * SLOT;
            const uint8_t* sy1 = sy0 + SLOT;
            const uint8_t* sc0 = buf + (2 * R + 2 * r) * SLOT;
            const uint32_t lY0j = lY0[j], lY1j = lY1[j], lC0j = lC0[j], lC1j = lC1[j], wpj = wp[j];
            uint32_t v[3];
            if constexpr (kYUV) {
                const int ya = y0 + lr.R0(Y - Y0), yb = y0 + lr.R1(Y - Y0);
                const bool share = (ya >> 1) == (yb >> 1);
                const uint8_t* sc1 = share ? sc0 : sc0 + SLOT;
                // NV12: U and V of a tap are adjacent bytes of the staged UV row; I420: same offset in the
                // U and V slots.
                const uint8_t* sv0 = FMT == kNV12 ? sc0 + 1 : sc0 + 2 * R * SLOT;
                const uint8_t* sv1 = FMT == kNV12 ? sc1 + 1 : sc1 + 2 * R * SLOT;
                const UVs tA = uv_terms_sat(sc0[lC0j], sv0[lC0j]);
                const UVs tB = uv_terms_sat(sc0[lC1j], sv0[lC1j]);
                const uint32_t yA = luma_term(sy0[lY0j]), yB = luma_term(sy0[lY1j]);
                const uint32_t yC = luma_term(sy1[lY0j]), yD = luma_term(sy1[lY1j]);
                const uint32_t h0[3] = {hpass_sat(yA, tA.b, yB, tB.b, wpj), hpass_sat(yA, tA.g, yB, tB.g, wpj),
                                        hpass_sat(yA, tA.r, yB, tB.r, wpj)};
                uint32_t h1[3];
                // both vertical taps in one chroma row (wave-uniform, ~half the rows of a 2:1 chroma
                // downscale): its terms are reused instead of read and converted again. The second row's
                // horizontal pass is written out in both branches, so the shared path carries no copies of
                // the chroma terms.
                if (share) {
                    h1[0] = hpass_sat(yC, tA.b, yD, tB.b, wpj);
                    h1[1] = hpass_sat(yC, tA.g, yD, tB.g, wpj);
                    h1[2] = hpass_sat(yC, tA.r, yD, tB.r, wpj);
                } else {
                    const UVs tC = uv_terms_sat(sc1[lC0j], sv1[lC0j]);
                    const UVs tD = uv_terms_sat(sc1[lC1j], sv1[lC1j]);
                    h1[0] = hpass_sat(yC, tC.b, yD, tD.b, wpj);
                    h1[1] = hpass_sat(yC, tC.g, yD, tD.g, wpj);
                    h1[2] = hpass_sat(yC, tC.r, yD, tD.r, wpj);
                }
#pragma unroll
                for (int c = 0; c < 3; c++) v[c] = vfinal<OUT>(h0[c], h1[c], wb0, wb1);
                if (anypadc) {  // wave-uniform: most launches have no padding column at all (C2, C4, C5)
#pragma unroll
                    for (int c = 0; c < 3; c++) v[c] = padc ? fillv[c] : v[c];
                }
                put(v);
                continue;
            }
            const uint32_t a0 = wa[j] & 0xFFFF, a1 = wa[j] >> 16;  // 15-bit
            int c[4][3];
            {  // packed sources (BGRx / BGR)
                const uint8_t* rowp[2] = {sy0, sy1};
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const uint8_t* sp = rowp[q >> 1] + ((q & 1) ? lY1j : lY0j);
                    if constexpr (FMT == kBGRX) {
                        const uint32_t px = *reinterpret_cast<const uint32_t*>(sp);
                        c[q][0] = px & 0xFF; c[q][1] = (px >> 8) & 0xFF; c[q][2] = (px >> 16) & 0xFF;
                    } else {
                        c[q][0] = sp[0]; c[q][1] = sp[1]; c[q][2] = sp[2];
                    }
                }
            }
#pragma unroll
            for (int ch3 = 0; ch3 < 3; ch3++) {
                const uint32_t D0 = __umul24(c[0][ch3], a0) + __umul24(c[1][ch3], a1);
                const uint32_t D1 = __umul24(c[2][ch3], a0) + __umul24(c[3][ch3], a1);
                v[ch3] = padc ? fillv[ch3] : vfinal<OUT>(D0, D1, wb0, wb1);
            }
            put(v);
        }
        return n;
    };

    uint8_t* const bufs = smem + P.offBuf;
    // Prologue: the first NBUF - 1 groups' DMA goes out before the LUT and column-table loads, so their
    // latencies overlap instead of adding up. q[j]: VMEM operations issued up to the end of the DMA of
    // group g + j (j < NBUF - 1), for the counted waits below.
    int issued = 0;
    int q[NBUF - 1];
#pragma unroll
    for (int j = 0; j < NBUF - 1; j++) {
        if (j < ngroups) issued += __builtin_amdgcn_readfirstlane(issue(j, bufs + j * P.buf_bytes));
        q[j] = issued;
    }
    asm volatile("" ::: "memory");
    if constexpr (OUT == 1) {  // sections in source channel order (B, G, R): see compute
        if (!(kAblate & 32))   // diagnostics: 32 skips the LUT load
            for (int i = tid; i < 768; i += kThreads) lut_s[i] = P.lut[P.color_rgb ? 512 - (i & ~255) + (i & 255) : i];
    }
#pragma unroll
    for (int j = 0; j < SPW; j++) {
        const XTab xt = P.xtab[xin[j] ? X[j] : 0];
        wa[j] = (uint32_t)xt.a0 | ((uint32_t)xt.a1 << 16);
        wp[j] = (wa[j] >> 4) & 0x0FFF0FFFu;
        if (xin[j] && wa[j] != 0) {
            const int ca = x0 + xt.s0, cb = x0 + xt.s1;
            lY0[j] = (uint32_t)(ca * T::bpp - fsY);
            lY1[j] = (uint32_t)(cb * T::bpp - fsY);
            lC0[j] = FMT == kNV12 ? (uint32_t)(2 * (ca >> 1) - fsC) : (uint32_t)((ca >> 1) - fsC);
            lC1[j] = FMT == kNV12 ? (uint32_t)(2 * (cb >> 1) - fsC) : (uint32_t)((cb >> 1) - fsC);
        }
    }
    int bi = 0;                 // buffer of group g
    int bn = NBUF - 1;          // buffer of group g + NBUF - 1
    if ((kAblate & 64) && ngroups != -7) {  // diagnostics: prologue only
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("" :: "v"(lY0[0]), "v"(lC0[0]), "v"(wa[0]), "v"(lY1[0]), "v"(lC1[0]));
        return;
    }
    // Stores this wave issues for a full group (3 per owned row; the padding select is branchless).
    int st_full = 0;
#pragma unroll
    for (int j = 0; j < SPW; j++) st_full += wave_stores[j] ? 3 * RPW : 0;
    st_full = __builtin_amdgcn_readfirstlane(st_full);
    for (int g = 0; g < ngroups; g++) {
        // This wave's share of group g's DMA landed; everything issued after it (later groups' DMA, the
        // previous groups' stores) may stay in flight. The first iteration also covers the prologue's
        // global loads (LUT, column table), which were issued after the DMA.
        if (g == 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else if constexpr (NBUF == 2) {
            // Two buffers: only the stores of group g - 1 (a full group: group g exists) were issued
            // after group g's DMA, and their count is a per-wave constant, so the wait is one
            // immediate, not the counted ladder (scalar instructions are shared by the CU's waves).
            if (st_full == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            else if (SPW == 1 || st_full == 3 * RPW) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(3 * RPW) : "memory");
            else asm volatile("s_waitcnt vmcnt(%0)" :: "n"(6 * RPW) : "memory");
        } else {
            vmcnt_at_most(issued - q[0]);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // every wave's DMA for g landed; every wave done reading g-1
#pragma unroll
        for (int j = 0; j + 1 < NBUF - 1; j++) q[j] = q[j + 1];
        if (g + NBUF - 1 < ngroups) issued += __builtin_amdgcn_readfirstlane(issue(g + NBUF - 1, bufs + bn * P.buf_bytes));
        q[NBUF - 2] = issued;
        asm volatile("" ::: "memory");  // the next groups' DMA stays ahead of this group's stores
        issued += __builtin_amdgcn_readfirstlane(compute(g, bufs + bi * P.buf_bytes));
        asm volatile("" ::: "memory");
        bi = bi + 1 == NBUF ? 0 : bi + 1;
        bn = bn + 1 == NBUF ? 0 : bn + 1;
    }
}

// ------------------------------------------------------------------------------------------------
// wave-row kernel (uniform geometry)
// ------------------------------------------------------------------------------------------------
struct WParams {
    ItemArg items[kArgItems];
    int ox, rw;          // uniform placement / resized width
    const float* lut;    // [3][256]
    const XTab* xtab;    // [DW]
    const YTab* ytab;    // [DH]
    void* dst;
    int slot_offset, slot_stride;  // output slot of item i = slot_offset + i * slot_stride
    int DW, DH;
    int TH, tiles_x, tiles_per_item;
    int offBuf;          // LDS offset of the per-wave staging areas (after the LUT)
    int segY, segC;      // bytes of one staged luma / chroma row segment (multiples of 16)
    int wave_bytes;      // one wave's staging area (two buffers)
    int color_rgb;
    uint32_t fill;
};

typedef int evam_v2i __attribute__((ext_vector_type(2)));
typedef int evam_v4i __attribute__((ext_vector_type(4)));

// PX adjacent output pixels of one channel from one lane: a single buffer store of PX x 4 bytes (fp32)
// or PX bytes (u8). lut == nullptr: u8 output.
template <int OUT, int PX>
__device__ __forceinline__ void store_vec(const __amdgpu_buffer_rsrc_t rs, uint32_t vo, int so, const float* lut,
                                          const int (&v)[PX]) {
    if constexpr (OUT == 1) {
        if constexpr (PX == 4) {
            evam_v4i q = {(int)__float_as_uint(lut[v[0]]), (int)__float_as_uint(lut[v[1]]),
                          (int)__float_as_uint(lut[v[2]]), (int)__float_as_uint(lut[v[3]])};
            __builtin_amdgcn_raw_buffer_store_b128(q, rs, vo, so, EVAM_PP_STORE_AUX);
        } else if constexpr (PX == 2) {
            evam_v2i q = {(int)__float_as_uint(lut[v[0]]), (int)__float_as_uint(lut[v[1]])};
            __builtin_amdgcn_raw_buffer_store_b64(q, rs, vo, so, EVAM_PP_STORE_AUX);
        } else {
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(lut[v[0]]), rs, vo, so, EVAM_PP_STORE_AUX);
        }
    } else {
        if constexpr (PX == 4)
            __builtin_amdgcn_raw_buffer_store_b32((uint32_t)v[0] | ((uint32_t)v[1] << 8) | ((uint32_t)v[2] << 16) |
                                                      ((uint32_t)v[3] << 24), rs, vo, so, EVAM_PP_STORE_AUX);
        else if constexpr (PX == 2)
            __builtin_amdgcn_raw_buffer_store_b16((uint16_t)(v[0] | (v[1] << 8)), rs, vo, so, EVAM_PP_STORE_AUX);
        else
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)v[0], rs, vo, so, EVAM_PP_STORE_AUX);
    }
}

// Same, with the fp32 values given as byte offsets into an LDS LUT section `lb` (vfinal<1>): the LUT
// read needs no address arithmetic (section base 0, 1024, 2048 is the instruction's immediate offset).
template <int OUT, int PX>
__device__ __forceinline__ void store_off(const __amdgpu_buffer_rsrc_t rs, uint32_t vo, const uint8_t* lb,
                                          const uint32_t (&v)[PX]) {
    if constexpr (OUT == 1) {
        auto L = [&](uint32_t o) { return (int)*reinterpret_cast<const uint32_t*>(lb + o); };
        if constexpr (PX == 4) {
            evam_v4i q = {L(v[0]), L(v[1]), L(v[2]), L(v[3])};
            __builtin_amdgcn_raw_buffer_store_b128(q, rs, vo, 0, EVAM_PP_STORE_AUX);
        } else if constexpr (PX == 2) {
            evam_v2i q = {L(v[0]), L(v[1])};
            __builtin_amdgcn_raw_buffer_store_b64(q, rs, vo, 0, EVAM_PP_STORE_AUX);
        } else {
            __builtin_amdgcn_raw_buffer_store_b32((uint32_t)L(v[0]), rs, vo, 0, EVAM_PP_STORE_AUX);
        }
    } else {
        if constexpr (PX == 4)
            __builtin_amdgcn_raw_buffer_store_b32(v[0] | (v[1] << 8) | (v[2] << 16) | (v[3] << 24), rs, vo, 0,
                                                  EVAM_PP_STORE_AUX);
        else if constexpr (PX == 2)
            __builtin_amdgcn_raw_buffer_store_b16((uint16_t)(v[0] | (v[1] << 8)), rs, vo, 0, EVAM_PP_STORE_AUX);
        else
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)v[0], rs, vo, 0, EVAM_PP_STORE_AUX);
    }
}

// Uniform-geometry kernel built around independent waves. A workgroup owns a 64·PX-column x TH-row
// tile of one item; each of its four waves owns a contiguous quarter of the tile's rows and walks it
// one output row at a time, every lane producing PX adjacent pixels:
//  * The wave stages the source row segments its next row needs (luma taps, chroma taps; each the
//    tile's 16 B-aligned footprint) into its own double-buffered LDS area by LDS-DMA while it converts
//    the current row. Nothing is shared between waves, so there is no workgroup barrier in the loop:
//    the wait for a row's DMA is this wave's vmcnt, with the previous row's three stores still in flight.
//  * Horizontal results are kept per source row (H = 11-bit weighted sum of the two converted taps, per
//    channel). With REUSE (vertical upscales, where consecutive output rows share source rows) a source
//    row that the previous output row already filtered is neither staged nor converted again.
//  * When both vertical taps read the same 4:2:0 chroma row, its BT.601 chroma terms are computed once.
//  * Each channel of a row leaves as one PX-wide store per lane (dwordx4 for fp32 at PX = 4).
template <int FMT, int OUT, int PX, bool REUSE>
__global__ __launch_bounds__(kThreads) void evam_pp_wave(const WParams P) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    using T = FmtTraits<FMT>;
    constexpr bool kYUV = FMT == kNV12 || FMT == kI420;
    constexpr int TW = 64 * PX;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int t = blockIdx.x;
    // the launch parameters of the prologue in one batch of scalar loads (one wait): without the empty
    // asm use, branches split them into dependent round trips ahead of the first DMA
    asm volatile("" ::"s"(P.tiles_per_item), "s"(P.tiles_x), "s"(P.ytab), "s"(P.xtab), "s"(P.TH),
                 "s"(P.DH), "s"(P.DW), "s"(P.ox), "s"(P.rw));
    const int item = t / P.tiles_per_item;
    const int tile = t - item * P.tiles_per_item;
    const int ty = tile / P.tiles_x;
    const int tx = tile - ty * P.tiles_x;
    const ItemArg& it = P.items[item];
    const __attribute__((address_space(4))) XTab* xtab_s = (const __attribute__((address_space(4))) XTab*)(P.xtab);
    const uint8_t* p0 = it.plane[0];
    const uint8_t* p1 = it.plane[1];
    const uint8_t* p2 = it.plane[2];
    const int pitch0 = it.pitch[0], pitch1 = it.pitch[1], pitch2 = it.pitch[2];
    const int x0 = it.x0, y0 = it.y0, ox = P.ox, rw = P.rw;
    const size_t plane = (size_t)P.DW * P.DH;
    const size_t esz = OUT == 1 ? 4 : 1;
    uint8_t* const d0 = reinterpret_cast<uint8_t*>(P.dst) + (size_t)(P.slot_offset + it.index * P.slot_stride) * 3 * plane * esz;
    uint8_t* const d1 = d0 + plane * esz;
    uint8_t* const d2 = d1 + plane * esz;
    const __amdgpu_buffer_rsrc_t rsY = __builtin_amdgcn_make_buffer_rsrc((void*)p0, (short)0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsC = __builtin_amdgcn_make_buffer_rsrc((void*)(p1 ? p1 : p0), (short)0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsV = __builtin_amdgcn_make_buffer_rsrc((void*)(p2 ? p2 : p0), (short)0, 0x7FFFFFFF, 0x00020000);
    // output planes in store order (BGR, or RGB: planes 0 and 2 exchanged)
    const __amdgpu_buffer_rsrc_t rsO0 = __builtin_amdgcn_make_buffer_rsrc((void*)(P.color_rgb ? d2 : d0), (short)0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsO1 = __builtin_amdgcn_make_buffer_rsrc((void*)d1, (short)0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsO2 = __builtin_amdgcn_make_buffer_rsrc((void*)(P.color_rgb ? d0 : d2), (short)0, 0x7FFFFFFF, 0x00020000);

    float* lut_s = reinterpret_cast<float*>(smem);
    // fill values in output plane order (P.fill is already in output channel order)
    const int fo0 = P.fill & 0xFF, fo1 = (P.fill >> 8) & 0xFF, fo2 = (P.fill >> 16) & 0xFF;
    const int fb0 = P.color_rgb ? fo2 : fo0, fb2 = P.color_rgb ? fo0 : fo2;  // same, in BGR order

    const int X0 = tx * TW, Y0 = ty * P.TH, Y1 = min(Y0 + P.TH, P.DH);
    // visible (non-padding) columns of the tile -> source footprint (wave-uniform)
    const int Xv0 = max(X0, ox), Xv1 = min(min(X0 + TW, P.DW), ox + rw) - 1;
    const bool cols = Xv0 <= Xv1;
    int fsY = 0, nY = 0, fsC = 0, nC = 0;
    // both footprint taps in one batch of scalar loads (clamped indices: read even for padding tiles)
    const int fs0 = xtab_s[max(min(Xv0, P.DW - 1), 0)].s0, fs1 = xtab_s[max(min(Xv1, P.DW - 1), 0)].s1;
    if (cols) footprint_chunks(FMT, T::bpp, x0 + fs0, x0 + fs1, fsY, nY, fsC, nC);
    // per-lane column state for the PX pixels of this lane: the PX table loads go out together here and
    // are consumed after the first DMA is issued
    const int Xl = X0 + lane * PX;
    const bool xin = Xl < P.DW;  // DW % PX == 0: a lane's pixels are all in or all out
    XTab xts[PX];
#pragma unroll
    for (int j = 0; j < PX; j++) xts[j] = P.xtab[xin ? Xl + j : 0];
    uint32_t lY[PX], lC[PX], wa[PX];
    const uint32_t vo = (uint32_t)(xin ? Xl : 0) * (uint32_t)esz;

    // this wave's rows
    const int thw = (P.TH + 3) >> 2;
    const int Yw0 = Y0 + wave * thw, Yw1 = min(Yw0 + thw, Y1);
    uint8_t* const wbuf = smem + P.offBuf + wave * P.wave_bytes;
    const int half = P.wave_bytes >> 1;
    const int segY = P.segY, segC = P.segC;
    // buffer layout: [Y tap0][Y tap1][C tap0][C tap1][V tap0][V tap1]
    const int oY1 = segY, oC0 = 2 * segY, oC1 = 2 * segY + segC, oV0 = 2 * segY + 2 * segC, oV1 = oV0 + segC;

    LaneRows lr;  // this wave's rows (<= 64, host)
    lr.load(P.ytab, Yw0, Yw1 - Yw0, lane);

    // Staging decision for output row Y, given the source rows (pa, pb) whose H the wave holds.
    struct Plan {
        int ya, yb, b0, b1;
        bool pad, stA, stB, stCB;  // stage luma tap0 / tap1 rows; chroma of tap1 in its own slot
    };
    auto plan = [&](int Y, int pa, int pb) {
        Plan q;
        q.b0 = lr.B0(Y - Yw0);
        q.b1 = lr.B1(Y - Yw0);
        q.ya = y0 + lr.R0(Y - Yw0);
        q.yb = y0 + lr.R1(Y - Yw0);
        q.pad = (q.b0 | q.b1) == 0 || !cols;
        if (REUSE) {
            q.stA = q.ya != pa && q.ya != pb;
            q.stB = q.yb != q.ya && q.yb != pa && q.yb != pb;
        } else {
            q.stA = true;
            q.stB = q.yb != q.ya;
        }
        q.stCB = q.stB && !(q.stA && (q.ya >> 1) == (q.yb >> 1));
        return q;
    };
    auto dma = [&](const __amdgpu_buffer_rsrc_t rs, uint8_t* dst, int nck, int soff) {
        for (int c = 0; c < nck; c += 64) {
            if (lane + c < nck)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(dst + c * 16), 16,
                                                         (lane + c) * 16, soff, EVAM_PP_LOAD_AUX, 0);
        }
    };
    auto issue = [&](const Plan& q, uint8_t* buf) {
        if (q.pad || (kAblate & 16)) return;
        if (q.stA) {
            dma(rsY, buf, nY, q.ya * pitch0 + fsY);
            if constexpr (kYUV) dma(rsC, buf + oC0, nC, (q.ya >> 1) * pitch1 + fsC);
            if constexpr (FMT == kI420) dma(rsV, buf + oV0, nC, (q.ya >> 1) * pitch2 + fsC);
        }
        if (q.stB) {
            dma(rsY, buf + oY1, nY, q.yb * pitch0 + fsY);
            if (q.stCB) {
                if constexpr (kYUV) dma(rsC, buf + oC1, nC, (q.yb >> 1) * pitch1 + fsC);
                if constexpr (FMT == kI420) dma(rsV, buf + oV1, nC, (q.yb >> 1) * pitch2 + fsC);
            }
        }
    };

    // Horizontal pass of one staged source row (or two sharing their chroma row).
    auto hrow = [&](const uint8_t* sy, const uint8_t* sc, const uint8_t* sv, uint32_t (&H)[PX][3]) {
#pragma unroll
        for (int j = 0; j < PX; j++) {
            const uint32_t tY0 = lY[j] & 0xFFFF, tY1 = lY[j] >> 16;
            int c0[3], c1[3];
            if constexpr (kYUV) {
                const uint32_t tC0 = lC[j] & 0xFFFF, tC1 = lC[j] >> 16;
                const uint8_t* svv = FMT == kNV12 ? sc + 1 : sv;
                hrow_sat(sy[tY0], sy[tY1], uv_terms_sat(sc[tC0], svv[tC0]), uv_terms_sat(sc[tC1], svv[tC1]),
                         (wa[j] >> 4) & 0x0FFF0FFFu, H[j]);
                continue;
            } else if constexpr (FMT == kBGRX) {
                const uint32_t q0 = *reinterpret_cast<const uint32_t*>(sy + tY0);
                const uint32_t q1 = *reinterpret_cast<const uint32_t*>(sy + tY1);
                c0[0] = q0 & 0xFF; c0[1] = (q0 >> 8) & 0xFF; c0[2] = (q0 >> 16) & 0xFF;
                c1[0] = q1 & 0xFF; c1[1] = (q1 >> 8) & 0xFF; c1[2] = (q1 >> 16) & 0xFF;
            } else {
                c0[0] = sy[tY0]; c0[1] = sy[tY0 + 1]; c0[2] = sy[tY0 + 2];
                c1[0] = sy[tY1]; c1[1] = sy[tY1 + 1]; c1[2] = sy[tY1 + 2];
            }
            const uint32_t a0 = wa[j] & 0xFFFF, a1 = wa[j] >> 16;
#pragma unroll
            for (int ch = 0; ch < 3; ch++) H[j][ch] = __umul24(c0[ch], a0) + __umul24(c1[ch], a1);
        }
    };
    auto hrow2 = [&](const uint8_t* sya, const uint8_t* syb, const uint8_t* sc, const uint8_t* sv,
                     uint32_t (&HA)[PX][3], uint32_t (&HB)[PX][3]) {
#pragma unroll
        for (int j = 0; j < PX; j++) {
            const uint32_t tY0 = lY[j] & 0xFFFF, tY1 = lY[j] >> 16;
            const uint32_t tC0 = lC[j] & 0xFFFF, tC1 = lC[j] >> 16;
            const uint8_t* svv = FMT == kNV12 ? sc + 1 : sv;
            const UVs sA = uv_terms_sat(sc[tC0], svv[tC0]), sB = uv_terms_sat(sc[tC1], svv[tC1]);
            const uint32_t wp = (wa[j] >> 4) & 0x0FFF0FFFu;
            hrow_sat(sya[tY0], sya[tY1], sA, sB, wp, HA[j]);
            hrow_sat(syb[tY0], syb[tY1], sA, sB, wp, HB[j]);
        }
    };

    auto store_row = [&](int Y, const int (&v)[3][PX]) {
        if (!xin || (kAblate & 4)) {
            if (kAblate & 4) asm volatile("" :: "v"(v[0][0]), "v"(v[1][0]), "v"(v[2][0]));
            return;
        }
        // Row offset in the VGPR offset, soffset 0. A >8-byte buffer store with an SGPR soffset is
        // exempt from the compiler's store-data hazard check, yet on gfx950 a VALU write right after
        // such a dwordx4 store corrupted the stored data (lanes 12-15 of each 16, first dword);
        // with soffset 0 the compiler inserts the wait state.
        const uint32_t off = vo + (uint32_t)(Y * P.DW) * (uint32_t)esz;
        // the LUT is per output plane: B lands in plane 2 when the output is RGB
        store_vec<OUT, PX>(rsO0, off, 0, lut_s + (P.color_rgb ? 512 : 0), v[0]);
        store_vec<OUT, PX>(rsO1, off, 0, lut_s + 256, v[1]);
        store_vec<OUT, PX>(rsO2, off, 0, lut_s + (P.color_rgb ? 0 : 512), v[2]);
    };

    uint32_t HA[PX][3], HB[PX][3];  // H of source rows pa, pb (REUSE) / of this row's taps
#pragma unroll
    for (int j = 0; j < PX; j++)
#pragma unroll
        for (int ch = 0; ch < 3; ch++) HA[j][ch] = HB[j][ch] = 0;
    int pa = -1, pb = -1;
    // Prologue order: the first row's DMA needs only the item, the footprint and the row table, so it goes
    // out before the LUT load, its barrier and the per-lane column math, whose latency it then covers.
    Plan cur{};
    if (Yw0 < Yw1) {
        cur = plan(Yw0, pa, pb);
        issue(cur, wbuf);
    }
    if constexpr (OUT == 1) {
        for (int i = tid; i < 768; i += kThreads) lut_s[i] = P.lut[i];
        __syncthreads();  // every wave, including those without rows
    }
    if (Yw0 >= Yw1) return;
#pragma unroll
    for (int j = 0; j < PX; j++) {
        const XTab& xt = xts[j];
        wa[j] = (uint32_t)xt.a0 | ((uint32_t)xt.a1 << 16);
        lY[j] = lC[j] = 0;
        if (xin && wa[j] != 0) {
            const int ca = x0 + xt.s0, cb = x0 + xt.s1;
            lY[j] = (uint32_t)(ca * T::bpp - fsY) | ((uint32_t)(cb * T::bpp - fsY) << 16);
            if constexpr (FMT == kNV12)
                lC[j] = (uint32_t)(2 * (ca >> 1) - fsC) | ((uint32_t)(2 * (cb >> 1) - fsC) << 16);
            else if constexpr (FMT == kI420)
                lC[j] = (uint32_t)((ca >> 1) - fsC) | ((uint32_t)((cb >> 1) - fsC) << 16);
        }
    }
    int i = 0;
    for (int Y = Yw0; Y < Yw1; Y++, i++) {
        // this row's DMA landed; the previous row's three stores may stay in flight
        if (i == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
        const uint8_t* buf = wbuf + (i & 1) * half;
        const int na = cur.pad ? pa : cur.ya, nb = cur.pad ? pb : cur.yb;
        Plan nxt{};
        if (Y + 1 < Yw1) {
            nxt = plan(Y + 1, na, nb);
            issue(nxt, wbuf + ((i + 1) & 1) * half);  // that buffer was last read by row Y - 1
        }
        // Keep every DMA of row Y + 1 ahead of row Y's stores: the vmcnt(3) above relies on that order.
        asm volatile("" ::: "memory");
        int v[3][PX];
        if (cur.pad || (kAblate & 2)) {
#pragma unroll
            for (int j = 0; j < PX; j++) { v[0][j] = fb0; v[1][j] = fo1; v[2][j] = fb2; }
        } else {
            uint32_t NA[PX][3], NB[PX][3];
            const bool shareC = kYUV && cur.stA && cur.stB && !cur.stCB;
            if (shareC) {
                if constexpr (kYUV) hrow2(buf, buf + oY1, buf + oC0, buf + oV0, NA, NB);
            } else {
                if (cur.stA) hrow(buf, buf + oC0, buf + oV0, NA);
                else {
#pragma unroll
                    for (int j = 0; j < PX; j++)
#pragma unroll
                        for (int ch = 0; ch < 3; ch++) NA[j][ch] = cur.ya == pa ? HA[j][ch] : HB[j][ch];
                }
                if (cur.stB) hrow(buf + oY1, buf + (cur.stCB ? oC1 : oC0), buf + (cur.stCB ? oV1 : oV0), NB);
                else {
#pragma unroll
                    for (int j = 0; j < PX; j++)
#pragma unroll
                        for (int ch = 0; ch < 3; ch++)
                            NB[j][ch] = cur.yb == cur.ya ? NA[j][ch] : (cur.yb == pa ? HA[j][ch] : HB[j][ch]);
                }
            }
            const uint32_t wb0 = (uint32_t)cur.b0, wb1 = (uint32_t)cur.b1;
#pragma unroll
            for (int j = 0; j < PX; j++) {
                const bool padc = wa[j] == 0;  // letterbox padding column
#pragma unroll
                for (int ch = 0; ch < 3; ch++) {
                    const int r = vresize(NA[j][ch], NB[j][ch], wb0, wb1);
                    v[ch][j] = padc ? (ch == 0 ? fb0 : (ch == 1 ? fo1 : fb2)) : r;
                }
            }
            if (REUSE) {
#pragma unroll
                for (int j = 0; j < PX; j++)
#pragma unroll
                    for (int ch = 0; ch < 3; ch++) { HA[j][ch] = NA[j][ch]; HB[j][ch] = NB[j][ch]; }
            }
        }
        store_row(Y, v);
        asm volatile("" ::: "memory");
        pa = na;
        pb = nb;
        cur = nxt;
    }
}

// Diagnostic builds only (-DEVAM_PP_TRACE): timestamps of the 100 MHz constant clock written by lane 0
// with a vector store, per workgroup (EVAM_STAMP: the ROI kernel, tools/roi_timeline.py) or per wave
// (EVAM_WSTAMP: the strip kernel, tools/wave_timeline.py). Product builds compile no stamp. In the strip
// kernel a stamp is one more VMEM operation than its counted waits assume, which only makes them wait
// longer (still exact data, slightly perturbed timing).
#ifdef EVAM_PP_TRACE
constexpr int kTraceWGs = 16384, kTraceSlots = 12;
__device__ unsigned long long g_evam_trace[kTraceWGs * kTraceSlots];
#define EVAM_STAMP(k)                                                                                  \
    do {                                                                                               \
        unsigned long long t_;                                                                         \
        __builtin_amdgcn_sched_barrier(0);                                                             \
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");               \
        __builtin_amdgcn_sched_barrier(0);                                                             \
        if (threadIdx.x == 0 && blockIdx.x < kTraceWGs) g_evam_trace[blockIdx.x * kTraceSlots + (k)] = t_; \
    } while (0)
#define EVAM_TRACE_VAL(k, v)                                                                           \
    do {                                                                                               \
        if (threadIdx.x == 0 && blockIdx.x < kTraceWGs) g_evam_trace[blockIdx.x * kTraceSlots + (k)] = (v); \
    } while (0)
#define EVAM_WSTAMP(k)                                                                                 \
    do {                                                                                               \
        unsigned long long t_;                                                                         \
        __builtin_amdgcn_sched_barrier(0);                                                             \
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");               \
        __builtin_amdgcn_sched_barrier(0);                                                             \
        const unsigned w_ = ((blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6); \
        if ((threadIdx.x & 63) == 0 && w_ < (unsigned)kTraceWGs) g_evam_trace[w_ * kTraceSlots + (k)] = t_; \
    } while (0)
#define EVAM_WTRACE_VAL(k, v)                                                                          \
    do {                                                                                               \
        const unsigned w_ = ((blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6); \
        if ((threadIdx.x & 63) == 0 && w_ < (unsigned)kTraceWGs) g_evam_trace[w_ * kTraceSlots + (k)] = (v); \
    } while (0)
#else
#define EVAM_STAMP(k) do { } while (0)
#define EVAM_TRACE_VAL(k, v) do { } while (0)
#define EVAM_WSTAMP(k) do { } while (0)
#define EVAM_WTRACE_VAL(k, v) do { } while (0)
#endif

static_assert(sizeof(evam_roi) == 20, "evam_roi layout");

// One ROI tile in launch order, self-contained: its source frame's planes and size next to the caller's
// rect, the item index (output slot) and the output rows the tile covers, so a workgroup needs one
// 64-byte scalar load (one round trip over PCIe from the pinned descriptor slot) before it can resolve
// the geometry. (A 16-byte record with the frames in the kernel arguments measured slower: the frame
// lookup is a second dependent load, profiles/r02r_c3_records.txt.)
struct alignas(64) RoiRec {  // 64 B
    const uint8_t* plane[3];
    int32_t pitch[3];
    uint16_t width, height;   // source frame (<= 32768, validated)
    int32_t x, y, w, h;       // the caller's rect
    int32_t item;
    uint16_t row0, row1;      // output rows [row0, row1) of this tile (DH <= 65535 for split tiles)
};
static_assert(sizeof(RoiRec) == 64, "RoiRec layout");
// The host builds a record as four 16-byte lines: the frame's first 40 bytes (planes, pitches, size; prepared once per
// source and call), the caller's rect (evam_roi x, y, w, h: 16 contiguous bytes), then the output index and rows.
static_assert(offsetof(RoiRec, x) == 40 && offsetof(RoiRec, item) == 56 && offsetof(RoiRec, row0) == 60, "RoiRec lines");
static_assert(offsetof(evam_roi, h) == offsetof(evam_roi, x) + 12, "evam_roi rect");
struct RecFrame { __m128i l[3]; };  // a record's bytes 0-47 for one source (bytes 40-47 zero)

// ------------------------------------------------------------------------------------------------
// strip kernel (uniform geometry, 4:2:0 sources, no shared source rows between output rows)
// ------------------------------------------------------------------------------------------------
constexpr int kMaxStrips = 32;  // per-strip footprints in the kernel arguments: DW <= 2048
constexpr int kSfoot = 64;      // footprint entries: strip kernel tile column x 8 + wave (<= 8 columns)
// One staged row segment of the strip kernel: a strip's footprint is at most one DMA instruction's 64
// 16-byte chunks, so every LDS offset of the ring is a compile-time immediate. 64-column 4:2:0 strips (PX = 1)
// use half-size slots (footprints <= 512 B, downscales <= ~7.7x): half the LDS per wave; BGRx rows are four
// bytes a pixel and always take whole 1 KB slots.
constexpr int strip_slot(int fmt, int px) { return px == 1 && fmt != kBGRX ? 512 : 1024; }

struct TParams {
    ItemArg items[kArgItems];
    double scale_x, scale_y;     // OpenCV: 1. / ((double)rw / cw), 1. / ((double)rh / ch)
    const float* lut;            // [3][256]
    void* dst;
    int slot_offset, slot_stride;  // output slot of item i = slot_offset + i * slot_stride
    int DW, DH;
    int cw, ch, rw, rh, ox, oy;  // the launch's crop size, resized size and placement (uniform)
    int nw;                      // waves (strips) per workgroup
    int TH, tiles_x, tiles_per_item;  // tile = nw strips x TH rows
    int wave_bytes;              // one wave's ring: D entries of strip_slot(PX)-byte segments
    int color_rgb;
    uint32_t fill;
    int2 sfoot[kSfoot];          // per strip: crop-relative source columns of the first visible column's
                                 // first tap and the last visible column's last tap; (-1, -1): padding only
                                 // (band kernel: per strip; strip kernel: per tile column x 8 + wave)
    // band kernel only: one wave per (item, band of TH rows, strip); LDS rows of one band
    int nstrips, units;          // strips per row; waves of work in the launch
    int segY, segC;              // bytes of one staged luma / chroma row (multiples of 16)
    int nrY;                     // most luma rows of one band (the chroma rows follow at nrY * segY)
    int prio;                    // 1: progress-based wave priority (s_setprio 3 -> 0 over the quarters of a wave's rows)
    int ahead;                   // band kernel: source rows issued ahead of the rows the current output row reads
};
static_assert(sizeof(TParams) <= 4000, "strip / band kernel arguments must fit the 4 KB kernarg segment");

// Row-strip kernel for uniform-geometry 4:2:0 batches whose output rows do not share source rows
// (downscales: C2, C4, C5). Every wave owns one strip of 64 x PX output columns of a tile (lane l holds
// columns l, l + 64, ...) and walks the tile's rows alone, one output row per step, with no workgroup
// barrier after the prologue:
//  * a ring of D row entries per wave (two luma row segments, one or two chroma row segments: the strip's
//    16-byte-aligned footprint) fed by LDS-DMA D rows ahead; the wait for a row is one counted vmcnt,
//    so the ring's other rows and the stores of the previous rows stay in flight;
//  * the OpenCV coefficient tables of the strip's columns (per lane) and of the tile's rows (one per
//    lane, read back with v_readlane) are computed in the prologue by the kernels' shared linear_coef, so
//    the first DMA waits for no table load;
//  * per pixel: four luma taps and two chroma taps per chroma row from LDS, BT.601 as saturating two-tap
//    registers, the 11-bit horizontal pass as one v_dot2 per channel, VResizeLinear 32s->8u as mulhi_u24,
//    the LUT (fp32) and three planar stores (256 contiguous bytes per store instruction).
// Strip width: the C2 data movement alone takes 39.4 us in 64-column strips and 36.4 us in 128-column
// strips (one 480-byte DMA segment per source row instead of 240: half the DMA instructions for the same
// bytes), the copy floor of those bytes on the same box (profiles/r03c_strip_bw.txt).
// Letterbox rows are plain fill stores outside the ring; letterbox columns are a per-lane select in the
// strips that have any. D = ring depth (rows of DMA in flight).
// Progress-based priority (EVAM_PP_PRIO): s_setprio 3 at the start, one level lower at each quarter of a wave's n
// steps (rows or row groups), so the waves behind get the issue slot when several are ready. One scalar compare per
// step against the next threshold; the level change sits in the rarely taken branch (the three-way compare chain it
// replaces cost six scalar instructions per step).
struct ProgressPrio {
    int next, q2, q3, level;
    __device__ __forceinline__ ProgressPrio(bool on, int n) : next(on ? n / 4 : -1), q2(n / 2), q3((3 * n) / 4), level(3) {
        if (on) __builtin_amdgcn_s_setprio(3);
    }
    __device__ __forceinline__ void step(int i) {
        if (__builtin_expect(i != next, 1)) return;
        if (level == 3) {
            __builtin_amdgcn_s_setprio(2);
            level = 2;
            next = q2;
        } else if (level == 2) {
            __builtin_amdgcn_s_setprio(1);
            level = 1;
            next = q3;
        } else {
            __builtin_amdgcn_s_setprio(0);
            level = 0;
            next = -1;
        }
    }
};

template <int FMT, int OUT, int D, int PX, int PR>
__global__ __launch_bounds__(512) void evam_pp_strip(const TParams P) {
    // the LUT at a static LDS address (folds into the reads' immediate offsets); the rings after it
    __shared__ __attribute__((aligned(16))) float lut_s[OUT == 1 ? 768 : 4];
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    static_assert(FMT == kNV12 || FMT == kI420 || FMT == kBGRX, "4:2:0 or BGRx sources");
    static_assert(D >= 1 && D <= 4, "ring depth");
    static_assert(PX == 1 || PX == 2, "pixels per lane");
    constexpr int SLOT = strip_slot(FMT, PX);
    constexpr bool PK = FMT == kBGRX;                 // packed BGRx: one plane, 4 bytes a pixel, no conversion
    constexpr int NPC = FMT == kI420 ? 2 : (PK ? 0 : 1);  // chroma planes
    // PR (paired taps): both source rows of a plane go out in ONE LDS-DMA instruction, lanes 0-31 the first
    // row's chunks and lanes 32-63 the second's (I420: U tap0 / U tap1 / V tap0 / V tap1 in lane quarters), so
    // every row costs exactly NI instructions. Without PR a row costs 2 + NPC (chroma row shared) or 2 + 2 NPC.
    static_assert(PR == 0 || PR == 1, "paired taps");
    constexpr int NMIN = PR ? (PK ? 1 : 2) : 2 + NPC;  // fewest DMA instructions of one row (PR: exact)
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (kAblate & 128) return;  // diagnostics: launch cost only
    EVAM_WSTAMP(0);
    const uint8_t *p0, *p1, *p2;
    int pitch0, pitch1, pitch2, x0, y0, index, p_nw, p_DH, p_DW, strip, Y0, Y1;
    int g_ox, g_rw, g_oy, g_rh, g_cw, k_ch, k_rgb;
    double k_scale_x, k_scale_y;
    const float* k_lut;
    int2 sf;
    // grid (tile column, tile row, item): every kernel-argument load of the prologue has an address known at
    // entry, so they all go out in one batch (one round trip before the first DMA)
    const int item = blockIdx.z, ty = blockIdx.y;
    const ItemArg& it = P.items[item];
    sf = P.sfoot[min((int)blockIdx.x * 8 + wave, kSfoot - 1)];
    const int p_TH = P.TH;
    p_nw = P.nw; p_DH = P.DH; p_DW = P.DW;
    p0 = it.plane[0];
    p1 = it.plane[1];
    p2 = it.plane[2];
    pitch0 = it.pitch[0]; pitch1 = it.pitch[1]; pitch2 = it.pitch[2];
    x0 = it.x0; y0 = it.y0;
    index = it.index;
    asm volatile("" ::"s"(p_nw), "s"(p_TH), "s"(p_DH), "s"(p_DW), "s"(P.ox), "s"(P.rw), "s"(P.oy), "s"(P.rh),
                 "s"(P.wave_bytes), "s"(p0), "s"(p1), "s"(p2), "s"(pitch0), "s"(pitch1), "s"(pitch2), "s"(x0), "s"(y0),
                 "s"(index), "s"(sf.x), "s"(sf.y), "s"(P.dst), "s"(P.slot_offset), "s"(P.slot_stride));
    // the row table's and the LUT DMA's parameters in the same batch, as opaque values the compiler cannot
    // reload: loaded where first used, they were one or two more dependent kernel-argument round trips before
    // the first DMA
    k_scale_y = P.scale_y;
    k_ch = P.ch; k_rgb = P.color_rgb;
    k_lut = P.lut;
    asm volatile("" : "+s"(k_scale_y), "+s"(k_ch), "+s"(k_lut), "+s"(k_rgb));
    strip = (int)blockIdx.x * p_nw + wave;
    Y0 = ty * p_TH; Y1 = min(Y0 + p_TH, p_DH);
    g_ox = P.ox; g_rw = P.rw; g_oy = P.oy; g_rh = P.rh; g_cw = P.cw;
    k_scale_x = P.scale_x;
    const int X0 = strip * 64 * PX;
    const bool live = X0 < p_DW;  // a wave past the last strip only joins the LUT barrier
    const bool cols = live && sf.x >= 0;
    int fsY = 0, nY = 0, fsC = 0, nC = 0;
    if (cols) footprint_chunks(FMT, PK ? 4 : 1, x0 + sf.x, x0 + sf.y, fsY, nY, fsC, nC);
    // visible output rows of the tile (the rest are letterbox fill)
    const int vr0 = max(Y0, g_oy), vr1 = min(Y1, g_oy + g_rh);
    const int n = cols && vr1 > vr0 ? vr1 - vr0 : 0;

    // row table, one visible row per lane: source rows relative to the crop, weights << 8
    int lr0 = 0, lr1 = 0, lb0 = 0, lb1 = 0;
    if (lane < n) {
        int sy, b0, b1;
        linear_coef(vr0 + lane - g_oy, k_scale_y, k_ch, false, sy, b0, b1);
        lr0 = min(max(sy, 0), k_ch - 1);
        lr1 = min(max(sy + 1, 0), k_ch - 1);
        lb0 = b0 << 8;
        lb1 = b1 << 8;
    }
    const __amdgpu_buffer_rsrc_t rsY = __builtin_amdgcn_make_buffer_rsrc((void*)p0, (short)0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsU = __builtin_amdgcn_make_buffer_rsrc((void*)p1, (short)0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsV = __builtin_amdgcn_make_buffer_rsrc((void*)(NPC == 2 ? p2 : p1), (short)0, 0x7FFFFFFF, 0x00020000);
    uint8_t* const wbuf = smem + wave * P.wave_bytes;
    // Ring entry layout. Without PR: [Y tap0][Y tap1][C tap0][C tap1] (+ [V tap0][V tap1] for I420), SLOT bytes
    // each; BGRx: [row tap0][row tap1]. With PR: [Y tap0 | Y tap1] (512 B halves) then, for 4:2:0,
    // [C tap0 | C tap1] (NV12, 512 B halves) or [U tap0 | U tap1 | V tap0 | V tap1] (I420, 256 B quarters).
    //   SY: Y tap1 - Y tap0; CB: chroma region; SC: C tap1 - C tap0; SV: I420 V tap0 - U tap0.
    constexpr int SY = PR ? 512 : SLOT;
    constexpr int CB = PR ? 1024 : 2 * SLOT;
    constexpr int SC = PR ? (NPC == 2 ? 256 : 512) : SLOT;
    constexpr int SV = PR ? 512 : 2 * SLOT;
    constexpr int GRP = PR ? (PK ? 1024 : 2048) : 2 * SLOT + 2 * NPC * SLOT;
    constexpr int segY = SY;
    // I420 with PR: one buffer resource over both chroma planes, based at the lower one. Every byte read lies below
    // (offset of the upper plane) + (its extent), which must stay under num_records 0x7FFFFFFF: the host admits the
    // pairing only when that holds for every item of the launch, else the group runs unpaired
    const uint8_t* const pcl = NPC == 2 && PR ? (p1 < p2 ? p1 : p2) : p1;
    const uint32_t dU = (uint32_t)(p1 - pcl), dV = (uint32_t)(p2 - pcl);
    const __amdgpu_buffer_rsrc_t rsC2 = __builtin_amdgcn_make_buffer_rsrc((void*)pcl, (short)0, 0x7FFFFFFF, 0x00020000);
    auto issue = [&](int i, int k) {
        if (kAblate & 16) return;  // diagnostics: no DMA
        const int ya = y0 + __builtin_amdgcn_readlane(lr0, i), yb = y0 + __builtin_amdgcn_readlane(lr1, i);
        uint8_t* e = wbuf + k * GRP;
        if constexpr (PR) {
            const int hi = lane >> 5, c = lane & 31;
            if (c < nY)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rsY, (__attribute__((address_space(3))) void*)e, 16,
                                                         (uint32_t)((hi ? yb : ya) * pitch0 + fsY + c * 16), 0,
                                                         EVAM_PP_LOAD_AUX, 0);
            if constexpr (NPC == 1) {
                const int ca = ya >> 1, cb = yb >> 1;
                if (c < nC && (!hi || ca != cb))
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsU, (__attribute__((address_space(3))) void*)(e + CB), 16,
                                                             (uint32_t)((hi ? cb : ca) * pitch1 + fsC + c * 16), 0,
                                                             EVAM_PP_LOAD_AUX, 0);
            } else if constexpr (NPC == 2) {
                const int ca = ya >> 1, cb = yb >> 1, q = lane >> 4, c4 = lane & 15, r = (q & 1) ? cb : ca;
                const uint32_t off = (q & 2) ? dV + (uint32_t)(r * pitch2) : dU + (uint32_t)(r * pitch1);
                if (c4 < nC && (!(q & 1) || ca != cb))
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsC2, (__attribute__((address_space(3))) void*)(e + CB), 16,
                                                             off + (uint32_t)(fsC + c4 * 16), 0, EVAM_PP_LOAD_AUX, 0);
            }
            return;
        }
        const uint32_t vo = (uint32_t)lane * 16u;
        if (lane < nY) {
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsY, (__attribute__((address_space(3))) void*)e, 16, vo,
                                                     ya * pitch0 + fsY, EVAM_PP_LOAD_AUX, 0);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsY, (__attribute__((address_space(3))) void*)(e + segY), 16, vo,
                                                     yb * pitch0 + fsY, EVAM_PP_LOAD_AUX, 0);
        }
        if constexpr (NPC == 0) return;
        const int ca = ya >> 1, cb = yb >> 1;
        if (lane < nC) {
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsU, (__attribute__((address_space(3))) void*)(e + CB), 16, vo,
                                                     ca * pitch1 + fsC, EVAM_PP_LOAD_AUX, 0);
            if constexpr (NPC == 2)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rsV, (__attribute__((address_space(3))) void*)(e + CB + SV),
                                                         16, vo, ca * pitch2 + fsC, EVAM_PP_LOAD_AUX, 0);
        }
        if (ca != cb && lane < nC) {
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsU, (__attribute__((address_space(3))) void*)(e + CB + SC), 16,
                                                     vo, cb * pitch1 + fsC, EVAM_PP_LOAD_AUX, 0);
            if constexpr (NPC == 2)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rsV, (__attribute__((address_space(3))) void*)(e + CB + SV + SC),
                                                         16, vo, cb * pitch2 + fsC, EVAM_PP_LOAD_AUX, 0);
        }
    };

    // The LUT first (oldest VMEM: the first row's wait covers it), then the ring's first D rows. With four or
    // more waves, waves 0-2 each bring one 1 KB section by LDS-DMA (source section swapped for RGB): no ds_write
    // follows the ring's DMA, so nothing makes the compiler drain the ring before the LUT barrier.
    const int nthr = p_nw * 64;
    const bool lut_early = nthr >= 256;
    if constexpr (OUT == 1) {
        if (lut_early && wave < 3) {
            const __amdgpu_buffer_rsrc_t rsL = __builtin_amdgcn_make_buffer_rsrc((void*)k_lut, (short)0, 3072, 0x00020000);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsL, (__attribute__((address_space(3))) void*)(lut_s + wave * 256), 16,
                                                     (uint32_t)lane * 16u, (k_rgb ? 2 - wave : wave) * 1024, 0, 0);
        }
    }
    const int npro = min(n, D);
    for (int i = 0; i < npro; i++) issue(i, i);
    EVAM_WSTAMP(1);
    EVAM_WTRACE_VAL(5, (unsigned long long)blockIdx.z | ((unsigned long long)strip << 16) |
                           ((unsigned long long)blockIdx.y << 32) | ((unsigned long long)n << 48));

    // per-lane column state of the lane's PX pixels: tap offsets inside the staged segments, packed
    // 11-bit weights, store offsets
    bool xin[PX], padc[PX];
    uint32_t lY[PX], lC0[PX], lC1[PX], wp[PX], vo[PX];
    bool anyp = false;
    const size_t esz = OUT == 1 ? 4 : 1;
#pragma unroll
    for (int j = 0; j < PX; j++) {
        const int X = X0 + lane + 64 * j;
        xin[j] = live && X < p_DW;
        vo[j] = (uint32_t)(xin[j] ? X : 0) * (uint32_t)esz;
        lY[j] = lC0[j] = lC1[j] = wp[j] = 0;
        padc[j] = true;
        const int dx = X - g_ox;
        if (cols && xin[j] && dx >= 0 && dx < g_rw) {
            int s0, a0, a1;
            linear_coef(dx, k_scale_x, g_cw, true, s0, a0, a1);
            const int ca = x0 + s0;  // tap 1 reads ca + 1: at the right edge (s0 = cw - 1) its weight a1 is 0
            lY[j] = (uint32_t)(ca * (PK ? 4 : 1) - fsY);
            if constexpr (FMT == kNV12) {
                lC0[j] = (uint32_t)(2 * (ca >> 1) - fsC);
                lC1[j] = (uint32_t)(2 * ((ca + 1) >> 1) - fsC);
            } else if constexpr (FMT == kI420) {
                lC0[j] = (uint32_t)((ca >> 1) - fsC);
                lC1[j] = (uint32_t)(((ca + 1) >> 1) - fsC);
            }
            // BGRx: the weights carry the 16x that the 4:2:0 path's saturating clamp leaves on its taps
            wp[j] = PK ? ((uint32_t)a0 << 4) | ((uint32_t)a1 << 20) : (uint32_t)a0 | ((uint32_t)a1 << 16);
            padc[j] = false;
        }
        anyp |= xin[j] && padc[j];
    }
    // some visible lane shows letterbox columns (wave-uniform): only then the per-pixel fill select
    const bool anypad = cols && __builtin_amdgcn_ballot_w64(anyp) != 0;
    // stores per row of this wave: 3 per pixel column group with any lane inside the output (counted waits)
    const bool full = X0 + 64 * (PX - 1) < p_DW;

    const size_t plane = (size_t)p_DW * p_DH;
    uint8_t* const d0 = reinterpret_cast<uint8_t*>(P.dst) + (size_t)(P.slot_offset + index * P.slot_stride) * 3 * plane * esz;
    uint8_t* const d1 = d0 + plane * esz;
    uint8_t* const d2 = d1 + plane * esz;
    // output planes in source channel order (B, G, R): planes 0 and 2 exchanged for RGB
    const __amdgpu_buffer_rsrc_t rsO0 = __builtin_amdgcn_make_buffer_rsrc((void*)(k_rgb ? d2 : d0), (short)0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsO1 = __builtin_amdgcn_make_buffer_rsrc((void*)d1, (short)0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsO2 = __builtin_amdgcn_make_buffer_rsrc((void*)(k_rgb ? d0 : d2), (short)0, 0x7FFFFFFF, 0x00020000);
    // fill in source channel order (P.fill is in output plane order)
    const uint32_t fq0 = P.fill & 0xFF, fq1 = (P.fill >> 8) & 0xFF, fq2 = (P.fill >> 16) & 0xFF;
    const uint32_t fsh = OUT == 1 ? 2 : 0;
    const uint32_t fill0 = (k_rgb ? fq2 : fq0) << fsh, fill1 = fq1 << fsh, fill2 = (k_rgb ? fq0 : fq2) << fsh;

    if constexpr (OUT == 1) {
        if (lut_early) {
            // this wave's LUT section landed once at most the ring's DMA instructions are outstanding; the
            // barrier then needs no vmcnt(0): each wave waits for its own ring rows in the loop
            if (npro == D) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NMIN * D) : "memory");
            else vmcnt_exact(NMIN * npro);
            lds_barrier();
        } else {  // workgroups of 1-3 waves (outputs narrower than 64 x PX x 3 + 1 columns)
            for (int idx = threadIdx.x; idx < 768; idx += nthr)
                lut_s[idx] = k_lut[k_rgb ? 512 - (idx & ~255) + (idx & 255) : idx];
            __syncthreads();
        }
    }
    EVAM_WSTAMP(2);
    if (!live) return;
    if (kAblate & 64) {  // diagnostics: prologue only (tables, LUT, the ring's first DMA)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("" ::"v"(lY[0]), "v"(lC0[0]), "v"(lC1[0]), "v"(wp[0]), "v"(vo[0]), "v"(lb0), "v"(lb1));
        return;
    }
    const uint8_t* lutb = reinterpret_cast<const uint8_t*>(lut_s);
    // per-lane LDS addresses of the taps in ring entry 0 (entry k adds k * GRP, an immediate offset)
    const uint8_t* aY[PX];
    const uint8_t* aC0[PX];
    const uint8_t* aC1[PX];
#pragma unroll
    for (int j = 0; j < PX; j++) {
        aY[j] = wbuf + lY[j];
        aC0[j] = wbuf + CB + lC0[j];
        aC1[j] = wbuf + CB + lC1[j];
    }
    // BT.601 chroma-term constants: the additive ones in VGPRs so every term is one v_mad (a VOP3 reads one
    // scalar operand: the multiplier)
    uint32_t kb = kKBs, kg = kKGs, kr = kKRs;
    int cvg = kCVG, cug = kCUG;
    asm volatile("" : "+v"(kb), "+v"(kg), "+v"(kr), "+s"(cvg), "+s"(cug));
    auto uvt = [&](uint32_t U, uint32_t V) {
        // g = V * CVG + (U * CUG + K): two v_mad_i32_i24 (the sum of two products would select mul, mul, add3)
        int gu = __mul24((int)U, cug) + (int)kg;
        asm("" : "+v"(gu));  // keeps the association (no asm volatile: still scheduled freely)
        return UVs{__umul24(U, (uint32_t)kCUB) + kb, (uint32_t)(__mul24((int)V, cvg) + gu), __umul24(V, (uint32_t)kCVR) + kr};
    };
    // pixel column group j of row Y; v: LUT byte offsets (fp32) or bytes (u8), source channel order
    auto put = [&](int Y, int j, uint32_t v0, uint32_t v1, uint32_t v2) {
        if (!xin[j]) return;
        if (kAblate & 4) {  // diagnostics: no stores
            asm volatile("" ::"v"(v0), "v"(v1), "v"(v2));
            return;
        }
        const int so = (int)((uint32_t)(Y * p_DW) * (uint32_t)esz);
        if constexpr (OUT == 1) {
            __builtin_amdgcn_raw_buffer_store_b32(*reinterpret_cast<const uint32_t*>(lutb + v0), rsO0, vo[j], so, EVAM_PP_STORE_AUX);
            __builtin_amdgcn_raw_buffer_store_b32(*reinterpret_cast<const uint32_t*>(lutb + 1024 + v1), rsO1, vo[j], so, EVAM_PP_STORE_AUX);
            __builtin_amdgcn_raw_buffer_store_b32(*reinterpret_cast<const uint32_t*>(lutb + 2048 + v2), rsO2, vo[j], so, EVAM_PP_STORE_AUX);
        } else {
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)v0, rsO0, vo[j], so, EVAM_PP_STORE_AUX);
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)v1, rsO1, vo[j], so, EVAM_PP_STORE_AUX);
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)v2, rsO2, vo[j], so, EVAM_PP_STORE_AUX);
        }
    };
    auto put_fill = [&](int Y) {
#pragma unroll
        for (int j = 0; j < PX; j++) put(Y, j, fill0, fill1, fill2);
    };
    // letterbox rows above the ring: before its DMA in issue order, so they never enter the counted waits
    const int ra = n ? vr0 : Y1;
    for (int Y = Y0; Y < ra; Y++) put_fill(Y);

    // Progress-based priority (EVAM_PP_PRIO): waves of a SIMD otherwise share issue by age, so the youngest
    // workgroups' waves lag and end the launch alone; a wave lowers its priority as it passes each quarter of its
    // rows, so the ones behind get the issue slots when several are ready.
    ProgressPrio prio(P.prio != 0, n);
    const int nst = full ? 3 * PX : 3;
    // one output row: row i of the tile's visible rows, ring entry kk (compile-time after unrolling)
    auto row = [&](int i, int kk, auto has_pad) {
        constexpr bool PADC = decltype(has_pad)::value;
        // row i's DMA landed. Issued after it: the DMA of rows i+1 .. i+D-1 (>= NMIN each) and the stores
        // of rows i-D+1 .. i-1 (nst each)
        constexpr int SD = D - 1;
        if (SD == 0) {  // nothing was issued after row i's DMA
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else if (i >= SD && i + D - 1 < n) {
            if (PX == 1 || !full) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((D - 1) * NMIN + SD * 3) : "memory");
            else asm volatile("s_waitcnt vmcnt(%0)" ::"n"((D - 1) * NMIN + SD * 3 * PX) : "memory");
        } else {
            vmcnt_exact(NMIN * (min(i + D - 1, n - 1) - i) + nst * min(i, SD));
        }
#ifdef EVAM_PP_TRACE
        if (i == 0) EVAM_WSTAMP(3);
#endif
        prio.step(i);
        const int Y = vr0 + i;
        const uint32_t wb0 = (uint32_t)__builtin_amdgcn_readlane(lb0, i), wb1 = (uint32_t)__builtin_amdgcn_readlane(lb1, i);
        const int ya = __builtin_amdgcn_readlane(lr0, i), yb = __builtin_amdgcn_readlane(lr1, i);
        const bool share = ((y0 + ya) >> 1) == ((y0 + yb) >> 1);
        if (kAblate & 2) {  // diagnostics: no pixel math (no tap reads)
            put_fill(Y);
        } else if constexpr (PK) {
            // BGRx: both taps of a source row are two adjacent dwords; channel c of the pair is one v_perm into
            // two u16 halves, and the horizontal pass one v_dot2 with the 16x weights
            const int eo = kk * GRP;
#pragma unroll
            for (int j = 0; j < PX; j++) {
                const uint32_t* ay = reinterpret_cast<const uint32_t*>(aY[j] + eo);
                const uint32_t qa0 = ay[0], qa1 = ay[1], qb0 = ay[SY / 4], qb1 = ay[SY / 4 + 1];
                uint32_t v[3];
#pragma unroll
                for (int c = 0; c < 3; c++) {
                    const uint32_t sel = 0x0C000C00u | ((uint32_t)(4 + c) << 16) | (uint32_t)c;
                    const uint32_t ha = __builtin_amdgcn_udot2(
                        __builtin_bit_cast(evam_u16x2, __builtin_amdgcn_perm(qa1, qa0, sel)),
                        __builtin_bit_cast(evam_u16x2, wp[j]), 0u, false);
                    const uint32_t hb = __builtin_amdgcn_udot2(
                        __builtin_bit_cast(evam_u16x2, __builtin_amdgcn_perm(qb1, qb0, sel)),
                        __builtin_bit_cast(evam_u16x2, wp[j]), 0u, false);
                    v[c] = vfinal<OUT>(ha, hb, wb0, wb1);
                }
                if constexpr (PADC) {
                    v[0] = padc[j] ? fill0 : v[0];
                    v[1] = padc[j] ? fill1 : v[1];
                    v[2] = padc[j] ? fill2 : v[2];
                }
                put(Y, j, v[0], v[1], v[2]);
            }
        } else {
            const int eo = kk * GRP;  // this entry's offset from entry 0
            // raw taps of the entry into registers: luma bytes of both source rows, chroma of the first
            // chroma row and, when the second source row has its own, of the second
            uint32_t rY[PX][4], rC[PX][2][2], rE[PX][2][2];
            auto raw_c = [&](const uint8_t* a, int o, uint32_t (&c)[2]) {
                c[0] = a[o];
                c[1] = FMT == kNV12 ? a[o + 1] : a[o + SV];  // NV12: interleaved UV; I420: the V slot
            };
#pragma unroll
            for (int j = 0; j < PX; j++) {
                const uint8_t* ay = aY[j] + eo;
                rY[j][0] = ay[0]; rY[j][1] = ay[1]; rY[j][2] = ay[SY]; rY[j][3] = ay[SY + 1];
                raw_c(aC0[j], eo, rC[j][0]);
                raw_c(aC1[j], eo, rC[j][1]);
            }
            if (!share) {
#pragma unroll
                for (int j = 0; j < PX; j++) {
                    raw_c(aC0[j], eo + SC, rE[j][0]);
                    raw_c(aC1[j], eo + SC, rE[j][1]);
                }
            }
#pragma unroll
            for (int j = 0; j < PX; j++) {
                const UVs tA = uvt(rC[j][0][0], rC[j][0][1]), tB = uvt(rC[j][1][0], rC[j][1][1]);
                const uint32_t yA = luma_term(rY[j][0]), yB = luma_term(rY[j][1]);
                const uint32_t yC = luma_term(rY[j][2]), yD = luma_term(rY[j][3]);
                uint32_t h0[3], h1[3];
                h0[0] = hpass_sat(yA, tA.b, yB, tB.b, wp[j]);
                h0[1] = hpass_sat(yA, tA.g, yB, tB.g, wp[j]);
                h0[2] = hpass_sat(yA, tA.r, yB, tB.r, wp[j]);
                if (share) {  // both vertical taps in one chroma row: its terms serve both source rows
                    h1[0] = hpass_sat(yC, tA.b, yD, tB.b, wp[j]);
                    h1[1] = hpass_sat(yC, tA.g, yD, tB.g, wp[j]);
                    h1[2] = hpass_sat(yC, tA.r, yD, tB.r, wp[j]);
                    // distinct markers end the two branches, so the compiler does not merge their common
                    // tail behind register copies of the chroma terms
                    asm volatile("; strip: shared chroma row" ::"v"(h1[0]), "v"(h1[1]), "v"(h1[2]));
                } else {
                    const UVs tC = uvt(rE[j][0][0], rE[j][0][1]), tE = uvt(rE[j][1][0], rE[j][1][1]);
                    h1[0] = hpass_sat(yC, tC.b, yD, tE.b, wp[j]);
                    h1[1] = hpass_sat(yC, tC.g, yD, tE.g, wp[j]);
                    h1[2] = hpass_sat(yC, tC.r, yD, tE.r, wp[j]);
                    asm volatile("; strip: two chroma rows" ::"v"(h1[0]), "v"(h1[1]), "v"(h1[2]));
                }
                uint32_t v[3];
#pragma unroll
                for (int c = 0; c < 3; c++) v[c] = vfinal<OUT>(h0[c], h1[c], wb0, wb1);
                if constexpr (PADC) {
                    v[0] = padc[j] ? fill0 : v[0];
                    v[1] = padc[j] ? fill1 : v[1];
                    v[2] = padc[j] ? fill2 : v[2];
                }
                put(Y, j, v[0], v[1], v[2]);
            }
        }
        asm volatile("" ::: "memory");  // issue order is what the counted waits assume
        if (i + D < n) issue(i + D, kk);  // this entry's reads are done: the stores consumed them
        asm volatile("" ::: "memory");
    };
    auto ring = [&](auto has_pad) {
        for (int i0 = 0; i0 < n; i0 += D) {
#pragma unroll
            for (int kk = 0; kk < D; kk++)
                if (i0 + kk < n) row(i0 + kk, kk, has_pad);
        }
    };
    if (anypad) ring(std::true_type{});
    else ring(std::false_type{});
    // letterbox rows below the ring
    for (int Y = max(ra, vr1); Y < Y1; Y++) put_fill(Y);
#ifdef EVAM_PP_TRACE
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the last stores retired
    EVAM_WSTAMP(4);
    {
        unsigned xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        EVAM_WTRACE_VAL(6, (unsigned long long)xcc);
    }
#endif
}

// Wait until at most n (>= 0, wave-uniform) vector-memory operations of this wave are outstanding, rounded down to
// 0-4, 6, 8, 12, 16 or 32: waiting for a few more operations than needed is always safe. A binary tree of scalar
// compares and branches in one asm block: 4-5 compares, one wait and one branch on every path. (The same tree in C was
// structurised by the compiler into flag registers carried through every level, ~25 scalar instructions per wait;
// same box, one launch at a time: C1 equal, C1 / I420 +2.2 %, profiles/r06n_vmcnt_asm_ab.txt. The tree itself costs a
// third of the scalar instructions of an exact 64-case jump, C1 +2 % against it: profiles/r04k2_vmcnt_coarse_ab.txt.)
__device__ __forceinline__ void vmcnt_le(int n) {
    n = __builtin_amdgcn_readfirstlane(n);
    asm volatile(
        "s_cmp_lt_i32 %0, 8\n\t"
        "s_cbranch_scc1 5f\n\t"
        "s_cmp_lt_i32 %0, 16\n\t"
        "s_cbranch_scc1 2f\n\t"
        "s_cmp_lt_i32 %0, 32\n\t"
        "s_cbranch_scc1 1f\n\t"
        "s_waitcnt vmcnt(32)\n\t"
        "s_branch 9f\n"
        "1:\n\t"
        "s_waitcnt vmcnt(16)\n\t"
        "s_branch 9f\n"
        "2:\n\t"
        "s_cmp_lt_i32 %0, 12\n\t"
        "s_cbranch_scc1 3f\n\t"
        "s_waitcnt vmcnt(12)\n\t"
        "s_branch 9f\n"
        "3:\n\t"
        "s_waitcnt vmcnt(8)\n\t"
        "s_branch 9f\n"
        "5:\n\t"
        "s_cmp_lt_i32 %0, 4\n\t"
        "s_cbranch_scc1 7f\n\t"
        "s_cmp_lt_i32 %0, 6\n\t"
        "s_cbranch_scc1 6f\n\t"
        "s_waitcnt vmcnt(6)\n\t"
        "s_branch 9f\n"
        "6:\n\t"
        "s_waitcnt vmcnt(4)\n\t"
        "s_branch 9f\n"
        "7:\n\t"
        "s_cmp_lt_i32 %0, 2\n\t"
        "s_cbranch_scc1 8f\n\t"
        "s_cmp_lt_i32 %0, 3\n\t"
        "s_cbranch_scc1 4f\n\t"
        "s_waitcnt vmcnt(3)\n\t"
        "s_branch 9f\n"
        "4:\n\t"
        "s_waitcnt vmcnt(2)\n\t"
        "s_branch 9f\n"
        "8:\n\t"
        "s_cmp_lt_i32 %0, 1\n\t"
        "s_cbranch_scc1 10f\n\t"
        "s_waitcnt vmcnt(1)\n\t"
        "s_branch 9f\n"
        "10:\n\t"
        "s_waitcnt vmcnt(0)\n"
        "9:"
        ::"s"(n)
        : "scc", "memory");
}

// Band kernel for uniform 4:2:0 batches whose consecutive output rows share source rows (vertical
// upscales: C1). One wave owns one band of TH output rows of one 64·PX-column strip (lane l: the PX
// adjacent columns X0 + PX l ..), with no workgroup barrier after the prologue:
//  * every source row the band reads (luma rows r0(first) .. r1(last), and their chroma rows) is staged
//    once, in need order, by one LDS-DMA instruction per row segment at the start; output row i then
//    waits with one counted vmcnt for the rows it needs, so its arithmetic overlaps the later rows' DMA;
//  * horizontal results stay in registers per source row (HA: row pa, HB: row pb) and the BT.601 chroma
//    terms per chroma row, so a source row is converted and filtered once however many output rows read
//    it (~0.84 source rows per output row at 432 -> 512);
//  * coefficients of the strip's columns (per lane) and of the band's rows (one per lane, v_readlane)
//    come from the kernels' shared linear_coef: no table loads (the host's column table loaded at entry instead
//    was 1.5 % slower on C1: the per-pixel setup then waits for the load, profiles/r05t_c1_band_table_dd_ab.txt);
//  * DD (six-column lanes, band_six_columns): a lane's 4 pixels read 6 source columns and 3 chroma columns, so a
//    source row costs 6 luma and 18 saturating sums instead of 8 and 24, a chroma row 3 conversions instead of 8;
//  * each channel of a row leaves as one PX-wide store per lane.
// Workgroups of up to four waves: the strips of one band of one item.
template <int FMT, int OUT, int PX, int DD>
__global__ __launch_bounds__(256) void evam_pp_band(const TParams P) {
    __shared__ __attribute__((aligned(16))) float lut_s[OUT == 1 ? 768 : 4];
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    if (kAblate & 128) return;  // diagnostics: launch cost only
    static_assert(FMT == kNV12 || FMT == kI420, "4:2:0 sources");
    static_assert(PX == 1 || PX == 2 || PX == 4, "pixels per lane");
    static_assert(!DD || PX == 4, "six-column lanes hold 4 pixels");
    constexpr int NPC = FMT == kI420 ? 2 : 1;  // chroma planes
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    EVAM_WSTAMP(0);
    // grid (strip group, band, item): every kernel-argument load of the prologue has an address known at entry,
    // so they all go out in one batch (one round trip before the first DMA)
    const int item = blockIdx.z, band = blockIdx.y;
    const ItemArg& it = P.items[item];
    const int2 sf = P.sfoot[min((int)blockIdx.x * 8 + wave, kSfoot - 1)];
    const int p_nw = P.nw, p_TH = P.TH, p_DH = P.DH, p_DW = P.DW;
    int p_ns = P.nstrips, k_wb = P.wave_bytes;
    const uint8_t* p0 = it.plane[0];
    const uint8_t* p1 = it.plane[1];
    const uint8_t* p2 = it.plane[2];
    const int pitch0 = it.pitch[0], pitch1 = it.pitch[1], pitch2 = it.pitch[2];
    const int x0 = it.x0, y0 = it.y0;
    // The row table's and the LUT DMA's parameters join the batch as opaque values the compiler cannot reload
    // (loaded where first used, they were two more dependent kernel-argument round trips before the first DMA);
    // one statement, so every load goes out before the one wait (30 operands at most: the output's
    // parameters, first needed at the first store, are left out).
    double k_scale_y = P.scale_y;
    int k_ch = P.ch, k_rgb = P.color_rgb;
    const float* k_lut = P.lut;
    asm volatile("" : "+s"(k_scale_y), "+s"(k_ch), "+s"(k_lut), "+s"(k_rgb), "+s"(p_ns), "+s"(k_wb)
                 : "s"(p_nw), "s"(p_TH), "s"(p_DH), "s"(p_DW), "s"(P.ox), "s"(P.rw), "s"(P.oy), "s"(P.rh),
                   "s"(P.segY), "s"(P.segC), "s"(P.nrY), "s"(p0), "s"(p1), "s"(p2), "s"(pitch0),
                   "s"(pitch1), "s"(pitch2), "s"(x0), "s"(y0), "s"(it.index), "s"(sf.x), "s"(sf.y));
    const int strip = (int)blockIdx.x * p_nw + wave;
    const bool live = strip < p_ns;
    const int Y0 = band * p_TH, Y1 = min(Y0 + p_TH, p_DH);
    const int X0 = strip * 64 * PX;
    const bool cols = live && sf.x >= 0;
    int fsY = 0, nY = 0, fsC = 0, nC = 0;
    if (cols) footprint_chunks(FMT, 1, x0 + sf.x, x0 + sf.y, fsY, nY, fsC, nC);
    const int vr0 = max(Y0, P.oy), vr1 = min(Y1, P.oy + P.rh);
    const int n = cols && vr1 > vr0 ? vr1 - vr0 : 0;  // visible rows of the band (<= 64)

    // row table, one visible row per lane: source rows relative to the crop, weights << 8
    int lr0 = 0, lr1 = 0, lb0 = 0, lb1 = 0;
    if (lane < n) {
        int sy, b0, b1;
        linear_coef(vr0 + lane - P.oy, k_scale_y, k_ch, false, sy, b0, b1);
        lr0 = min(max(sy, 0), k_ch - 1);
        lr1 = min(max(sy + 1, 0), k_ch - 1);
        lb0 = b0 << 8;
        lb1 = b1 << 8;
    }
    const __amdgpu_buffer_rsrc_t rsY = __builtin_amdgcn_make_buffer_rsrc((void*)p0, (short)0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsU = __builtin_amdgcn_make_buffer_rsrc((void*)p1, (short)0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsV = __builtin_amdgcn_make_buffer_rsrc((void*)(NPC == 2 ? p2 : p1), (short)0, 0x7FFFFFFF, 0x00020000);
    uint8_t* const wbuf = smem + wave * k_wb;
    const int segY = P.segY, segC = P.segC;
    uint8_t* const cbuf = wbuf + P.nrY * segY;  // chroma rows; I420: V row k at + segC / 2 (segC holds U | V)
    // source rows of the band (rows are monotonic in the output row): luma [rlo, rhi], chroma [clo, chi]
    const int rlo = n ? __builtin_amdgcn_readlane(lr0, 0) : 0;
    const int rhi = n ? __builtin_amdgcn_readlane(lr1, n - 1) : -1;
    const int clo = (y0 + rlo) >> 1;
    // The wave counts every vector-memory operation it issues (pos) and remembers pos right after each luma row's
    // DMA (lane r - rlo of dpos), so every wait below is exact.
    int pos = 0, dpos = 0;
    // fp32: the LUT (3 KB, sections in source channel order) by LDS-DMA ahead of the rows, so no VGPR waits
    // on it and the rows' counted waits are unaffected (it is older)
    if constexpr (OUT == 1) {
        for (int c0 = wave * 64; c0 < 192; c0 += (int)(blockDim.x >> 6) * 64, pos++) {
            const int c = c0 + lane, sec = c >> 6;
            const int src = ((k_rgb ? 2 - sec : sec) * 64 + (c & 63)) * 16;
            const __amdgpu_buffer_rsrc_t rsL = __builtin_amdgcn_make_buffer_rsrc((void*)k_lut, (short)0, 3072, 0x00020000);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsL, (__attribute__((address_space(3))) void*)((uint8_t*)lut_s + c0 * 16),
                                                     16, (uint32_t)src, 0, 0, 0);
        }
    }
    const int lut_pos = pos;
    // DMA in need order: luma row r, then its chroma row when r is the first row reading it. Rows go out up to
    // `ahead` source rows past the last row the current output row reads (EVAM_PP_BAND_AHEAD; 64: the whole band
    // at once), so a wave's first rows do not queue behind the rest of the band in the launch's opening burst.
    int rnext = rlo, cprev = -1;
    const int ahead = P.ahead;
    auto issue_to = [&](int rmax) {
        const uint32_t vo = (uint32_t)lane * 16u;
        for (; rnext <= rmax; rnext++) {
            const int r = rnext, ya = y0 + r, c = ya >> 1;
            if (lane < nY)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rsY, (__attribute__((address_space(3))) void*)(wbuf + (r - rlo) * segY),
                                                         16, vo, ya * pitch0 + fsY, EVAM_PP_LOAD_AUX, 0);
            pos++;
            if (c != cprev) {
                uint8_t* cb = cbuf + (c - clo) * segC;
                if (lane < nC) {
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsU, (__attribute__((address_space(3))) void*)cb, 16, vo,
                                                             c * pitch1 + fsC, EVAM_PP_LOAD_AUX, 0);
                    if constexpr (NPC == 2)
                        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsV, (__attribute__((address_space(3))) void*)(cb + segC / 2),
                                                                 16, vo, c * pitch2 + fsC, EVAM_PP_LOAD_AUX, 0);
                }
                pos += NPC;
                cprev = c;
            }
            dpos = lane == r - rlo ? pos : dpos;
        }
    };
    if (n) issue_to(min(rhi, __builtin_amdgcn_readlane(lr1, 0) + ahead));
    EVAM_WSTAMP(1);
    EVAM_WTRACE_VAL(5, (unsigned long long)n << 48);

    if constexpr (OUT == 1) {
        vmcnt_le(pos - lut_pos);  // this wave's LUT pieces landed (issued before every row)
        lds_barrier();            // ... and every other wave's (LDS only: the rows' DMA stays in flight)
    }
    if (!live) return;

    // per-lane column state: tap offsets in the staged rows (tap 0 low, tap 1 high half), packed 11-bit
    // weights, padding columns
    const int X = X0 + lane * PX;
    const bool xin = X < p_DW;  // DW % PX == 0: a lane's pixels are all in or all out
    uint32_t lY[PX], lC[PX], wp[PX];
    bool padc[PX];
    bool anyp = false;
#pragma unroll
    for (int j = 0; j < PX; j++) {
        lY[j] = lC[j] = wp[j] = 0;
        padc[j] = true;
        const int dx = X + j - P.ox;
        if (cols && xin && dx >= 0 && dx < P.rw) {
            int s0, a0, a1;
            linear_coef(dx, P.scale_x, P.cw, true, s0, a0, a1);
            const int ca = x0 + s0, cb = x0 + min(s0 + 1, P.cw - 1);
            lY[j] = (uint32_t)(ca - fsY) | ((uint32_t)(cb - fsY) << 16);
            if constexpr (FMT == kNV12)
                lC[j] = (uint32_t)(2 * (ca >> 1) - fsC) | ((uint32_t)(2 * (cb >> 1) - fsC) << 16);
            else
                lC[j] = (uint32_t)((ca >> 1) - fsC) | ((uint32_t)((cb >> 1) - fsC) << 16);
            wp[j] = (uint32_t)a0 | ((uint32_t)a1 << 16);
            padc[j] = false;
        }
        anyp |= xin && padc[j];
    }
    const bool anypad = __builtin_amdgcn_ballot_w64(anyp) != 0;
    if (kAblate & 64) {  // diagnostics: prologue only (row / column coefficients, the first rows' DMA landed)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("" ::"v"(lY[0]), "v"(lC[0]), "v"(wp[0]), "v"(lb0), "v"(lb1), "v"((int)anypad));
        return;
    }
    const size_t esz = OUT == 1 ? 4 : 1;
    const uint32_t vo = (uint32_t)(xin ? X : 0) * (uint32_t)esz;
    const size_t plane = (size_t)p_DW * p_DH;
    uint8_t* const d0 = reinterpret_cast<uint8_t*>(P.dst) + (size_t)(P.slot_offset + it.index * P.slot_stride) * 3 * plane * esz;
    uint8_t* const d1 = d0 + plane * esz;
    uint8_t* const d2 = d1 + plane * esz;
    const __amdgpu_buffer_rsrc_t rsO0 = __builtin_amdgcn_make_buffer_rsrc((void*)(k_rgb ? d2 : d0), (short)0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsO1 = __builtin_amdgcn_make_buffer_rsrc((void*)d1, (short)0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsO2 = __builtin_amdgcn_make_buffer_rsrc((void*)(k_rgb ? d0 : d2), (short)0, 0x7FFFFFFF, 0x00020000);
    const uint32_t fq0 = P.fill & 0xFF, fq1 = (P.fill >> 8) & 0xFF, fq2 = (P.fill >> 16) & 0xFF;
    const uint32_t fsh = OUT == 1 ? 2 : 0;
    const uint32_t fill0 = (k_rgb ? fq2 : fq0) << fsh, fill1 = fq1 << fsh, fill2 = (k_rgb ? fq0 : fq2) << fsh;
    const uint8_t* lutb = reinterpret_cast<const uint8_t*>(lut_s);
    // one row of the strip: v[c][j] = LUT byte offsets (fp32) or bytes (u8) in source channel order; the
    // row offset in the VGPR offset (soffset 0: the store-data hazard of wide stores, see evam_pp_wave)
    auto put = [&](int Y, const uint32_t (&v)[3][PX]) {
        if (!xin) return;
        const uint32_t off = vo + (uint32_t)(Y * p_DW) * (uint32_t)esz;
        store_off<OUT, PX>(rsO0, off, lutb, v[0]);
        store_off<OUT, PX>(rsO1, off, lutb + 1024, v[1]);
        store_off<OUT, PX>(rsO2, off, lutb + 2048, v[2]);
    };
    auto put_fill = [&](int Y) {
        uint32_t v[3][PX];
#pragma unroll
        for (int j = 0; j < PX; j++) { v[0][j] = fill0; v[1][j] = fill1; v[2][j] = fill2; }
        put(Y, v);
    };
    for (int Y = Y0; Y < (n ? vr0 : Y1); Y++) {  // letterbox rows above
        put_fill(Y);
        pos += 3;
    }

    uint32_t kb = kKBs, kg = kKGs, kr = kKRs;
    int cvg = kCVG, cug = kCUG;
    asm volatile("" : "+v"(kb), "+v"(kg), "+v"(kr), "+s"(cvg), "+s"(cug));
    auto uvt = [&](uint32_t U, uint32_t V) {
        int gu = __mul24((int)U, cug) + (int)kg;
        asm("" : "+v"(gu));
        return UVs{__umul24(U, (uint32_t)kCUB) + kb, (uint32_t)(__mul24((int)V, cvg) + gu), __umul24(V, (uint32_t)kCVR) + kr};
    };
    // chroma terms of the chroma row cc for both taps of every pixel (kept across source rows)
    UVs tA[PX], tB[PX];
    int cc = -1;
    auto chroma_row = [&](int c) {
        const uint8_t* cb = cbuf + (c - clo) * segC;
        cc = c;
        if constexpr (DD) {  // the chroma columns of (c0, c1), (c2, c3), (c4, c5) in tA[0..2]
            const uint32_t o[3] = {lC[0] & 0xFFFF, lC[1] >> 16, lC[2] >> 16};
#pragma unroll
            for (int k = 0; k < 3; k++) {
                const uint8_t* a = cb + o[k];
                tA[k] = uvt(a[0], FMT == kNV12 ? a[1] : a[segC / 2]);
            }
            return;
        }
#pragma unroll
        for (int j = 0; j < PX; j++) {
            const uint8_t* a0 = cb + (lC[j] & 0xFFFF);
            const uint8_t* a1 = cb + (lC[j] >> 16);
            if constexpr (FMT == kNV12) {
                tA[j] = uvt(a0[0], a0[1]);
                tB[j] = uvt(a1[0], a1[1]);
            } else {
                tA[j] = uvt(a0[0], a0[segC / 2]);
                tB[j] = uvt(a1[0], a1[segC / 2]);
            }
        }
    };
    // A source row's 3 PX filtered values travel as 64-bit register pairs (value k of pixel j at flat index
    // 3 j + k), so the HA <- HB copy of a one-row step is one v_pk_mov_b32 per two values.
    constexpr int NH = (3 * PX + 1) / 2;
    struct HRow { uint64_t p[NH]; };
    auto hget = [](const HRow& h, int j, int k) -> uint32_t {
        const int f = 3 * j + k;
        return (uint32_t)(h.p[f >> 1] >> (32 * (f & 1)));
    };
    auto hpack = [](HRow& h, const uint32_t (&H)[PX][3]) {
#pragma unroll
        for (int i = 0; i < NH; i++) {
            const int f0 = 2 * i, f1 = 2 * i + 1;
            const uint32_t lo = H[f0 / 3][f0 % 3], hi = f1 < 3 * PX ? H[f1 / 3][f1 % 3] : 0u;
            h.p[i] = (uint64_t)lo | ((uint64_t)hi << 32);
        }
    };
    // horizontal pass of source row r (crop-relative) into HR
    auto hrow = [&](int r, HRow& HR) {
        uint32_t H[PX][3];
        const int c = (y0 + r) >> 1;
        if (c != cc) chroma_row(c);
        const uint8_t* yb = wbuf + (r - rlo) * segY;
        if constexpr (DD) {  // columns c0..c5: pixel 0 (c0, c1), 1 (c1, c2), 2 (c3, c4), 3 (c4, c5)
            const uint32_t yl[6] = {luma_term(yb[lY[0] & 0xFFFF]), luma_term(yb[lY[0] >> 16]), luma_term(yb[lY[1] >> 16]),
                                    luma_term(yb[lY[2] & 0xFFFF]), luma_term(yb[lY[2] >> 16]), luma_term(yb[lY[3] >> 16])};
#pragma unroll
            for (int ch3 = 0; ch3 < 3; ch3++) {
                uint32_t sm[6];
#pragma unroll
                for (int k = 0; k < 6; k++) {
                    const UVs& t = tA[k >> 1];
                    sm[k] = __builtin_elementwise_add_sat(yl[k], ch3 == 0 ? t.b : (ch3 == 1 ? t.g : t.r));
                }
                H[0][ch3] = hpass_sums(sm[0], sm[1], wp[0]) & kVMask;
                H[1][ch3] = hpass_sums(sm[1], sm[2], wp[1]) & kVMask;
                H[2][ch3] = hpass_sums(sm[3], sm[4], wp[2]) & kVMask;
                H[3][ch3] = hpass_sums(sm[4], sm[5], wp[3]) & kVMask;
            }
            hpack(HR, H);
            return;
        }
#pragma unroll
        for (int j = 0; j < PX; j++) {
            const uint32_t yA = luma_term(yb[lY[j] & 0xFFFF]), yB = luma_term(yb[lY[j] >> 16]);
            // masked once per source row here rather than per output row in vfinal (each row serves ~2.4 output rows)
            H[j][0] = hpass_sat(yA, tA[j].b, yB, tB[j].b, wp[j]) & kVMask;
            H[j][1] = hpass_sat(yA, tA[j].g, yB, tB[j].g, wp[j]) & kVMask;
            H[j][2] = hpass_sat(yA, tA[j].r, yB, tB[j].r, wp[j]) & kVMask;
        }
        hpack(HR, H);
    };
    HRow HA, HB;
    int pa = -1, pb = -1;
    const int nst = 3;  // stores per output row (one PX-wide store per channel)
    // progress-based priority (EVAM_PP_PRIO), as in the strip kernel
    ProgressPrio prio(P.prio != 0, n);
    for (int i = 0; i < n; i++) {
        prio.step(i);
        const int ra = __builtin_amdgcn_readlane(lr0, i), rb = __builtin_amdgcn_readlane(lr1, i);
        issue_to(rb);  // (issued already unless `ahead` is 0)
        vmcnt_le(pos - __builtin_amdgcn_readlane(dpos, rb - rlo));  // rows up to rb landed
#ifdef EVAM_PP_TRACE
        if (i == 0) {
            EVAM_WSTAMP(2);
            EVAM_WSTAMP(3);
        }
#endif
        const uint32_t wb0 = (uint32_t)__builtin_amdgcn_readlane(lb0, i), wb1 = (uint32_t)__builtin_amdgcn_readlane(lb1, i);
        if (kAblate & 2) {  // diagnostics: no pixel math (no tap reads), stores and DMA kept
            put_fill(vr0 + i);
            pos += nst;
            asm volatile("" ::: "memory");
            if (i + 1 < n) issue_to(min(rhi, __builtin_amdgcn_readlane(lr1, i + 1) + ahead));
            asm volatile("" ::: "memory");
            continue;
        }
        // HA <- row ra, HB <- row rb, reusing what the previous output row filtered (wave-uniform branches)
        if (ra != pa) {
            if (ra == pb) {
                HA = HB;
            } else {
                hrow(ra, HA);
            }
        }
        if (rb == ra) {
            HB = HA;
        } else if (rb != pb || ra == pb) {  // HB was overwritten into HA above, or holds another row
            hrow(rb, HB);
        }
        pa = ra;
        pb = rb;
        uint32_t v[3][PX];
#pragma unroll
        for (int j = 0; j < PX; j++)
#pragma unroll
            for (int c = 0; c < 3; c++) v[c][j] = vfinal_masked<OUT>(hget(HA, j, c), hget(HB, j, c), wb0, wb1);
        if constexpr (OUT == 0 && PX == 4) {  // u8, 4 pixels per lane: the sums packed by pack4_u8_sums
            uint32_t x[3][4];
#pragma unroll
            for (int j = 0; j < 4; j++)
#pragma unroll
                for (int c = 0; c < 3; c++) x[c][j] = mulhi_u24(wb0, hget(HA, j, c)) + mulhi_u24(wb1, hget(HB, j, c)) + 2u;
            if (anypad) {  // padding columns: the fill byte as a sum (x >> 2 == fill)
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    x[0][j] = padc[j] ? fill0 << 2 : x[0][j];
                    x[1][j] = padc[j] ? fill1 << 2 : x[1][j];
                    x[2][j] = padc[j] ? fill2 << 2 : x[2][j];
                }
            }
            if (xin) {
                const uint32_t off = vo + (uint32_t)((vr0 + i) * p_DW);
                __builtin_amdgcn_raw_buffer_store_b32(pack4_u8_sums(x[0][0], x[0][1], x[0][2], x[0][3]), rsO0, off, 0,
                                                      EVAM_PP_STORE_AUX);
                __builtin_amdgcn_raw_buffer_store_b32(pack4_u8_sums(x[1][0], x[1][1], x[1][2], x[1][3]), rsO1, off, 0,
                                                      EVAM_PP_STORE_AUX);
                __builtin_amdgcn_raw_buffer_store_b32(pack4_u8_sums(x[2][0], x[2][1], x[2][2], x[2][3]), rsO2, off, 0,
                                                      EVAM_PP_STORE_AUX);
            }
            pos += nst;
            asm volatile("" ::: "memory");  // issue order is what the counted waits assume
            if (i + 1 < n) issue_to(min(rhi, __builtin_amdgcn_readlane(lr1, i + 1) + ahead));
            asm volatile("" ::: "memory");
            continue;
        }
        if (anypad) {
#pragma unroll
            for (int j = 0; j < PX; j++) {
                v[0][j] = padc[j] ? fill0 : v[0][j];
                v[1][j] = padc[j] ? fill1 : v[1][j];
                v[2][j] = padc[j] ? fill2 : v[2][j];
            }
        }
        put(vr0 + i, v);
        pos += nst;
        asm volatile("" ::: "memory");  // issue order is what the counted waits assume
        if (i + 1 < n) issue_to(min(rhi, __builtin_amdgcn_readlane(lr1, i + 1) + ahead));
        asm volatile("" ::: "memory");
    }
    for (int Y = max(n ? vr1 : Y1, Y0); Y < Y1; Y++) put_fill(Y);  // letterbox rows below
#ifdef EVAM_PP_TRACE
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    EVAM_WSTAMP(4);
    {
        unsigned xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        EVAM_WTRACE_VAL(6, (unsigned long long)xcc);
    }
#endif
}


#ifndef EVAM_PP_ROI_K
#define EVAM_PP_ROI_K 6
#endif
constexpr int kRoiK = EVAM_PP_ROI_K;  // max pixels per lane per row group in the ROI kernel

struct QParams {
    const RoiRec* recs;       // this launch's ROI tiles in launch order (largest work first)
    const float* lut;         // [3][256]
    void* dst;
    int DW, DH;
    int TH;                   // most output rows of one tile (the LDS row table's size)
    int mode, placement;      // evam_resize_mode, evam_placement
    int slot_offset, slot_stride;
    int offXT, offYT, offBuf; // LDS carve: [LUT][XTab x DW][YTab x TH][buf0][buf1]
    int buf_bytes;            // one staging buffer
    int color_rgb;
    uint32_t fill;
    int prio;                 // progress-based priority (as the strip kernel's), over the quarters of the row groups
    uint32_t mqw;             // q / QW as mulhi(q, mqw) for the lane quads (QW = DW / PX > 1): ceil(2^32 / QW)
};


template <int N>
__device__ __forceinline__ void wait_vmcnt_stores(int nk) {
    // s_waitcnt takes an immediate: vmcnt(N * nk) for the wave-uniform store-step count nk.
    switch (nk) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * N) : "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(%0)" :: "n"(3 * N) : "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(%0)" :: "n"(4 * N) : "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(%0)" :: "n"(5 * N) : "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(%0)" :: "n"(6 * N) : "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(%0)" :: "n"(7 * N) : "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(%0)" :: "n"(8 * N) : "memory"); break;
    }
}

// Staged kernel for batches whose items differ in geometry (gvaclassify ROI batches, mixed crops).
// The host passes the caller's raw ROI array; each workgroup resolves its item's crop, resized size
// and placement on the device (roi_geometry, the host's own rules) and owns all DW columns x TH rows
// of that item:
//  * OpenCV coefficient tables for its columns / rows are built in LDS (exact double/float sequence);
//  * rows are walked in groups whose size R adapts to the item: as many output rows as the staging
//    buffer holds for this crop's width (narrow crops: many rows per group, few barriers), capped so
//    the R x DW pixels cover the 256 lanes at most kRoiK times;
//  * a group's source row segments (luma taps and chroma taps, each exactly the item's footprint)
//    are packed back to back in LDS and arrive by LDS-DMA while the previous group is converted;
//  * the group's R x DW output pixels are packed densely onto the lanes (pixel p = tid + 256 k), so a
//    72-wide classifier row keeps every lane busy and every store is row-contiguous.
// 7 resident workgroups per CU need <= 96 SGPRs (800 / (96 + 16)); the occupancy API does not count
// SGPRs (MI355X_MICROARCH.md, Residency): uncapped, the kernel's ~106 allowed only 6 and a 1,600-ROI
// batch ran a second round (profiles/r02r_c3_roi_timeline_before.json).
template <int FMT, int OUT, int PX, int NB>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_num_sgpr(96))) void evam_pp_roi(const QParams P) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    static_assert(NB == 2, "two staging buffers (three were retired in round 5)");
    using T = FmtTraits<FMT>;
    constexpr bool kYUV = FMT == kNV12 || FMT == kI420;
    constexpr int NP = FMT == kI420 ? 3 : (FMT == kNV12 ? 2 : 1);

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // the parameters of the prologue in one batch of scalar loads, so the record's PCIe read below is not
    // queued behind a kernarg round trip for the diagnostics test
    asm volatile("" ::"s"(P.recs), "s"(P.lut), "s"(P.color_rgb), "s"(P.mode), "s"(P.placement),
                 "s"(P.DW), "s"(P.DH));
    if (kAblate & 128) return;  // diagnostics: launch cost only
    EVAM_STAMP(0);
    // The whole 64-byte record in one scalar load, issued first (field-by-field loads became up to three
    // dependent round trips per wave). The record slot is device memory the host wrote through its BAR
    // mapping (PinRing, HipRings::pinned_alloc), or pinned host memory read over PCIe where the platform does
    // not map device memory (~1-2 us more under load). Its latency overlaps the LUT load below.
    typedef unsigned int u32x16 __attribute__((ext_vector_type(16)));
    const u32x16 rec = *((const __attribute__((address_space(4))) u32x16*)(P.recs) + blockIdx.x);
    // The LUT by LDS-DMA, issued first: no VGPR waits on it, and group 0's wait (everything older than its
    // DMA) covers it. Loaded into registers and stored it held the row-table barrier, and so the first DMA,
    // up to ~15 us for the last workgroups behind the chip's first DMA burst (profiles/r03l_c3_roi_timeline.json).
    // Sections in source channel order (B, G, R): RGB output swaps the B / R output planes instead of the
    // values (see rsD0 / rsD2), so the per-pixel path carries no swap.
    float* lut_s = reinterpret_cast<float*>(smem);
    if constexpr (OUT == 1) {
        const int c0 = wave * 48, c = c0 + lane, sec = c >> 6;  // 192 chunks of 16 B: 48 per wave
        const __amdgpu_buffer_rsrc_t rsL = __builtin_amdgcn_make_buffer_rsrc((void*)P.lut, (short)0, 3072, 0x00020000);
        if (lane < 48)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsL, (__attribute__((address_space(3))) void*)(smem + c0 * 16), 16,
                                                     (uint32_t)(((P.color_rgb ? 2 - sec : sec) * 64 + (c & 63)) * 16), 0, 0, 0);
    }
    // RoiRec as dwords: plane[0..2] 0-5, pitch[0..2] 6-8, width | height << 16 9, x y w h 10-13, item 14,
    // row0 | row1 << 16 15
    static_assert(offsetof(RoiRec, pitch) == 24 && offsetof(RoiRec, width) == 36 && offsetof(RoiRec, x) == 40 &&
                  offsetof(RoiRec, item) == 56 && offsetof(RoiRec, row0) == 60, "RoiRec dword map");
    auto ptr_of = [](unsigned lo, unsigned hi) {
        return reinterpret_cast<const uint8_t*>(((uint64_t)hi << 32) | lo);
    };
    const int item = (int)rec[14];
    const uint32_t wh = rec[9];
    const uint32_t rr01 = rec[15];
    const int fw = wh & 0xFFFF, fh = wh >> 16;
    const int rx = (int)rec[10], ry = (int)rec[11], rwd = (int)rec[12], rht = (int)rec[13];
    const uint8_t* p0 = ptr_of(rec[0], rec[1]);
    const uint8_t* p1 = ptr_of(rec[2], rec[3]);
    const uint8_t* p2 = ptr_of(rec[4], rec[5]);
    const int pitch0 = (int)rec[6], pitch1 = (int)rec[7], pitch2 = (int)rec[8];
    Geom g;
    roi_geometry(FMT, fw, fh, true, rx, ry, rwd, rht, P.mode, P.placement, P.DW, P.DH,
                 g);  // never empty: the host validated every item
    const int x0 = __builtin_amdgcn_readfirstlane(g.x0), y0 = __builtin_amdgcn_readfirstlane(g.y0);
    const int cw = __builtin_amdgcn_readfirstlane(g.cw), ch = __builtin_amdgcn_readfirstlane(g.ch);
    const int rw = __builtin_amdgcn_readfirstlane(g.rw), rh = __builtin_amdgcn_readfirstlane(g.rh);
    const int ox = __builtin_amdgcn_readfirstlane(g.ox), oy = __builtin_amdgcn_readfirstlane(g.oy);
    EVAM_STAMP(1);
    // diagnostics: stop after the geometry (64) / after the per-lane setup (32)
    if ((kAblate & 64) && rw != -7) return;
    const double scx = 1. / ((double)rw / cw), scy = 1. / ((double)rh / ch);
    const size_t plane = (size_t)P.DW * P.DH;
    const size_t esz = OUT == 1 ? 4 : 1;
    const int slot = P.slot_offset + item * P.slot_stride;
    uint8_t* const d0 = reinterpret_cast<uint8_t*>(P.dst) + (size_t)slot * 3 * plane * esz;
    uint8_t* const d1 = d0 + plane * esz;
    uint8_t* const d2 = d1 + plane * esz;
    const __amdgpu_buffer_rsrc_t rsY = __builtin_amdgcn_make_buffer_rsrc((void*)p0, (short)0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsC = __builtin_amdgcn_make_buffer_rsrc((void*)(p1 ? p1 : p0), (short)0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsV = __builtin_amdgcn_make_buffer_rsrc((void*)(p2 ? p2 : p0), (short)0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsD0 = __builtin_amdgcn_make_buffer_rsrc((void*)(P.color_rgb ? d2 : d0), (short)0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsD1 = __builtin_amdgcn_make_buffer_rsrc((void*)d1, (short)0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsD2 = __builtin_amdgcn_make_buffer_rsrc((void*)(P.color_rgb ? d0 : d2), (short)0, 0x7FFFFFFF, 0x00020000);

    // Prologue order: the row table is built first; group 0's DMA (it needs only the row table and the
    // analytic footprint) goes out before the column table and the per-lane setup are built, so its
    // latency overlaps them. The column table holds each column's packed tap offsets into the staged rows and
    // weights (lY, lC, wa: what every lane reading the column needs), so the per-lane setup is table reads.
    uint4* ct = reinterpret_cast<uint4*>(smem + P.offXT);
    YTab* yt = reinterpret_cast<YTab*>(smem + P.offYT);
    const int DW = P.DW;
    const int Y0 = __builtin_amdgcn_readfirstlane(rr01 & 0xFFFF), Y1 = __builtin_amdgcn_readfirstlane(rr01 >> 16);
    const int rows = Y1 - Y0;
    for (int ly = tid; ly < rows; ly += kThreads) {
        YTab e;
        e.r0 = 0; e.r1 = 0; e.b0 = 0; e.b1 = 0;
        const int dy = Y0 + ly - oy;
        if (dy >= 0 && dy < rh) {
            int sy, b0, b1;
            linear_coef(dy, scy, ch, false, sy, b0, b1);
            e.r0 = min(max(sy, 0), ch - 1);
            e.r1 = min(max(sy + 1, 0), ch - 1);
            e.b0 = b0 << 8;
            e.b1 = b1 << 8;
        }
        yt[ly] = e;
    }
    int fsY, nY, fsC, nC;
    item_footprint(FMT, T::bpp, x0, cw, rw, ox, scx, DW, fsY, nY, fsC, nC);
    fsY = __builtin_amdgcn_readfirstlane(fsY);
    nY = __builtin_amdgcn_readfirstlane(nY);
    fsC = __builtin_amdgcn_readfirstlane(fsC);
    nC = __builtin_amdgcn_readfirstlane(nC);
    // Staging buffer layout for a group of R output rows, one plane region after the other:
    //   Y: segment (2 r + tap) at (2 r + tap) * segY;   C (U / UV): at offC + (2 r + tap) * segC;
    //   V (I420): at offC + 2 R segC + (2 r + tap) * segC.
    // Each plane region is contiguous, so its 16-byte chunks are staged by wave-wide LDS-DMA with one
    // per-lane source offset each: 64 chunks (of any rows and taps) per instruction.
    const int segY = nY * 16, segC = nC * 16;
    const int rowb = 2 * segY + 2 * (NP - 1) * segC;
    // Lanes own runs of PX adjacent pixels of one row (DW % PX == 0, host): a "quad" q of the
    // group's R x QW quads covers row q / QW, columns PX * (q % QW) ...
    constexpr int KQ = kRoiK / PX;                // max quads per lane per group
    const int QW = DW / PX;
    int R = rowb > 0 ? P.buf_bytes / rowb : rows;
    R = min(R, (KQ * kThreads) / QW);
    R = max(1, min(R, rows));
    const int offC = 2 * R * segY;
    const int nq = R * QW;                        // quads per full group
    const int K = (nq + kThreads - 1) / kThreads;
    // store steps this wave issues in a full group: k with some lane of the wave holding a quad
    int nk_w = 0;
    for (int k = 0; k < K; k++) nk_w += (k * kThreads + wave * 64 < nq) ? 1 : 0;
    // q / n for q < 2^16 by one mul_hi: m = ceil(2^32 / n) is exact there (n = 1: the identity).
    const uint32_t mY = nY > 1 ? (uint32_t)((0x100000000ull + nY - 1) / nY) : 0u;
    const uint32_t mC = nC > 1 ? (uint32_t)((0x100000000ull + nC - 1) / nC) : 0u;
    // Row table visible: LDS writes only (lgkmcnt) and a raw barrier. __syncthreads() would add vmcnt(0) and
    // hold every wave until the LUT's LDS-DMA landed; group 0's wait below covers the LUT instead.
    lds_barrier();
    EVAM_STAMP(8);
    // One plane region of group grp: chunk q -> (segment, chunk) -> (row, tap) -> source offset.
    // Returns the number of DMA instructions this wave issued (wave-uniform: an instruction with no active
    // lane is skipped), for the counted waits of the three-buffer pipeline.
    auto issue_plane = [&](int grp, uint8_t* base, int nr, int n, uint32_t m, int pl) -> int {
        const int nq = 2 * nr * n;
        int cnt = 0;
        for (int q0 = wave * 64; q0 < nq; q0 += 4 * 64) {
            const int q = q0 + lane;
            const int seg = n > 1 ? (int)__umulhi((uint32_t)q, m) : q;
            const int c = q - seg * n;
            const int r = seg >> 1, tap = seg & 1;
            const YTab e = yt[min(grp * R + r, rows - 1)];
            const int ya = y0 + e.r0, yb = y0 + e.r1;
            bool on = q < nq && (e.b0 | e.b1) != 0;           // padding rows stage nothing
            if (pl > 0) on = on && !(tap && (ya >> 1) == (yb >> 1));  // chroma row shared by both taps
            __attribute__((address_space(3))) void* dstl = (__attribute__((address_space(3))) void*)(base + q0 * 16);
            if (on) {
                const int yr = tap ? yb : ya;
                if (pl == 0)
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsY, dstl, 16, yr * pitch0 + fsY + c * 16, 0, EVAM_PP_LOAD_AUX, 0);
                else if (pl == 1)
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsC, dstl, 16, (yr >> 1) * pitch1 + fsC + c * 16, 0, EVAM_PP_LOAD_AUX, 0);
                else
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsV, dstl, 16, (yr >> 1) * pitch2 + fsC + c * 16, 0, EVAM_PP_LOAD_AUX, 0);
            }
        }
        return cnt;
    };
    auto issue = [&](int grp, uint8_t* buf) -> int {
        if (nY == 0 || (kAblate & 16)) return 0;  // no visible columns: every pixel is fill
        const int nr = min(R, rows - grp * R);
        int cnt = issue_plane(grp, buf, nr, nY, mY, 0);
        if constexpr (NP >= 2) cnt += issue_plane(grp, buf + offC, nr, nC, mC, 1);
        if constexpr (NP >= 3) cnt += issue_plane(grp, buf + offC + 2 * R * segC, nr, nC, mC, 2);
        return __builtin_amdgcn_readfirstlane(cnt);
    };
    uint8_t* const buf0 = smem + P.offBuf;
    uint8_t* const buf1 = buf0 + P.buf_bytes;
    issue(0, buf0);
    static_assert(sizeof(uint4) == sizeof(XTab), "column entries take the host's XTab carve");
    for (int X = tid; X < DW; X += kThreads) {
        uint4 e = {0u, 0u, 0u, 0u};  // (lY, lC, wa, 0); all 0: padding column
        const int dx = X - ox;
        if (dx >= 0 && dx < rw) {
            int sx, a0, a1;
            linear_coef(dx, scx, cw, true, sx, a0, a1);
            const int ca = x0 + sx, cb = x0 + min(sx + 1, cw - 1);
            e.x = (uint32_t)(ca * T::bpp - fsY) | ((uint32_t)(cb * T::bpp - fsY) << 16);
            if constexpr (FMT == kNV12)
                e.y = (uint32_t)(2 * (ca >> 1) - fsC) | ((uint32_t)(2 * (cb >> 1) - fsC) << 16);
            else if constexpr (FMT == kI420)
                e.y = (uint32_t)((ca >> 1) - fsC) | ((uint32_t)((cb >> 1) - fsC) << 16);
            e.z = ((uint32_t)a0 << 4) | ((uint32_t)a1 << 20);
        }
        ct[X] = e;
    }
    lds_barrier();  // column table visible to the per-lane setup; group 0's DMA stays in flight
    EVAM_STAMP(9);
    // fill in source channel order (P.fill is in output plane order); fp32: LUT byte offsets
    const uint32_t fsh = OUT == 1 ? 2 : 0;
    const uint32_t fq0 = P.fill & 0xFF, fq1 = (P.fill >> 8) & 0xFF, fq2 = (P.fill >> 16) & 0xFF;
    const uint32_t f0 = (P.color_rgb ? fq2 : fq0) << fsh, f1 = fq1 << fsh, f2 = (P.color_rgb ? fq0 : fq2) << fsh;
    // Per-lane state for quad steps k < K, identical for every group: row of the quad inside the
    // group; per pixel packed LDS tap offsets (tap 0 low, tap 1 high half) and horizontal weights.
    uint32_t lY[KQ][PX], lC[KQ][PX], wa[KQ][PX];
    int rr[KQ];
#pragma unroll
    for (int k = 0; k < KQ; k++) {
        const uint32_t q = (uint32_t)(tid + k * kThreads);  // < 2^16: mulhi by ceil(2^32 / QW) is q / QW exactly
        const bool v = k < K && (int)q < nq;
        const int r = v ? (QW > 1 ? (int)__umulhi(q, P.mqw) : (int)q) : 0;
        const int c0 = v ? ((int)q - r * QW) * PX : 0;
        rr[k] = v ? r : -1;
#pragma unroll
        for (int j = 0; j < PX; j++) {
            const uint4 e = ct[c0 + j];
            lY[k][j] = e.x;
            lC[k][j] = e.y;
            wa[k][j] = e.z;
        }
    }
    const int ngroups = (rows + R - 1) / R;
#ifdef EVAM_PP_TRACE
    {
        EVAM_STAMP(2);
        unsigned xcc, hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        EVAM_TRACE_VAL(4, (unsigned long long)cw | ((unsigned long long)ch << 32));
        EVAM_TRACE_VAL(5, (unsigned long long)ngroups | ((unsigned long long)R << 32));
        EVAM_TRACE_VAL(6, (unsigned long long)xcc | ((unsigned long long)hw << 32));
    }
#endif
    if ((kAblate & 32) && ngroups != -7) {
        asm volatile("" :: "v"(lY[0][0]), "v"(lC[0][0]), "v"(wa[0][0]), "v"(rr[0]), "s"(mY), "s"(mC));
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // group 0's DMA lands before the LDS is released
        return;
    }

    auto compute = [&](int grp, const uint8_t* buf) {
        const uint32_t gbase = (uint32_t)((Y0 + grp * R) * DW);
#pragma unroll
        for (int k = 0; k < KQ; k++) {
            if (k >= K) break;
            const int ly = grp * R + rr[k];
            if (rr[k] < 0 || ly >= rows) continue;
            const YTab e = yt[ly];
            const bool padrow = (e.b0 | e.b1) == 0 || (kAblate & 2);  // letterbox padding row
            const uint8_t* sy0 = buf + 2 * rr[k] * segY;
            const uint8_t* sy1 = sy0 + segY;
            const uint8_t* sc0 = buf + offC + 2 * rr[k] * segC;
            const uint8_t* sc1 = sc0;
            if constexpr (kYUV) {
                const int ya = y0 + e.r0, yb = y0 + e.r1;
                sc1 = (ya >> 1) == (yb >> 1) ? sc0 : sc0 + segC;
            }
            const uint32_t wb0 = (uint32_t)e.b0, wb1 = (uint32_t)e.b1;
            uint32_t v[3][PX];  // source channel c (B, G, R); fp32: 4 x value, the LUT byte offset
#pragma unroll
            for (int j = 0; j < PX; j++) {
                if (padrow || wa[k][j] == 0) {  // padding row / column
                    v[0][j] = f0; v[1][j] = f1; v[2][j] = f2;
                    continue;
                }
                const uint32_t a0 = wa[k][j] & 0xFFFF, a1 = wa[k][j] >> 16;
                const uint32_t tY0 = lY[k][j] & 0xFFFF, tY1 = lY[k][j] >> 16;
                int c[4][3];
                if constexpr (kYUV) {
                    const uint32_t tC0 = lC[k][j] & 0xFFFF, tC1 = lC[k][j] >> 16;
                    const uint8_t* sv0 = FMT == kNV12 ? sc0 + 1 : sc0 + 2 * R * segC;
                    const uint8_t* sv1 = FMT == kNV12 ? sc1 + 1 : sc1 + 2 * R * segC;
                    const uint32_t wp = (wa[k][j] >> 4) & 0x0FFF0FFFu;
                    uint32_t H0[3], H1[3];
                    hrow_sat(sy0[tY0], sy0[tY1], uv_terms_sat(sc0[tC0], sv0[tC0]), uv_terms_sat(sc0[tC1], sv0[tC1]), wp, H0);
                    hrow_sat(sy1[tY0], sy1[tY1], uv_terms_sat(sc1[tC0], sv1[tC0]), uv_terms_sat(sc1[tC1], sv1[tC1]), wp, H1);
#pragma unroll
                    for (int ch3 = 0; ch3 < 3; ch3++) v[ch3][j] = vfinal<OUT>(H0[ch3], H1[ch3], wb0, wb1);
                    continue;
                }
                {  // packed sources (BGRx / BGR)
                    const uint8_t* tap[4] = {sy0 + tY0, sy0 + tY1, sy1 + tY0, sy1 + tY1};
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        if constexpr (FMT == kBGRX) {
                            const uint32_t px = *reinterpret_cast<const uint32_t*>(tap[q]);
                            c[q][0] = px & 0xFF; c[q][1] = (px >> 8) & 0xFF; c[q][2] = (px >> 16) & 0xFF;
                        } else {
                            c[q][0] = tap[q][0]; c[q][1] = tap[q][1]; c[q][2] = tap[q][2];
                        }
                    }
                }
#pragma unroll
                for (int ch3 = 0; ch3 < 3; ch3++) {
                    const uint32_t D0 = __umul24(c[0][ch3], a0) + __umul24(c[1][ch3], a1);
                    const uint32_t D1 = __umul24(c[2][ch3], a0) + __umul24(c[3][ch3], a1);
                    v[ch3][j] = vfinal<OUT>(D0, D1, wb0, wb1);
                }
            }
            // soffset 0: the row offset is in voffset (a > 8-byte store with an SGPR soffset misses
            // the compiler's store-data hazard wait on gfx950, see evam_pp_wave)
            const uint32_t vo = (gbase + (uint32_t)(tid + k * kThreads) * PX) * (uint32_t)esz;
            if (kAblate & 4) {
                asm volatile("" :: "v"(v[0][0]), "v"(v[1][0]), "v"(v[2][0]));
                continue;
            }
            const uint8_t* lb = reinterpret_cast<const uint8_t*>(lut_s);
            store_off<OUT, PX>(rsD0, vo, lb, v[0]);
            store_off<OUT, PX>(rsD1, vo, lb + 1024, v[1]);
            store_off<OUT, PX>(rsD2, vo, lb + 2048, v[2]);
        }
    };


    // progress-based priority (EVAM_PP_PRIO): 3 -> 0 over the quarters of the workgroup's row groups
    ProgressPrio prio(P.prio != 0, ngroups);
    for (int grp = 0; grp < ngroups; grp++) {
        prio.step(grp);
        // Wait for this wave's share of group grp's DMA. Group grp-1 was full (only the last group can
        // be partial), so this wave issued at least 3 stores for each of its nk_w store steps after
        // that DMA: those may stay in flight.
        if (grp > 0) wait_vmcnt_stores<3>(nk_w);
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // every wave's DMA for grp landed; every wave done reading grp-1
        if (grp == 0) EVAM_STAMP(10);
        if (grp + 1 < ngroups) issue(grp + 1, (grp & 1) ? buf0 : buf1);
        asm volatile("" ::: "memory");  // the next group's DMA stays ahead of this group's stores
        compute(grp, (grp & 1) ? buf1 : buf0);
        asm volatile("" ::: "memory");
    }
    EVAM_STAMP(3);
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


int item_geometry(int f, int W, int H, const evam_roi* roi, const evam_preproc& cfg, int DW, int DH, Geom& g) {
    return roi_geometry(f, W, H, roi != nullptr, roi ? roi->x : 0, roi ? roi->y : 0, roi ? roi->w : 0,
                        roi ? roi->h : 0, cfg.resize_mode, cfg.placement, DW, DH, g);
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


struct TileCfg {
    int TW, TH, offCol, offRow, lds;
};

int env_int(const char* name, int dflt) {
    const char* v = getenv(name);
    return (v && *v) ? atoi(v) : dflt;
}

// Tuning and diagnostic knobs. Read from the environment once, when a handle is
// created (evam_pp_create), never on the per-call path. -1 = the measured heuristic default.
struct Knobs {
    int staged = 1, wave = 1, rows = 1, roi = 1;   // kernel families allowed (wave 2 = force)
    int th = -1, tw = -1, xcd = -1;                // staged / generic tiles, XCD-contiguous order
    int nsegx = 0;                                 // staged tile width in 64-column segments (0: widest that fits)
    int stage_r = -1;                              // staged pipeline: rows per group
    int wth = -1, px = 0, reuse = 1, wave_lds = 40 * 1024;
    int roi_th = -1, roi_buf = -1, roi_px = 2;     // roi_buf -1: sized for one round; pixels per lane (1 for odd DW)
    int roi_sort = 1;  // 1: largest estimated bytes first before the stable sort by row groups (alone: equal or
                       // slower, profiles/r04k_ab_lines.txt; with the snake deal below C3 +1.5-2 %,
                       // profiles/r05zf_c3_snake_ab.txt)
    int roi_tail = 4;                              // row tiles per ROI of the uneven tail over the CUs (1: no split)
    int roi_snake = 1;                             // snake deal of the sorted units over the CUs (0: bands in one direction)
    int roi_xcd = 0;                               // 1: each frame's ROIs on one XCD, snake-dealt over its CUs (experiment)
    int strip = 1, strip_th = -1, strip_nw = -1, strip_px = 0;  // strip kernel: allowed (2: forced), rows per
                                                                // tile, waves, px
    int strip_pair = 1;                            // strip kernel: paired-tap DMA where the footprints allow it
    int strip_waves = 16;                          // strip / band kernels: resident waves per CU the tiles are sized for
    int band = 1, band_px = 0;                     // band kernel: allowed (2: forced), pixels per lane
    int band_dd = 1;                               // band kernel: six-column lanes where the column table allows
    int rec_device = 1;                            // ROI records in host-written device memory where mapped (0: pinned host)
    int prio = 1;                                  // progress-based wave priority (strip, band, ROI kernels): C2 +3 %,
                                                   // C4 +3 %, C5 +3-5 %, C1 +9 % (profiles/r04k_ab_lines.txt)
    int band_ahead = 2;                            // band kernel: source rows issued ahead of the current output row's
                                                   // (64: the whole band at once; 2 measured +2 % on C1)
    int host_simd = 1;                             // ROI calls: pass 1 on AVX2 (0: scalar)
    void read() {
        host_simd = env_int("EVAM_PP_HOST_SIMD", host_simd);
        prio = env_int("EVAM_PP_PRIO", prio);
        band_ahead = env_int("EVAM_PP_BAND_AHEAD", band_ahead);
        band = env_int("EVAM_PP_BAND", band); band_px = env_int("EVAM_PP_BAND_PX", band_px);
        band_dd = env_int("EVAM_PP_BAND_DD", band_dd);
        rec_device = env_int("EVAM_PP_REC_DEVICE", rec_device);
        strip = env_int("EVAM_PP_STRIP", strip); strip_th = env_int("EVAM_PP_STRIP_TH", strip_th);
        strip_waves = env_int("EVAM_PP_STRIP_WAVES", strip_waves);
        strip_pair = env_int("EVAM_PP_STRIP_PAIR", strip_pair); strip_nw = env_int("EVAM_PP_STRIP_NW", strip_nw);
        strip_px = env_int("EVAM_PP_STRIP_PX", strip_px);
        staged = env_int("EVAM_PP_STAGED", staged); wave = env_int("EVAM_PP_WAVE", wave);
        rows = env_int("EVAM_PP_ROWS", rows); roi = env_int("EVAM_PP_ROI", roi);
        th = env_int("EVAM_PP_TH", th); tw = env_int("EVAM_PP_TW", tw); xcd = env_int("EVAM_PP_XCD", xcd);
        nsegx = env_int("EVAM_PP_NSEGX", nsegx);
        stage_r = env_int("EVAM_PP_STAGE_R", stage_r);
        wth = env_int("EVAM_PP_WTH", wth); px = env_int("EVAM_PP_PX", px);
        reuse = env_int("EVAM_PP_REUSE", reuse); wave_lds = env_int("EVAM_PP_WAVE_LDS", wave_lds);
        roi_th = env_int("EVAM_PP_ROI_TH", roi_th); roi_buf = env_int("EVAM_PP_ROI_BUF", roi_buf);
        roi_px = env_int("EVAM_PP_ROI_PX", roi_px); roi_sort = env_int("EVAM_PP_ROI_SORT", roi_sort);
        roi_tail = env_int("EVAM_PP_ROI_TAIL", roi_tail); roi_snake = env_int("EVAM_PP_ROI_SNAKE", roi_snake);
        roi_xcd = env_int("EVAM_PP_ROI_XCD", roi_xcd);
    }
};

// Tile shape: up to 512 columns (a whole model-input row when it fits) x enough rows for ~4096 output
// pixels per 256-thread workgroup, so the per-tile table setup is amortised over ~16 pixels per lane.
// EVAM_PP_TW / EVAM_PP_TH override (tuning).
TileCfg choose_tiles(int DW, int DH, int out_dtype, const Knobs& k) {
    TileCfg t{};
    t.TW = std::min(DW, 512);
    t.TH = std::max(1, std::min(DH, 4096 / t.TW));
    if (k.tw > 0) t.TW = std::max(1, std::min(DW, k.tw));
    if (k.th > 0) t.TH = std::max(1, std::min(DH, k.th));
    t.offCol = out_dtype == EVAM_DTYPE_F32 ? kLutBytes : 0;
    t.offRow = t.offCol + (int)sizeof(ColEntry) * t.TW;
    t.lds = t.offRow + (int)sizeof(RowEntry) * t.TH;
    return t;
}

struct TabCache {
    int key[8] = {-1, -1, -1, -1, -1, -1, -1, -1};
    std::vector<XTab> x;
    std::vector<YTab> y;
};

// OpenCV coefficient tables for the uniform-geometry kernel, indexed by output column / row of the
// DW x DH plane (padding columns / rows get zero weights). Cached: rebuilt only when the geometry changes.
void build_tables(const Geom& g, int DW, int DH, TabCache& c, XTab* xt, YTab* yt) {
    const int key[8] = {g.cw, g.ch, g.rw, g.rh, g.ox, g.oy, DW, DH};
    if (memcmp(key, c.key, sizeof(key)) != 0) {
        c.x.assign(DW, XTab{});
        c.y.assign(DH, YTab{});
        build_tables_into(g, DW, DH, c.x.data(), c.y.data());
        memcpy(c.key, key, sizeof(key));
    }
    memcpy(xt, c.x.data(), sizeof(XTab) * DW);
    memcpy(yt, c.y.data(), sizeof(YTab) * DH);
}

struct RowCfg {
    int TW, TH;
};

// Row-kernel tile: TW in {512, 256, 128, 64} (whole 64-pixel segments; 4 waves split them) chosen for
// the least padding lanes, and enough rows for ~4096 pixels per 256-thread workgroup.
RowCfg choose_row_tiles(int DW, int DH, const Knobs& k) {
    RowCfg r{512, 8};
    int best = 1 << 30;
    for (int tw : {512, 256, 128, 64}) {
        const int waste = ((DW + tw - 1) / tw) * tw - DW;
        if (waste < best) { best = waste; r.TW = tw; }
    }
    if (k.tw > 0) r.TW = k.tw;
    if (r.TW != 64 && r.TW != 128 && r.TW != 256 && r.TW != 512) r.TW = 512;
    r.TH = std::max(1, std::min(DH, k.th > 0 ? k.th : 4096 / r.TW));
    return r;
}

// Staged-kernel pipeline shapes: (output rows per group R, staging buffers NBUF). One variant per
// (format, dtype, column segments) is instantiated for each shape listed here.
struct StagedShape { int R, nbuf; };
// (Three staging buffers, 512-column tiles and 2 KB row slots measured neutral or slower for two rounds and were
// retired in round 5.)
constexpr StagedShape kStagedShapes[] = {{2, 2}, {1, 2}};

// Valid (column segments, rows per group): four waves split NSEGX x R evenly.
constexpr bool staged_valid(int nsegx, int R) { return nsegx > 4 ? R == 1 : (nsegx == 4 ? true : R % (4 / nsegx) == 0); }

template <int FMT, int OUT, int NSEGX, int R, int NBUF>
hipError_t launch_staged_t(const SParams& p, int grid, int lds, hipStream_t s) {
    if constexpr (staged_valid(NSEGX, R)) {
        if (lds > 64 * 1024) {
            hipError_t e = hipFuncSetAttribute((const void*)evam_pp_staged<FMT, OUT, R, NSEGX, NBUF>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, lds);
            if (e != hipSuccess) return e;
        }
        hipLaunchKernelGGL((evam_pp_staged<FMT, OUT, R, NSEGX, NBUF>), dim3(grid), dim3(kThreads), lds, s, p);
        return hipGetLastError();
    } else {
        return hipErrorInvalidValue;  // never selected: staged_plan() only returns compatible shapes
    }
}

template <int FMT, int OUT, int NSEGX>
hipError_t launch_staged_s(int R, int nbuf, const SParams& p, int grid, int lds, hipStream_t s) {
    (void)nbuf;
    if (R == 2) return launch_staged_t<FMT, OUT, NSEGX, 2, 2>(p, grid, lds, s);
    if (R == 1) return launch_staged_t<FMT, OUT, NSEGX, 1, 2>(p, grid, lds, s);
    return hipErrorInvalidValue;
}

template <int FMT, int OUT>
hipError_t launch_staged_n(int nsegx, int R, int nbuf, const SParams& p, int grid, int lds, hipStream_t s) {
    switch (nsegx) {
    case 4: return launch_staged_s<FMT, OUT, 4>(R, nbuf, p, grid, lds, s);
    case 2: return launch_staged_s<FMT, OUT, 2>(R, nbuf, p, grid, lds, s);
    default: return launch_staged_s<FMT, OUT, 1>(R, nbuf, p, grid, lds, s);
    }
}

hipError_t launch_staged(int f, int out, int nsegx, int R, int nbuf, const SParams& p, int grid, int lds,
                         hipStream_t s) {
    switch (f * 2 + out) {
    case kNV12 * 2 + 0: return launch_staged_n<kNV12, 0>(nsegx, R, nbuf, p, grid, lds, s);
    case kNV12 * 2 + 1: return launch_staged_n<kNV12, 1>(nsegx, R, nbuf, p, grid, lds, s);
    case kI420 * 2 + 0: return launch_staged_n<kI420, 0>(nsegx, R, nbuf, p, grid, lds, s);
    case kI420 * 2 + 1: return launch_staged_n<kI420, 1>(nsegx, R, nbuf, p, grid, lds, s);
    case kBGRX * 2 + 0: return launch_staged_n<kBGRX, 0>(nsegx, R, nbuf, p, grid, lds, s);
    case kBGRX * 2 + 1: return launch_staged_n<kBGRX, 1>(nsegx, R, nbuf, p, grid, lds, s);
    case kBGR * 2 + 0: return launch_staged_n<kBGR, 0>(nsegx, R, nbuf, p, grid, lds, s);
    default: return launch_staged_n<kBGR, 1>(nsegx, R, nbuf, p, grid, lds, s);
    }
}


template <int FMT, int OUT>
hipError_t launch_rows_t(const RParams& p, int grid, int lds, hipStream_t s) {
    hipLaunchKernelGGL((evam_pp_rows<FMT, OUT>), dim3(grid), dim3(kThreads), lds, s, p);
    return hipGetLastError();
}

hipError_t launch_rows(int f, int out, const RParams& p, int grid, int lds, hipStream_t s) {
    switch (f * 2 + out) {
    case kNV12 * 2 + 0: return launch_rows_t<kNV12, 0>(p, grid, lds, s);
    case kNV12 * 2 + 1: return launch_rows_t<kNV12, 1>(p, grid, lds, s);
    case kI420 * 2 + 0: return launch_rows_t<kI420, 0>(p, grid, lds, s);
    case kI420 * 2 + 1: return launch_rows_t<kI420, 1>(p, grid, lds, s);
    case kBGRX * 2 + 0: return launch_rows_t<kBGRX, 0>(p, grid, lds, s);
    case kBGRX * 2 + 1: return launch_rows_t<kBGRX, 1>(p, grid, lds, s);
    case kBGR * 2 + 0: return launch_rows_t<kBGR, 0>(p, grid, lds, s);
    default: return launch_rows_t<kBGR, 1>(p, grid, lds, s);
    }
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

template <int FMT, int OUT, int PX, int NB>
hipError_t launch_roi_px(const QParams& p, int grid, int lds, hipStream_t s) {
    if (lds > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void*)evam_pp_roi<FMT, OUT, PX, NB>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL((evam_pp_roi<FMT, OUT, PX, NB>), dim3(grid), dim3(kThreads), lds, s, p);
    return hipGetLastError();
}

// PX = 2 adjacent pixels per lane by default (round 5; 1 for odd output widths): one dwordx2 store per channel and
// one row setup per 2 pixels, C3 +3.7 % over PX = 1 on one box (profiles/r05p_c3_roi_px_rmax_ab.txt; PX = 4 equals
// PX = 1 there, round 2 measured it 8 % slower: lanes 4 pixels apart spread their LDS tap reads over more dwords).
// (Three staging buffers, EVAM_PP_ROI_NBUF=3, measured neutral or slower for two rounds: retired in round 5.)
template <int FMT, int OUT>
hipError_t launch_roi_t(int px, int nb, const QParams& p, int grid, int lds, hipStream_t s) {
    (void)nb;
    if (px == 4 && p.DW % 4 == 0) return launch_roi_px<FMT, OUT, 4, 2>(p, grid, lds, s);
    if (px == 2 && p.DW % 2 == 0) return launch_roi_px<FMT, OUT, 2, 2>(p, grid, lds, s);
    return launch_roi_px<FMT, OUT, 1, 2>(p, grid, lds, s);
}

hipError_t launch_roi(int f, int out, int px, int nb, const QParams& p, int grid, int lds, hipStream_t s) {
    switch (f * 2 + out) {
    case kNV12 * 2 + 0: return launch_roi_t<kNV12, 0>(px, nb, p, grid, lds, s);
    case kNV12 * 2 + 1: return launch_roi_t<kNV12, 1>(px, nb, p, grid, lds, s);
    case kI420 * 2 + 0: return launch_roi_t<kI420, 0>(px, nb, p, grid, lds, s);
    case kI420 * 2 + 1: return launch_roi_t<kI420, 1>(px, nb, p, grid, lds, s);
    case kBGRX * 2 + 0: return launch_roi_t<kBGRX, 0>(px, nb, p, grid, lds, s);
    case kBGRX * 2 + 1: return launch_roi_t<kBGRX, 1>(px, nb, p, grid, lds, s);
    case kBGR * 2 + 0: return launch_roi_t<kBGR, 0>(px, nb, p, grid, lds, s);
    default: return launch_roi_t<kBGR, 1>(px, nb, p, grid, lds, s);
    }
}

template <int FMT, int OUT, int PX>
hipError_t launch_wave_r(bool reuse, const WParams& p, int grid, int lds, hipStream_t s) {
    if (reuse) hipLaunchKernelGGL((evam_pp_wave<FMT, OUT, PX, true>), dim3(grid), dim3(kThreads), lds, s, p);
    else hipLaunchKernelGGL((evam_pp_wave<FMT, OUT, PX, false>), dim3(grid), dim3(kThreads), lds, s, p);
    return hipGetLastError();
}

template <int FMT, int OUT>
hipError_t launch_wave_p(int px, bool reuse, const WParams& p, int grid, int lds, hipStream_t s) {
    switch (px) {
    case 4: return launch_wave_r<FMT, OUT, 4>(reuse, p, grid, lds, s);
    case 2: return launch_wave_r<FMT, OUT, 2>(reuse, p, grid, lds, s);
    default: return launch_wave_r<FMT, OUT, 1>(reuse, p, grid, lds, s);
    }
}

hipError_t launch_wave(int f, int out, int px, bool reuse, const WParams& p, int grid, int lds, hipStream_t s) {
    switch (f * 2 + out) {
    case kNV12 * 2 + 0: return launch_wave_p<kNV12, 0>(px, reuse, p, grid, lds, s);
    case kNV12 * 2 + 1: return launch_wave_p<kNV12, 1>(px, reuse, p, grid, lds, s);
    case kI420 * 2 + 0: return launch_wave_p<kI420, 0>(px, reuse, p, grid, lds, s);
    case kI420 * 2 + 1: return launch_wave_p<kI420, 1>(px, reuse, p, grid, lds, s);
    case kBGRX * 2 + 0: return launch_wave_p<kBGRX, 0>(px, reuse, p, grid, lds, s);
    case kBGRX * 2 + 1: return launch_wave_p<kBGRX, 1>(px, reuse, p, grid, lds, s);
    case kBGR * 2 + 0: return launch_wave_p<kBGR, 0>(px, reuse, p, grid, lds, s);
    default: return launch_wave_p<kBGR, 1>(px, reuse, p, grid, lds, s);
    }
}

template <int FMT, int OUT>
const void* wave_fn_t(int px, bool reuse) {
    switch (px * 2 + (reuse ? 1 : 0)) {
    case 9: return (const void*)evam_pp_wave<FMT, OUT, 4, true>;
    case 8: return (const void*)evam_pp_wave<FMT, OUT, 4, false>;
    case 5: return (const void*)evam_pp_wave<FMT, OUT, 2, true>;
    case 4: return (const void*)evam_pp_wave<FMT, OUT, 2, false>;
    case 3: return (const void*)evam_pp_wave<FMT, OUT, 1, true>;
    default: return (const void*)evam_pp_wave<FMT, OUT, 1, false>;
    }
}
const void* wave_fn(int f, int out, int px, bool reuse) {
    switch (f * 2 + out) {
    case kNV12 * 2 + 0: return wave_fn_t<kNV12, 0>(px, reuse);
    case kNV12 * 2 + 1: return wave_fn_t<kNV12, 1>(px, reuse);
    case kI420 * 2 + 0: return wave_fn_t<kI420, 0>(px, reuse);
    case kI420 * 2 + 1: return wave_fn_t<kI420, 1>(px, reuse);
    case kBGRX * 2 + 0: return wave_fn_t<kBGRX, 0>(px, reuse);
    case kBGRX * 2 + 1: return wave_fn_t<kBGRX, 1>(px, reuse);
    case kBGR * 2 + 0: return wave_fn_t<kBGR, 0>(px, reuse);
    default: return wave_fn_t<kBGR, 1>(px, reuse);
    }
}

// Workgroups of `fn` (256 threads, `lds` bytes of dynamic LDS) resident per CU: registers and LDS both
// count. Cached per (kernel, LDS size): the query runs once per shape, not per call.
int resident_per_cu(const void* fn, int lds, int threads = kThreads) {
    static std::mutex mu;
    static std::map<std::tuple<const void*, int, int>, int> cache;
    std::lock_guard<std::mutex> lock(mu);
    auto it = cache.find({fn, lds, threads});
    if (it != cache.end()) return it->second;
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, threads, (size_t)lds) != hipSuccess || n <= 0)
        n = std::max(1, std::min(8, (160 * 1024) / std::max(lds, 1)));
    cache[{fn, lds, threads}] = n;
    return n;
}

// Wave-row kernel plan for a uniform-geometry group: pixels per lane PX (the widest whose staging
// fits the LDS budget and divides DW), the exact per-tile footprint from the host tables, REUSE when
// consecutive output rows share source rows, and a tile height that gives every CU enough workgroups.
// The kernel stages each item's footprint from that item's own crop origin x0, and the number of
// 16-byte chunks a footprint spans depends on x0's alignment: the segments are sized for the worst
// case over every residue x0 mod 32 present in the group (x0_mask bit r), which covers the 16-byte
// phase of every plane (luma / packed at bpp 1, 3, 4; NV12 chroma 2 (x >> 1); I420 chroma x >> 1).
bool plan_wave(int f, const Geom& g, int DW, int DH, int count, int out_dtype, int n_cu, const XTab* xt,
               const YTab* yt, uint32_t x0_mask, const Knobs& kn, WParams& w, int& px, bool& reuse, int& lds,
               int& grid) {
    const int npc = f == kI420 ? 2 : (f == kNV12 ? 1 : 0);
    const int lut = out_dtype == EVAM_DTYPE_F32 ? kLutBytes : 0;
    const int budget = kn.wave_lds;
    const int want_px = kn.px;
    if (!x0_mask) x0_mask = 1u << (g.x0 & 31);
    reuse = false;
    for (int Y = 0; Y + 1 < DH; Y++) {
        const bool pad0 = (yt[Y].b0 | yt[Y].b1) == 0, pad1 = (yt[Y + 1].b0 | yt[Y + 1].b1) == 0;
        if (!pad0 && !pad1 && yt[Y + 1].r0 <= yt[Y].r1) { reuse = true; break; }
    }
    if (kn.reuse == 0) reuse = false;
    px = 0;
    for (int cand : {4, 2, 1}) {
        if (want_px && cand != want_px) continue;
        if (cand > 1 && DW % cand) continue;
        const int tw = 64 * cand;
        int mY = 0, mC = 0;
        wave_segments(f, g.ox, g.rw, DW, xt, x0_mask, tw, mY, mC);
        const int segY = std::max(16, 16 * mY), segC = npc ? std::max(16, 16 * mC) : 0;
        const int wave_bytes = 2 * (2 * segY + 2 * npc * segC);
        const int need = lut + 4 * wave_bytes;
        if (need > budget && !(want_px && need <= 64 * 1024)) continue;
        px = cand;
        w.segY = segY;
        w.segC = segC;
        w.wave_bytes = wave_bytes;
        w.offBuf = lut;
        lds = need;
        break;
    }
    if (!px) return false;
    w.DW = DW; w.DH = DH;
    w.tiles_x = (DW + 64 * px - 1) / (64 * px);
    // Rows per wave: enough that the whole grid is resident at once (one round: a second round repeats
    // every workgroup's prologue latency at the tail), counting at most 4 resident workgroups per CU —
    // longer per-wave row runs amortise the prologue better than more waves hide latency. C1: 16-row
    // tiles at the 5 workgroups per CU its registers allow ran 1.6 rounds, 31.9 us; 28-row tiles (one
    // round at 5 per CU) 31.6 us; 32-row tiles (one round at 4 per CU) 29.6 us (profiles/r02r_c1_sweep.txt).
    const int per_cu = std::min(4, resident_per_cu(wave_fn(f, out_dtype, px, reuse), lds));
    const int64_t slots = (int64_t)n_cu * per_cu;
    int64_t rpw = ((int64_t)count * w.tiles_x * DH + 4 * slots - 1) / (4 * slots);
    rpw = std::max<int64_t>(2, std::min<int64_t>(32, rpw));
    w.TH = std::max(1, std::min(std::min(DH, 4 * 64), kn.wth > 0 ? kn.wth : (int)(4 * rpw)));  // <= 64 rows per wave
    w.tiles_per_item = w.tiles_x * ((DH + w.TH - 1) / w.TH);
    const int64_t gr = (int64_t)count * w.tiles_per_item;
    if (gr > 0x7FFFFFFF) return false;
    grid = (int)gr;
    return true;
}

// Ring depth: D = 2 (D 1 / 3 / 4 measured slower on C2 and C5, rounds 2-3: profiles/r03f_bench_lines.txt, C2 D 3
// +2.7 us; the other depths were retired in round 5).
#ifndef EVAM_PP_STRIP_DEPTH
#define EVAM_PP_STRIP_DEPTH 2  // A/B builds only (tools/build_variant.sh -DEVAM_PP_STRIP_DEPTH=3)
#endif
constexpr int kStripD = EVAM_PP_STRIP_DEPTH;
template <int FMT, int OUT, int PX>
const void* strip_fn_p(int pr) {
    return pr ? (const void*)evam_pp_strip<FMT, OUT, kStripD, PX, 1> : (const void*)evam_pp_strip<FMT, OUT, kStripD, PX, 0>;
}
const void* strip_fn(int f, int out, int pr, int px) {
    switch ((f * 2 + out) * 2 + (px == 2)) {
    case (kNV12 * 2 + 0) * 2: return strip_fn_p<kNV12, 0, 1>(pr);
    case (kNV12 * 2 + 0) * 2 + 1: return strip_fn_p<kNV12, 0, 2>(pr);
    case (kNV12 * 2 + 1) * 2: return strip_fn_p<kNV12, 1, 1>(pr);
    case (kNV12 * 2 + 1) * 2 + 1: return strip_fn_p<kNV12, 1, 2>(pr);
    case (kI420 * 2 + 0) * 2: return strip_fn_p<kI420, 0, 1>(pr);
    case (kI420 * 2 + 0) * 2 + 1: return strip_fn_p<kI420, 0, 2>(pr);
    case (kI420 * 2 + 1) * 2: return strip_fn_p<kI420, 1, 1>(pr);
    case (kI420 * 2 + 1) * 2 + 1: return strip_fn_p<kI420, 1, 2>(pr);
    case (kBGRX * 2 + 0) * 2: return strip_fn_p<kBGRX, 0, 1>(pr);
    case (kBGRX * 2 + 0) * 2 + 1: return strip_fn_p<kBGRX, 0, 2>(pr);
    case (kBGRX * 2 + 1) * 2: return strip_fn_p<kBGRX, 1, 1>(pr);
    default: return strip_fn_p<kBGRX, 1, 2>(pr);
    }
}

// Strip-kernel plan for a uniform 4:2:0 group (fills everything in TParams but the items, LUT, output
// and colour fields).
//  * Pixels per lane PX: 2 (128-column strips: one ~480-byte DMA segment per source row at 3.75x) where
//    the output has at least 4 such strips per row and a strip's footprint fits one 1 KB DMA instruction;
//    the strip pattern's data movement alone is 3 us faster at 128 columns than at 64
//    (profiles/r03c_strip_bw.txt).
//  * Waves per workgroup: 4..8 strips with the fewest idle waves.
//  * Tile height: about EVAM_PP_STRIP_WAVES (16) waves per CU over the whole launch (the data-movement
//    microbenchmark's best: fewer, longer-lived waves beat a full 32), at most 64 rows (the lane-held row
//    table).
//  * Ring depth: kStripD = 2.
//  * Paired taps (pr): both source rows of a plane in one LDS-DMA instruction when every strip's footprint is at
//    most 32 chunks (512 B) per row (I420 chroma: 16, four segments per instruction): 2 instructions per row
//    instead of 4 (NV12) or 6 (I420), 1 instead of 2 (BGRx). EVAM_PP_STRIP_PAIR=0 keeps one row per instruction.
// Returns false when the geometry does not suit it: outputs wider than kMaxStrips strips, footprints over
// 1 KB per strip, or consecutive output rows that share source rows (vertical upscales: the wave kernel's
// REUSE path).
bool plan_strip(int f, const Geom& g, int DW, int DH, int count, int out_dtype, int n_cu, const XTab* xt,
                const YTab* yt, uint32_t x0_mask, const Knobs& kn, bool pair_ok, TParams& p, int& pr, int& px, int& lds,
                int& grid) {
    if (f != kNV12 && f != kI420 && f != kBGRX) return false;
    int shared = 0, vis = 0;
    for (int Y = 0; Y + 1 < DH; Y++) {
        const bool pad0 = (yt[Y].b0 | yt[Y].b1) == 0, pad1 = (yt[Y + 1].b0 | yt[Y + 1].b1) == 0;
        if (pad0 || pad1) continue;
        vis++;
        shared += yt[Y + 1].r0 <= yt[Y].r1;
    }
    if (kn.strip != 2 && shared * 8 > vis) return false;  // more than 1 in 8 rows re-stages a row
    if (!x0_mask) x0_mask = 1u << (g.x0 & 31);
    const int npc = f == kI420 ? 2 : (f == kBGRX ? 0 : 1);
    int mY = 0, mC = 0;
    px = 0;
    for (int cand : {2, 1}) {
        if (kn.strip_px > 0 && cand != kn.strip_px) continue;
        // 128-column strips only where they still give a workgroup 4 strips per row: C5 (224 columns: two
        // 128-column strips, the second 3/4 full) runs 13.0 us in four 64-column strips and 15.6 us in
        // two 128-column ones (profiles/r03g_c5_px.txt)
        if (cand == 2 && (DW + 127) / 128 < 4 && kn.strip_px != 2) continue;
        wave_segments(f, g.ox, g.rw, DW, xt, x0_mask, 64 * cand, mY, mC);
        const int cap = strip_slot(f, cand) / 16;  // chunks of one slot
        if (mY <= cap && mC <= cap) { px = cand; break; }
    }
    if (!px) return false;
    const int nstrips = (DW + 64 * px - 1) / (64 * px);
    if (nstrips > kMaxStrips) return false;
    pr = kn.strip_pair && pair_ok && mY <= 32 && (npc == 0 || (npc == 1 && mC <= 32) || (npc == 2 && mC <= 16)) ? 1 : 0;
    // one ring entry: 2 luma + 2 x npc chroma segments (paired: 1 KB per plane group)
    const int grp_bytes = pr ? (npc ? 2048 : 1024) : (2 + 2 * npc) * strip_slot(f, px);
    int nw = 4, best = 1 << 30;
    for (int c = 4; c <= 8; c++) {
        const int idle = (nstrips + c - 1) / c * c - nstrips;
        if (idle < best) { best = idle; nw = c; }
    }
    if (nstrips < 4) nw = nstrips;
    if (kn.strip_nw > 0) nw = std::min(8, kn.strip_nw);
    p.nw = nw;
    p.tiles_x = (nstrips + nw - 1) / nw;
    const int lut_static = out_dtype == EVAM_DTYPE_F32 ? kLutBytes : 16;  // the kernel's static LDS
    const int wg_target = std::max(1, std::min(32, kn.strip_waves) / nw);
    p.wave_bytes = kStripD * grp_bytes;
    lds = nw * p.wave_bytes + 16;  // dynamic LDS; + 16: a right-edge tap reads past its footprint (weight 0)
    if (lds + lut_static > 64 * 1024) return false;
    const int res = std::max(1, std::min(wg_target, resident_per_cu(strip_fn(f, out_dtype, pr, px), lds)));
    const int64_t slots = (int64_t)n_cu * res;
    const int64_t work = (int64_t)std::min(count, kArgItems) * p.tiles_x * DH;
    int th = (int)std::max<int64_t>(1, (work + slots - 1) / slots);
    th = std::max(th, std::min(DH, kStripD));
    if (kn.strip_th > 0) th = kn.strip_th;
    p.TH = std::max(1, std::min(std::min(DH, 64), th));
    p.tiles_per_item = p.tiles_x * ((DH + p.TH - 1) / p.TH);
    p.DW = DW; p.DH = DH;
    p.cw = g.cw; p.ch = g.ch; p.rw = g.rw; p.rh = g.rh; p.ox = g.ox; p.oy = g.oy;
    p.scale_x = 1. / ((double)g.rw / g.cw);
    p.scale_y = 1. / ((double)g.rh / g.ch);
    const int sw = 64 * px;
    for (int k = 0; k < kSfoot; k++) {  // entry tile column x 8 + wave (nw <= 8, tiles_x <= 8)
        const int tx = k >> 3, w = k & 7, s = tx * nw + w;
        const int Xv0 = std::max(s * sw, g.ox), Xv1 = std::min(std::min(s * sw + sw, DW), g.ox + g.rw) - 1;
        p.sfoot[k] = w < nw && s < nstrips && Xv0 <= Xv1 ? int2{xt[Xv0].s0, xt[Xv1].s1} : int2{-1, -1};
    }
    if ((p.tiles_x - 1) * 8 + nw > kSfoot) return false;
    const int64_t gr = (int64_t)std::min(count, kArgItems) * p.tiles_per_item;
    if (gr > 0x7FFFFFFF) return false;
    grid = (int)gr;
    return true;
}

template <int FMT, int OUT, int PX>
hipError_t launch_strip_t(int pr, const TParams& p, dim3 grid, int lds, hipStream_t s) {
    const dim3 blk(64 * p.nw);
    if (pr) hipLaunchKernelGGL((evam_pp_strip<FMT, OUT, kStripD, PX, 1>), grid, blk, lds, s, p);
    else hipLaunchKernelGGL((evam_pp_strip<FMT, OUT, kStripD, PX, 0>), grid, blk, lds, s, p);
    return hipGetLastError();
}

hipError_t launch_strip(int f, int out, int pr, int px, const TParams& p, dim3 grid, int lds, hipStream_t s) {
    switch ((f * 2 + out) * 2 + (px == 2)) {
    case (kNV12 * 2 + 0) * 2: return launch_strip_t<kNV12, 0, 1>(pr, p, grid, lds, s);
    case (kNV12 * 2 + 0) * 2 + 1: return launch_strip_t<kNV12, 0, 2>(pr, p, grid, lds, s);
    case (kNV12 * 2 + 1) * 2: return launch_strip_t<kNV12, 1, 1>(pr, p, grid, lds, s);
    case (kNV12 * 2 + 1) * 2 + 1: return launch_strip_t<kNV12, 1, 2>(pr, p, grid, lds, s);
    case (kI420 * 2 + 0) * 2: return launch_strip_t<kI420, 0, 1>(pr, p, grid, lds, s);
    case (kI420 * 2 + 0) * 2 + 1: return launch_strip_t<kI420, 0, 2>(pr, p, grid, lds, s);
    case (kI420 * 2 + 1) * 2: return launch_strip_t<kI420, 1, 1>(pr, p, grid, lds, s);
    case (kI420 * 2 + 1) * 2 + 1: return launch_strip_t<kI420, 1, 2>(pr, p, grid, lds, s);
    case (kBGRX * 2 + 0) * 2: return launch_strip_t<kBGRX, 0, 1>(pr, p, grid, lds, s);
    case (kBGRX * 2 + 0) * 2 + 1: return launch_strip_t<kBGRX, 0, 2>(pr, p, grid, lds, s);
    case (kBGRX * 2 + 1) * 2: return launch_strip_t<kBGRX, 1, 1>(pr, p, grid, lds, s);
    default: return launch_strip_t<kBGRX, 1, 2>(pr, p, grid, lds, s);
    }
}

// Band-kernel plan for a uniform 4:2:0 group whose consecutive output rows share source rows (vertical
// upscales, C1). Fills the geometry, strips, bands and LDS fields of TParams (not items, LUT, output,
// colour).
//  * PX: the widest of 4 / 2 / 1 adjacent columns per lane that divides DW and whose strip footprint fits
//    one DMA instruction (64 chunks) per row.
//  * Band height TH: about EVAM_PP_STRIP_WAVES (16) waves per CU over the launch (one round), at most 64
//    (the lane-held row table), lowered until the band's staged rows fit the LDS.
//  * LDS per wave: the most luma rows any band reads (nrY, from the host's row table) and the chroma rows
//    they can span at either crop-origin parity (nrY / 2 + 1).
// Returns false for geometries it does not suit (fewer than 1 in 8 rows sharing source rows, footprints
// over 1 KB, outputs wider than kMaxStrips strips).
bool plan_band(int f, const Geom& g, int DW, int DH, int count, int out_dtype, int n_cu, const XTab* xt,
               const YTab* yt, uint32_t x0_mask, const Knobs& kn, TParams& p, int& px, bool& dd, int& nw, int& lds) {
    if (f != kNV12 && f != kI420) return false;
    int shared = 0, vis = 0;
    for (int Y = 0; Y + 1 < DH; Y++) {
        const bool pad0 = (yt[Y].b0 | yt[Y].b1) == 0, pad1 = (yt[Y + 1].b0 | yt[Y + 1].b1) == 0;
        if (pad0 || pad1) continue;
        vis++;
        shared += yt[Y + 1].r0 <= yt[Y].r1;
    }
    if (kn.band != 2 && shared * 8 <= vis) return false;
    if (!x0_mask) x0_mask = 1u << (g.x0 & 31);
    const int npc = f == kI420 ? 2 : 1;
    int mY = 0, mC = 0;
    px = 0;
    for (int cand : {4, 2, 1}) {
        if (kn.band_px > 0 && cand != kn.band_px) continue;
        if (DW % cand) continue;
        wave_segments(f, g.ox, g.rw, DW, xt, x0_mask, 64 * cand, mY, mC);
        if (mY <= 64 && mC <= 64) { px = cand; break; }
    }
    if (!px) return false;
    const int nstrips = (DW + 64 * px - 1) / (64 * px);
    if (nstrips > kMaxStrips) return false;
    p.segY = 16 * std::max(1, mY);
    p.segC = 16 * std::max(1, mC) * npc;  // I420: the U and V rows side by side
    const int lut_static = out_dtype == EVAM_DTYPE_F32 ? kLutBytes : 16;
    const int per_launch = std::min(count, kArgItems);
    const int64_t want = (int64_t)std::max(1, std::min(64, kn.strip_waves)) * n_cu;
    const int64_t band_rows = (int64_t)per_launch * nstrips * DH;
    // Small batches (fewer band rows than the waves the chip is sized for: C1 at 1-4 frames) run faster on the wave
    // kernel: 7.4 vs 8.1 us per launch at 1, 2 and 4 frames, while at 8 frames the band kernel is 19 % ahead
    // (profiles/r04i_c1_small_batch_ab.txt)
    if (band_rows <= want && kn.band != 2 && kn.strip_th <= 0) return false;
    int th = (int)std::max<int64_t>(2, (band_rows + want - 1) / want);
    if (kn.strip_th > 0) th = kn.strip_th;
    th = std::max(1, std::min(std::min(DH, 64), th));
    for (;; th--) {
        int nrY = 1;
        for (int Y0 = 0; Y0 < DH; Y0 += th) {
            int lo = -1, hi = -1;
            for (int Y = Y0; Y < std::min(DH, Y0 + th); Y++) {
                if ((yt[Y].b0 | yt[Y].b1) == 0) continue;  // letterbox row
                if (lo < 0) lo = yt[Y].r0;
                hi = yt[Y].r1;
            }
            if (lo >= 0) nrY = std::max(nrY, hi - lo + 1);
        }
        p.nrY = nrY;
        p.wave_bytes = nrY * p.segY + (nrY / 2 + 1) * p.segC;
        nw = std::min(4, nstrips);  // a workgroup: up to four strips of one band
        lds = nw * p.wave_bytes + 16;  // + 16: a right-edge tap reads past its footprint (weight 0)
        if (lds + lut_static <= 64 * 1024 && nrY <= 64) break;  // <= 64 rows: one lane of the wait table per row
        if (th == 1) return false;
    }
    p.TH = th;
    p.nstrips = nstrips;
    p.tiles_per_item = nstrips * ((DH + th - 1) / th);  // wave units per item
    p.DW = DW; p.DH = DH;
    p.cw = g.cw; p.ch = g.ch; p.rw = g.rw; p.rh = g.rh; p.ox = g.ox; p.oy = g.oy;
    p.scale_x = 1. / ((double)g.rw / g.cw);
    p.scale_y = 1. / ((double)g.rh / g.ch);
    p.nw = nw;
    p.tiles_x = (nstrips + nw - 1) / nw;  // strip groups
    if ((p.tiles_x - 1) * 8 + nw > kSfoot) return false;
    const int sw = 64 * px;
    for (int k = 0; k < kSfoot; k++) {  // entry strip group x 8 + wave
        const int w = k & 7, s = (k >> 3) * nw + w;
        const int Xv0 = std::max(s * sw, g.ox), Xv1 = std::min(std::min(s * sw + sw, DW), g.ox + g.rw) - 1;
        p.sfoot[k] = w < nw && s < nstrips && Xv0 <= Xv1 ? int2{xt[Xv0].s0, xt[Xv1].s1} : int2{-1, -1};
    }
    dd = px == 4 && kn.band_dd && band_six_columns(xt, DW, x0_mask);
    return (int64_t)per_launch * p.tiles_per_item <= 0x7FFFFFFF;
}

template <int FMT, int OUT>
hipError_t launch_band_t(int px, bool dd, const TParams& p, dim3 grid, int nw, int lds, hipStream_t s) {
    const dim3 blk(64 * nw);
    if (px == 4 && dd) hipLaunchKernelGGL((evam_pp_band<FMT, OUT, 4, 1>), grid, blk, lds, s, p);
    else if (px == 4) hipLaunchKernelGGL((evam_pp_band<FMT, OUT, 4, 0>), grid, blk, lds, s, p);
    else if (px == 2) hipLaunchKernelGGL((evam_pp_band<FMT, OUT, 2, 0>), grid, blk, lds, s, p);
    else hipLaunchKernelGGL((evam_pp_band<FMT, OUT, 1, 0>), grid, blk, lds, s, p);
    return hipGetLastError();
}
hipError_t launch_band(int f, int out, int px, bool dd, const TParams& p, dim3 grid, int nw, int lds, hipStream_t s) {
    switch (f * 2 + out) {
    case kNV12 * 2 + 0: return launch_band_t<kNV12, 0>(px, dd, p, grid, nw, lds, s);
    case kNV12 * 2 + 1: return launch_band_t<kNV12, 1>(px, dd, p, grid, nw, lds, s);
    case kI420 * 2 + 0: return launch_band_t<kI420, 0>(px, dd, p, grid, nw, lds, s);
    default: return launch_band_t<kI420, 1>(px, dd, p, grid, nw, lds, s);
    }
}

template <int FMT, int OUT>
const void* roi_fn_t(int px, int nb) {
    (void)nb;
    return px == 4 ? (const void*)evam_pp_roi<FMT, OUT, 4, 2>
         : px == 2 ? (const void*)evam_pp_roi<FMT, OUT, 2, 2> : (const void*)evam_pp_roi<FMT, OUT, 1, 2>;
}
const void* roi_fn(int f, int out, int px, int nb) {
    switch (f * 2 + out) {
    case kNV12 * 2 + 0: return roi_fn_t<kNV12, 0>(px, nb);
    case kNV12 * 2 + 1: return roi_fn_t<kNV12, 1>(px, nb);
    case kI420 * 2 + 0: return roi_fn_t<kI420, 0>(px, nb);
    case kI420 * 2 + 1: return roi_fn_t<kI420, 1>(px, nb);
    case kBGRX * 2 + 0: return roi_fn_t<kBGRX, 0>(px, nb);
    case kBGRX * 2 + 1: return roi_fn_t<kBGRX, 1>(px, nb);
    case kBGR * 2 + 0: return roi_fn_t<kBGR, 0>(px, nb);
    default: return roi_fn_t<kBGR, 1>(px, nb);
    }
}

// ROI-kernel plan for one format group with per-item geometry: the tile height, the LDS carve and the
// staging buffer size, sized for the widest crop of the group (max_row_bytes = row_bytes_bound of it).
// Returns false when the group needs the generic kernel (outputs wider than kRoiK x 256 pixels, taller
// than 65535 rows, or a crop so wide that one output row's segments overflow the LDS budget).
// The staging buffers are sized so that the whole grid fits on the chip in one round when it can: a ROI
// batch is about one workgroup per CU slot (C3: 1,600 ROIs), and a second round starts its workgroups
// only when first-round ones finish, paying record, geometry and setup latency again at the tail
// (C3 with 6 instead of 7 resident per CU: the 64 smallest ROIs started at ~32 us and ended the launch,
// profiles/r02r_c3_roi_timeline_before.json). Occupancy is capped by the kernel's registers
// (kRoiWavesPerSimd); the buffers take what that occupancy leaves of the LDS (allocated in 1 KB
// granules, checked against the runtime's occupancy calculator), between the widest crop's row and
// 12 KB (EVAM_PP_ROI_BUF fixes it). `slots`: workgroups resident at once with that carve.
constexpr int kRoiWavesPerSimd = 7;  // evam_pp_roi<*, *, 1> at kRoiK = 6: <= 72 VGPRs
bool plan_roi(int f, int DW, int DH, int out_dtype, int px, int max_row_bytes, int count, int n_cu, const Knobs& kn,
              QParams& q, int& base_tiles, int& lds, int64_t& slots) {
    if (DW > kRoiK * kThreads || DH > 65535) return false;
    q.DW = DW; q.DH = DH;
    q.TH = (int64_t)DW * DH <= 32768 ? DH : std::max(8, std::min(DH, 16384 / DW));
    if (kn.roi_th > 0) q.TH = std::max(1, std::min(DH, kn.roi_th));
    base_tiles = (DH + q.TH - 1) / q.TH;
    q.offXT = out_dtype == EVAM_DTYPE_F32 ? kLutBytes : 0;
    q.offYT = q.offXT + (int)sizeof(XTab) * DW;
    q.offBuf = q.offYT + (int)sizeof(YTab) * q.TH;
    const int64_t grid = (int64_t)count * base_tiles;
    const int per_cu = (int)std::max<int64_t>(1, std::min<int64_t>(kRoiWavesPerSimd, (grid + n_cu - 1) / n_cu));
    const int pxv = (px == 4 || px == 2) && DW % px == 0 ? px : 1;
    const uint32_t qw = (uint32_t)(DW / pxv);
    q.mqw = qw > 1 ? (uint32_t)((0x100000000ull + qw - 1) / qw) : 0u;
    const int nb = 2;
    int buf = kn.roi_buf;
    if (buf <= 0) buf = std::min(12 * 1024, ((((160 * 1024) / per_cu) & ~1023) - q.offBuf) / nb & ~15);
    q.buf_bytes = (std::max(buf, max_row_bytes) + 15) & ~15;
    lds = q.offBuf + nb * q.buf_bytes;
    if (q.buf_bytes > 32 * 1024 || lds > 160 * 1024) return false;
    const void* fn = roi_fn(f, out_dtype, pxv, nb);
    int res = resident_per_cu(fn, lds);
    while (kn.roi_buf <= 0 && res < per_cu && q.buf_bytes - 512 >= max_row_bytes) {
        q.buf_bytes -= 512;
        lds -= 512 * nb;
        res = resident_per_cu(fn, lds);
    }
    slots = (int64_t)n_cu * res;
    return true;
}

// HIP backend of the descriptor rings (evam_rings.h): events, streams, pinned and device memory. Every
// failure is reported through fail() with the HIP error string.
struct HipRings {
    using Event = hipEvent_t;
    using Stream = hipStream_t;
    static int err(hipError_t e, const char* what) {
        return e == hipSuccess ? 0 : fail(EVAM_PP_ERR_HIP, "%s failed: %s", what, hipGetErrorString(e));
    }
    int event_create(Event* e) { return err(hipEventCreateWithFlags(e, hipEventDisableTiming), "hipEventCreate"); }
    int event_destroy(Event e) { return err(hipEventDestroy(e), "hipEventDestroy"); }
    int event_record(Event e, Stream s) { return err(hipEventRecord(e, s), "hipEventRecord"); }
    int event_sync(Event e) { return err(hipEventSynchronize(e), "hipEventSynchronize"); }
    int stream_create(Stream* s) { return err(hipStreamCreateWithFlags(s, hipStreamNonBlocking), "hipStreamCreate"); }
    int stream_destroy(Stream s) { return err(hipStreamDestroy(s), "hipStreamDestroy"); }
    int stream_wait(Stream s, Event e) { return err(hipStreamWaitEvent(s, e, 0), "hipStreamWaitEvent"); }
    int stream_sync(Stream s) { return err(hipStreamSynchronize(s), "hipStreamSynchronize"); }
    // ROI record slots: fine-grained device memory that the host writes through the platform's BAR mapping of it
    // (one 64-byte scalar load per workgroup from device memory instead of a PCIe read from host memory: ~4.5 us
    // less per 1,600-workgroup launch, tools/microbench/rec_hostwrite.hip), where the allocation is mapped
    // read-write into this process; else pinned, coherent host memory (EVAM_PP_REC_DEVICE=0 forces that).
    bool rec_device = true;
    static bool host_mapped_rw(const void* p, size_t n) {
        FILE* f = fopen("/proc/self/maps", "r");
        if (!f) return false;
        const uintptr_t a = reinterpret_cast<uintptr_t>(p), e = a + n;
        char line[512];
        bool ok = false;
        while (!ok && fgets(line, sizeof(line), f)) {
            unsigned long lo = 0, hi = 0;
            char perm[8] = {};
            if (sscanf(line, "%lx-%lx %7s", &lo, &hi, perm) == 3 && lo <= a && e <= hi) ok = perm[0] == 'r' && perm[1] == 'w';
        }
        fclose(f);
        return ok;
    }
    int pinned_alloc(uint8_t** h, const uint8_t** d, size_t n, bool* wc) {
        *wc = false;
        if (rec_device) {
            void* p = nullptr;
            if (hipExtMallocWithFlags(&p, n, hipDeviceMallocFinegrained) == hipSuccess) {
                if (host_mapped_rw(p, n)) {
                    *h = static_cast<uint8_t*>(p);
                    *d = static_cast<const uint8_t*>(p);
                    *wc = true;
                    return 0;
                }
                (void)hipFree(p);
            } else {
                (void)hipGetLastError();
            }
        }
        if (hipHostMalloc((void**)h, n, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
            *h = nullptr;
            return fail(EVAM_PP_ERR_OOM, "evam_pp_run: hipHostMalloc(%zu) failed", n);
        }
        void* dp = nullptr;
        if (int rc = err(hipHostGetDevicePointer(&dp, *h, 0), "hipHostGetDevicePointer")) return rc;
        *d = reinterpret_cast<const uint8_t*>(dp);
        return 0;
    }
    int pinned_free(uint8_t* h, bool wc) { return wc ? err(hipFree(h), "hipFree") : err(hipHostFree(h), "hipHostFree"); }
    int host_alloc(uint8_t** h, size_t n) {
        if (hipHostMalloc((void**)h, n, hipHostMallocDefault) != hipSuccess) {
            *h = nullptr;
            return fail(EVAM_PP_ERR_OOM, "evam_pp_run: hipHostMalloc(%zu) failed", n);
        }
        return 0;
    }
    int host_free(uint8_t* h) { return err(hipHostFree(h), "hipHostFree"); }
    int dev_alloc(uint8_t** d, size_t n) {
        if (hipMalloc((void**)d, n) != hipSuccess) {
            *d = nullptr;
            return fail(EVAM_PP_ERR_OOM, "evam_pp_run: hipMalloc(%zu) failed", n);
        }
        return 0;
    }
    int dev_free(uint8_t* d) { return err(hipFree(d), "hipFree"); }
    int copy_h2d(uint8_t* dst, const uint8_t* src, size_t n, Stream s) {
        return err(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, s), "hipMemcpyAsync");
    }
};
using DescRing = DescRingT<HipRings>;
using PinRing = PinRingT<HipRings>;

}  // namespace

#ifdef EVAM_PP_HOST_PROF
// Diagnostic build: cumulative host time from entry to each mark of evam_pp_run, printed at destroy.
#include <chrono>
static double g_hp[12];
static long g_hp_n;
#define HP_START const auto hp_t0 = std::chrono::steady_clock::now(); double hp_t[12] = {}
#define HP(i) (hp_t[i] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - hp_t0).count())
#else
#define HP_START (void)0
#define HP(i) (void)0
#endif

struct evam_pp {
    int device = 0;
    int n_cu = 256;
    hipStream_t stream = nullptr;
    int opt_stats = 0, opt_timing = 0;
    evam_pp_stats stats{};
    std::vector<uint8_t> h_block;  // this call's descriptor block, built on the host
    DescRing ring;
    PinRing pin;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    hipEvent_t ev_switch = nullptr;
    bool timed = false;
    TabCache tab_cache;
    evam_preproc lut_key{};        // cfg the cached LUT was built from (norm fields + dtype)
    bool lut_valid = false;
    float lut[768];
    Knobs knobs;                   // EVAM_PP_* tuning knobs, read once at evam_pp_create
    std::vector<int> sc_fmt;       // per-call scratch, kept to avoid reallocation
    std::vector<int> sc_bucket;
    std::vector<int> sc_sfmt;      // per-call source format ids
    std::vector<int> sc_order;
    std::vector<int> sc_members;   // item indices grouped by source format
    std::vector<Geom> sc_geo;
    std::vector<int> sc_units;     // ROI work units: (item, row0, row1, cost)
    std::vector<int> sc_start;     // ROI unit counting sort: bucket starts
    std::vector<int> sc_slot;      // ROI units in launch order
    std::vector<uint8_t> sc_seen;  // evam_pp_run_slots: output slots taken
    std::vector<uint32_t> sc_plan; // roi_launch_order scratch
    std::vector<RecFrame> sc_frames;  // per source: the frame half of its ROI records
    int memo_key[4] = {-1, -1, -1, -1};  // (format, staging buffer, row cap, DH) of memo_rg
    std::vector<uint32_t> memo_rg;       // per crop width: rows per group | groups of the whole height << 16
    TParams sc_tparams;            // strip-kernel arguments (3.5 KB: kept off the stack)
};

namespace {

// A failed evam_pp_run after its pinned slot was taken: drain the stream (PinRingT::abandon), so a run
// whose fence the failed call should have recorded cannot leave slots that kernels still read.
struct PinGuard {
    evam_pp* h;
    bool armed = false;
    ~PinGuard() {
        if (armed) {
            HipRings b;
            (void)h->pin.abandon(b, h->stream);
        }
    }
};

}  // namespace

extern "C" {

int evam_pp_abi_version(void) { return EVAM_PP_ABI_VERSION; }

#ifdef EVAM_PP_TRACE
// Diagnostic builds: copy the first n_wg workgroups' trace records (kTraceSlots x u64 each) of the last
// traced launch.
// host == NULL: clear the trace buffer (before the launch to trace).
int evam_pp_debug_trace(unsigned long long* host, int n_wg) {
    if (!host) {
        void* a = nullptr;
        HIP_TRY(hipDeviceSynchronize());
        HIP_TRY(hipGetSymbolAddress(&a, HIP_SYMBOL(g_evam_trace)));
        HIP_TRY(hipMemset(a, 0, sizeof(g_evam_trace)));
        return EVAM_PP_OK;
    }
    if (n_wg <= 0 || n_wg > kTraceWGs) return EVAM_PP_ERR_INVALID_ARG;
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_evam_trace),
                                sizeof(unsigned long long) * kTraceSlots * (size_t)n_wg));
    return EVAM_PP_OK;
}
#endif

const char* evam_pp_last_error(void) { return g_last_error.c_str(); }

int evam_pp_create(int hip_device, void* hip_stream, evam_pp** out) {
    if (!out) return fail(EVAM_PP_ERR_INVALID_ARG, "evam_pp_create: out is NULL");
    *out = nullptr;
    if (kAblate != 0) {  // a stage-removal diagnostic build computes invalid tensors: never by accident
        const char* ok = getenv("EVAM_PP_DIAGNOSTIC_BUILD_OK");
        if (!ok || strcmp(ok, "1") != 0)
            return fail(EVAM_PP_ERR_UNSUPPORTED, "evam_pp_create: diagnostic build (EVAM_PP_ABLATE=%d) refused; "
                        "set EVAM_PP_DIAGNOSTIC_BUILD_OK=1 for profiling runs", kAblate);
        fprintf(stderr, "[evam_pp] DIAGNOSTIC BUILD (EVAM_PP_ABLATE=%d): outputs are invalid\n", kAblate);
    }
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
        return fail(EVAM_PP_ERR_NO_DEVICE, "evam_pp_create: no HIP device");
    if (hip_device < 0 || hip_device >= n)
        return fail(EVAM_PP_ERR_NO_DEVICE, "evam_pp_create: device %d out of range [0,%d)", hip_device, n);
    HIP_TRY(hipSetDevice(hip_device));
    evam_pp* h = new (std::nothrow) evam_pp();
    if (!h) return fail(EVAM_PP_ERR_OOM, "evam_pp_create: out of host memory");
    h->device = hip_device;
    h->knobs.read();
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
#ifdef EVAM_PP_HOST_PROF
    if (g_hp_n) {
        fprintf(stderr, "[host prof] %ld steady calls, mean us from entry at marks 1..10:", g_hp_n);
        for (int i = 1; i <= 10; i++) fprintf(stderr, " %.2f", g_hp[i] / g_hp_n);
        fprintf(stderr, "\n");
    }
#endif
    (void)hipSetDevice(h->device);
    if (h->ring.have_copy || h->pin.cur >= 0) {
        (void)hipStreamSynchronize(h->stream);
        if (h->ring.have_copy) (void)hipStreamSynchronize(h->ring.copy);
    }
    HipRings b;
    h->ring.release(b);
    h->pin.release(b);
    if (h->ev_switch) (void)hipEventDestroy(h->ev_switch);
    if (h->ev0) (void)hipEventDestroy(h->ev0);
    if (h->ev1) (void)hipEventDestroy(h->ev1);
    delete h;
}

int evam_pp_set_stream(evam_pp* h, void* hip_stream) {
    if (!h) return fail(EVAM_PP_ERR_INVALID_ARG, "evam_pp_set_stream: NULL handle");
    hipStream_t ns = reinterpret_cast<hipStream_t>(hip_stream);
    if (ns != h->stream && (h->ring.cur >= 0 || h->pin.cur >= 0)) {
        // Order the new stream behind everything already launched on the old one, so the descriptor
        // slots' fences (recorded on the current stream) keep covering earlier kernels.
        HIP_TRY(hipSetDevice(h->device));
        if (!h->ev_switch) HIP_TRY(hipEventCreateWithFlags(&h->ev_switch, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(h->ev_switch, h->stream));
        HIP_TRY(hipStreamWaitEvent(ns, h->ev_switch, 0));
    }
    h->stream = ns;
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

}  // extern "C"

namespace {

// evam_pp_run and evam_pp_run_slots. slots == NULL: item i -> slot dst->slot_offset + i * dst->slot_stride; else item i
// -> slot slots[i]. The kernels read one output index per item (ItemArg / ItemDesc .index, RoiRec .item) and compute
// slot = slot_offset + index * slot_stride, so an explicit table travels as index = slots[i], offset 0, stride 1.
int run_impl(evam_pp* h, const evam_image* srcs, int n_srcs, const evam_roi* items, int n_items, const evam_preproc* cfg,
             const evam_tensor* dst, const int32_t* slots, evam_transform* out_xform) {
    HP_START;
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
    const int esz = cfg->out_dtype == EVAM_DTYPE_F32 ? 4 : 1;
    // The kernels address one output plane with 32-bit byte offsets.
    if (plane * esz > INT32_MAX)
        return fail(EVAM_PP_ERR_INVALID_ARG, "evam_pp_run: dst plane %dx%d exceeds 2 GiB", DW, DH);
    const Knobs& kn = h->knobs;

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
            const int rows = p == 0 ? s.height : s.height / 2;
            if (!s.planes[p]) return fail(EVAM_PP_ERR_INVALID_ARG, "evam_pp_run: srcs[%d].planes[%d] is NULL", i, p);
            if (((uintptr_t)s.planes[p] & 15) || (s.pitch[p] & 15))
                return fail(EVAM_PP_ERR_ALIGNMENT, "evam_pp_run: srcs[%d] plane %d pointer/pitch (%d) not 16-byte aligned", i, p, s.pitch[p]);
            if (s.pitch[p] < row_bytes)
                return fail(EVAM_PP_ERR_INVALID_ARG, "evam_pp_run: srcs[%d] plane %d pitch %d < row bytes %d", i, p, s.pitch[p], row_bytes);
            // the kernels address a plane through buffer resources with 32-bit byte offsets
            if ((int64_t)s.pitch[p] * rows > INT32_MAX)
                return fail(EVAM_PP_ERR_INVALID_ARG, "evam_pp_run: srcs[%d] plane %d (%d x %d B) exceeds 2 GiB", i, p, rows, s.pitch[p]);
        }
    }

    HP(1);
    // ---- pass 1 (integer only): item -> source, format, clipped crop; validation ----
    std::vector<int>& fmt = h->sc_fmt;
    std::vector<Geom>& geo = h->sc_geo;
    fmt.resize(n_items);
    geo.resize(n_items);
    int count[4] = {0, 0, 0, 0};
    int rep[4] = {-1, -1, -1, -1};
    int max_cw[4] = {0, 0, 0, 0}, max_ch[4] = {0, 0, 0, 0};
    uint32_t x0_mask[4] = {0, 0, 0, 0};  // crop origins x0 mod 32 present (wave-kernel staging bound)
    bool uniform[4] = {true, true, true, true};
    if (slots) {
        // an explicit slot per item: each inside the batch, no two items into one slot
        std::vector<uint8_t>& seen = h->sc_seen;
        seen.assign((size_t)dst->n, 0);
        for (int i = 0; i < n_items; i++) {
            const int32_t sl = slots[i];
            if (sl < 0 || sl >= dst->n)
                return fail(EVAM_PP_ERR_INVALID_ARG, "evam_pp_run_slots: slots[%d] = %d outside tensor batch %d", i, sl,
                            dst->n);
            if (seen[sl]++)
                return fail(EVAM_PP_ERR_INVALID_ARG, "evam_pp_run_slots: slot %d given to two items (slots[%d])", sl, i);
        }
    } else {
        // output slots are linear in the item index: the first and the last bound them all
        for (int i : {0, n_items - 1}) {
            const int64_t slot = (int64_t)dst->slot_offset + (int64_t)i * dst->slot_stride;
            if (slot < 0 || slot >= dst->n)
                return fail(EVAM_PP_ERR_INVALID_ARG, "evam_pp_run: item %d -> slot %lld outside tensor batch %d", i,
                            (long long)slot, dst->n);
        }
    }
    const int slot_offset = slots ? 0 : dst->slot_offset, slot_stride = slots ? 1 : dst->slot_stride;
    std::vector<int>& sfmt = h->sc_sfmt;  // per source: format id (looked up once, not per ROI)
    sfmt.resize(n_srcs);
    bool one_fmt = true, one_size = true;
    for (int i = 0; i < n_srcs; i++) {
        sfmt[i] = fmt_id(srcs[i].fourcc);
        one_fmt &= sfmt[i] == sfmt[0];
        one_size &= srcs[i].width == srcs[0].width && srcs[i].height == srcs[0].height;
    }
    static const bool has_avx2 = __builtin_cpu_supports("avx2");
    if (one_fmt && one_size && items && n_items >= 8 && has_avx2 && kn.host_simd &&
        clip_rois_avx2(items, n_items, n_srcs, srcs[0].width, srcs[0].height, sfmt[0] == kNV12 || sfmt[0] == kI420,
                       geo.data(), max_cw[sfmt[0]], max_ch[sfmt[0]], x0_mask[sfmt[0]], uniform[sfmt[0]])) {
        const int f = sfmt[0];
        std::fill(fmt.begin(), fmt.end(), f);
        count[f] = n_items; rep[f] = 0;
    } else if (one_fmt && items && n_items > 0 && n_srcs > 0) {
        // every source in one format (the common case: one decoder): the group's counters live in registers
        // instead of arrays indexed by the item's format (a store-to-load chain per ROI: C3 pass 1 ~7 -> ~4 us)
        const int f = sfmt[0];
        int mcw = 0, mch = 0, rcw = 0, rch = 0;
        uint32_t xm = 0;
        bool uni = true;
        for (int i = 0; i < n_items; i++) {
            const evam_roi& r = items[i];
            if ((unsigned)r.src_index >= (unsigned)n_srcs)
                return fail(EVAM_PP_ERR_INVALID_ARG, "evam_pp_run: items[%d].src_index %d out of range", i, r.src_index);
            const evam_image& s = srcs[r.src_index];
            fmt[i] = f;
            Geom& g = geo[i];
            if (roi_clip(f, s.width, s.height, true, r.x, r.y, r.w, r.h, g))
                return fail(EVAM_PP_ERR_EMPTY_ROI, "evam_pp_run: items[%d] ROI (%d,%d,%d,%d) is empty after clipping to %dx%d",
                            i, r.x, r.y, r.w, r.h, s.width, s.height);
            mcw = std::max(mcw, g.cw);
            mch = std::max(mch, g.ch);
            xm |= 1u << (g.x0 & 31);
            if (i == 0) { rcw = g.cw; rch = g.ch; }
            uni &= g.cw == rcw && g.ch == rch;  // geometry = f(cw, ch)
        }
        count[f] = n_items; max_cw[f] = mcw; max_ch[f] = mch; x0_mask[f] = xm; rep[f] = 0; uniform[f] = uni;
    } else
    for (int i = 0; i < n_items; i++) {
        const evam_roi* r = items ? &items[i] : nullptr;
        const int si = items ? r->src_index : i;
        if ((unsigned)si >= (unsigned)n_srcs)
            return fail(EVAM_PP_ERR_INVALID_ARG, "evam_pp_run: items[%d].src_index %d out of range", i, si);
        const evam_image& s = srcs[si];
        const int f = sfmt[si];
        fmt[i] = f;
        Geom& g = geo[i];
        if (roi_clip(f, s.width, s.height, r != nullptr, r ? r->x : 0, r ? r->y : 0, r ? r->w : 0, r ? r->h : 0, g))
            return fail(EVAM_PP_ERR_EMPTY_ROI, "evam_pp_run: items[%d] ROI (%d,%d,%d,%d) is empty after clipping to %dx%d",
                        i, r ? r->x : 0, r ? r->y : 0, r ? r->w : 0, r ? r->h : 0, s.width, s.height);
        count[f]++;
        max_cw[f] = std::max(max_cw[f], g.cw);
        max_ch[f] = std::max(max_ch[f], g.ch);
        x0_mask[f] |= 1u << (g.x0 & 31);
        if (rep[f] < 0) rep[f] = i;
        else if (g.cw != geo[rep[f]].cw || g.ch != geo[rep[f]].ch) uniform[f] = false;  // geometry = f(cw, ch)
    }
    HP(2);
    // item indices grouped by format, in call order within a format
    std::vector<int>& members = h->sc_members;
    members.resize(n_items);
    int mfirst[5] = {0, 0, 0, 0, 0};
    for (int f = 0; f < 4; f++) mfirst[f + 1] = mfirst[f] + count[f];
    if (n_items == count[fmt[0]]) {  // one format: call order
        for (int i = 0; i < n_items; i++) members[i] = i;
    } else {
        int fill_at[4] = {mfirst[0], mfirst[1], mfirst[2], mfirst[3]};
        for (int i = 0; i < n_items; i++) members[fill_at[fmt[i]]++] = i;
    }

    // ---- per format group: kernel choice ----
    //   uniform geometry        -> staged / wave / row kernels: host-built tables, items in kernel arguments
    //   per-item geometry       -> ROI kernel: raw ROI rect + source (RoiRec), geometry resolved on the device
    //   ROI plan impossible     -> generic kernel, per-item ItemDesc in the descriptor block
    enum { kPathNone, kPathUniform, kPathRoi, kPathGeneric };
    int path[4];
    QParams qp[4];
    int qlds[4] = {0, 0, 0, 0}, qbase[4] = {1, 1, 1, 1}, qrec[4] = {0, 0, 0, 0};
    int64_t qslots[4] = {0, 0, 0, 0};
    bool any_generic = false, any_roi = false;
    for (int f = 0; f < 4; f++) {
        path[f] = kPathNone;
        if (!count[f]) continue;
        if (uniform[f] && kn.rows) path[f] = kPathUniform;
        else if (kn.roi && plan_roi(f, DW, DH, cfg->out_dtype, kn.roi_px, row_bytes_bound(f, max_cw[f]), count[f], h->n_cu,
                                    kn, qp[f], qbase[f], qlds[f], qslots[f])) path[f] = kPathRoi;
        else path[f] = kPathGeneric;
        any_generic |= path[f] == kPathGeneric;
        any_roi |= path[f] == kPathRoi;
    }
    // Full geometry on the host only where something consumes it.
    const bool all_geo = out_xform != nullptr || h->opt_stats;
    int64_t src_bytes = 0;
    for (int i = 0; i < n_items; i++) {
        const int f = fmt[i];
        if (!all_geo && path[f] == kPathRoi) continue;
        if (!all_geo && path[f] == kPathUniform && i != rep[f]) continue;  // same crop size: rep's geometry
        Geom& g = geo[i];
        const evam_roi* r = items ? &items[i] : nullptr;
        const evam_image& s = srcs[items ? r->src_index : i];
        roi_geometry(f, s.width, s.height, r != nullptr, r ? r->x : 0, r ? r->y : 0, r ? r->w : 0, r ? r->h : 0,
                     cfg->resize_mode, cfg->placement, DW, DH, g);
        if (out_xform) {
            evam_transform& t = out_xform[i];
            t.scale_x = (float)((double)g.rw / g.cw);
            t.scale_y = (float)((double)g.rh / g.ch);
            t.crop_x = g.x0; t.crop_y = g.y0; t.crop_w = g.cw; t.crop_h = g.ch;
            t.pad_x = g.ox; t.pad_y = g.oy;
            t.resized_w = g.rw; t.resized_h = g.rh;
        }
        if (h->opt_stats) src_bytes += item_src_bytes(f, g, DW, DH);
    }

    HP(3);
    // ---- descriptor block (device-resident, re-uploaded only when its bytes change) ----
    // [LUT][ItemDesc x (items of generic groups)][per uniform group: XTab x DW, YTab x DH]
    // Everything in it is a function of the configuration and the geometry, not of the frames, so a new
    // set of frames of the same geometry reuses the resident block.
    size_t nbytes = kLutBytes;
    const size_t desc_off = nbytes;
    int n_desc = 0;
    for (int f = 0; f < 4; f++)
        if (path[f] == kPathGeneric) n_desc += count[f];
    nbytes += sizeof(ItemDesc) * (size_t)n_desc;
    size_t tab_off[4] = {0, 0, 0, 0};
    for (int f = 0; f < 4; f++) {
        if (path[f] != kPathUniform) continue;
        tab_off[f] = nbytes;
        nbytes += sizeof(XTab) * (size_t)DW + sizeof(YTab) * (size_t)DH;
    }
    // ROI groups: [per ROI group: RoiRec x tiles], in a pinned zero-copy slot (PinRing). A group has
    // count x base tiles, plus up to one extra tile per ROI when its longest crops are split in two.
    size_t rec_off[4] = {0, 0, 0, 0}, dyn_bytes = 0;
    if (any_roi) {
        for (int f = 0; f < 4; f++) {
            if (path[f] != kPathRoi) continue;
            rec_off[f] = dyn_bytes;
            dyn_bytes += sizeof(RoiRec) * (size_t)count[f] * (size_t)qbase[f];
            // tail split: up to n_cu ROIs become kn.roi_tail row tiles each
            if (qbase[f] == 1 && kn.roi_tail > 1)
                dyn_bytes += sizeof(RoiRec) * (size_t)std::min(count[f], h->n_cu) * (size_t)(kn.roi_tail - 1);
        }
    }
    h->h_block.resize(nbytes);
    uint8_t* blk = h->h_block.data();
    if (cfg->out_dtype == EVAM_DTYPE_F32) {
        // The LUT depends only on the normalisation fields: rebuilt when they change.
        evam_preproc key{};
        key.out_dtype = cfg->out_dtype;
        key.norm_flags = cfg->norm_flags;
        memcpy(key.range, cfg->range, sizeof(key.range));
        memcpy(key.mean, cfg->mean, sizeof(key.mean));
        memcpy(key.std, cfg->std, sizeof(key.std));
        if (!h->lut_valid || memcmp(&key, &h->lut_key, sizeof(key)) != 0) {
            build_lut(*cfg, h->lut);
            h->lut_key = key;
            h->lut_valid = true;
        }
        memcpy(blk, h->lut, kLutBytes);
    } else {
        memset(blk, 0, kLutBytes);
    }
    int first[4] = {0, 0, 0, 0};
    {
        ItemDesc* desc = reinterpret_cast<ItemDesc*>(blk + desc_off);
        int order = 0;
        for (int f = 0; f < 4; f++) {
            if (path[f] == kPathGeneric) {
                first[f] = order;
                for (int m = mfirst[f]; m < mfirst[f + 1]; m++) {
                    const int i = members[m];
                    const evam_image& s = srcs[items ? items[i].src_index : i];
                    ItemDesc& d = desc[order++];
                    for (int p = 0; p < 3; p++) { d.plane[p] = s.planes[p]; d.pitch[p] = s.pitch[p]; }
                    const Geom& g = geo[i];
                    d.x0 = g.x0; d.y0 = g.y0; d.cw = g.cw; d.ch = g.ch;
                    d.rw = g.rw; d.rh = g.rh; d.ox = g.ox; d.oy = g.oy;
                    d.index = slots ? slots[i] : i;  // the slot offset / stride are launch parameters: the block survives clip-ring steps
                    d.pad_ = 0;
                    d.scale_x = 1. / ((double)g.rw / g.cw);
                    d.scale_y = 1. / ((double)g.rh / g.ch);
                }
            } else if (path[f] == kPathUniform) {
                XTab* xt = reinterpret_cast<XTab*>(blk + tab_off[f]);
                YTab* yt = reinterpret_cast<YTab*>(xt + DW);
                build_tables(geo[rep[f]], DW, DH, h->tab_cache, xt, yt);
            }
        }
    }
    (void)any_generic;
    HP(4);
    HIP_TRY(hipSetDevice(h->device));
    uint8_t* dyn = nullptr;
    const uint8_t* d_dyn = nullptr;
    PinGuard pin_guard{h};
    bool dyn_wc = false;
    if (any_roi) {
        HipRings b;
        b.rec_device = kn.rec_device != 0;
        if (int rc = h->pin.acquire(b, dyn_bytes, &dyn, &d_dyn, &dyn_wc)) return rc;
        pin_guard.armed = true;
        HP(5);
        // Launch order: largest estimated work first (counting sort on 64 buckets of the staged
        // bytes, crop width x touched rows). Workgroups are dispatched in order as slots free, so
        // the long ROIs start first and the short ones fill the tail.
        const bool sort = kn.roi_sort != 0;
        // the frame half of the records, once per source (a record then takes three of its lines from here)
        std::vector<RecFrame>& rfr = h->sc_frames;
        rfr.resize((size_t)n_srcs);
        for (int s = 0; s < n_srcs; s++) {
            RoiRec r;
            memset(&r, 0, sizeof(r));
            r.plane[0] = srcs[s].planes[0]; r.plane[1] = srcs[s].planes[1]; r.plane[2] = srcs[s].planes[2];
            r.pitch[0] = srcs[s].pitch[0]; r.pitch[1] = srcs[s].pitch[1]; r.pitch[2] = srcs[s].pitch[2];
            r.width = (uint16_t)srcs[s].width; r.height = (uint16_t)srcs[s].height;
            memcpy(&rfr[s], &r, sizeof(RecFrame));
        }
        for (int f = 0; f < 4; f++) {
            if (path[f] != kPathRoi) continue;
            RoiRec* rr = reinterpret_cast<RoiRec*>(dyn + rec_off[f]);
            // One record per work unit, assembled in four XMM registers and written as one 64-byte line into its
            // launch slot: the frame's lines, the caller's rect (w <= 0 without items: the full frame), the output
            // index and the tile's rows.
            const RecFrame* rf = rfr.data();
            auto put_rec = [&](int pos, int i, int row0, int row1) {
                const RecFrame& F = rf[items ? items[i].src_index : i];
                const __m128i rect = items ? _mm_loadu_si128(reinterpret_cast<const __m128i*>(&items[i].x)) : _mm_setzero_si128();
                const uint64_t tail = (uint64_t)(uint32_t)(slots ? slots[i] : i) |
                                      ((uint64_t)((uint32_t)(uint16_t)row0 | ((uint32_t)(uint16_t)row1 << 16)) << 32);
                const __m128i l2 = _mm_unpacklo_epi64(F.l[2], rect);
                const __m128i l3 = _mm_unpackhi_epi64(rect, _mm_set_epi64x((long long)tail, 0));
                __m128i* dst = reinterpret_cast<__m128i*>(&rr[pos]);
                if (dyn_wc) {  // write-combined device memory: the 64-byte line as four streaming stores
                    _mm_stream_si128(dst + 0, F.l[0]);
                    _mm_stream_si128(dst + 1, F.l[1]);
                    _mm_stream_si128(dst + 2, l2);
                    _mm_stream_si128(dst + 3, l3);
                } else {
                    _mm_store_si128(dst + 0, F.l[0]);
                    _mm_store_si128(dst + 1, F.l[1]);
                    _mm_store_si128(dst + 2, l2);
                    _mm_store_si128(dst + 3, l3);
                }
            };
            // Work units (one workgroup each): one per ROI, or per row tile of TH rows for outputs taller than one
            // tile. Units launch largest first; beyond the resident workgroups the dispatcher starts each remaining
            // unit as a slot frees up. (Row tiles of a few row groups per ROI, EVAM_PP_ROI_UNIT, measured slower for
            // two rounds and were retired in round 5.)
            const QParams& q = qp[f];
            const int base = qbase[f];
            const int pxr = (kn.roi_px == 4 || kn.roi_px == 2) && DW % kn.roi_px == 0 ? kn.roi_px : 1;
            const int rcap = std::max(1, ((kRoiK / pxr) * kThreads) / (DW / pxr));
            int nu = 0;
            if (base == 1) {
                // One unit per ROI (the default), planned in four passes over the ROIs with no unit list
                // (roi_launch_order, evam_geom.h): row groups per ROI, the bytes pre-order, the tail split, one
                // counting sort by (row groups, bytes), the snake deal, and each record written into its slot.
                // Tail split: every ROI does the same pixel work (DW x DH), so when the ROIs do not divide
                // evenly over the CUs the last `tail` ROIs in launch order land as one extra workgroup on
                // `tail` CUs, whose SIMDs then convert 1 / floor(count / n_cu) more pixels than the others and
                // end the launch (profiles/r03s_c3_roi_timeline_lut_dma.json: the last workgroups to finish
                // are those narrow, compute-dense crops). Splitting those ROIs into kn.roi_tail row tiles —
                // as long as every unit stays resident — gives each of the CUs a fraction of an ROI instead.
                // Snake deal: workgroup p starts on XCD p % 8 and within it on CU (p / 8) % 32, so each band of n_cu
                // consecutive positions puts one unit on every CU; reversing every other band gives each CU one large
                // and one small unit per two bands instead of always the k-th largest of every band (per-CU work
                // balance is what bounds a one-round launch: profiles/r05ze_c3_head_split_ab.txt,
                // r05zd_c3_xcd_frames_devrec_ab.txt).
                // Rows per group and groups per ROI depend on an ROI only through its crop width: memoised per
                // handle for this launch's (format, staging buffer, row cap, DH).
                const int mkey[4] = {f, q.buf_bytes, rcap, DH};
                if (memcmp(mkey, h->memo_key, sizeof(mkey)) != 0) {
                    memcpy(h->memo_key, mkey, sizeof(mkey));
                    h->memo_rg.clear();
                }
                if ((int)h->memo_rg.size() <= max_cw[f]) h->memo_rg.resize((size_t)max_cw[f] + 1, 0u);
                uint32_t* rgm = h->memo_rg.data();  // R | groups of the whole height << 16 (0: not yet known)
                auto rg = [&](int cw) {
                    uint32_t& e = rgm[cw];
                    if (!e) {
                        const int R = std::max(1, std::min(std::min(q.buf_bytes / row_bytes_bound(f, cw), rcap), DH));
                        e = (uint32_t)R | ((uint32_t)((DH + R - 1) / R) << 16);
                    }
                    return e;
                };
                HP(6);
                if (kn.roi_xcd && items && h->n_cu >= 8) {
                    // experiment (EVAM_PP_ROI_XCD=1): the sorted units, then each frame's units on one XCD
                    std::vector<int>& un = h->sc_units;  // per sorted position: item, row0, row1, cost
                    un.assign(4 * ((size_t)count[f] * (size_t)std::max(1, kn.roi_tail) + 1), -1);
                    nu = roi_launch_order(members.data() + mfirst[f], count[f], geo.data(), DH, h->n_cu, qslots[f],
                                          kn.roi_tail, sort, false, rg, h->sc_plan, [&](int q, int i, int r0, int r1) {
                                              const int R = (int)(rg(geo[i].cw) & 0xFFFF);
                                              int* u = &un[4 * (size_t)q];
                                              u[0] = i; u[1] = r0; u[2] = r1; u[3] = (r1 - r0 + R - 1) / R;
                                          });
                    std::vector<int>& fr = h->sc_start;
                    std::vector<int>& co = h->sc_bucket;
                    fr.resize(nu);
                    co.resize(nu);
                    for (int q = 0; q < nu; q++) { fr[q] = items[un[4 * q]].src_index; co[q] = un[4 * q + 3]; }
                    roi_xcd_deal(fr.data(), co.data(), nu, n_srcs, h->n_cu, 8, h->sc_slot, h->sc_order);
                    for (int q = 0; q < nu; q++) put_rec(h->sc_slot[q], un[4 * q], un[4 * q + 1], un[4 * q + 2]);
                } else {
                    nu = roi_launch_order(members.data() + mfirst[f], count[f], geo.data(), DH, h->n_cu, qslots[f],
                                          kn.roi_tail, sort, kn.roi_snake != 0, rg, h->sc_plan, put_rec);
                }
                HP(7);
            } else {
                // outputs taller than one tile (DH > TH): row tiles of TH rows per ROI, the same order rules
                std::vector<int>& bucket = h->sc_bucket;
                bucket.resize(n_items);
                std::vector<int>& ord = h->sc_order;
                roi_largest_first(members.data() + mfirst[f], count[f], geo.data(), DH, sort, bucket.data(), ord);
                HP(6);
                std::vector<int>& un = h->sc_units;  // (item, row0, row1, cost) per unit
                un.clear();
                int maxcost = 1;
                for (size_t p = 0; p < ord.size(); p++) {
                    const int i = ord[p];
                    const int R = std::max(1, std::min(std::min(q.buf_bytes / row_bytes_bound(f, geo[i].cw), rcap), DH));
                    for (int t = 0; t < base; t++) {
                        const int y0 = t * q.TH;
                        const int y1 = std::min(DH, (t + 1) * q.TH);
                        const int cost = (y1 - y0 + R - 1) / R;
                        maxcost = std::max(maxcost, cost);
                        un.insert(un.end(), {i, y0, y1, cost});
                    }
                }
                HP(7);
                // stable counting sort of the units by cost, largest first, then the snake deal
                nu = (int)(un.size() / 4);
                std::vector<int>& start = h->sc_start;
                start.assign((size_t)maxcost + 2, 0);
                for (int u = 0; u < nu; u++) start[maxcost - un[4 * u + 3] + 1]++;
                for (int c = 0; c <= maxcost; c++) start[c + 1] += start[c];
                std::vector<int>& order = h->sc_slot;
                order.resize(nu);
                for (int u = 0; u < nu; u++) order[start[maxcost - un[4 * u + 3]]++] = u;
                if (kn.roi_snake) {
                    const int band = std::max(1, h->n_cu);
                    for (int b0 = band; b0 < nu; b0 += 2 * band) std::reverse(order.begin() + b0, order.begin() + std::min(nu, b0 + band));
                }
                for (int pos = 0; pos < nu; pos++) {
                    const int u = order[pos];
                    put_rec(pos, un[4 * u], un[4 * u + 1], un[4 * u + 2]);
                }
            }
            if (dyn_wc && nu > 0) {
                // The records reach device memory before the launch's doorbell. The fence only drains this core's
                // write-combining buffers into the PCIe posted-write stream; a read from the slot cannot complete
                // ahead of those posted writes (PCIe ordering: a read does not pass posted writes), so once it
                // returns every record is in device memory (the HIP runtime publishes host-written device kernel
                // arguments the same way: a read-back of the last byte after the fence).
                _mm_sfence();
                _mm_mfence();
                (void)*reinterpret_cast<const volatile uint32_t*>(reinterpret_cast<const uint8_t*>(&rr[nu - 1]) +
                                                                  sizeof(RoiRec) - 4);
            }
            const int nrec = nu;
            qrec[f] = nrec;
        }
    }
    HP(8);
    const uint8_t* d_block = nullptr;
    {
        HipRings b;
        if (int rc = h->ring.upload(b, h->stream, h->h_block.data(), h->h_block.size(), &d_block)) return rc;
    }
    HP(9);

    // ---- launches ----
    if (h->opt_timing) HIP_TRY(hipEventRecord(h->ev0, h->stream));
    int launches = 0;
    uint32_t kmask = 0;
    const uint32_t fill = (uint32_t)cfg->fill[0] | ((uint32_t)cfg->fill[1] << 8) | ((uint32_t)cfg->fill[2] << 16);
    const int color_rgb = cfg->color_order == EVAM_COLOR_RGB;
    const float* lut_d = reinterpret_cast<const float*>(d_block);
    // Kernel-argument items of one uniform launch: members [m0, m0 + n) of format group f.
    auto fill_args = [&](ItemArg* a, int m0, int n) {
        for (int k = 0; k < n; k++) {
            const int i = members[m0 + k];
            const evam_image& s = srcs[items ? items[i].src_index : i];
            for (int p = 0; p < 3; p++) { a[k].plane[p] = s.planes[p]; a[k].pitch[p] = s.pitch[p]; }
            a[k].x0 = geo[i].x0;
            a[k].y0 = geo[i].y0;
            a[k].index = slots ? slots[i] : i;
        }
    };
    for (int f = 0; f < 4; f++) {
        if (path[f] == kPathNone) continue;
        if (path[f] == kPathRoi) {
            QParams& q = qp[f];
            q.recs = reinterpret_cast<const RoiRec*>(d_dyn + rec_off[f]);
            q.lut = lut_d;
            q.dst = dst->data;
            q.mode = cfg->resize_mode;
            q.placement = cfg->placement;
            q.slot_offset = slot_offset;
            q.slot_stride = slot_stride;
            q.color_rgb = color_rgb;
            q.fill = fill;
            q.prio = kn.prio;
            const int64_t grid = qrec[f];
            if (grid > 0x7FFFFFFF) return fail(EVAM_PP_ERR_INVALID_ARG, "evam_pp_run: too many tiles");
            hipError_t e = launch_roi(f, cfg->out_dtype, kn.roi_px, 2, q, (int)grid, qlds[f], h->stream);
            if (e != hipSuccess) return fail(EVAM_PP_ERR_HIP, "kernel launch failed: %s", hipGetErrorString(e));
            launches++; kmask |= EVAM_KERNEL_ROI;
            continue;
        }
        if (path[f] == kPathUniform) {
            const Geom& g0 = geo[rep[f]];
            const XTab* xt_d = reinterpret_cast<const XTab*>(d_block + tab_off[f]);
            const YTab* yt_d = reinterpret_cast<const YTab*>(xt_d + DW);
            const int per_launch = std::min(count[f], kArgItems);
            if (kn.strip && kn.wave != 2) {
                TParams* tp = &h->sc_tparams;
                int pr = 0, spx = 0, lds = 0, grid = 0;
                const XTab* hx = reinterpret_cast<const XTab*>(h->h_block.data() + tab_off[f]);
                // I420 paired chroma addresses both chroma planes from one buffer resource based at the lower one:
                // for every item, the upper plane's offset from the lower plus its extent must fit the resource's
                // 0x7FFFFFFF bytes (else no pairing for the group)
                bool pair_ok = true;
                if (f == kI420 && kn.strip_pair)
                    for (int m = mfirst[f]; m < mfirst[f + 1] && pair_ok; m++) {
                        const int i = members[m];
                        const evam_image& sr = srcs[items ? items[i].src_index : i];
                        const int64_t d = (int64_t)((intptr_t)sr.planes[2] - (intptr_t)sr.planes[1]);
                        const int64_t ext = (int64_t)sr.pitch[d >= 0 ? 2 : 1] * (sr.height / 2);
                        pair_ok = (d >= 0 ? d : -d) + ext <= (int64_t)0x7FFFFFFF;
                    }
                if (plan_strip(f, g0, DW, DH, count[f], cfg->out_dtype, h->n_cu, hx, reinterpret_cast<const YTab*>(hx + DW),
                               x0_mask[f], kn, pair_ok, *tp, pr, spx, lds, grid)) {
                    tp->lut = lut_d;
                    tp->dst = dst->data;
                    tp->slot_offset = slot_offset;
                    tp->slot_stride = slot_stride;
                    tp->color_rgb = color_rgb;
                    tp->fill = fill;
                    tp->prio = kn.prio;
                    for (int m0 = mfirst[f]; m0 < mfirst[f + 1]; m0 += kArgItems) {
                        const int nm = std::min(kArgItems, mfirst[f + 1] - m0);
                        fill_args(tp->items, m0, nm);
                        // grid (tile column, tile row, item), dispatched in that order (the C2 data movement in
                        // the strip pattern takes 1.7 us longer with each XCD on its own run of tiles,
                        // profiles/r03c_strip_bw.txt)
                        const dim3 gr((unsigned)tp->tiles_x, (unsigned)((DH + tp->TH - 1) / tp->TH), (unsigned)nm);
                        hipError_t e = launch_strip(f, cfg->out_dtype, pr, spx, *tp, gr, lds, h->stream);
                        if (e != hipSuccess) return fail(EVAM_PP_ERR_HIP, "kernel launch failed: %s", hipGetErrorString(e));
                        launches++; kmask |= EVAM_KERNEL_STRIP;
                    }
                    (void)grid;
                    continue;
                }
            }
            if (kn.band && kn.wave != 2 && kn.strip != 2) {
                TParams* tp = &h->sc_tparams;
                int bpx = 0, nw = 0, lds = 0;
                bool dd = false;
                const XTab* hx = reinterpret_cast<const XTab*>(h->h_block.data() + tab_off[f]);
                if (plan_band(f, g0, DW, DH, count[f], cfg->out_dtype, h->n_cu, hx, reinterpret_cast<const YTab*>(hx + DW),
                              x0_mask[f], kn, *tp, bpx, dd, nw, lds)) {
                    tp->lut = lut_d;
                    tp->dst = dst->data;
                    tp->slot_offset = slot_offset;
                    tp->slot_stride = slot_stride;
                    tp->color_rgb = color_rgb;
                    tp->fill = fill;
                    tp->prio = kn.prio;
                    tp->ahead = std::max(0, kn.band_ahead);
                    for (int m0 = mfirst[f]; m0 < mfirst[f + 1]; m0 += kArgItems) {
                        const int nm = std::min(kArgItems, mfirst[f + 1] - m0);
                        fill_args(tp->items, m0, nm);
                        tp->units = nm * tp->tiles_per_item;
                        const dim3 gr((unsigned)tp->tiles_x, (unsigned)((DH + tp->TH - 1) / tp->TH), (unsigned)nm);
                        hipError_t e = launch_band(f, cfg->out_dtype, bpx, dd, *tp, gr, nw, lds, h->stream);
                        if (e != hipSuccess) return fail(EVAM_PP_ERR_HIP, "kernel launch failed: %s", hipGetErrorString(e));
                        launches++; kmask |= EVAM_KERNEL_BAND;
                    }
                    continue;
                }
            }
            if (kn.wave) {
                WParams w{};
                int px = 0, lds = 0, grid = 0;
                bool reuse = false;
                const XTab* hx = reinterpret_cast<const XTab*>(h->h_block.data() + tab_off[f]);
                // The wave kernel wins where consecutive output rows share source rows (vertical
                // upscale: REUSE); for downscales the staged kernel's deeper shared staging is faster.
                if (plan_wave(f, g0, DW, DH, count[f], cfg->out_dtype, h->n_cu, hx,
                              reinterpret_cast<const YTab*>(hx + DW), x0_mask[f], kn, w, px, reuse, lds, grid) &&
                    (reuse || kn.wave == 2)) {
                    w.ox = g0.ox;
                    w.rw = g0.rw;
                    w.lut = lut_d;
                    w.xtab = xt_d;
                    w.ytab = yt_d;
                    w.dst = dst->data;
                    w.slot_offset = slot_offset;
                    w.slot_stride = slot_stride;
                    w.color_rgb = color_rgb;
                    w.fill = fill;
                    for (int m0 = mfirst[f]; m0 < mfirst[f + 1]; m0 += kArgItems) {
                        const int n = std::min(kArgItems, mfirst[f + 1] - m0);
                        fill_args(w.items, m0, n);
                        hipError_t e = launch_wave(f, cfg->out_dtype, px, reuse, w, n * w.tiles_per_item, lds, h->stream);
                        if (e != hipSuccess) return fail(EVAM_PP_ERR_HIP, "kernel launch failed: %s", hipGetErrorString(e));
                        launches++; kmask |= EVAM_KERNEL_WAVE;
                    }
                    continue;
                }
            }
            // Tile width: the widest of 256 / 128 columns whose staged row segment (the exact widest footprint of
            // any tile and crop origin of this group) fits the kernel's 1 KB slot.
            const XTab* hx = reinterpret_cast<const XTab*>(h->h_block.data() + tab_off[f]);
            auto seg_bytes = [&](int tw) {
                int mY = 0, mC = 0;
                wave_segments(f, g0.ox, g0.rw, DW, hx, x0_mask[f], tw, mY, mC);
                return 16 * std::max(1, std::max(mY, mC));
            };
            int nsegx = 0;
            if (kn.staged)
                for (int n : {4, 2}) {  // (64 columns would need R % 4 == 0: the row kernel serves those)
                    if (seg_bytes(64 * n) <= kSlot) { nsegx = n; break; }
                }
            if (nsegx && kn.nsegx > 0 && kn.nsegx < nsegx && 2 % (4 / kn.nsegx) == 0) nsegx = kn.nsegx;
            if (nsegx) {
                // Pipeline shape: R output rows per group, NBUF staging buffers (NBUF - 1 groups of DMA in
                // flight).
                int R = kn.stage_r > 0 ? kn.stage_r : 2, nbuf = 2;
                bool shape_ok = false;
                for (const StagedShape& ss : kStagedShapes) shape_ok |= ss.R == R && ss.nbuf == nbuf;
                if (!shape_ok || !staged_valid(nsegx, R)) { R = 2; nbuf = 2; }
                SParams sp{};
                sp.ox = g0.ox;
                sp.rw = g0.rw;
                sp.lut = lut_d;
                sp.xtab = xt_d;
                sp.ytab = yt_d;
                sp.dst = dst->data;
                sp.slot_offset = slot_offset;
                sp.slot_stride = slot_stride;
                sp.DW = DW; sp.DH = DH;
                const int tw = 64 * nsegx;
                sp.tiles_x = (DW + tw - 1) / tw;
                // ~4096 pixels per workgroup, but short enough tiles that small batches still put
                // 8 workgroups on every CU (a whole clip-ring step is only 32 x 224 x 224 pixels).
                // At most 16 rows: C4 (tw 128) runs 3-7 % faster at 16 than at 32 (profiles/r01ad_sweep_th*.txt).
                int th = std::max(2, std::min(16, 4096 / tw));
                const int64_t cols = (int64_t)per_launch * sp.tiles_x;
                const int64_t want = 8 * (int64_t)h->n_cu;
                if (cols * ((DH + th - 1) / th) < want) th = (int)std::max<int64_t>(2, cols * DH / want);
                sp.TH = std::max(1, std::min(std::min(DH, 64), kn.th > 0 ? kn.th : th));  // <= 64: lane-held rows
                sp.TH = std::min(64, (sp.TH + R - 1) / R * R);
                sp.tiles_per_item = sp.tiles_x * ((DH + sp.TH - 1) / sp.TH);
                const int np = f == kI420 ? 3 : (f == kNV12 ? 2 : 1);
                sp.offBuf = cfg->out_dtype == EVAM_DTYPE_F32 ? kLutBytes : 0;
                sp.slot_bytes = seg_bytes(tw);  // <= the kernel's SLOT_MAX (tile choice above)
                sp.buf_bytes = 2 * R * np * sp.slot_bytes;
                sp.ntcol = sp.tiles_x <= kTCols ? sp.tiles_x : 0;
                for (int c = 0; c < sp.ntcol; c++) {
                    const int Xv0 = std::max(c * tw, g0.ox), Xv1 = std::min(std::min(c * tw + tw, DW), g0.ox + g0.rw) - 1;
                    sp.tcol[c] = Xv0 <= Xv1 ? int2{hx[Xv0].s0, hx[Xv1].s1} : int2{-1, -1};
                }
                sp.color_rgb = color_rgb;
                sp.fill = fill;
                const int lds = sp.offBuf + nbuf * sp.buf_bytes;
                for (int m0 = mfirst[f]; m0 < mfirst[f + 1]; m0 += kArgItems) {
                    const int n = std::min(kArgItems, mfirst[f + 1] - m0);
                    fill_args(sp.items, m0, n);
                    const int64_t grid = (int64_t)n * sp.tiles_per_item;
                    if (grid > 0x7FFFFFFF) return fail(EVAM_PP_ERR_INVALID_ARG, "evam_pp_run: too many tiles");
                    // XCD-contiguous tiles: C2 -1.4 %, C4 -3 % kernel time; a grid of one workgroup round or
                    // less (C5) gains nothing (profiles/r01ae_sweep_xcd.txt). EVAM_PP_XCD=0/1 forces it.
                    sp.xcd_remap = kn.xcd >= 0 ? kn.xcd : (int)(grid >= 8 * (int64_t)h->n_cu);
                    hipError_t e = launch_staged(f, cfg->out_dtype, nsegx, R, nbuf, sp, (int)grid, lds, h->stream);
                    if (e != hipSuccess) return fail(EVAM_PP_ERR_HIP, "kernel launch failed: %s", hipGetErrorString(e));
                    launches++; kmask |= EVAM_KERNEL_STAGED;
                }
                continue;
            }
            const RowCfg rc = choose_row_tiles(DW, DH, kn);
            RParams r{};
            r.ox = g0.ox;
            r.rw = g0.rw;
            r.lut = lut_d;
            r.xtab = xt_d;
            r.ytab = yt_d;
            r.dst = dst->data;
            r.slot_offset = slot_offset;
            r.slot_stride = slot_stride;
            r.DW = DW; r.DH = DH;
            r.TW = rc.TW; r.TH = rc.TH;
            r.tiles_x = (DW + rc.TW - 1) / rc.TW;
            r.tiles_per_item = r.tiles_x * ((DH + rc.TH - 1) / rc.TH);
            r.nsegx = rc.TW / 64;
            r.color_rgb = color_rgb;
            r.fill = fill;
            const int lds = cfg->out_dtype == EVAM_DTYPE_F32 ? kLutBytes : 0;
            for (int m0 = mfirst[f]; m0 < mfirst[f + 1]; m0 += kArgItems) {
                const int n = std::min(kArgItems, mfirst[f + 1] - m0);
                fill_args(r.items, m0, n);
                const int64_t grid = (int64_t)n * r.tiles_per_item;
                if (grid > 0x7FFFFFFF) return fail(EVAM_PP_ERR_INVALID_ARG, "evam_pp_run: too many tiles");
                hipError_t e = launch_rows(f, cfg->out_dtype, r, (int)grid, lds, h->stream);
                if (e != hipSuccess) return fail(EVAM_PP_ERR_HIP, "kernel launch failed: %s", hipGetErrorString(e));
                launches++; kmask |= EVAM_KERNEL_ROWS;
            }
            continue;
        }
        const ItemDesc* items_d = reinterpret_cast<const ItemDesc*>(d_block + desc_off) + first[f];
        const TileCfg t = choose_tiles(DW, DH, cfg->out_dtype, kn);
        KParams p{};
        p.items = items_d;
        p.lut = lut_d;
        p.dst = dst->data;
        p.slot_offset = slot_offset;
        p.slot_stride = slot_stride;
        p.DW = DW; p.DH = DH;
        p.TW = t.TW; p.TH = t.TH;
        p.tiles_x = (DW + t.TW - 1) / t.TW;
        const int tiles_y = (DH + t.TH - 1) / t.TH;
        p.tiles_per_item = p.tiles_x * tiles_y;
        const int64_t n_tiles = (int64_t)count[f] * p.tiles_per_item;
        if (n_tiles > 0x7FFFFFFF) return fail(EVAM_PP_ERR_INVALID_ARG, "evam_pp_run: too many tiles");
        p.n_tiles = (int)n_tiles;
        p.tw_magic = t.TW > 1 ? (uint32_t)(0xFFFFFFFFu / (uint32_t)t.TW) + 1u : 0u;
        p.offCol = t.offCol; p.offRow = t.offRow;
        p.color_rgb = color_rgb;
        p.fill = fill;
        const int lds = t.lds;
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
        hipError_t e = launch(f, cfg->out_dtype, p, (int)n_tiles, lds, h->stream);
        if (e != hipSuccess) return fail(EVAM_PP_ERR_HIP, "kernel launch failed: %s", hipGetErrorString(e));
        launches++; kmask |= EVAM_KERNEL_GENERIC;
    }
    if (any_roi) {
        HipRings b;
        if (int rc = h->pin.fence(b, h->stream)) return rc;
        pin_guard.armed = false;
    }
    if (h->opt_timing) HIP_TRY(hipEventRecord(h->ev1, h->stream));
    h->timed = h->opt_timing != 0;
#ifdef EVAM_PP_HOST_PROF
    HP(10);
    static long hp_calls = 0;
    if (++hp_calls > 200) {  // steady state: past warm-up, allocations and code-object loading
        for (int i = 0; i < 12; i++) g_hp[i] += hp_t[i];
        g_hp_n++;
    }
#endif

    h->stats.n_items = n_items;
    h->stats.n_launches = launches;
    h->stats.kernels = kmask;
    h->stats.src_bytes = h->opt_stats ? src_bytes : 0;
    h->stats.dst_bytes = (int64_t)n_items * plane * 3 * esz;
    return EVAM_PP_OK;
}

}  // namespace

extern "C" {

int evam_pp_run(evam_pp* h, const evam_image* srcs, int n_srcs, const evam_roi* items, int n_items,
                const evam_preproc* cfg, const evam_tensor* dst, evam_transform* out_xform) {
    return run_impl(h, srcs, n_srcs, items, n_items, cfg, dst, nullptr, out_xform);
}

int evam_pp_run_slots(evam_pp* h, const evam_image* srcs, int n_srcs, const evam_roi* items, int n_items,
                      const evam_preproc* cfg, const evam_tensor* dst, const int32_t* slots, evam_transform* out_xform) {
    if (!slots) return fail(EVAM_PP_ERR_INVALID_ARG, "evam_pp_run_slots: slots is NULL");
    return run_impl(h, srcs, n_srcs, items, n_items, cfg, dst, slots, out_xform);
}

}  // extern "C"
