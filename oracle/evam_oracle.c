/*
 * evam_oracle.c — CPU ORACLE. TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library, and
 * only as the checker / the timed CPU baseline. The product path (libevam_pp.so) never links it.
 *
 * What it restates. The reference (intel/edge-video-analytics-microservice v0.7.2) has no native code:
 * its pre-process hot path is DL Streamer 2022.1's `opencv` pre-proc backend inside gvadetect /
 * gvaclassify / gvaactionrecognitionbin (selected at pipelines/object_detection/vehicle/pipeline.json:5,
 * pipelines/object_classification/vehicle_attributes/pipeline.json:4-5,
 * pipelines/action_recognition/general/pipeline.json:3-4), which calls OpenCV. Both are third-party
 * dependencies pinned by the base image intel/dlstreamer-pipeline-server:2022.1.1-ubuntu20
 * (docker-compose-build.yml:37; OpenCV 4.5.x bundled) and are NOT present in /root/reference or in
 * this container. This file restates their published algorithms:
 *   - OpenCV modules/imgproc/src/color_yuv.simd.hpp: ITU-R BT.601 YUV420 -> BGR, 20-bit fixed point
 *     (uvToRGBuv / yRGBuvToRGBA), chroma nearest (one UV sample per 2x2 luma block).
 *   - OpenCV modules/imgproc/src/resize.cpp: hal::resize coefficient tables (fx = (float)((dx+0.5)*
 *     scale-0.5), scale = 1/(dsize/ssize) in double, 11-bit saturate_cast<short> weights, x-border fx
 *     reset, y rows clipped but fy kept) + HResizeLinear<uchar,int,short,2048> +
 *     VResizeLinear<uchar,int,short,FixedPtCast<int,uchar,22>,VResizeLinearVec_32s8u> specialisation:
 *     dst = (((b0*(D0>>4))>>16) + ((b1*(D1>>4))>>16) + 2) >> 2.
 *   - OpenCV Mat::convertTo(CV_32F, alpha, beta) then per-channel subtract(mean) / divide(std).
 *   - DL Streamer 2022.1 opencv pre-proc order: crop -> colour convert -> resize (no-aspect |
 *     aspect-ratio [+ central crop]) -> colour-space swap -> range / mean / std -> planar split into
 *     batch slot. The in-tree model-procs that pin the parameters are
 *     models_list/vehicle-detection-0202.json:3 and models_list/action-recognition-0001.json:3-13.
 *
 * PARITY UNPINNED. The reference has no tests, fixtures or golden vectors for this path (SURVEY.md
 * §4, §8c), OpenCV / DL Streamer cannot be built or imported here, and no cv2 exists on the GPU box.
 * This restatement is checked against the known-answer values of SURVEY.md §8(a) (BT.601 KATs and
 * resize coefficient tables), against an independent numpy restatement (oracle/oracle.py), and against
 * torch bilinear (+-1 LSB) — not against reference outputs.
 *
 * Build: make -C oracle   (gcc -O2 -fopenmp -ffp-contract=off; no FMA contraction, matching OpenCV's
 * scalar table code).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define ORC_NV12 0x3231564E
#define ORC_I420 0x30323449
#define ORC_BGRX 0x58524742
#define ORC_BGRA 0x41524742
#define ORC_BGR 0x20524742

/* OpenCV color_yuv.simd.hpp ITUR_BT_601_* */
#define BT601_SHIFT 20
#define BT601_CY 1220542
#define BT601_CUB 2116026
#define BT601_CUG (-409993)
#define BT601_CVG (-852492)
#define BT601_CVR 1673527

#define RESIZE_COEF_BITS 11
#define RESIZE_COEF_SCALE (1 << RESIZE_COEF_BITS)

static inline int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
static inline uint8_t sat8(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

/* OpenCV uvToRGBuv + yRGBuvToRGBA, output B,G,R. */
void orc_yuv_pixel(int Y, int U, int V, uint8_t bgr[3]) {
    int uu = U - 128, vv = V - 128;
    int ruv = (1 << (BT601_SHIFT - 1)) + BT601_CVR * vv;
    int guv = (1 << (BT601_SHIFT - 1)) + BT601_CVG * vv + BT601_CUG * uu;
    int buv = (1 << (BT601_SHIFT - 1)) + BT601_CUB * uu;
    int y = (Y - 16 > 0 ? Y - 16 : 0) * BT601_CY;
    bgr[0] = sat8((y + buv) >> BT601_SHIFT);
    bgr[1] = sat8((y + guv) >> BT601_SHIFT);
    bgr[2] = sat8((y + ruv) >> BT601_SHIFT);
}

/* OpenCV cvFloor(float) */
static inline int cv_floor_f(float v) {
    int i = (int)v;
    return i - (i > v);
}

/* saturate_cast<short>(float): cvRound (round half to even under the default FP environment). */
static inline short sat_short_f(float v) {
    long r = lrintf(v);
    return (short)(r < -32768 ? -32768 : (r > 32767 ? 32767 : r));
}

/*
 * OpenCV hal::resize INTER_LINEAR table for one axis (resize.cpp, the `for(dx...)` / `for(dy...)`
 * loops of the generic path with ksize = 2, area_mode = false, fixpt = true).
 * x axis: sx < 0 -> sx = 0, fx = 0; sx >= ssize-1 -> sx = ssize-1, fx = 0.
 * y axis: sy kept raw (rows are clipped later by resizeGeneric_Invoker), fy kept.
 */
void orc_linear_table(int ssize, int dsize, int is_x, int32_t* ofs, int16_t* c0, int16_t* c1) {
    double inv_scale = (double)dsize / ssize;
    double scale = 1. / inv_scale;
    for (int d = 0; d < dsize; d++) {
        float f = (float)((d + 0.5) * scale - 0.5);
        int s = cv_floor_f(f);
        f -= s;
        if (is_x) {
            if (s < 0) { f = 0.f; s = 0; }
            if (s >= ssize - 1) { f = 0.f; s = ssize - 1; }
        }
        ofs[d] = s;
        c0[d] = sat_short_f((1.f - f) * RESIZE_COEF_SCALE);
        c1[d] = sat_short_f(f * RESIZE_COEF_SCALE);
    }
}

/* Colour-convert a w x h window (origin x0,y0, even for 4:2:0) of a frame to packed BGR (cvtColor). */
void orc_to_bgr(int fourcc, const uint8_t* const planes[3], const int pitch[3], int x0, int y0, int w,
                int h, uint8_t* bgr) {
    #pragma omp parallel for schedule(static)
    for (int i = 0; i < h; i++) {
        int y = y0 + i;
        uint8_t* out = bgr + (size_t)i * w * 3;
        const uint8_t* prow = planes[0] + (size_t)y * pitch[0];
        for (int j = 0; j < w; j++) {
            int x = x0 + j;
            switch (fourcc) {
            case ORC_NV12: {
                const uint8_t* uv = planes[1] + (size_t)(y >> 1) * pitch[1] + 2 * (x >> 1);
                orc_yuv_pixel(prow[x], uv[0], uv[1], out + 3 * j);
                break;
            }
            case ORC_I420: {
                int U = planes[1][(size_t)(y >> 1) * pitch[1] + (x >> 1)];
                int V = planes[2][(size_t)(y >> 1) * pitch[2] + (x >> 1)];
                orc_yuv_pixel(prow[x], U, V, out + 3 * j);
                break;
            }
            case ORC_BGRX:
            case ORC_BGRA:
                memcpy(out + 3 * j, prow + 4 * x, 3); /* COLOR_BGRA2BGR */
                break;
            default: /* ORC_BGR */
                memcpy(out + 3 * j, prow + 3 * x, 3);
                break;
            }
        }
    }
}

/*
 * cv::resize(src, dst, Size(dw, dh), 0, 0, INTER_LINEAR) on packed u8 BGR (resizeGeneric_ with
 * HResizeLinear / VResizeLinear 32s8u). Equal sizes are a copy in OpenCV; the table path gives the same
 * bytes. An exact 2x2 downscale switches OpenCV to INTER_AREA fast, which is also byte-identical to the
 * table path ((p+q+r+s+2)>>2 both ways), so no special case is needed.
 */
void orc_resize_linear_c3(const uint8_t* src, int sw, int sh, int sstep, uint8_t* dst, int dw, int dh,
                          int dstep) {
    int32_t* xofs = (int32_t*)malloc(sizeof(int32_t) * dw);
    int16_t* xa0 = (int16_t*)malloc(sizeof(int16_t) * dw);
    int16_t* xa1 = (int16_t*)malloc(sizeof(int16_t) * dw);
    int32_t* yofs = (int32_t*)malloc(sizeof(int32_t) * dh);
    int16_t* yb0 = (int16_t*)malloc(sizeof(int16_t) * dh);
    int16_t* yb1 = (int16_t*)malloc(sizeof(int16_t) * dh);
    orc_linear_table(sw, dw, 1, xofs, xa0, xa1);
    orc_linear_table(sh, dh, 0, yofs, yb0, yb1);
    #pragma omp parallel
    {
        int32_t* D0 = (int32_t*)malloc(sizeof(int32_t) * dw * 3);
        int32_t* D1 = (int32_t*)malloc(sizeof(int32_t) * dw * 3);
        #pragma omp for schedule(static)
        for (int dy = 0; dy < dh; dy++) {
            int sy0 = clampi(yofs[dy], 0, sh - 1);     /* clip(sy0 - ksize2 + 1 + k, 0, ssize.height) */
            int sy1 = clampi(yofs[dy] + 1, 0, sh - 1);
            const uint8_t* S0 = src + (size_t)sy0 * sstep;
            const uint8_t* S1 = src + (size_t)sy1 * sstep;
            for (int dx = 0; dx < dw; dx++) {
                int sx = xofs[dx];
                int sx1 = sx + 1 < sw ? sx + 1 : sw - 1; /* weight is 0 whenever this clamps */
                int a0 = xa0[dx], a1 = xa1[dx];
                for (int c = 0; c < 3; c++) {
                    D0[dx * 3 + c] = S0[sx * 3 + c] * a0 + S0[sx1 * 3 + c] * a1;
                    D1[dx * 3 + c] = S1[sx * 3 + c] * a0 + S1[sx1 * 3 + c] * a1;
                }
            }
            int b0 = yb0[dy], b1 = yb1[dy];
            uint8_t* out = dst + (size_t)dy * dstep;
            for (int k = 0; k < dw * 3; k++)
                out[k] = (uint8_t)((((b0 * (D0[k] >> 4)) >> 16) + ((b1 * (D1[k] >> 4)) >> 16) + 2) >> 2);
        }
        free(D0);
        free(D1);
    }
    free(xofs); free(xa0); free(xa1); free(yofs); free(yb0); free(yb1);
}

/*
 * Normalisation table: the fp32 value of a u8 sample in output channel c, computed in the reference's
 * operation order with one rounding per operation (convertTo: (float)u*alpha + beta; subtract; divide).
 */
void orc_norm_lut(int norm_flags, const float range[2], const float mean[3], const float std_[3],
                  float* lut /* [3][256] */) {
    float alpha = (float)(((double)range[1] - (double)range[0]) / 255.0);
    float beta = range[0];
    for (int c = 0; c < 3; c++) {
        for (int u = 0; u < 256; u++) {
            volatile float v = (float)u;
            if (norm_flags & 1) {
                volatile float m = v * alpha;
                v = m + beta;
            }
            if (norm_flags & 2) {
                volatile float s = v - mean[c];
                v = s / std_[c];
            }
            lut[c * 256 + u] = v;
        }
    }
}

/* Geometry of one item (shared semantics with the C ABI's evam_roi / evam_preproc docs). */
typedef struct orc_geom {
    int x0, y0, cw, ch; /* effective crop */
    int rw, rh;         /* resized size   */
    int ox, oy;         /* placement of the resized image in the DW x DH plane */
} orc_geom;

int orc_item_geometry(int fourcc, int W, int H, int x, int y, int w, int h, int mode, int placement,
                      int DW, int DH, orc_geom* g) {
    int x0, y0, x1, y1;
    if (w <= 0 || h <= 0) {
        x0 = 0; y0 = 0; x1 = W; y1 = H;
    } else {
        x0 = clampi(x, 0, W); y0 = clampi(y, 0, H);
        /* x + w in 64 bits: caller-supplied int32 rects may overflow int */
        long long xe = (long long)x + w, ye = (long long)y + h;
        x1 = xe < 0 ? 0 : (xe > W ? W : (int)xe);
        y1 = ye < 0 ? 0 : (ye > H ? H : (int)ye);
        if (fourcc == ORC_NV12 || fourcc == ORC_I420) {
            x0 &= ~1; y0 &= ~1;
            x1 = (x1 + 1) & ~1; if (x1 > W) x1 = W;
            y1 = (y1 + 1) & ~1; if (y1 > H) y1 = H;
        }
    }
    if (x1 - x0 <= 0 || y1 - y0 <= 0) return -4;
    g->x0 = x0; g->y0 = y0; g->cw = x1 - x0; g->ch = y1 - y0;
    int cw = g->cw, ch = g->ch;
    g->ox = 0; g->oy = 0;
    if (mode == 0) {
        g->rw = DW; g->rh = DH;
    } else {
        double sx = (double)DW / cw, sy = (double)DH / ch;
        int x_dominant = (mode == 1) ? (sx <= sy) : (sx >= sy);
        if (x_dominant) {
            g->rw = DW;
            g->rh = (int)(ch * sx);
        } else {
            g->rh = DH;
            g->rw = (int)(cw * sy);
        }
        if (g->rw < 1) g->rw = 1;
        if (g->rh < 1) g->rh = 1;
        if (mode == 1) {
            if (g->rw > DW) g->rw = DW;
            if (g->rh > DH) g->rh = DH;
            if (placement == 1) { g->ox = (DW - g->rw) / 2; g->oy = (DH - g->rh) / 2; }
        } else {
            if (g->rw < DW) g->rw = DW;
            if (g->rh < DH) g->rh = DH;
            g->ox = -((g->rw - DW) / 2);
            g->oy = -((g->rh - DH) / 2);
        }
    }
    return 0;
}

/*
 * Full reference path for one item, writing planar slot `slot` of an N x 3 x DH x DW tensor
 * (u8 when out_f32 == 0, else fp32 through `lut`). color_rgb swaps B and R in the output planes.
 * fill[c] is the u8 value of padded pixels in OUTPUT channel c.
 */
int orc_preprocess_item(int fourcc, const uint8_t* const planes[3], const int pitch[3], int W, int H,
                        int x, int y, int w, int h, int mode, int placement, int color_rgb, int out_f32,
                        const float* lut, const uint8_t fill[3], void* dst, int slot, int DW, int DH,
                        int32_t* geom_out /* 8 ints or NULL */) {
    orc_geom g;
    int rc = orc_item_geometry(fourcc, W, H, x, y, w, h, mode, placement, DW, DH, &g);
    if (rc) return rc;
    if (geom_out) {
        geom_out[0] = g.x0; geom_out[1] = g.y0; geom_out[2] = g.cw; geom_out[3] = g.ch;
        geom_out[4] = g.rw; geom_out[5] = g.rh; geom_out[6] = g.ox; geom_out[7] = g.oy;
    }
    uint8_t* bgr = (uint8_t*)malloc((size_t)g.cw * g.ch * 3);
    uint8_t* rs = (uint8_t*)malloc((size_t)g.rw * g.rh * 3);
    orc_to_bgr(fourcc, planes, pitch, g.x0, g.y0, g.cw, g.ch, bgr);
    orc_resize_linear_c3(bgr, g.cw, g.ch, g.cw * 3, rs, g.rw, g.rh, g.rw * 3);
    size_t plane = (size_t)DW * DH;
    #pragma omp parallel for schedule(static)
    for (int Y = 0; Y < DH; Y++) {
        int dy = Y - g.oy;
        for (int X = 0; X < DW; X++) {
            int dx = X - g.ox;
            uint8_t px[3];
            if (dx >= 0 && dx < g.rw && dy >= 0 && dy < g.rh) {
                const uint8_t* s = rs + ((size_t)dy * g.rw + dx) * 3;
                px[0] = color_rgb ? s[2] : s[0];
                px[1] = s[1];
                px[2] = color_rgb ? s[0] : s[2];
            } else {
                px[0] = fill[0]; px[1] = fill[1]; px[2] = fill[2];
            }
            for (int c = 0; c < 3; c++) {
                size_t idx = ((size_t)slot * 3 + c) * plane + (size_t)Y * DW + X;
                if (out_f32)
                    ((float*)dst)[idx] = lut[c * 256 + px[c]];
                else
                    ((uint8_t*)dst)[idx] = px[c];
            }
        }
    }
    free(bgr);
    free(rs);
    return 0;
}

int orc_num_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

void orc_set_num_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}
