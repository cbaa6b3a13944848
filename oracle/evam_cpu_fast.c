/*
 * evam_cpu_fast.c — CPU BASELINE. TEST / BENCH INFRASTRUCTURE ONLY (linked into libevam_oracle.so).
 *
 * Only bench.py's cpu_baseline leg and tests/ load it; the product path (libevam_pp.so) never does.
 *
 * The same arithmetic as evam_oracle.c (OpenCV 4.5.x color_yuv BT.601 20-bit fixed point, resize.cpp
 * INTER_LINEAR 11-bit tables with HResizeLinear / VResizeLinearVec_32s8u, convertTo + subtract/divide
 * through the reference-order LUT; DL Streamer 2022.1 opencv pre-proc order crop -> convert -> resize ->
 * swap -> normalise -> planar slot), organised the way OpenCV's own optimised CPU path runs it, so that
 * the bench's CPU column is what a host can actually do rather than a scalar restatement:
 *   - one OpenMP region over (item, stripe of output rows) tasks for the whole batch (OpenCV's
 *     parallel_for_ stripes), per-thread scratch reused across tasks, no per-item allocation;
 *   - resizeGeneric_Invoker's row cache: each needed source row is converted and horizontally resized
 *     once into an int row (two-row ring keyed by source row), then every output row is one vertical
 *     pass over two cached rows;
 *   - planar B / G / R rows and branch-free inner loops that gcc auto-vectorises (-O3, AVX2 target).
 * It must stay byte-identical to evam_oracle.c (tests/test_oracle.py::test_cpu_fast_matches_oracle).
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

#define BT601_SHIFT 20
#define BT601_CY 1220542
#define BT601_CUB 2116026
#define BT601_CUG (-409993)
#define BT601_CVG (-852492)
#define BT601_CVR 1673527

typedef struct orc_frame {
    const uint8_t* planes[3];
    int32_t pitch[3];
    int32_t fourcc, width, height, pad_;
} orc_frame;

/* from evam_oracle.c (same translation unit family, same rules) */
typedef struct orc_geom {
    int x0, y0, cw, ch, rw, rh, ox, oy;
} orc_geom;
int orc_item_geometry(int fourcc, int W, int H, int x, int y, int w, int h, int mode, int placement, int DW,
                      int DH, orc_geom* g);
void orc_linear_table(int ssize, int dsize, int is_x, int32_t* ofs, int16_t* c0, int16_t* c1);

static inline uint8_t sat8(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }
static inline int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

typedef struct scratch {
    size_t cap_w, cap_r, cap_t;
    uint8_t* bgr;   /* 3 planar rows of the crop width */
    int32_t* D;     /* 2 cached rows x 3 channels x rw */
    int32_t* xofs;  /* tables */
    int16_t* xa;    /* xa0 | xa1 */
    int32_t* yofs;
    int16_t* yb;
} scratch;

static void scratch_fit(scratch* s, int cw, int rw, int rh) {
    if ((size_t)cw > s->cap_w) {
        free(s->bgr);
        s->cap_w = (size_t)cw;
        s->bgr = (uint8_t*)malloc(3 * s->cap_w + 64);
    }
    if ((size_t)rw > s->cap_r) {
        free(s->D); free(s->xofs); free(s->xa);
        s->cap_r = (size_t)rw;
        s->D = (int32_t*)malloc(sizeof(int32_t) * 6 * s->cap_r);
        s->xofs = (int32_t*)malloc(sizeof(int32_t) * s->cap_r);
        s->xa = (int16_t*)malloc(sizeof(int16_t) * 2 * s->cap_r);
    }
    if ((size_t)rh > s->cap_t) {
        free(s->yofs); free(s->yb);
        s->cap_t = (size_t)rh;
        s->yofs = (int32_t*)malloc(sizeof(int32_t) * s->cap_t);
        s->yb = (int16_t*)malloc(sizeof(int16_t) * 2 * s->cap_t);
    }
}

/* cvtColor of crop row `r` (absolute row y0 + r) into planar B, G, R rows of cw pixels. */
static void convert_row(const orc_frame* f, int x0, int y, int cw, uint8_t* restrict B, uint8_t* restrict G,
                        uint8_t* restrict R) {
    const uint8_t* restrict Y = f->planes[0] + (size_t)y * f->pitch[0];
    if (f->fourcc == ORC_NV12 || f->fourcc == ORC_I420) {
        const uint8_t* restrict Yr = Y + x0;
        const uint8_t* restrict U;
        const uint8_t* restrict V;
        int step;
        if (f->fourcc == ORC_NV12) {
            U = f->planes[1] + (size_t)(y >> 1) * f->pitch[1] + x0;  /* x0 even: UV pair of column x0 */
            V = U + 1;
            step = 2;
        } else {
            U = f->planes[1] + (size_t)(y >> 1) * f->pitch[1] + (x0 >> 1);
            V = f->planes[2] + (size_t)(y >> 1) * f->pitch[2] + (x0 >> 1);
            step = 1;
        }
        const int half = 1 << (BT601_SHIFT - 1);
        for (int k = 0; k < cw / 2; k++) {
            const int u = U[step * k] - 128, v = V[step * k] - 128;
            const int ruv = half + BT601_CVR * v;
            const int guv = half + BT601_CVG * v + BT601_CUG * u;
            const int buv = half + BT601_CUB * u;
            const int ya = (Yr[2 * k] > 16 ? Yr[2 * k] - 16 : 0) * BT601_CY;
            const int yb = (Yr[2 * k + 1] > 16 ? Yr[2 * k + 1] - 16 : 0) * BT601_CY;
            B[2 * k] = sat8((ya + buv) >> BT601_SHIFT);
            G[2 * k] = sat8((ya + guv) >> BT601_SHIFT);
            R[2 * k] = sat8((ya + ruv) >> BT601_SHIFT);
            B[2 * k + 1] = sat8((yb + buv) >> BT601_SHIFT);
            G[2 * k + 1] = sat8((yb + guv) >> BT601_SHIFT);
            R[2 * k + 1] = sat8((yb + ruv) >> BT601_SHIFT);
        }
        return;
    }
    const int bpp = f->fourcc == ORC_BGR ? 3 : 4;  /* COLOR_BGRA2BGR drops X / A */
    const uint8_t* restrict p = Y + (size_t)x0 * bpp;
    for (int j = 0; j < cw; j++) {
        B[j] = p[bpp * j];
        G[j] = p[bpp * j + 1];
        R[j] = p[bpp * j + 2];
    }
}

/* HResizeLinear<uchar, int, short, 2048> of one planar channel row. */
static void hresize(const uint8_t* restrict S, int cw, const int32_t* restrict xofs, const int16_t* restrict xa0,
                    const int16_t* restrict xa1, int rw, int32_t* restrict D) {
    for (int dx = 0; dx < rw; dx++) {
        const int sx = xofs[dx];
        const int sx1 = sx + 1 < cw ? sx + 1 : cw - 1;  /* its weight is 0 whenever this clamps */
        D[dx] = S[sx] * xa0[dx] + S[sx1] * xa1[dx];
    }
}

/* One (item, output rows [Y0, Y1)) task. */
static void run_task(const orc_frame* f, const orc_geom* g, int color_rgb, int out_f32, const float* lut,
                     const uint8_t fill[3], void* dst, size_t slot, int DW, int DH, int Y0, int Y1, scratch* s) {
    const int cw = g->cw, ch = g->ch, rw = g->rw, rh = g->rh;
    scratch_fit(s, cw, rw, rh);
    int32_t* xofs = s->xofs;
    int16_t* xa0 = s->xa;
    int16_t* xa1 = s->xa + rw;
    int32_t* yofs = s->yofs;
    int16_t* yb0 = s->yb;
    int16_t* yb1 = s->yb + rh;
    orc_linear_table(cw, rw, 1, xofs, xa0, xa1);
    orc_linear_table(ch, rh, 0, yofs, yb0, yb1);
    uint8_t* Bc = s->bgr;
    uint8_t* Gc = Bc + s->cap_w;
    uint8_t* Rc = Gc + s->cap_w;
    int tag[2] = {-1, -1};  /* source row held by cache slot k */
    const size_t plane = (size_t)DW * DH;
    /* output plane of source channel c (B, G, R), RGB order swaps B and R */
    const int oc[3] = {color_rgb ? 2 : 0, 1, color_rgb ? 0 : 2};
    for (int Y = Y0; Y < Y1; Y++) {
        const int dy = Y - g->oy;
        const int inrow = dy >= 0 && dy < rh;
        int32_t *D0[3] = {0, 0, 0}, *D1[3] = {0, 0, 0};
        int b0 = 0, b1 = 0;
        if (inrow) {
            const int sy[2] = {clampi(yofs[dy], 0, ch - 1), clampi(yofs[dy] + 1, 0, ch - 1)};
            int slotk[2];
            for (int t = 0; t < 2; t++) {
                int k = tag[0] == sy[t] ? 0 : (tag[1] == sy[t] ? 1 : -1);
                if (k < 0) {
                    /* evict a slot the other tap does not use: for tap 1 the slot tap 0 did not take; for
                       tap 0 the slot not holding tap 1's row (if cached) */
                    if (t == 1) k = 1 - slotk[0];
                    else k = tag[0] == sy[1] ? 1 : 0;
                    convert_row(f, g->x0, g->y0 + sy[t], cw, Bc, Gc, Rc);
                    int32_t* D = s->D + (size_t)k * 3 * rw;
                    hresize(Bc, cw, xofs, xa0, xa1, rw, D);
                    hresize(Gc, cw, xofs, xa0, xa1, rw, D + rw);
                    hresize(Rc, cw, xofs, xa0, xa1, rw, D + 2 * rw);
                    tag[k] = sy[t];
                }
                slotk[t] = k;
            }
            for (int c = 0; c < 3; c++) {
                D0[c] = s->D + (size_t)slotk[0] * 3 * rw + (size_t)c * rw;
                D1[c] = s->D + (size_t)slotk[1] * 3 * rw + (size_t)c * rw;
            }
            b0 = yb0[dy];
            b1 = yb1[dy];
        }
        for (int c = 0; c < 3; c++) {
            const int o = oc[c];
            const size_t base = (slot * 3 + (size_t)o) * plane + (size_t)Y * DW;
            const int fv = fill[o];
            const float* L = out_f32 ? lut + o * 256 : 0;
            /* columns: [0, xa) fill, [xa, xb) resized, [xb, DW) fill */
            const int xa = inrow ? clampi(g->ox, 0, DW) : DW;
            const int xb = inrow ? clampi(g->ox + rw, 0, DW) : DW;
            if (out_f32) {
                float* restrict out = (float*)dst + base;
                const float fvf = L[fv];
                for (int X = 0; X < xa; X++) out[X] = fvf;
                const int32_t* restrict d0 = D0[c];
                const int32_t* restrict d1 = D1[c];
                for (int X = xa; X < xb; X++) {
                    const int dx = X - g->ox;
                    const int v = (((b0 * (d0[dx] >> 4)) >> 16) + ((b1 * (d1[dx] >> 4)) >> 16) + 2) >> 2;
                    out[X] = L[v];
                }
                for (int X = xb; X < DW; X++) out[X] = fvf;
            } else {
                uint8_t* restrict out = (uint8_t*)dst + base;
                if (xa > 0) memset(out, fv, (size_t)xa);
                const int32_t* restrict d0 = D0[c];
                const int32_t* restrict d1 = D1[c];
                for (int X = xa; X < xb; X++) {
                    const int dx = X - g->ox;
                    out[X] = (uint8_t)((((b0 * (d0[dx] >> 4)) >> 16) + ((b1 * (d1[dx] >> 4)) >> 16) + 2) >> 2);
                }
                if (xb < DW) memset(out + xb, fv, (size_t)(DW - xb));
            }
        }
    }
}

/*
 * The whole batch: items[i] = (src_index, x, y, w, h) (w <= 0: full frame) into slot
 * slot_offset + i * slot_stride of an N x 3 x DH x DW tensor (u8, or fp32 through lut [3][256] indexed
 * by output channel). fill[c]: u8 pad value of output channel c. Returns 0 or -4 (empty ROI).
 */
int orc_fast_batch(int n_items, const orc_frame* frames, const int32_t* items, int mode, int placement,
                   int color_rgb, int out_f32, const float* lut, const uint8_t fill[3], void* dst, int slot_offset,
                   int slot_stride, int DW, int DH) {
    orc_geom* geo = (orc_geom*)malloc(sizeof(orc_geom) * (size_t)(n_items > 0 ? n_items : 1));
    for (int i = 0; i < n_items; i++) {
        const int32_t* it = items + 5 * (size_t)i;
        const orc_frame* f = frames + it[0];
        if (orc_item_geometry(f->fourcc, f->width, f->height, it[1], it[2], it[3], it[4], mode, placement, DW, DH,
                              &geo[i])) {
            free(geo);
            return -4;
        }
    }
    int threads = 1;
#ifdef _OPENMP
    threads = omp_get_max_threads();
#endif
    /* stripes per item: about 4 tasks per thread over the batch, stripes of >= 8 output rows */
    int stripes = (4 * threads + n_items - 1) / (n_items > 0 ? n_items : 1);
    if (stripes > DH / 8) stripes = DH / 8;
    if (stripes < 1) stripes = 1;
    const long ntask = (long)n_items * stripes;
    #pragma omp parallel
    {
        scratch s;
        memset(&s, 0, sizeof(s));
        #pragma omp for schedule(dynamic, 1)
        for (long t = 0; t < ntask; t++) {
            const int i = (int)(t / stripes), k = (int)(t % stripes);
            const int Y0 = (int)((long)DH * k / stripes), Y1 = (int)((long)DH * (k + 1) / stripes);
            run_task(frames + items[5 * (size_t)i], &geo[i], color_rgb, out_f32, lut, fill, dst,
                     (size_t)slot_offset + (size_t)i * slot_stride, DW, DH, Y0, Y1, &s);
        }
        free(s.bgr); free(s.D); free(s.xofs); free(s.xa); free(s.yofs); free(s.yb);
    }
    free(geo);
    return 0;
}
