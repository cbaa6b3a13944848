/*
 * evam_pp.h — C ABI of the MI355X-native frame pre-processing backend.
 *
 * This is the drop-in boundary for the EVAM pre-process hot path:
 *   decoded NV12 / I420 / BGRx / BGR frame (device memory)
 *     -> optional ROI crop (gvaclassify)
 *     -> BT.601 colour conversion to BGR      (OpenCV cvtColor YUV2BGR_NV12 / _I420, BGRA2BGR)
 *     -> INTER_LINEAR resize                  (OpenCV resize, 8U fixed-point path)
 *     -> aspect-ratio letterbox / central crop (DL Streamer model-proc "resize"/"crop")
 *     -> optional BGR->RGB                    (model-proc "color_space")
 *     -> optional range + mean/std to fp32    (model-proc "range"/"mean"/"std")
 *     -> planar NCHW write into batch slot n  (DL Streamer MatToMultiPlaneImage)
 *
 * Reference interface replaced (all paths relative to the reference tree):
 *   - element selection surface: pipelines/object_detection/vehicle/pipeline.json:5,13-18
 *     ("detection-properties" element-properties passthrough), pipelines/object_classification/
 *     vehicle_attributes/pipeline.json:4-5,12-23, pipelines/action_recognition/general/pipeline.json:3-4,24-29;
 *     the parameters arrive through evas/manager.py:127-141 (pipeline.start(..., parameters=)).
 *   - native boundary [third party, not vendored]: DL Streamer 2022.1
 *     ImagePreprocessor::Convert(const Image& src, Image& dst, pre_proc_info, transform, make_planar,
 *     allocate_destination) selected by the element property "pre-process-backend" (SURVEY.md §8b).
 *     evam_pp_run() is that call batched over frames/ROIs; evam_image mirrors DLS `Image`,
 *     evam_preproc mirrors `InputImageLayerDesc`, evam_transform mirrors `ImageTransformationParams`.
 *
 * Conventions: every function returns EVAM_PP_OK (0) or a negative evam_pp_status; no C++ exception
 * crosses the ABI; the message of the last failure on the calling thread is evam_pp_last_error().
 * The caller owns every device buffer. A handle is bound to one HIP device and one HIP stream, is not
 * thread-safe, and launches asynchronously on that stream (evam_pp_sync() waits for it).
 */
#ifndef EVAM_PP_H
#define EVAM_PP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define EVAM_PP_ABI_VERSION 2 /* 2: evam_pp_run_slots */

/* DL Streamer FourCC values: fourcc(a,b,c,d) = a | b<<8 | c<<16 | d<<24. */
enum evam_fourcc {
    EVAM_FOURCC_NV12 = 0x3231564E, /* Y plane + interleaved UV plane (4:2:0), VA-API decode output   */
    EVAM_FOURCC_I420 = 0x30323449, /* Y, U, V planes (4:2:0), avdec_h264 output                       */
    EVAM_FOURCC_BGRX = 0x58524742, /* packed 4-byte BGRx (videoconvert, action_recognition template)  */
    EVAM_FOURCC_BGRA = 0x41524742, /* packed 4-byte BGRA, treated as BGRx                             */
    EVAM_FOURCC_BGR  = 0x20524742  /* packed 3-byte BGR                                               */
};

enum evam_pp_status {
    EVAM_PP_OK = 0,
    EVAM_PP_ERR_INVALID_ARG = -1, /* null pointer, bad size, bad enum, index out of range       */
    EVAM_PP_ERR_UNSUPPORTED = -2, /* fourcc / channel count / dtype not supported               */
    EVAM_PP_ERR_ALIGNMENT   = -3, /* plane pointer or pitch not a multiple of 16 bytes          */
    EVAM_PP_ERR_EMPTY_ROI   = -4, /* ROI is empty after clipping to the frame                   */
    EVAM_PP_ERR_HIP         = -5, /* a HIP runtime call failed (message has the HIP error)      */
    EVAM_PP_ERR_NO_DEVICE   = -6, /* no HIP device / bad device ordinal                         */
    EVAM_PP_ERR_OOM         = -7  /* device or host allocation failed                           */
};

/* A decoded frame. Planes are DEVICE pointers; plane i has pitch[i] bytes per row.
 * NV12: planes[0]=Y, planes[1]=UV.  I420: Y, U, V.  BGRx/BGRA/BGR: planes[0] only.
 * YUV 4:2:0 frames must have even width and height (as OpenCV's YUV420 conversions require).
 * Every used plane pointer and pitch must be a multiple of 16 bytes. */
typedef struct evam_image {
    int32_t fourcc;
    int32_t width;
    int32_t height;
    int32_t pitch[3];
    const uint8_t* planes[3];
} evam_image;

/* One unit of work: a region of srcs[src_index]. w<=0 or h<=0 means the full frame.
 * ROIs are clipped to the frame; for 4:2:0 sources the clipped rect is then widened to even
 * coordinates: x0 = x & ~1, y0 = y & ~1, x1 = min(W, (x+w+1) & ~1), y1 = min(H, (y+h+1) & ~1). */
typedef struct evam_roi {
    int32_t src_index;
    int32_t x, y, w, h;
} evam_roi;

enum evam_resize_mode {
    EVAM_RESIZE_NO_ASPECT   = 0, /* plain resize to the tensor H x W (model-proc default)          */
    EVAM_RESIZE_ASPECT      = 1, /* model-proc resize=aspect-ratio: scale = min ratio, pad (letterbox) */
    EVAM_RESIZE_ASPECT_CROP = 2  /* resize=aspect-ratio + crop=central: scale = max ratio, centre crop */
};

enum evam_placement {
    EVAM_PLACE_TOP_LEFT = 0, /* letterbox image at (0,0), fill right/bottom (build default) */
    EVAM_PLACE_CENTER   = 1  /* letterbox image centred                                     */
};

enum evam_color_order { EVAM_COLOR_BGR = 0, EVAM_COLOR_RGB = 1 };
enum evam_dtype { EVAM_DTYPE_U8 = 0, EVAM_DTYPE_F32 = 1 };

#define EVAM_NORM_RANGE    1 /* f = (float)u8 * ((max-min)/255) + min      (OpenCV convertTo) */
#define EVAM_NORM_MEAN_STD 2 /* f = (f - mean[c]) / std[c]                 (cv::subtract/divide) */

typedef struct evam_preproc {
    int32_t resize_mode;   /* evam_resize_mode                                                  */
    int32_t placement;     /* evam_placement (letterbox only)                                   */
    int32_t color_order;   /* evam_color_order of the output planes                             */
    int32_t out_dtype;     /* evam_dtype of the output tensor                                   */
    int32_t norm_flags;    /* EVAM_NORM_* bits; ignored for U8 output                           */
    uint8_t fill[4];       /* u8 fill value of padded pixels, per OUTPUT channel, before normalisation */
    float range[2];        /* {min, max}                                                        */
    float mean[3];         /* per OUTPUT channel                                                */
    float std[3];          /* per OUTPUT channel                                                */
} evam_preproc;

/* Contiguous NCHW device tensor. Item i is written to slot  slot_offset + i * slot_stride.
 * (slot_stride = 16, slot_offset = t % 16 packs a [S,16,3,H,W] clip ring.) */
typedef struct evam_tensor {
    void* data;
    int32_t n, c, h, w;
    int32_t slot_offset;
    int32_t slot_stride;
} evam_tensor;

/* Per-item transform for post-processing (DLS ImageTransformationParams): a resized-image pixel
 * (u, v) = ((x - crop_x) * scale_x, (y - crop_y) * scale_y); tensor pixel = (u + pad_x, v + pad_y). */
typedef struct evam_transform {
    float scale_x, scale_y;
    int32_t crop_x, crop_y, crop_w, crop_h;
    int32_t pad_x, pad_y;
    int32_t resized_w, resized_h;
} evam_transform;

/* Host-side accounting of the last evam_pp_run (filled when EVAM_OPT_STATS is on). */
typedef struct evam_pp_stats {
    int64_t src_bytes;   /* algorithmic source bytes: distinct touched rows x crop-window row bytes */
    int64_t dst_bytes;   /* output bytes written, padding included                                 */
    int32_t n_items;
    int32_t n_launches;
    float last_kernel_ms;/* duration of the last run's kernel(s) from HIP events (EVAM_OPT_TIMING) */
    uint32_t kernels;    /* kernel families the last run launched: EVAM_KERNEL_* bits (always filled)      */
} evam_pp_stats;

/* evam_pp_stats.kernels bits (diagnostics: which kernel family served a call). */
enum evam_kernel_family {
    EVAM_KERNEL_GENERIC = 1, EVAM_KERNEL_ROWS = 2, EVAM_KERNEL_STAGED = 4, EVAM_KERNEL_WAVE = 8,
    EVAM_KERNEL_STRIP = 16, EVAM_KERNEL_BAND = 32, EVAM_KERNEL_ROI = 64
};

enum evam_pp_option {
    EVAM_OPT_STATS  = 1, /* compute evam_pp_stats byte accounting on every run           */
    EVAM_OPT_TIMING = 2  /* bracket each run's kernels with HIP events on the handle's stream */
};

typedef struct evam_pp evam_pp;

/* Bind a handle to HIP device `hip_device` and stream `hip_stream` (NULL = the null stream). */
int evam_pp_create(int hip_device, void* hip_stream, evam_pp** out);

/* Pre-process n_items items (items == NULL: one full-frame item per src, n_items = n_srcs)
 * into dst. out_xform: NULL or an array of n_items. Asynchronous on the handle's stream. */
int evam_pp_run(evam_pp* h, const evam_image* srcs, int n_srcs, const evam_roi* items, int n_items,
                const evam_preproc* cfg, const evam_tensor* dst, evam_transform* out_xform);

/* evam_pp_run with an explicit output slot per item: item i is written to slot slots[i] of dst (dst->slot_offset
 * and dst->slot_stride are ignored). slots is a HOST array of n_items distinct values in [0, dst->n); a value
 * outside it or a slot given twice is EVAM_PP_ERR_INVALID_ARG. One launch can then write the new frames of many
 * camera streams into a shared [S,16,3,H,W] clip ring, each at its own stream's slot s*16 + t_s % 16, where the
 * reference's gvaactionrecognitionbin (pipelines/action_recognition/general/pipeline.json:3-4) pre-processes one
 * stream's frame per encoder call. */
int evam_pp_run_slots(evam_pp* h, const evam_image* srcs, int n_srcs, const evam_roi* items, int n_items,
                      const evam_preproc* cfg, const evam_tensor* dst, const int32_t* slots,
                      evam_transform* out_xform);

int evam_pp_sync(evam_pp* h);
int evam_pp_set_stream(evam_pp* h, void* hip_stream);
int evam_pp_set_option(evam_pp* h, int option, int value);
int evam_pp_get_stats(evam_pp* h, evam_pp_stats* out);
void evam_pp_destroy(evam_pp* h);
const char* evam_pp_last_error(void);
int evam_pp_abi_version(void);

/* Exact OpenCV INTER_LINEAR coefficient tables for a src_size -> dst_size axis, as the kernels compute
 * them on the device: ofs = clamped first tap (x axis) or raw floor (y axis), c0/c1 = 11-bit weights.
 * is_x != 0 applies OpenCV's x-axis border rule (fx = 0 at clamped taps). Host-only helper. */
int evam_pp_linear_table(int src_size, int dst_size, int is_x, int32_t* ofs, int16_t* c0, int16_t* c1);

#ifdef __cplusplus
}
#endif

#endif /* EVAM_PP_H */
