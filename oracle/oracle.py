"""CPU ORACLE for the EVAM pre-process hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
module, and only as the checker (or as the timed CPU baseline). The product path never imports it.

Two independent restatements of the same third-party arithmetic (see oracle/evam_oracle.c header for
the full provenance and the "parity unpinned" status):

* :class:`COracle` — ctypes binding of ``oracle/build/libevam_oracle.so`` (C + OpenMP). It is the
  fast checker for GPU parity tests and the timed CPU baseline ("port").
* ``np_*`` functions — a vectorised numpy restatement written separately from the C one, used to
  cross-check it and to generate ``tests/golden`` fixtures.

Reference anchors (paths relative to the reference tree): pre-proc call sites
``pipelines/object_detection/vehicle/pipeline.json:5``,
``pipelines/object_classification/vehicle_attributes/pipeline.json:4-5``,
``pipelines/action_recognition/general/pipeline.json:3-4``; parameters
``models_list/vehicle-detection-0202.json:3`` (default: plain resize, BGR, u8, no normalisation) and
``models_list/action-recognition-0001.json:3-13`` (BGR, resize aspect-ratio, crop central).
Third-party algorithm: OpenCV 4.5.x ``color_yuv.simd.hpp`` (BT.601, 20-bit) and ``resize.cpp``
(INTER_LINEAR, 11-bit coefficients, VResizeLinear 32s->8u), as bundled in
intel/dlstreamer-pipeline-server:2022.1.1-ubuntu20 (``docker-compose-build.yml:37``).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass, field

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libevam_oracle.so")

NV12 = 0x3231564E
I420 = 0x30323449
BGRX = 0x58524742
BGRA = 0x41524742
BGR = 0x20524742

# OpenCV ITUR_BT_601_* constants
CY, CUB, CUG, CVG, CVR, SHIFT = 1220542, 2116026, -409993, -852492, 1673527, 20


# ----------------------------------------------------------------------------------------------
# Host frame representation shared by the oracle restatements
# ----------------------------------------------------------------------------------------------
@dataclass
class HostFrame:
    """A decoded frame in host memory: planes are 2-D uint8 arrays of shape (rows, pitch)."""

    fourcc: int
    width: int
    height: int
    planes: list = field(default_factory=list)

    @property
    def pitches(self):
        return [p.shape[1] for p in self.planes]


def bpp(fourcc: int) -> int:
    return {BGRX: 4, BGRA: 4, BGR: 3}.get(fourcc, 1)


def plane_shapes(fourcc: int, width: int, height: int, pitch_align: int = 16):
    """(rows, row_bytes) of each plane; pitches rounded up to ``pitch_align``."""

    def al(n):
        return (n + pitch_align - 1) // pitch_align * pitch_align

    if fourcc == NV12:
        return [(height, al(width)), (height // 2, al(width))]
    if fourcc == I420:
        return [(height, al(width)), (height // 2, al(width // 2)), (height // 2, al(width // 2))]
    return [(height, al(width * bpp(fourcc)))]


def random_frame(rng: np.random.Generator, fourcc: int, width: int, height: int,
                 pitch_align: int = 16, pattern: str = "uniform") -> HostFrame:
    """Seeded synthetic frame: i.i.d. uniform bytes, or a smooth gradient (+ noise)."""
    planes = []
    for i, (rows, pitch) in enumerate(plane_shapes(fourcc, width, height, pitch_align)):
        if pattern == "uniform":
            p = rng.integers(0, 256, size=(rows, pitch), dtype=np.uint8)
        else:
            yy, xx = np.mgrid[0:rows, 0:pitch]
            base = (xx * 255 // max(pitch - 1, 1) + yy * 97 // max(rows - 1, 1) + 37 * i) % 256
            p = (base + rng.integers(0, 8, size=(rows, pitch))).clip(0, 255).astype(np.uint8)
        planes.append(p)
    return HostFrame(fourcc, width, height, planes)


# ----------------------------------------------------------------------------------------------
# numpy restatement
# ----------------------------------------------------------------------------------------------
def np_yuv_pixel(Y, U, V):
    """BT.601 20-bit fixed point (OpenCV uvToRGBuv / yRGBuvToRGBA). Returns B, G, R arrays."""
    Y = np.asarray(Y, dtype=np.int64)
    uu = np.asarray(U, dtype=np.int64) - 128
    vv = np.asarray(V, dtype=np.int64) - 128
    half = 1 << (SHIFT - 1)
    ruv = half + CVR * vv
    guv = half + CVG * vv + CUG * uu
    buv = half + CUB * uu
    y = np.maximum(Y - 16, 0) * CY
    f = lambda t: np.clip((y + t) >> SHIFT, 0, 255).astype(np.uint8)  # noqa: E731
    return f(buv), f(guv), f(ruv)


def np_linear_table(ssize: int, dsize: int, is_x: bool):
    """OpenCV hal::resize INTER_LINEAR per-axis table with float32/float64 semantics."""
    scale = 1.0 / (float(dsize) / float(ssize))
    d = np.arange(dsize, dtype=np.float64)
    f = ((d + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(np.float32)).astype(np.float32)
    if is_x:
        lo = s < 0
        f[lo] = 0.0
        s[lo] = 0
        hi = s >= ssize - 1
        f[hi] = 0.0
        s[hi] = ssize - 1
    one = np.float32(1.0)
    k = np.float32(2048.0)
    c0 = np.rint((one - f) * k).astype(np.int64)
    c1 = np.rint(f * k).astype(np.int64)
    return s, c0, c1


def np_to_bgr(frame: HostFrame, x0: int, y0: int, w: int, h: int) -> np.ndarray:
    fc = frame.fourcc
    ys = np.arange(y0, y0 + h)
    xs = np.arange(x0, x0 + w)
    if fc in (NV12, I420):
        Y = frame.planes[0][y0:y0 + h, x0:x0 + w]
        if fc == NV12:
            uv = frame.planes[1]
            U = uv[(ys >> 1)[:, None], (2 * (xs >> 1))[None, :]]
            V = uv[(ys >> 1)[:, None], (2 * (xs >> 1) + 1)[None, :]]
        else:
            U = frame.planes[1][(ys >> 1)[:, None], (xs >> 1)[None, :]]
            V = frame.planes[2][(ys >> 1)[:, None], (xs >> 1)[None, :]]
        b, g, r = np_yuv_pixel(Y, U, V)
        return np.stack([b, g, r], axis=-1)
    n = bpp(fc)
    p = frame.planes[0][y0:y0 + h, x0 * n:(x0 + w) * n].reshape(h, w, n)
    return np.ascontiguousarray(p[..., :3])


def np_resize_linear(src: np.ndarray, dw: int, dh: int) -> np.ndarray:
    """cv::resize INTER_LINEAR for HxWx3 uint8 (HResizeLinear + VResizeLinear 32s8u)."""
    sh, sw = src.shape[:2]
    sx, a0, a1 = np_linear_table(sw, dw, True)
    sy, b0, b1 = np_linear_table(sh, dh, False)
    sx1 = np.minimum(sx + 1, sw - 1)
    s = src.astype(np.int64)
    # horizontal pass on every source row
    D = s[:, sx, :] * a0[None, :, None] + s[:, sx1, :] * a1[None, :, None]
    r0 = np.clip(sy, 0, sh - 1)
    r1 = np.clip(sy + 1, 0, sh - 1)
    D0 = D[r0] >> 4
    D1 = D[r1] >> 4
    out = (((b0[:, None, None] * D0) >> 16) + ((b1[:, None, None] * D1) >> 16) + 2) >> 2
    return out.astype(np.uint8)


def np_norm_lut(norm_flags: int, rng_=(0.0, 255.0), mean=(0.0, 0.0, 0.0), std=(1.0, 1.0, 1.0)):
    """[3,256] float32 LUT: ((float)u*alpha + beta - mean[c]) / std[c], one rounding per op."""
    alpha = np.float32((float(rng_[1]) - float(rng_[0])) / 255.0)
    beta = np.float32(rng_[0])
    u = np.arange(256, dtype=np.float32)
    out = np.empty((3, 256), dtype=np.float32)
    for c in range(3):
        v = u.copy()
        if norm_flags & 1:
            v = (v * alpha).astype(np.float32)
            v = (v + beta).astype(np.float32)
        if norm_flags & 2:
            v = (v - np.float32(mean[c])).astype(np.float32)
            v = (v / np.float32(std[c])).astype(np.float32)
        out[c] = v
    return out


def item_geometry(fourcc, W, H, x, y, w, h, mode, placement, DW, DH):
    """Crop / resize / placement geometry (same rules as include/evam_pp.h). None if the ROI is empty."""
    if w <= 0 or h <= 0:
        x0, y0, x1, y1 = 0, 0, W, H
    else:
        cl = lambda v, hi: max(0, min(v, hi))  # noqa: E731
        x0, y0, x1, y1 = cl(x, W), cl(y, H), cl(x + w, W), cl(y + h, H)
        if fourcc in (NV12, I420):
            x0 &= ~1
            y0 &= ~1
            x1 = min(W, (x1 + 1) & ~1)
            y1 = min(H, (y1 + 1) & ~1)
    cw, ch = x1 - x0, y1 - y0
    if cw <= 0 or ch <= 0:
        return None
    ox = oy = 0
    if mode == 0:
        rw, rh = DW, DH
    else:
        sx, sy = DW / cw, DH / ch
        x_dom = (sx <= sy) if mode == 1 else (sx >= sy)
        if x_dom:
            rw, rh = DW, int(ch * sx)
        else:
            rw, rh = int(cw * sy), DH
        rw, rh = max(rw, 1), max(rh, 1)
        if mode == 1:
            rw, rh = min(rw, DW), min(rh, DH)
            if placement == 1:
                ox, oy = (DW - rw) // 2, (DH - rh) // 2
        else:
            rw, rh = max(rw, DW), max(rh, DH)
            ox, oy = -((rw - DW) // 2), -((rh - DH) // 2)
    return dict(x0=x0, y0=y0, cw=cw, ch=ch, rw=rw, rh=rh, ox=ox, oy=oy)


def np_preprocess_item(frame: HostFrame, roi, DW, DH, mode=0, placement=0, color_rgb=False,
                       lut=None, fill=(0, 0, 0)):
    """One item through the reference order. Returns [3, DH, DW] uint8 (lut None) or float32."""
    x, y, w, h = roi if roi is not None else (0, 0, 0, 0)
    g = item_geometry(frame.fourcc, frame.width, frame.height, x, y, w, h, mode, placement, DW, DH)
    if g is None:
        raise ValueError("empty ROI")
    bgr = np_to_bgr(frame, g["x0"], g["y0"], g["cw"], g["ch"])
    rs = np_resize_linear(bgr, g["rw"], g["rh"])
    if color_rgb:
        rs = rs[..., ::-1]
    out = np.empty((3, DH, DW), dtype=np.uint8)
    out[...] = np.asarray(fill, dtype=np.uint8)[:, None, None]
    X = np.arange(DW) - g["ox"]
    Yr = np.arange(DH) - g["oy"]
    xm = (X >= 0) & (X < g["rw"])
    ym = (Yr >= 0) & (Yr < g["rh"])
    sub = rs[Yr[ym]][:, X[xm]]
    out[:, np.where(ym)[0][:, None], np.where(xm)[0][None, :]] = np.moveaxis(sub, -1, 0)
    if lut is None:
        return out
    return np.stack([lut[c][out[c]] for c in range(3)])


# ----------------------------------------------------------------------------------------------
# C oracle (ctypes)
# ----------------------------------------------------------------------------------------------
def build_c_oracle(force: bool = False) -> str:
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-C", HERE, "-s"], check=True)
    return LIB_PATH


class COracle:
    """ctypes wrapper of oracle/build/libevam_oracle.so."""

    def __init__(self, path: str = LIB_PATH):
        if not os.path.exists(path):
            build_c_oracle()
        L = self.lib = ctypes.CDLL(path)
        P = ctypes.POINTER
        u8p = P(ctypes.c_uint8)
        L.orc_linear_table.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, P(ctypes.c_int32),
                                       P(ctypes.c_int16), P(ctypes.c_int16)]
        L.orc_yuv_pixel.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, u8p]
        L.orc_resize_linear_c3.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, u8p,
                                           ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.orc_norm_lut.argtypes = [ctypes.c_int, P(ctypes.c_float), P(ctypes.c_float),
                                   P(ctypes.c_float), P(ctypes.c_float)]
        L.orc_preprocess_item.argtypes = [
            ctypes.c_int, P(u8p), P(ctypes.c_int), ctypes.c_int, ctypes.c_int,
            ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
            ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
            P(ctypes.c_float), u8p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
            P(ctypes.c_int32)]
        L.orc_preprocess_item.restype = ctypes.c_int
        L.orc_num_threads.restype = ctypes.c_int
        L.orc_set_num_threads.argtypes = [ctypes.c_int]
        L.orc_fast_batch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.orc_fast_batch.restype = ctypes.c_int

    @staticmethod
    def _ptr(a, t=ctypes.c_uint8):
        return a.ctypes.data_as(ctypes.POINTER(t))

    def set_num_threads(self, n: int):
        self.lib.orc_set_num_threads(n)

    def num_threads(self) -> int:
        return self.lib.orc_num_threads()

    def linear_table(self, ssize, dsize, is_x):
        ofs = np.zeros(dsize, np.int32)
        c0 = np.zeros(dsize, np.int16)
        c1 = np.zeros(dsize, np.int16)
        self.lib.orc_linear_table(ssize, dsize, int(is_x), self._ptr(ofs, ctypes.c_int32),
                                  self._ptr(c0, ctypes.c_int16), self._ptr(c1, ctypes.c_int16))
        return ofs, c0, c1

    def yuv_pixel(self, Y, U, V):
        out = np.zeros(3, np.uint8)
        self.lib.orc_yuv_pixel(Y, U, V, self._ptr(out))
        return tuple(int(v) for v in out)

    def resize_linear(self, src: np.ndarray, dw: int, dh: int) -> np.ndarray:
        src = np.ascontiguousarray(src)
        sh, sw = src.shape[:2]
        dst = np.zeros((dh, dw, 3), np.uint8)
        self.lib.orc_resize_linear_c3(self._ptr(src), sw, sh, sw * 3, self._ptr(dst), dw, dh, dw * 3)
        return dst

    def norm_lut(self, norm_flags, rng_=(0.0, 255.0), mean=(0, 0, 0), std=(1, 1, 1)):
        r = np.asarray(rng_, np.float32)
        m = np.asarray(mean, np.float32)
        s = np.asarray(std, np.float32)
        lut = np.zeros((3, 256), np.float32)
        self.lib.orc_norm_lut(norm_flags, self._ptr(r, ctypes.c_float), self._ptr(m, ctypes.c_float),
                              self._ptr(s, ctypes.c_float), self._ptr(lut, ctypes.c_float))
        return lut

    def preprocess_item(self, frame: HostFrame, roi, out: np.ndarray, slot: int, mode=0, placement=0,
                        color_rgb=False, lut=None, fill=(0, 0, 0)):
        """Write item into out[slot] (out: [N,3,DH,DW] uint8 or float32). Returns geometry tuple."""
        planes = [np.ascontiguousarray(p) for p in frame.planes]
        arr = (ctypes.POINTER(ctypes.c_uint8) * 3)(*([self._ptr(p) for p in planes]
                                                    + [None] * (3 - len(planes))))
        pitches = (ctypes.c_int * 3)(*([p.shape[1] for p in planes] + [0] * (3 - len(planes))))
        x, y, w, h = roi if roi is not None else (0, 0, 0, 0)
        out_f32 = out.dtype == np.float32
        if out_f32:
            lut = np.ascontiguousarray(lut if lut is not None else np_norm_lut(0), np.float32)
        fl = np.asarray(fill, np.uint8)
        geom = np.zeros(8, np.int32)
        DH, DW = out.shape[2], out.shape[3]
        rc = self.lib.orc_preprocess_item(
            frame.fourcc, arr, pitches, frame.width, frame.height, x, y, w, h, mode, placement,
            int(color_rgb), int(out_f32), self._ptr(lut, ctypes.c_float) if out_f32 else None,
            self._ptr(fl), out.ctypes.data_as(ctypes.c_void_p), slot, DW, DH,
            self._ptr(geom, ctypes.c_int32))
        if rc != 0:
            raise ValueError(f"oracle rejected item (rc={rc})")
        return tuple(int(v) for v in geom)


class OrcFrame(ctypes.Structure):
    """orc_frame of oracle/evam_cpu_fast.c."""

    _fields_ = [("planes", ctypes.c_void_p * 3), ("pitch", ctypes.c_int32 * 3), ("fourcc", ctypes.c_int32),
                ("width", ctypes.c_int32), ("height", ctypes.c_int32), ("pad_", ctypes.c_int32)]


class FastBatch:
    """The CPU baseline (oracle/evam_cpu_fast.c, same arithmetic as the oracle, OpenCV-style organisation):
    a whole batch of items in one call. The frames and ROI array are marshalled once, so a timed loop
    measures the C code, not ctypes."""

    def __init__(self, coracle: "COracle", frames, rois=None):
        self.lib = coracle.lib
        self.planes = [[np.ascontiguousarray(p) for p in f.planes] for f in frames]
        self.frames = (OrcFrame * len(frames))()
        for k, (f, pl) in enumerate(zip(frames, self.planes)):
            for i, p in enumerate(pl):
                self.frames[k].planes[i] = p.ctypes.data
                self.frames[k].pitch[i] = p.shape[1]
            self.frames[k].fourcc, self.frames[k].width, self.frames[k].height = f.fourcc, f.width, f.height
        items = rois if rois is not None else [(i, 0, 0, 0, 0) for i in range(len(frames))]
        self.items = np.ascontiguousarray(np.asarray(items, np.int32).reshape(-1, 5))

    def run(self, out: np.ndarray, mode=0, placement=0, color_rgb=False, lut=None, fill=(0, 0, 0), slot_offset=0,
            slot_stride=1):
        out_f32 = out.dtype == np.float32
        if out_f32:
            self._lut = np.ascontiguousarray(lut if lut is not None else np_norm_lut(0), np.float32)
        self._fill = np.asarray(fill, np.uint8)
        DH, DW = out.shape[2], out.shape[3]
        rc = self.lib.orc_fast_batch(len(self.items), ctypes.addressof(self.frames), self.items.ctypes.data, mode,
                                     placement, int(color_rgb), int(out_f32),
                                     self._lut.ctypes.data if out_f32 else None, self._fill.ctypes.data,
                                     out.ctypes.data, slot_offset, slot_stride, DW, DH)
        if rc != 0:
            raise ValueError(f"CPU baseline rejected the batch (rc={rc})")

