"""CPU tests of the oracle itself (no GPU): known answers, cross-checks of the two restatements,
OpenCV special cases, geometry rules. These pin the checker before it is trusted.

Provenance of the known answers: SURVEY.md §8(a) "a3 restated" / "a5 restated" KATs, derived from the
OpenCV 4.5 constants (third party, absent here) — the reference tree itself holds no golden vectors, so
parity with the reference is UNPINNED (see oracle/evam_oracle.c header and DESIGN.md).
"""
import zlib

import numpy as np
import pytest

BT601_KATS = [((16, 128, 128), (0, 0, 0)), ((235, 128, 128), (255, 255, 255)), ((128, 128, 128), (130, 130, 130)),
              ((81, 90, 240), (0, 0, 254)), ((145, 54, 34), (1, 255, 0)), ((41, 240, 110), (255, 0, 0)),
              ((0, 0, 0), (0, 154, 0)), ((255, 255, 255), (255, 125, 255))]


@pytest.mark.parametrize("yuv,bgr", BT601_KATS)
def test_bt601_kat(O, coracle, yuv, bgr):
    assert coracle.yuv_pixel(*yuv) == bgr
    assert tuple(int(v) for v in O.np_yuv_pixel(*yuv)) == bgr


def test_bt601_c_vs_numpy_exhaustive(O, coracle):
    # all (U, V) pairs for a spread of Y values, C vs numpy
    rng = np.random.default_rng(0)
    for Y in (0, 15, 16, 17, 100, 128, 234, 235, 255):
        U, V = rng.integers(0, 256, 64), rng.integers(0, 256, 64)
        npb = np.stack(O.np_yuv_pixel(np.full(64, Y), U, V), -1)
        cb = np.array([coracle.yuv_pixel(Y, int(u), int(v)) for u, v in zip(U, V)])
        assert (npb == cb).all()


def test_resize_table_kats(coracle):
    sx, a0, a1 = coracle.linear_table(1920, 512, True)
    assert list(zip(sx[:3], a0[:3], a1[:3])) == [(1, 1280, 768), (5, 1792, 256), (8, 256, 1792)]
    assert (sx[-1], a0[-1], a1[-1]) == (1917, 768, 1280)
    sy, b0, b1 = coracle.linear_table(1080, 512, False)
    assert list(zip(sy[:3], b0[:3], b1[:3])) == [(0, 912, 1136), (2, 688, 1360), (4, 464, 1584)]
    assert (sy[-1], b0[-1], b1[-1]) == (1078, 1136, 912)
    sx, a0, a1 = coracle.linear_table(3840, 640, True)
    assert (sx == 6 * np.arange(640) + 2).all() and (a0 == 1024).all() and (a1 == 1024).all()


def test_resize_table_borders(coracle):
    # upscale: x taps clamp with fx reset; y keeps the raw (negative) floor and its weights
    sx, a0, a1 = coracle.linear_table(432, 512, True)
    assert sx[0] == 0 and (a0[0], a1[0]) == (2048, 0)
    sy, b0, b1 = coracle.linear_table(432, 512, False)
    assert sy[0] == -1 and b0[0] + b1[0] == 2048 and b1[0] > 0
    assert sx[-1] == 431 and a1[-1] == 0


@pytest.mark.parametrize("s,d", [(1920, 512), (1080, 512), (432, 512), (768, 512), (7, 13), (400, 72), (24, 72),
                                 (3840, 640), (2160, 360), (1920, 398), (1080, 224), (1, 5), (5, 1), (2, 1)])
@pytest.mark.parametrize("is_x", [True, False])
def test_tables_c_vs_numpy(O, coracle, s, d, is_x):
    A = coracle.linear_table(s, d, is_x)
    B = O.np_linear_table(s, d, is_x)
    for a, b in zip(A, B):
        assert (np.asarray(a, np.int64) == np.asarray(b, np.int64)).all()


def test_tables_library_helper_matches(O, coracle, evam):
    """libevam_pp.so's host helper (same code the kernels run) agrees with the oracle — no GPU needed."""
    import ctypes

    lib = evam.load_library()
    for s, d in [(1920, 512), (1080, 512), (432, 512), (400, 72), (3840, 640), (1080, 224), (33, 17)]:
        for is_x in (0, 1):
            ofs = np.zeros(d, np.int32)
            c0 = np.zeros(d, np.int16)
            c1 = np.zeros(d, np.int16)
            rc = lib.evam_pp_linear_table(s, d, is_x, ofs.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                          c0.ctypes.data_as(ctypes.POINTER(ctypes.c_int16)),
                                          c1.ctypes.data_as(ctypes.POINTER(ctypes.c_int16)))
            assert rc == 0
            ro, r0, r1 = coracle.linear_table(s, d, is_x)
            assert (ofs == ro).all() and (c0 == r0).all() and (c1 == r1).all()


@pytest.mark.parametrize("shape,dsize", [((48, 64), (512, 512)), ((50, 66), (33, 17)), ((30, 40), (40, 30)),
                                         ((90, 160), (72, 72)), ((17, 9), (5, 31)), ((1, 1), (3, 2))])
def test_resize_c_vs_numpy(O, coracle, shape, dsize):
    rng = np.random.default_rng(1)
    src = rng.integers(0, 256, size=shape + (3,), dtype=np.uint8)
    a = coracle.resize_linear(src, *dsize)
    b = O.np_resize_linear(src, *dsize)
    assert (a == b).all()


def test_resize_identity_is_copy(O, coracle):
    src = np.random.default_rng(2).integers(0, 256, size=(37, 53, 3), dtype=np.uint8)
    assert (coracle.resize_linear(src, 53, 37) == src).all()


def test_resize_exact_2x_equals_area_fast(O, coracle):
    """OpenCV switches exact 2x INTER_LINEAR to INTER_AREA fast; the table path gives the same bytes."""
    src = np.random.default_rng(3).integers(0, 256, size=(48, 64, 3), dtype=np.uint8).astype(np.int64)
    area = (src[0::2, 0::2] + src[0::2, 1::2] + src[1::2, 0::2] + src[1::2, 1::2] + 2) >> 2
    assert (coracle.resize_linear(src.astype(np.uint8), 32, 24) == area).all()


def test_resize_close_to_torch_bilinear(O, coracle):
    """Independent approximate cross-check: within 1 LSB of torch half-pixel bilinear on
    interior pixels."""
    import torch

    rng = np.random.default_rng(4)
    src = rng.integers(0, 256, size=(108, 192, 3), dtype=np.uint8)
    out = coracle.resize_linear(src, 51, 51).astype(np.int64)
    t = torch.from_numpy(src).permute(2, 0, 1)[None].double()
    ref = torch.nn.functional.interpolate(t, size=(51, 51), mode="bilinear", align_corners=False)
    ref = ref[0].permute(1, 2, 0).numpy()
    d = np.abs(out[1:-1, 1:-1] - ref[1:-1, 1:-1])
    assert d.max() <= 1.0 + 1e-9


def test_norm_lut_c_vs_numpy(O, coracle):
    for flags, r, m, s in [(0, (0, 255), (0, 0, 0), (1, 1, 1)), (1, (0.0, 1.0), (0, 0, 0), (1, 1, 1)),
                           (3, (0.0, 1.0), (0.406, 0.456, 0.485), (0.225, 0.224, 0.229)),
                           (2, (0, 255), (103.94, 116.78, 123.68), (57.4, 57.1, 58.4)), (3, (-1.0, 1.0), (0.1, 0.2, 0.3), (0.5, 0.25, 2.0))]:
        a = coracle.norm_lut(flags, r, m, s)
        b = O.np_norm_lut(flags, r, m, s)
        assert (a.view(np.uint32) == b.view(np.uint32)).all()
    lut = O.np_norm_lut(1, (0.0, 1.0))
    assert lut[0, 0] == 0.0 and lut[0, 255] == np.float32(255) * np.float32(1 / 255.0)


def test_geometry_rules(O):
    # C4 letterbox: 3840x2160 -> 640x640, top-left
    g = O.item_geometry(O.NV12, 3840, 2160, 0, 0, 0, 0, 1, 0, 640, 640)
    assert (g["rw"], g["rh"], g["ox"], g["oy"]) == (640, 360, 0, 0)
    g = O.item_geometry(O.NV12, 3840, 2160, 0, 0, 0, 0, 1, 1, 640, 640)
    assert (g["ox"], g["oy"]) == (0, 140)
    # C5 aspect + central crop: 1920x1080 and 768x432 -> 398x224, offset 87
    for W, H in ((1920, 1080), (768, 432)):
        g = O.item_geometry(O.NV12, W, H, 0, 0, 0, 0, 2, 0, 224, 224)
        assert (g["rw"], g["rh"], g["ox"], g["oy"]) == (398, 224, -87, 0)
    # ROI: clip, then 4:2:0 even alignment
    g = O.item_geometry(O.NV12, 100, 80, 5, 7, 10, 10, 0, 0, 72, 72)
    assert (g["x0"], g["y0"], g["cw"], g["ch"]) == (4, 6, 12, 12)
    g = O.item_geometry(O.BGRX, 100, 80, 5, 7, 10, 10, 0, 0, 72, 72)
    assert (g["x0"], g["y0"], g["cw"], g["ch"]) == (5, 7, 10, 10)
    g = O.item_geometry(O.NV12, 100, 80, -10, 70, 30, 30, 0, 0, 72, 72)
    assert (g["x0"], g["y0"], g["cw"], g["ch"]) == (0, 70, 20, 10)
    assert O.item_geometry(O.NV12, 100, 80, 120, 10, 5, 5, 0, 0, 72, 72) is None


@pytest.mark.parametrize("fmt", ["NV12", "I420", "BGRX", "BGR"])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_item_c_vs_numpy(O, coracle, fmt, mode):
    fc = {"NV12": O.NV12, "I420": O.I420, "BGRX": O.BGRX, "BGR": O.BGR}[fmt]
    rng = np.random.default_rng(6)
    f = O.random_frame(rng, fc, 66, 50)
    lut = O.np_norm_lut(3, (0.0, 1.0), (0.406, 0.456, 0.485), (0.225, 0.224, 0.229))
    for roi in [None, (3, 5, 31, 17), (60, 40, 20, 20)]:
        out = np.zeros((1, 3, 24, 40), np.float32)
        coracle.preprocess_item(f, roi, out, 0, mode=mode, lut=lut, fill=(1, 2, 3), color_rgb=(mode == 1))
        ref = O.np_preprocess_item(f, roi, 40, 24, mode=mode, lut=lut, fill=(1, 2, 3), color_rgb=(mode == 1))
        assert (out[0].view(np.uint32) == ref.view(np.uint32)).all()


def test_nv12_equals_i420_same_samples(O, coracle):
    """Chroma is nearest (one UV sample per 2x2 block): the same samples as NV12 or I420 give the same BGR."""
    rng = np.random.default_rng(7)
    nv = O.random_frame(rng, O.NV12, 64, 48)
    U = nv.planes[1][:, 0:64:2]
    V = nv.planes[1][:, 1:64:2]
    pad = lambda a: np.pad(a, ((0, 0), (0, 16 - a.shape[1] % 16 if a.shape[1] % 16 else 0)))  # noqa: E731
    i4 = O.HostFrame(O.I420, 64, 48, [nv.planes[0], pad(np.ascontiguousarray(U)), pad(np.ascontiguousarray(V))])
    assert (O.np_to_bgr(nv, 0, 0, 64, 48) == O.np_to_bgr(i4, 0, 0, 64, 48)).all()
    b = O.np_to_bgr(nv, 0, 0, 64, 48)
    # a 2x2 block with equal luma shares one colour
    nv.planes[0][:] = 100
    b = O.np_to_bgr(nv, 0, 0, 64, 48)
    assert (b[0::2, 0::2] == b[1::2, 1::2]).all() and (b[0::2, 0::2] == b[0::2, 1::2]).all()


def test_saturating_clamp_identity():
    """The kernels' packed saturating clamp (evam_pp.hip hpass_sat) equals clamp255(S >> 20) on all (Y, U, V)."""
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location(
        "check_sat_clamp", os.path.join(os.path.dirname(__file__), "..", "tools", "check_sat_clamp.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    assert mod.check() == 0


@pytest.mark.parametrize("fmt", ["NV12", "I420", "BGRX", "BGR"])
@pytest.mark.parametrize("mode,placement,rgb,dst,dtype", [
    (0, 0, False, (72, 72), "f32"), (1, 1, True, (96, 64), "u8"), (2, 0, False, (40, 56), "f32"),
    (1, 0, False, (33, 17), "u8"), (0, 0, True, (300, 170), "f32")])
def test_cpu_fast_matches_oracle(O, coracle, fmt, mode, placement, rgb, dst, dtype):
    """The bench's CPU baseline (oracle/evam_cpu_fast.c: batch-parallel, row-cached, vectorised) is
    byte-identical to the oracle on ROI batches with edge, odd, partly outside and full-frame items,
    up- and downscales, letterbox / central crop, RGB order and clip-ring slot strides."""
    f = {"NV12": O.NV12, "I420": O.I420, "BGRX": O.BGRX, "BGR": O.BGR}[fmt]
    rng = np.random.default_rng(zlib.crc32(repr((fmt, mode, dst)).encode()))
    frames = [O.random_frame(rng, f, 160, 90, pattern=p) for p in ("uniform", "gradient", "uniform")]
    rois = [(0, 0, 0, 0, 0), (1, 0, 0, 0, 0), (2, -5, -3, 40, 30), (1, 151, 81, 20, 20), (0, 3, 5, 1, 1),
            (2, 17, 9, 131, 77), (1, 60, 40, 7, 45)]
    for _ in range(13):  # clipped rects stay non-empty (the oracle rejects an empty crop)
        x, y = int(rng.integers(-10, 150)), int(rng.integers(-10, 80))
        rois.append((int(rng.integers(0, 3)), x, y, int(rng.integers(1, 170)) + max(0, -x),
                     int(rng.integers(1, 100)) + max(0, -y)))
    lut = O.np_norm_lut(3, (0.0, 1.0), (0.1, 0.2, 0.3), (0.3, 0.2, 0.1)) if dtype == "f32" else None
    npd = np.float32 if dtype == "f32" else np.uint8
    stride = 2 if dst == (33, 17) else 1
    shape = (len(rois) * stride + 1, 3, dst[1], dst[0])
    ref = np.full(shape, 7, npd)
    for i, r in enumerate(rois):
        coracle.preprocess_item(frames[r[0]], r[1:], ref, 1 + i * stride, mode=mode, placement=placement,
                                color_rgb=rgb, lut=lut, fill=(4, 5, 6))
    got = np.full(shape, 7, npd)
    O.FastBatch(coracle, frames, rois).run(got, mode=mode, placement=placement, color_rgb=rgb, lut=lut,
                                           fill=(4, 5, 6), slot_offset=1, slot_stride=stride)
    if dtype == "f32":
        assert (got.view(np.uint32) == ref.view(np.uint32)).all()
    else:
        assert (got == ref).all()


# Unit-scale model-proc ranges (DL Streamer "range": [min, max]) with non-zero minima, and the bench's
# mean / std (ImageNet values in BGR order) next to a neutral setting.
_RANGES = [(0.0, 1.0), (-1.0, 1.0), (-0.5, 0.5), (0.1, 0.9), (-2.0, 2.0), (0.25, 3.0), (-8.0, 8.0)]
_MEAN_STD = [((0.406, 0.456, 0.485), (0.225, 0.224, 0.229)), ((0.0, 0.0, 0.0), (1.0, 1.0, 1.0)),
             ((0.5, 0.5, 0.5), (0.5, 0.5, 0.5))]


@pytest.mark.parametrize("rng_", _RANGES)
@pytest.mark.parametrize("mean,std", _MEAN_STD)
def test_norm_lut_within_tolerance_of_single_fma(O, rng_, mean, std):
    """SURVEY.md §8 a8 / north_star fp32 bar. The LUT (oracle and kernels) rounds u * alpha and + beta
    separately, as the scalar convertTo does; OpenCV's SIMD convertTo may fuse them into one FMA [3P,
    unverified]. The two differ by at most one rounding of u * alpha + beta; here both forms are built for
    every u and channel and the result stays within 1e-6 relative under SURVEY's max(|b|, 1/std) guard
    (b = the reference value). Holds for ranges of magnitude <= 8 (every model-proc range in the reference
    tree is [0, 1] or unset); a [16, 235]-scale range would exceed it near b = 0 (1 ulp of 235 is 1.5e-5)."""
    two = O.np_norm_lut(3, rng_, mean, std)
    alpha = np.float32((float(rng_[1]) - float(rng_[0])) / 255.0)
    beta = np.float32(rng_[0])
    u = np.arange(256, dtype=np.float64)
    fused = (u * np.float64(alpha) + np.float64(beta)).astype(np.float32)  # exact product + sum, one rounding
    for c in range(3):
        b = ((fused - np.float32(mean[c])).astype(np.float32) / np.float32(std[c])).astype(np.float32)
        guard = np.maximum(np.abs(b.astype(np.float64)), 1.0 / std[c])
        err = np.abs(two[c].astype(np.float64) - b.astype(np.float64))
        assert (err <= 1e-6 * guard).all(), (c, float((err / guard).max()))
    if rng_[0] == 0.0:  # beta = 0: the two forms are the same rounding
        for c in range(3):
            b = ((fused - np.float32(mean[c])).astype(np.float32) / np.float32(std[c])).astype(np.float32)
            assert np.array_equal(two[c].view(np.uint32), b.view(np.uint32))
