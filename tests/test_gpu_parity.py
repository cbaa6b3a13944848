"""GPU parity: the HIP path (through the C ABI) against the CPU oracle, bit-exact.

u8 outputs must be byte-identical; fp32 outputs are compared bitwise too (the kernel maps the u8 result
through a host-built LUT computed in the reference's operation order, so the bar north_star states —
1e-6 relative — is met with zero error). Sizes are small enough for the oracle to finish in seconds, plus
the full BASELINE configs through size-independent properties.
"""
import os
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FORMATS = ["NV12", "I420", "BGRX", "BGR"]


def fc(O, name):
    return {"NV12": O.NV12, "I420": O.I420, "BGRX": O.BGRX, "BGR": O.BGR}[name]


def upload(evam, frames, device):
    return [evam.Image.from_host(f.fourcc, f.width, f.height, f.planes, device=device) for f in frames]


def run_hip(evam, torch, imgs, shape, dtype, info=None, rois=None, slot_offset=0, slot_stride=1,
            want_transform=False, pp=None, init=None):
    out = torch.full(shape, init if init is not None else 7, dtype=dtype, device=imgs[0].planes[0].device)
    own = pp is None
    pp = pp or evam.HipPreProcessor(device=0)
    xf = pp.convert(imgs, out, info, rois=rois, slot_offset=slot_offset, slot_stride=slot_stride,
                    want_transform=want_transform)
    torch.cuda.synchronize()
    if own:
        pp.close()
    return out.cpu().numpy(), xf


def info_lut(O, info):
    if info is None:
        return None
    flags = (1 if info.range is not None else 0) | (2 if (info.mean is not None or info.std is not None) else 0)
    return O.np_norm_lut(flags, info.range or (0.0, 255.0), info.mean or (0, 0, 0), info.std or (1, 1, 1))


def run_oracle(O, coracle, frames, shape, dtype, info=None, rois=None, slot_offset=0, slot_stride=1, init=7):
    ref = np.full(shape, init, dtype=np.float32 if dtype == "f32" else np.uint8)
    mode = placement = 0
    rgb = False
    fill = (0, 0, 0)
    if info is not None:
        mode = info.resize_mode()
        placement = 1 if info.placement == "center" else 0
        rgb = info.color_space == "RGB"
        fill = info.fill
    lut = info_lut(O, info) if dtype == "f32" else None
    if dtype == "f32" and lut is None:
        lut = O.np_norm_lut(0)
    items = rois if rois is not None else [(i, 0, 0, 0, 0) for i in range(len(frames))]
    geoms = []
    for i, (si, x, y, w, h) in enumerate(items):
        g = coracle.preprocess_item(frames[si], (x, y, w, h), ref, slot_offset + i * slot_stride, mode=mode,
                                    placement=placement, color_rgb=rgb, lut=lut, fill=fill)
        geoms.append(g)
    return ref, geoms


def assert_same(got, ref, what=""):
    if got.dtype == np.float32:
        same = (got.view(np.uint32) == ref.view(np.uint32))
    else:
        same = got == ref
    if not same.all():
        bad = np.argwhere(~same)
        i = tuple(bad[0])
        raise AssertionError(f"{what}: {len(bad)} mismatches of {got.size}; first at {i}: got {got[i]} ref {ref[i]}")


@pytest.mark.parametrize("fmt", FORMATS)
@pytest.mark.parametrize("src,dst", [((64, 48), (512, 512)), ((66, 50), (33, 17)), ((160, 90), (72, 72)),
                                     ((320, 180), (160, 90)), ((96, 64), (96, 64)), ((200, 120), (300, 70)),
                                     ((64, 48), (1, 1)), ((64, 48), (1, 37)), ((2, 2), (40, 3)), ((1920, 1080), (3, 2))])
@pytest.mark.parametrize("dtype", ["u8", "f32"])
def test_full_frame(evam, O, coracle, gpu, fmt, src, dst, dtype):
    import torch

    rng = np.random.default_rng(zlib.crc32(repr((fmt, src, dst)).encode()))
    frames = [O.random_frame(rng, fc(O, fmt), src[0], src[1], pattern=p) for p in ("uniform", "gradient")]
    info = evam.PreProcInfo(range=(0.0, 1.0), mean=(0.406, 0.456, 0.485), std=(0.225, 0.224, 0.229)) \
        if dtype == "f32" else None
    shape = (2, 3, dst[1], dst[0])
    got, _ = run_hip(evam, torch, upload(evam, frames, gpu), shape, torch.float32 if dtype == "f32" else torch.uint8,
                     info)
    ref, _ = run_oracle(O, coracle, frames, shape, dtype, info)
    assert_same(got, ref, f"{fmt} {src}->{dst} {dtype}")


def test_numpy_restatement_agrees(evam, O, coracle, gpu):
    """Third leg: the GPU output also equals the independent numpy restatement."""
    import torch

    rng = np.random.default_rng(5)
    f = O.random_frame(rng, O.NV12, 130, 74)
    got, _ = run_hip(evam, torch, upload(evam, [f], gpu), (1, 3, 40, 56), torch.uint8)
    ref = O.np_preprocess_item(f, None, 56, 40)
    assert_same(got[0], ref, "numpy restatement")


@pytest.mark.parametrize("fmt", FORMATS)
def test_roi_batch(evam, O, coracle, gpu, fmt):
    """gvaclassify: ~50 variable ROIs per frame, incl. frame-edge, odd and partially outside rects."""
    import torch

    rng = np.random.default_rng(11)
    W, H = 320, 240
    frames = [O.random_frame(rng, fc(O, fmt), W, H) for _ in range(2)]
    rois = []
    for si in range(2):
        for _ in range(50):
            w = int(rng.integers(3, 200))
            h = int(rng.integers(3, 150))
            x = int(rng.integers(-20, W - 2))
            y = int(rng.integers(-20, H - 2))
            w, h = max(w, 3 - x), max(h, 3 - y)  # keep at least a sliver inside the frame
            rois.append((si, x, y, w, h))
    rois += [(0, 0, 0, W, H), (1, W - 3, H - 3, 10, 10), (0, 1, 1, 1, 1), (1, 5, 7, 9, 11)]
    info = evam.PreProcInfo(range=(0.0, 1.0))
    shape = (len(rois), 3, 72, 72)
    got, _ = run_hip(evam, torch, upload(evam, frames, gpu), shape, torch.float32, info,
                     rois=[evam.Roi(*r) for r in rois])
    ref, _ = run_oracle(O, coracle, frames, shape, "f32", info, rois=rois)
    assert_same(got, ref, f"roi batch {fmt}")


@pytest.mark.parametrize("fmt", FORMATS)
@pytest.mark.parametrize("dst,dtype,resize,placement", [
    ((72, 72), "u8", "no-aspect-ratio", "top_left"),     # ROI kernel, R=4, K=2
    ((300, 120), "f32", "aspect-ratio", "center"),       # ROI kernel, R=2 (DW > 256), letterbox columns+rows
    ((600, 40), "u8", "no-aspect-ratio", "top_left"),    # DW > 512: generic kernel
    ((17, 5), "f32", "aspect-ratio", "top_left"),        # K=1, nfull=0
    ((64, 64), "f32", "aspect-ratio", "center"),         # R*DW = 256 exactly
])
@pytest.mark.parametrize("roi_kernel", ["roi", "generic"])
def test_roi_kernels(evam, O, coracle, gpu, fmt, dst, dtype, resize, placement, roi_kernel, monkeypatch):
    """Per-item-geometry batches through the staged ROI kernel (the default) and the generic one (EVAM_PP_ROI=0)."""
    import torch

    monkeypatch.setenv("EVAM_PP_ROI", "0" if roi_kernel == "generic" else "1")
    rng = np.random.default_rng(zlib.crc32(f"{fmt}{dst}{resize}".encode()))
    W, H = 480, 270
    frames = [O.random_frame(rng, fc(O, fmt), W, H, pattern="gradient" if i else "uniform") for i in range(3)]
    rois = []
    for si in range(3):
        for _ in range(12):
            w, h = int(rng.integers(2, 420)), int(rng.integers(2, 260))
            x, y = int(rng.integers(-30, W - 1)), int(rng.integers(-30, H - 1))
            rois.append((si, x, y, max(w, 2 - x), max(h, 2 - y)))
    rois += [(0, 0, 0, W, H), (2, W - 2, H - 2, 9, 9), (1, 100, 50, 1, 1)]
    info = evam.PreProcInfo(resize=resize, placement=placement, fill=(9, 99, 199), color_space="RGB",
                            **({"range": (0.0, 1.0), "mean": (0.1, 0.2, 0.3), "std": (0.3, 0.2, 0.1)}
                               if dtype == "f32" else {}))
    DW, DH = dst
    shape = (len(rois), 3, DH, DW)
    tdt = torch.float32 if dtype == "f32" else torch.uint8
    got, _ = run_hip(evam, torch, upload(evam, frames, gpu), shape, tdt, info, rois=[evam.Roi(*r) for r in rois])
    ref, _ = run_oracle(O, coracle, frames, shape, dtype, info, rois=rois)
    assert_same(got, ref, f"roi {fmt} {dst} {resize} kernel={roi_kernel}")


@pytest.mark.parametrize("placement", ["top_left", "center"])
@pytest.mark.parametrize("fill", [(0, 0, 0), (114, 114, 114), (1, 2, 3)])
def test_letterbox(evam, O, coracle, gpu, placement, fill):
    import torch

    rng = np.random.default_rng(3)
    frames = [O.random_frame(rng, O.NV12, 384, 216), O.random_frame(rng, O.NV12, 216, 384)]
    info = evam.PreProcInfo(resize="aspect-ratio", placement=placement, fill=fill)
    shape = (2, 3, 160, 160)
    got, xf = run_hip(evam, torch, upload(evam, frames, gpu), shape, torch.uint8, info, want_transform=True)
    ref, geoms = run_oracle(O, coracle, frames, shape, "u8", info)
    assert_same(got, ref, f"letterbox {placement} {fill}")
    for t, g in zip(xf, geoms):
        assert (t.crop_x, t.crop_y, t.crop_w, t.crop_h, t.resized_w, t.resized_h, t.pad_x, t.pad_y) == g


@pytest.mark.parametrize("fmt", FORMATS)
@pytest.mark.parametrize("dtype", ["u8", "f32"])
@pytest.mark.parametrize("placement", ["top_left", "center"])
def test_letterbox_strong_downscale(evam, O, coracle, gpu, fmt, dtype, placement):
    """Letterbox columns and rows at > 15x downscales, where the kernel choice falls to the direct-tap row kernel
    (evam_pp_rows): its padding columns carry the fill (round 6: found by test_random_calls_in_flight, the row kernel
    wrote 0 there)."""
    import torch

    rng = np.random.default_rng(zlib.crc32(repr((fmt, dtype, placement)).encode()))
    info = evam.PreProcInfo(resize="aspect-ratio", placement=placement, fill=(241, 17, 99), color_space="RGB",
                            **({"range": (0.0, 1.0), "mean": (0.1, 0.2, 0.3), "std": (0.3, 0.2, 0.1)}
                               if dtype == "f32" else {}))
    for (W, H), (DW, DH) in (((1178, 566), (433, 26)), ((566, 1178), (26, 433)), ((1178, 566), (40, 40)),
                             ((566, 1178), (40, 40))):
        frames = [O.random_frame(rng, fc(O, fmt), W, H) for _ in range(2)]  # one size: a uniform-geometry launch
        shape = (3, 3, DH, DW)
        got, _ = run_hip(evam, torch, upload(evam, frames, gpu), shape, torch.float32 if dtype == "f32" else torch.uint8,
                         info, slot_offset=1)
        ref, _ = run_oracle(O, coracle, frames, shape, dtype, info, slot_offset=1)
        assert_same(got, ref, f"strong downscale letterbox {fmt} {dtype} {placement} -> {DW}x{DH}")


@pytest.mark.parametrize("fmt,src", [("NV12", (1920, 1080)), ("BGRX", (768, 432)), ("I420", (640, 480))])
def test_aspect_central_crop(evam, O, coracle, gpu, fmt, src):
    """action-recognition-0001 model-proc: BGR, resize aspect-ratio, crop central, 224x224."""
    import torch

    rng = np.random.default_rng(4)
    frames = [O.random_frame(rng, fc(O, fmt), *src)]
    info = evam.PreProcInfo.from_model_proc({"format": "image", "layer_name": "0", "params": {
        "color_space": "BGR", "resize": "aspect-ratio", "crop": "central"}})
    shape = (1, 3, 224, 224)
    got, xf = run_hip(evam, torch, upload(evam, frames, gpu), shape, torch.float32, info, want_transform=True)
    ref, geoms = run_oracle(O, coracle, frames, shape, "f32", info)
    assert_same(got, ref, f"aspect crop {fmt} {src}")
    if src == (1920, 1080):
        assert (xf[0].resized_w, xf[0].resized_h, xf[0].pad_x) == (398, 224, -87)


def test_clip_ring_slots(evam, O, coracle, gpu):
    """C5 packing: frame t of stream s goes to slot s*16 + t%16 of a [S*16,3,H,W] ring."""
    import torch

    rng = np.random.default_rng(8)
    S = 3
    shape = (S * 16, 3, 32, 32)
    out = torch.zeros(shape, dtype=torch.float32, device=gpu)
    ref = np.zeros(shape, np.float32)
    pp = evam.HipPreProcessor(device=0)
    info = evam.PreProcInfo(resize="aspect-ratio", crop="central")
    lut = O.np_norm_lut(0)
    for t in range(18):
        frames = [O.random_frame(rng, O.BGRX, 96, 54) for _ in range(S)]
        pp.convert(upload(evam, frames, gpu), out, info, slot_offset=t % 16, slot_stride=16)
        for s, f in enumerate(frames):
            coracle.preprocess_item(f, None, ref, s * 16 + t % 16, mode=2, lut=lut)
    torch.cuda.synchronize()
    assert_same(out.cpu().numpy(), ref, "clip ring")
    pp.close()


def test_rgb_order_and_mixed_formats(evam, O, coracle, gpu):
    """color_space=RGB swaps planes; one call may mix source formats (one launch per format)."""
    import torch

    rng = np.random.default_rng(9)
    frames = [O.random_frame(rng, fc(O, n), 120, 68) for n in FORMATS]
    info = evam.PreProcInfo(color_space="RGB", range=(-1.0, 1.0), mean=(0.1, 0.2, 0.3), std=(0.5, 0.25, 2.0))
    shape = (4, 3, 50, 70)
    got, _ = run_hip(evam, torch, upload(evam, frames, gpu), shape, torch.float32, info)
    ref, _ = run_oracle(O, coracle, frames, shape, "f32", info)
    assert_same(got, ref, "rgb mixed formats")


def test_reuse_handle_changing_inputs(evam, O, coracle, gpu):
    """The descriptor block cache must re-upload when frames / config change between calls."""
    import torch

    rng = np.random.default_rng(10)
    pp = evam.HipPreProcessor(device=0)
    for k in range(4):
        frames = [O.random_frame(rng, O.NV12, 64 + 16 * k, 48 + 8 * k) for _ in range(2)]
        info = evam.PreProcInfo(range=(0.0, float(k + 1)))
        shape = (2, 3, 40, 40)
        got, _ = run_hip(evam, torch, upload(evam, frames, gpu), shape, torch.float32, info, pp=pp)
        ref, _ = run_oracle(O, coracle, frames, shape, "f32", info)
        assert_same(got, ref, f"iteration {k}")
    pp.close()


def test_pitch_variants(evam, O, coracle, gpu):
    """1080p NV12 with pitch 1920 and 2048 (C2 variants)."""
    import torch

    rng = np.random.default_rng(12)
    for align in (16, 256):
        f = O.random_frame(rng, O.NV12, 1920, 1080, pitch_align=align)
        assert f.planes[0].shape[1] == (1920 if align == 16 else 2048)
        got, _ = run_hip(evam, torch, upload(evam, [f], gpu), (1, 3, 512, 512), torch.uint8)
        ref, _ = run_oracle(O, coracle, [f], (1, 3, 512, 512), "u8")
        assert_same(got, ref, f"pitch {f.planes[0].shape[1]}")


def test_c2_full_size_parity_and_properties(evam, O, coracle, gpu):
    """Headline config at full size: 1080p NV12 batch -> 512x512 fp32 normalised.
    Bit-exact vs the oracle on 4 distinct frames, and slot independence on a 32-frame batch."""
    import torch

    rng = np.random.default_rng(0)
    frames = [O.random_frame(rng, O.NV12, 1920, 1080, pattern=p) for p in ("uniform", "gradient") * 2]
    info = evam.PreProcInfo(range=(0.0, 1.0), mean=(0.406, 0.456, 0.485), std=(0.225, 0.224, 0.229))
    imgs = upload(evam, frames, gpu)
    got, _ = run_hip(evam, torch, imgs, (4, 3, 512, 512), torch.float32, info)
    ref, _ = run_oracle(O, coracle, frames, (4, 3, 512, 512), "f32", info)
    assert_same(got, ref, "C2 full size")
    # 32 slots = the 4 frames repeated: every slot equals its frame's slot, whatever its position.
    batch = [imgs[i % 4] for i in range(32)]
    got32, _ = run_hip(evam, torch, batch, (32, 3, 512, 512), torch.float32, info)
    for i in range(32):
        assert_same(got32[i], got[i % 4], f"slot {i}")


def test_constant_frame_property(evam, O, gpu):
    """Size-independent property at the C4 size: a constant-colour 4K frame letterboxed to 640x640 gives the
    constant's BT.601 colour in the 640x360 image and the fill value in the padding."""
    import torch

    W, H = 3840, 2160
    f = O.random_frame(np.random.default_rng(0), O.NV12, W, H)
    f.planes[0][:] = 150
    f.planes[1][:, 0::2] = 90
    f.planes[1][:, 1::2] = 200
    img = upload(evam, [f], gpu)
    info = evam.PreProcInfo(resize="aspect-ratio", fill=(9, 9, 9))
    got, xf = run_hip(evam, torch, img, (1, 3, 640, 640), torch.uint8, info, want_transform=True)
    b, g, r = (int(v) for v in O.np_yuv_pixel(150, 90, 200))
    assert (xf[0].resized_w, xf[0].resized_h) == (640, 360)
    assert (got[0, 0, :360] == b).all() and (got[0, 1, :360] == g).all() and (got[0, 2, :360] == r).all()
    assert (got[0, :, 360:] == 9).all()


@pytest.mark.parametrize("case", ["empty_roi", "bad_fourcc", "misaligned_pitch", "slot_oob", "odd_yuv",
                                  "bad_dtype", "src_index"])
def test_errors(evam, O, gpu, case):
    import torch

    rng = np.random.default_rng(1)
    f = O.random_frame(rng, O.NV12, 64, 48)
    img = upload(evam, [f], gpu)[0]
    out = torch.zeros((1, 3, 16, 16), dtype=torch.uint8, device=gpu)
    rois = None
    if case == "empty_roi":
        rois = [evam.Roi(0, 100, 100, 10, 10)]
    elif case == "bad_fourcc":
        img = evam.Image(0x12345678, 64, 48, img.planes)
    elif case == "misaligned_pitch":
        p = torch.zeros((48, 72), dtype=torch.uint8, device=gpu)
        img = evam.Image(O.NV12, 64, 48, [p, img.planes[1]])
    elif case == "slot_oob":
        rois = [evam.Roi(0, 0, 0, 0, 0), evam.Roi(0, 0, 0, 0, 0)]
    elif case == "odd_yuv":
        img = evam.Image(O.NV12, 63, 48, img.planes)
    elif case == "bad_dtype":
        out = torch.zeros((1, 3, 16, 16), dtype=torch.float16, device=gpu)
    elif case == "src_index":
        rois = [evam.Roi(3, 0, 0, 0, 0)]
    pp = evam.HipPreProcessor(device=0)
    with pytest.raises(evam.PreProcError) as ei:
        pp.convert([img], out, rois=rois)
    expected = {"empty_roi": -4, "bad_fourcc": -2, "misaligned_pitch": -3, "slot_oob": -1, "odd_yuv": -1,
                "bad_dtype": -2, "src_index": -1}[case]
    assert ei.value.status == expected, str(ei.value)
    pp.close()


def test_stats_and_timing(evam, O, gpu):
    """Byte accounting of SURVEY §8(d) for C2: 6,148,608 algorithmic bytes per frame."""
    import torch

    f = O.random_frame(np.random.default_rng(0), O.NV12, 1920, 1080)
    img = upload(evam, [f], gpu)
    pp = evam.HipPreProcessor(device=0)
    pp.set_option(evam.native.OPT_STATS, 1)
    pp.set_option(evam.native.OPT_TIMING, 1)
    out = torch.empty((2, 3, 512, 512), dtype=torch.float32, device=gpu)
    pp.convert(img * 2, out, evam.PreProcInfo(range=(0.0, 1.0)))
    st = pp.stats()
    assert st.src_bytes == 2 * 3_002_880 and st.dst_bytes == 2 * 3_145_728
    assert st.n_launches == 1 and st.last_kernel_ms > 0
    pp.close()


@pytest.mark.parametrize("fmt", FORMATS)
@pytest.mark.parametrize("src,dst,resize", [
    ((768, 432), (512, 512), "no-aspect-ratio"),    # C1 shape: vertical upscale -> REUSE
    ((640, 360), (256, 128), "no-aspect-ratio"),    # downscale, DW % 4 == 0
    ((320, 200), (226, 150), "aspect-ratio"),       # DW % 4 != 0 -> PX 2, letterbox rows
    ((300, 180), (131, 97), "aspect-ratio"),        # odd DW -> PX 1, letterbox
    ((480, 270), (224, 224), "aspect-crop"),        # C5 shape: central crop
])
@pytest.mark.parametrize("variant", ["auto", "wave", "px1", "px2", "noreuse", "staged", "staged_xcd", "staged_r1",
                                     "strip", "strip_unpaired", "strip_th5", "strip_nw8", "strip_px1", "strip_px2",
                                     "strip_px1_unpaired", "strip_px2_unpaired_th7", "strip_noprio", "band", "band_px1",
                                     "band_px2", "band_th5", "band_th64", "band_ahead64", "band_noprio", "rows"])
def test_wave_kernel_variants(evam, O, coracle, gpu, fmt, src, dst, resize, variant, monkeypatch):
    """Uniform-geometry batches through the default kernel choice, the wave-row kernel forced
    (EVAM_PP_WAVE=2; every PX / REUSE choice), the staged kernel (EVAM_PP_WAVE=0 EVAM_PP_STRIP=0; with the
    XCD-contiguous tile order forced on small, non-multiple-of-8 grids: EVAM_PP_XCD=1) and the strip kernel
    (EVAM_PP_STRIP=2: forced even where output rows share source rows; every ring depth, an odd tile height,
    8 waves per workgroup, XCD order, 1 and 2 pixels per lane) and the band kernel (EVAM_PP_BAND=2: forced
    on downscales too, every PX, short and 64-row bands), the direct-tap row kernel (every other family off), RGB
    order, fp32 with normalisation and u8."""
    import torch

    env = {"wave": {"EVAM_PP_WAVE": "2"}, "px1": {"EVAM_PP_WAVE": "2", "EVAM_PP_PX": "1"},
           "px2": {"EVAM_PP_WAVE": "2", "EVAM_PP_PX": "2"}, "noreuse": {"EVAM_PP_WAVE": "2", "EVAM_PP_REUSE": "0"},
           "staged": {"EVAM_PP_WAVE": "0"}, "staged_xcd": {"EVAM_PP_WAVE": "0", "EVAM_PP_XCD": "1"},
           "staged_r1": {"EVAM_PP_WAVE": "0", "EVAM_PP_STAGE_R": "1"},
           "strip": {"EVAM_PP_STRIP": "2"}, "strip_unpaired": {"EVAM_PP_STRIP": "2", "EVAM_PP_STRIP_PAIR": "0"},
           "strip_th5": {"EVAM_PP_STRIP": "2", "EVAM_PP_STRIP_TH": "5"},
           "strip_nw8": {"EVAM_PP_STRIP": "2", "EVAM_PP_STRIP_NW": "8"},
           "strip_px1": {"EVAM_PP_STRIP": "2", "EVAM_PP_STRIP_PX": "1"},
           "strip_px2": {"EVAM_PP_STRIP": "2", "EVAM_PP_STRIP_PX": "2"},
           "strip_px1_unpaired": {"EVAM_PP_STRIP": "2", "EVAM_PP_STRIP_PX": "1", "EVAM_PP_STRIP_PAIR": "0"},
           "strip_px2_unpaired_th7": {"EVAM_PP_STRIP": "2", "EVAM_PP_STRIP_PX": "2", "EVAM_PP_STRIP_PAIR": "0",
                                      "EVAM_PP_STRIP_TH": "7"},
           "band": {"EVAM_PP_BAND": "2"}, "band_px1": {"EVAM_PP_BAND": "2", "EVAM_PP_BAND_PX": "1"},
           "band_px2": {"EVAM_PP_BAND": "2", "EVAM_PP_BAND_PX": "2"},
           "band_th5": {"EVAM_PP_BAND": "2", "EVAM_PP_STRIP_TH": "5"},
           "band_th64": {"EVAM_PP_BAND": "2", "EVAM_PP_STRIP_TH": "64"},
           "strip_noprio": {"EVAM_PP_STRIP": "2", "EVAM_PP_PRIO": "0"},
           "band_ahead64": {"EVAM_PP_BAND": "2", "EVAM_PP_BAND_AHEAD": "64", "EVAM_PP_STRIP_TH": "20"},
           "band_noprio": {"EVAM_PP_BAND": "2", "EVAM_PP_PRIO": "0"},
           "rows": {"EVAM_PP_WAVE": "0", "EVAM_PP_STAGED": "0", "EVAM_PP_BAND": "0"}}.get(variant, {})
    if variant.startswith(("staged", "band", "rows")):
        env["EVAM_PP_STRIP"] = "0"
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    if variant == "px2" and dst[0] % 2:
        pytest.skip("PX 2 needs an even output width")
    rng = np.random.default_rng(zlib.crc32(repr((fmt, src, dst, resize)).encode()))
    frames = [O.random_frame(rng, fc(O, fmt), src[0], src[1], pattern=p) for p in ("uniform", "gradient", "uniform")]
    kw = {"resize": "aspect-ratio", "crop": "central"} if resize == "aspect-crop" else {"resize": resize}
    for dtype in ("u8", "f32"):
        info = evam.PreProcInfo(color_space="RGB", fill=(5, 50, 250), placement="center", **kw,
                                **({"range": (0.0, 1.0), "mean": (0.1, 0.2, 0.3), "std": (0.3, 0.2, 0.1)}
                                   if dtype == "f32" else {}))
        shape = (3, 3, dst[1], dst[0])
        got, _ = run_hip(evam, torch, upload(evam, frames, gpu), shape,
                         torch.float32 if dtype == "f32" else torch.uint8, info)
        ref, _ = run_oracle(O, coracle, frames, shape, dtype, info)
        assert_same(got, ref, f"wave {fmt} {src}->{dst} {resize} {variant} {dtype}")


@pytest.mark.parametrize("fmt", ["NV12", "I420"])
@pytest.mark.parametrize("src,dst,resize", [
    ((768, 432), (512, 512), "no-aspect-ratio"),   # C1: every lane reads 6 source columns
    ((432, 768), (512, 512), "aspect-ratio"),      # 3:2 with letterbox columns (whole padding lanes)
    ((600, 338), (400, 400), "no-aspect-ratio"),   # 3:2 horizontal, 338 -> 400 vertical
    ((630, 300), (420, 420), "aspect-ratio"),      # 3:2 with letterbox rows
    ((700, 400), (500, 500), "no-aspect-ratio"),   # 7:5: per-pixel taps (not admitted)
])
@pytest.mark.parametrize("dd", ["1", "0"])
def test_band_six_column_lanes(evam, O, coracle, gpu, fmt, src, dst, resize, dd, monkeypatch):
    """The band kernel's six-column lanes (4 pixels per lane reading 6 luma and 3 chroma columns, admitted by
    band_six_columns on the host) against the oracle, next to the per-pixel taps (EVAM_PP_BAND_DD=0), on 3:2
    horizontal scales with and without letterbox columns and rows, and one geometry the check refuses."""
    import torch

    monkeypatch.setenv("EVAM_PP_BAND", "2")
    monkeypatch.setenv("EVAM_PP_STRIP", "0")
    monkeypatch.setenv("EVAM_PP_BAND_DD", dd)
    rng = np.random.default_rng(zlib.crc32(repr(("dd", fmt, src, dst, resize)).encode()))
    frames = [O.random_frame(rng, fc(O, fmt), src[0], src[1], pattern=p) for p in ("uniform", "gradient", "uniform")]
    for dtype in ("u8", "f32"):
        info = evam.PreProcInfo(color_space="BGR" if dtype == "u8" else "RGB", fill=(5, 50, 250), placement="center",
                                resize=resize, **({"range": (0.0, 1.0), "mean": (0.1, 0.2, 0.3), "std": (0.3, 0.2, 0.1)}
                                                  if dtype == "f32" else {}))
        shape = (3, 3, dst[1], dst[0])
        got, _ = run_hip(evam, torch, upload(evam, frames, gpu), shape,
                         torch.float32 if dtype == "f32" else torch.uint8, info)
        ref, _ = run_oracle(O, coracle, frames, shape, dtype, info)
        assert_same(got, ref, f"band dd={dd} {fmt} {src}->{dst} {resize} {dtype}")


@pytest.mark.parametrize("rec_device", ["1", "0"])
def test_stream_switch_and_descriptor_churn(evam, O, coracle, gpu, rec_device, monkeypatch):
    """Descriptor slots stay valid across torch stream switches and many changing ROI sets / geometries
    (the upload ring and the ROI record ring wrap; slot fences, one per run of ROI slots, follow the stream), with
    the record slots in host-written device memory (default) and in pinned host memory (EVAM_PP_REC_DEVICE=0)."""
    import torch

    monkeypatch.setenv("EVAM_PP_REC_DEVICE", rec_device)

    rng = np.random.default_rng(11)
    frames = [O.random_frame(rng, O.NV12, 320, 180) for _ in range(2)]
    imgs = upload(evam, frames, gpu)
    pp = evam.HipPreProcessor(device=0)
    streams = [torch.cuda.Stream(device=gpu) for _ in range(3)]
    outs, refs = [], []
    for it in range(40):  # 20 ROI calls: the 16-slot pinned ROI ring wraps
        s = streams[it % 3]
        with torch.cuda.stream(s):
            if it % 2:
                rois = [(int(rng.integers(0, 2)), int(rng.integers(0, 200)), int(rng.integers(0, 100)),
                         int(rng.integers(8, 120)), int(rng.integers(8, 80))) for _ in range(9)]
                shape = (9, 3, 24, 40)
                out = torch.full(shape, 7, dtype=torch.uint8, device=gpu)
                pp.convert(imgs, out, None, rois=[evam.Roi(*r) for r in rois])
                ref, _ = run_oracle(O, coracle, frames, shape, "u8", None, rois=rois)
            else:
                dw, dh = 32 + 8 * it, 16 + 4 * it  # a new uniform geometry (new tables) every time
                shape = (2, 3, dh, dw)
                out = torch.full(shape, 7, dtype=torch.uint8, device=gpu)
                pp.convert(imgs, out)
                ref, _ = run_oracle(O, coracle, frames, shape, "u8")
            outs.append((out, s))
            refs.append(ref)
    torch.cuda.synchronize()
    for i, ((out, _), ref) in enumerate(zip(outs, refs)):
        assert_same(out.cpu().numpy(), ref, f"call {i}")
    pp.close()


@pytest.mark.parametrize("px", ["4", "2"])
@pytest.mark.parametrize("fmt", FORMATS)
@pytest.mark.parametrize("dst,dtype", [((72, 72), "f32"), ((64, 36), "u8"), ((45, 30), "f32")])
def test_roi_kernel_px4(evam, O, coracle, gpu, fmt, dst, dtype, px, monkeypatch):
    """The ROI kernel's 4- and 2-pixels-per-lane variants (EVAM_PP_ROI_PX) on a ROI batch (an odd output width falls
    back to one pixel per lane)."""
    import torch

    monkeypatch.setenv("EVAM_PP_ROI_PX", px)
    rng = np.random.default_rng(zlib.crc32(f"px4{fmt}{dst}".encode()))
    W, H = 320, 200
    frames = [O.random_frame(rng, fc(O, fmt), W, H, pattern="gradient" if i else "uniform") for i in range(2)]
    rois = [(int(rng.integers(0, 2)), int(rng.integers(-10, W - 4)), int(rng.integers(-10, H - 4)),
             int(rng.integers(4, 260)), int(rng.integers(4, 180))) for _ in range(20)]
    rois = [(s, x, y, max(w, 4 - x), max(h, 4 - y)) for s, x, y, w, h in rois]
    info = evam.PreProcInfo(resize="aspect-ratio", placement="center", fill=(1, 2, 3), color_space="RGB",
                            **({"range": (0.0, 1.0), "mean": (0.1, 0.2, 0.3), "std": (0.3, 0.2, 0.1)}
                               if dtype == "f32" else {}))
    shape = (len(rois), 3, dst[1], dst[0])
    got, _ = run_hip(evam, torch, upload(evam, frames, gpu), shape,
                     torch.float32 if dtype == "f32" else torch.uint8, info, rois=[evam.Roi(*r) for r in rois])
    ref, _ = run_oracle(O, coracle, frames, shape, dtype, info, rois=rois)
    assert_same(got, ref, f"roi px{px} {fmt} {dst} {dtype}")


@pytest.mark.parametrize("fmt", FORMATS)
@pytest.mark.parametrize("kind", ["inside", "mixed"])
@pytest.mark.parametrize("simd", ["1", "0"])
def test_roi_host_pass1_simd(evam, O, coracle, gpu, fmt, kind, simd, monkeypatch):
    """The host's ROI pass 1 on AVX2 (csrc/evam_clip_simd.h, EVAM_PP_HOST_SIMD=1, the default) and the scalar pass
    against the oracle: 61 ROIs (not a multiple of 8) on frames of one size. "inside" sets take the AVX2 pass;
    "mixed" sets add rects straddling or beyond the frame edges and a full-frame item (w = 0), which the AVX2 pass
    hands back to the scalar one."""
    import torch

    monkeypatch.setenv("EVAM_PP_HOST_SIMD", simd)
    rng = np.random.default_rng(zlib.crc32(f"simd{fmt}{kind}".encode()))
    W, H = 160, 96
    frames = [O.random_frame(rng, fc(O, fmt), W, H, pattern="gradient" if i % 2 else "uniform") for i in range(5)]
    rois = []
    for k in range(61):
        w, h = int(rng.integers(2, W)), int(rng.integers(2, H))
        x, y = int(rng.integers(0, W - w + 1)), int(rng.integers(0, H - h + 1))
        if kind == "mixed" and k % 5 == 1:
            x, y = int(rng.integers(-40, W)), int(rng.integers(-30, H))
            w, h = int(rng.integers(41, 2 * W)), int(rng.integers(31, 2 * H))
        if kind == "mixed" and k == 37:
            x = y = w = h = 0  # the full frame
        rois.append((int(rng.integers(0, len(frames))), x, y, w, h))
    info = evam.PreProcInfo(resize="aspect-ratio", placement="center", fill=(1, 2, 3),
                            range=(0.0, 1.0), mean=(0.1, 0.2, 0.3), std=(0.3, 0.2, 0.1))
    shape = (len(rois), 3, 24, 32)
    got, _ = run_hip(evam, torch, upload(evam, frames, gpu), shape, torch.float32, info,
                     rois=[evam.Roi(*r) for r in rois])
    ref, _ = run_oracle(O, coracle, frames, shape, "f32", info, rois=rois)
    assert_same(got, ref, f"roi host pass 1 simd={simd} {kind} {fmt}")


@pytest.mark.parametrize("fmt", FORMATS)
@pytest.mark.parametrize("variant", ["wave", "staged", "strip"])
def test_uniform_rois_varied_x0(evam, O, coracle, gpu, fmt, variant, monkeypatch):
    """Equal-size ROIs (one uniform-geometry group) at crop origins covering every x0 mod 32 residue, upscaled
    so the wave kernel's REUSE path runs: its LDS row segments must hold the widest 16-byte-aligned footprint
    of ANY item's origin, not just the first item's (a misaligned origin needs one more chunk)."""
    import torch

    monkeypatch.setenv("EVAM_PP_WAVE", "2" if variant == "wave" else "0")
    monkeypatch.setenv("EVAM_PP_STRIP", "2" if variant == "strip" else "0")
    rng = np.random.default_rng(zlib.crc32(f"x0{fmt}".encode()))
    W, H = 256, 120
    frames = [O.random_frame(rng, fc(O, fmt), W, H, pattern="gradient" if i else "uniform") for i in range(2)]
    yuv = fmt in ("NV12", "I420")
    cw, ch = 40, 24  # even: 4:2:0 origins stay on even x (same clipped size for every ROI)
    xs = list(range(0, 64, 2 if yuv else 1))
    rois = [(k % 2, x, (7 * k) % (H - ch) & ~1, cw, ch) for k, x in enumerate(xs)]
    for dst, dtype in (((96, 64), "u8"), ((120, 72), "f32")):
        info = evam.PreProcInfo(**({"range": (0.0, 1.0), "mean": (0.1, 0.2, 0.3), "std": (0.3, 0.2, 0.1)}
                                   if dtype == "f32" else {}))
        shape = (len(rois), 3, dst[1], dst[0])
        got, _ = run_hip(evam, torch, upload(evam, frames, gpu), shape,
                         torch.float32 if dtype == "f32" else torch.uint8, info, rois=[evam.Roi(*r) for r in rois])
        ref, _ = run_oracle(O, coracle, frames, shape, dtype, info, rois=rois)
        assert_same(got, ref, f"uniform ROIs varied x0 {fmt} {dst} {variant}")


def test_many_items_chunked_launches(evam, O, coracle, gpu):
    """Uniform batches larger than one launch's kernel-argument item table (64) split into several
    launches; every item still lands in its own slot, including clip-ring slot strides."""
    import torch

    rng = np.random.default_rng(21)
    frames = [O.random_frame(rng, O.NV12, 96, 54) for _ in range(7)]
    imgs = upload(evam, frames, gpu)
    n = 150
    batch = [imgs[i % 7] for i in range(n)]
    info = evam.PreProcInfo(range=(0.0, 1.0))
    pp = evam.HipPreProcessor(device=0)
    pp.set_option(evam.native.OPT_STATS, 1)
    got, _ = run_hip(evam, torch, batch, (n, 3, 40, 64), torch.float32, info, pp=pp)
    assert pp.stats().n_launches == 3
    ref1, _ = run_oracle(O, coracle, frames, (7, 3, 40, 64), "f32", info)
    for i in range(n):
        assert_same(got[i], ref1[i % 7], f"item {i}")
    pp.close()


@pytest.mark.parametrize("fmt", ["NV12", "I420", "BGRX"])
@pytest.mark.parametrize("n_frames", [64, 70])
def test_roi_batches_many_frames(evam, O, coracle, gpu, fmt, n_frames):
    """ROI batches over many frames (self-contained records per ROI tile, the widest crops split into two
    row tiles): oracle-exact, including ROIs on the last frame and partially outside rects."""
    import torch

    rng = np.random.default_rng(zlib.crc32(f"rec{fmt}{n_frames}".encode()))
    W, H = 96, 64
    frames = [O.random_frame(rng, fc(O, fmt), W, H, pattern="gradient" if i % 3 else "uniform")
              for i in range(n_frames)]
    rois = []
    for k in range(90):
        si = n_frames - 1 if k % 9 == 0 else int(rng.integers(0, n_frames))
        w, h = int(rng.integers(2, 90)), int(rng.integers(2, 60))
        x, y = int(rng.integers(-8, W - 2)), int(rng.integers(-8, H - 2))
        rois.append((si, x, y, max(w, 2 - x), max(h, 2 - y)))
    info = evam.PreProcInfo(resize="aspect-ratio", placement="center", fill=(5, 6, 7),
                            range=(0.0, 1.0), mean=(0.1, 0.2, 0.3), std=(0.3, 0.2, 0.1))
    shape = (len(rois), 3, 32, 48)
    got, _ = run_hip(evam, torch, upload(evam, frames, gpu), shape, torch.float32, info,
                     rois=[evam.Roi(*r) for r in rois])
    ref, _ = run_oracle(O, coracle, frames, shape, "f32", info, rois=rois)
    assert_same(got, ref, f"roi records {fmt} frames={n_frames}")


@pytest.mark.parametrize("fmt", ["NV12", "I420", "BGR"])
def test_staged_many_tile_columns(evam, O, coracle, gpu, fmt, monkeypatch):
    """A staged launch with more tile columns than the kernel-argument footprint table holds (tiles_x >
    16: each tile's footprint comes from the column table in device memory instead)."""
    import torch

    monkeypatch.setenv("EVAM_PP_WAVE", "0")
    monkeypatch.setenv("EVAM_PP_STRIP", "0")
    monkeypatch.setenv("EVAM_PP_NSEGX", "2")  # 128-column tiles: 2200 / 128 -> 18 tile columns
    rng = np.random.default_rng(zlib.crc32(f"tcol{fmt}".encode()))
    frames = [O.random_frame(rng, fc(O, fmt), 2400, 64, pattern=p) for p in ("uniform", "gradient")]
    info = evam.PreProcInfo(resize="aspect-ratio", placement="center", fill=(3, 4, 5))
    shape = (2, 3, 40, 2200)
    got, _ = run_hip(evam, torch, upload(evam, frames, gpu), shape, torch.uint8, info)
    ref, _ = run_oracle(O, coracle, frames, shape, "u8", info)
    assert_same(got, ref, f"staged >16 tile columns {fmt}")


@pytest.mark.parametrize("tail", ["1", "2", "4", "7"])
@pytest.mark.parametrize("dst", [(72, 72), (37, 29)])
def test_roi_tail_split(evam, O, coracle, gpu, tail, dst, monkeypatch):
    """ROI batches whose uneven tail over the CUs is split into row tiles (EVAM_PP_ROI_TAIL): with fewer ROIs
    than CUs every ROI is in the tail, so each becomes `tail` row tiles (any DH, including heights that do not
    divide evenly) and every tile lands in its own rows of the ROI's slot."""
    import torch

    monkeypatch.setenv("EVAM_PP_ROI_TAIL", tail)
    rng = np.random.default_rng(zlib.crc32(f"tail{tail}{dst}".encode()))
    W, H = 640, 360
    frames = [O.random_frame(rng, O.NV12, W, H, pattern="gradient" if i else "uniform") for i in range(2)]
    rois = [(int(rng.integers(0, 2)), int(rng.integers(0, W - 8)), int(rng.integers(0, H - 8)),
             int(rng.integers(8, 400)), int(rng.integers(8, 300))) for _ in range(40)]
    info = evam.PreProcInfo(range=(0.0, 1.0), mean=(0.1, 0.2, 0.3), std=(0.3, 0.2, 0.1))
    shape = (len(rois), 3, dst[1], dst[0])
    got, _ = run_hip(evam, torch, upload(evam, frames, gpu), shape, torch.float32, info,
                     rois=[evam.Roi(*r) for r in rois])
    ref, _ = run_oracle(O, coracle, frames, shape, "f32", info, rois=rois)
    assert_same(got, ref, f"roi tail split {tail} {dst}")




@pytest.mark.parametrize("layout", ["v_first", "u_first", "far_apart", "beyond_2g"])
def test_i420_paired_chroma_plane_layouts(evam, O, coracle, gpu, layout):
    """Strip kernel with paired taps on I420: both chroma planes are read through one buffer resource based at the
    lower plane (U and V segments of both source rows in one LDS-DMA instruction). V below U, U below V, planes 1 GiB
    apart (still paired: the upper plane ends inside the resource's 0x7FFFFFFF bytes) and planes 2 GiB apart (no
    pairing for that group: one row per instruction) all equal the oracle."""
    import torch

    rng = np.random.default_rng(2024)
    W, H = 960, 540
    frames = [O.random_frame(rng, O.I420, W, H, pattern=p) for p in ("uniform", "gradient")]
    imgs = []
    for f in frames:
        y, u, v = (np.ascontiguousarray(p) for p in f.planes)
        gap = {"far_apart": (1 << 30) + 4096, "beyond_2g": (2 << 30) + 4096}.get(layout, 4096)
        total = y.nbytes + u.nbytes + v.nbytes + gap + 3 * 256
        buf = torch.zeros(total, dtype=torch.uint8, device=gpu)

        def put(off, a):
            t = buf[off:off + a.nbytes].view(a.shape)
            t.copy_(torch.from_numpy(a))
            return t, (off + a.nbytes + 255) // 256 * 256

        o = 0
        if layout == "v_first":
            vt, o = put(o, v)
            ut, o = put(o, u)
        else:
            ut, o = put(o, u)
            o = (o + gap) // 256 * 256 if layout in ("far_apart", "beyond_2g") else o
            vt, o = put(o, v)
        yt, o = put(o, y)
        imgs.append(evam.Image(O.I420, W, H, [yt, ut, vt]))
    info = evam.PreProcInfo(range=(0.0, 1.0), mean=(0.406, 0.456, 0.485), std=(0.225, 0.224, 0.229))
    pp = evam.HipPreProcessor(device=0)
    got, _ = run_hip(evam, torch, imgs, (2, 3, 256, 256), torch.float32, info, pp=pp)
    assert pp.stats().kernels == evam.native.KERNEL_STRIP
    pp.close()
    ref, _ = run_oracle(O, coracle, frames, (2, 3, 256, 256), "f32", info)
    assert_same(got, ref, f"I420 paired chroma, {layout}")


@pytest.mark.parametrize("kind", ["strip", "band", "wave", "staged", "roi", "generic"])
def test_run_slots_explicit_output_slots(evam, O, coracle, gpu, kind, monkeypatch):
    """evam_pp_run_slots: item i lands in slot slots[i] (a permutation with gaps over a larger tensor, as a shared
    clip ring indexed s*16 + t_s % 16 gets), on every kernel family; untouched slots keep their value. Out-of-range
    and repeated slots are refused before anything launches."""
    import torch

    env = {"strip": {}, "band": {"EVAM_PP_BAND": "2", "EVAM_PP_STRIP": "0"}, "wave": {"EVAM_PP_WAVE": "2"},
           "staged": {"EVAM_PP_STRIP": "0", "EVAM_PP_WAVE": "0"}, "roi": {}, "generic": {"EVAM_PP_ROI": "0"}}[kind]
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    rng = np.random.default_rng(zlib.crc32(f"slots{kind}".encode()))
    up = kind in ("band", "wave")
    W, H = (120, 64) if up else (640, 360)
    frames = [O.random_frame(rng, O.NV12, W, H, pattern="gradient" if i % 2 else "uniform") for i in range(6)]
    imgs = upload(evam, frames, gpu)
    info = evam.PreProcInfo(resize="aspect-ratio", crop="central", range=(0.0, 1.0), mean=(0.1, 0.2, 0.3),
                            std=(0.3, 0.2, 0.1))
    rois = None
    if kind in ("roi", "generic"):
        rois = [(i % 6, int(rng.integers(0, W // 2)), int(rng.integers(0, H // 2)), int(rng.integers(16, W // 2)),
                 int(rng.integers(16, H // 2))) for i in range(9)]
    n = len(rois) if rois else 6
    dst = (96, 96) if not up else (200, 160)
    slots = [5 * 16 + 3, 0, 17, 2 * 16 + 15, 31, 3 * 16 + 8, 4 * 16, 1, 70][:n]
    out = torch.full((96, 3, dst[1], dst[0]), 7.0, device=gpu)
    pp = evam.HipPreProcessor(device=0)
    pp.convert(imgs, out, info, rois=[evam.Roi(*r) for r in rois] if rois else None, slots=slots)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    ref, _ = run_oracle(O, coracle, frames, (n, 3, dst[1], dst[0]), "f32", info, rois=rois)
    for i, s in enumerate(slots):
        assert_same(got[s], ref[i], f"run_slots {kind} item {i} -> slot {s}")
    rest = np.setdiff1d(np.arange(96), slots)
    assert (got[rest] == 7.0).all()
    for bad in ([0] * n, [96] + slots[1:], [-1] + slots[1:]):
        with pytest.raises(evam.PreProcError):
            pp.convert(imgs, out, info, rois=[evam.Roi(*r) for r in rois] if rois else None, slots=bad)
    with pytest.raises(evam.PreProcError):
        pp.convert(imgs, out, info, rois=[evam.Roi(*r) for r in rois] if rois else None, slots=slots[:-1])
    pp.close()


@pytest.fixture(scope="module")
def fuzz_pp(evam, gpu):
    """One handle for every fuzz case: descriptor-block, LUT, record-ring and convert-side caches all see churn."""
    pp = evam.HipPreProcessor(device=0)
    yield pp
    pp.close()


def random_case(evam, O, rng):
    """One seeded random call over the whole input space the boundary accepts (test_random_configurations):
    returns (fmt, frames, shape, dtype, info, rois or None, slot offset, slot stride)."""
    fmt = FORMATS[int(rng.integers(0, len(FORMATS)))]
    yuv = fmt in ("NV12", "I420")
    n_src = int(rng.integers(1, 4))
    one_size = rng.random() < 0.4  # every source one size: full-frame calls take the uniform-geometry kernels
    frames = []
    for k in range(n_src):
        big = rng.random() < 0.25
        W = int(rng.integers(2, 1300 if big else 400))
        H = int(rng.integers(2, 760 if big else 300))
        if yuv:
            W, H = W + (W & 1), H + (H & 1)
        if one_size and k:
            W, H = frames[0].width, frames[0].height
        frames.append(O.random_frame(rng, fc(O, fmt), W, H, pitch_align=int(rng.choice([16, 64, 256])),
                                     pattern="gradient" if rng.random() < 0.3 else "uniform"))
    DW, DH = int(rng.integers(1, 700)), int(rng.integers(1, 500))
    if rng.random() < 0.3:
        DW = DH = int(rng.choice([72, 224, 256, 512]))
    dtype = "f32" if rng.random() < 0.6 else "u8"
    mode = ["no-aspect-ratio", "aspect-ratio", "crop"][int(rng.integers(0, 3))]
    kw = {"resize": "aspect-ratio", "crop": "central"} if mode == "crop" else {"resize": mode}
    kw["placement"] = "center" if rng.random() < 0.5 else "top_left"
    kw["color_space"] = "RGB" if rng.random() < 0.5 else "BGR"
    kw["fill"] = tuple(int(v) for v in rng.integers(0, 256, 3))
    if dtype == "f32":
        if rng.random() < 0.7:
            kw["range"] = (0.0, float(rng.choice([1.0, 255.0])))
        if rng.random() < 0.6:
            kw["mean"] = tuple(float(v) for v in rng.uniform(0, 1, 3))
            kw["std"] = tuple(float(v) for v in rng.uniform(0.1, 1, 3))
    info = evam.PreProcInfo(**kw)
    rois = None
    if rng.random() < 0.6:
        rois = []
        for _ in range(int(rng.integers(1, 41))):
            si = int(rng.integers(0, n_src))
            W, H = frames[si].width, frames[si].height
            r = rng.random()
            if r < 0.1:
                rois.append((si, 0, 0, W, H))
            elif r < 0.15:
                rois.append((si, 0, 0, 0, 0))  # w <= 0: the full frame
            else:
                x, y = int(rng.integers(-W // 4 - 1, W)), int(rng.integers(-H // 4 - 1, H))
                w = int(rng.integers(1, max(2, W + W // 4)))
                h = int(rng.integers(1, max(2, H + H // 4)))
                rois.append((si, x, y, max(w, 1 - x), max(h, 1 - y)))  # at least one pixel inside
        n_items = len(rois)
    else:
        n_items = n_src
    stride = int(rng.integers(1, 3))
    offset = int(rng.integers(0, 3))
    shape = (offset + (n_items - 1) * stride + 1 + int(rng.integers(0, 2)), 3, DH, DW)
    return fmt, frames, shape, dtype, info, rois, offset, stride


@pytest.mark.parametrize("seed", range(int(os.environ.get("EVAM_FUZZ_CASES", "96"))))
def test_random_configurations(evam, O, coracle, gpu, fuzz_pp, seed):
    """Seeded random calls over the whole input space the boundary accepts, each bit-exact against the oracle: any
    source format, frame sizes from 2 to ~1,300 (odd widths for packed formats), pitch padding, tensor sizes from 1 to
    ~700 (up- and downscales), the three resize modes and two placements, BGR / RGB order, fill values, u8 or fp32
    with random range / mean / std, full frames or ROI lists (partly outside the frame, slivers, whole frames) over
    several sources of mixed sizes, and slot offsets / strides; one handle for all cases."""
    import torch

    fmt, frames, shape, dtype, info, rois, offset, stride = random_case(evam, O, np.random.default_rng(1000 + seed))
    tdt = torch.float32 if dtype == "f32" else torch.uint8
    what = f"seed {seed}: {fmt} {[(f.width, f.height) for f in frames]} -> {shape} {dtype} {info} " \
           f"{'%d rois' % len(rois) if rois else 'frames'} offset {offset} stride {stride}"
    got, _ = run_hip(evam, torch, upload(evam, frames, gpu), shape, tdt, info,
                     rois=[evam.Roi(*r) for r in rois] if rois else None, slot_offset=offset, slot_stride=stride,
                     pp=fuzz_pp)
    ref, _ = run_oracle(O, coracle, frames, shape, dtype, info, rois=rois, slot_offset=offset, slot_stride=stride)
    assert_same(got, ref, what)


@pytest.mark.parametrize("n_handles", [1, 3])
def test_random_calls_in_flight(evam, O, coracle, gpu, n_handles):
    """40 random calls (random_case) enqueued back to back with no synchronisation, round-robin over handles bound to
    their own HIP streams (the device runner's shape), each into its own output: the descriptor-block ring, the ROI
    record ring and the LUT are reused while earlier kernels still run. After one synchronize every output equals the
    oracle bit for bit."""
    import torch

    streams = [torch.cuda.Stream(device=gpu) for _ in range(n_handles)]
    pps = [evam.HipPreProcessor(device=0, stream=s) for s in streams]
    rng = np.random.default_rng(77 + n_handles)
    cases = [random_case(evam, O, rng) for _ in range(int(os.environ.get("EVAM_FUZZ_INFLIGHT_CALLS", "40")))]
    try:
        # inputs and outputs first (default stream), then one synchronize: the calls below go out back to back
        imgs = [upload(evam, c[1], gpu) for c in cases]
        outs = [torch.full(c[2], 7, dtype=torch.float32 if c[3] == "f32" else torch.uint8, device=gpu) for c in cases]
        torch.cuda.synchronize()
        first = int(os.environ.get("EVAM_FUZZ_INFLIGHT_FIRST", "0"))  # (diagnostics: a sub-range of the calls,
        sync_each = os.environ.get("EVAM_FUZZ_INFLIGHT_SYNC") == "1"    # or a synchronize after every call)
        for k, (case, im, out) in enumerate(zip(cases, imgs, outs)):
            if k < first:
                continue
            fmt, frames, shape, dtype, info, rois, offset, stride = case
            pps[k % n_handles].convert(im, out, info, rois=[evam.Roi(*r) for r in rois] if rois else None,
                                       slot_offset=offset, slot_stride=stride)
            if sync_each:
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        for k, (case, out) in enumerate(zip(cases, outs)):
            if k < first:
                continue
            fmt, frames, shape, dtype, info, rois, offset, stride = case
            ref, _ = run_oracle(O, coracle, frames, shape, dtype, info, rois=rois, slot_offset=offset,
                                slot_stride=stride)
            assert_same(out.cpu().numpy(), ref, f"call {k} on handle {k % n_handles}: {fmt} -> {shape} {dtype}")
    finally:
        for pp in pps:
            pp.close()


# Kernel families switched off (the planner then chooses among the rest by its own feasibility rules) and the ROI
# path's options: random calls through every family the product can reach, not only the one the default plan picks.
FAMILY_ENVS = {
    "no_strip": {"EVAM_PP_STRIP": "0"},
    "no_strip_band": {"EVAM_PP_STRIP": "0", "EVAM_PP_BAND": "0"},
    "staged_rows": {"EVAM_PP_STRIP": "0", "EVAM_PP_BAND": "0", "EVAM_PP_WAVE": "0"},
    "rows_only": {"EVAM_PP_STRIP": "0", "EVAM_PP_BAND": "0", "EVAM_PP_WAVE": "0", "EVAM_PP_STAGED": "0"},
    "no_uniform": {"EVAM_PP_ROWS": "0"},
    "generic_only": {"EVAM_PP_ROWS": "0", "EVAM_PP_ROI": "0"},
    "roi_px1": {"EVAM_PP_ROI_PX": "1"},
    "roi_px4": {"EVAM_PP_ROI_PX": "4"},
    "roi_unsorted": {"EVAM_PP_ROI_SORT": "0", "EVAM_PP_ROI_SNAKE": "0"},
    "roi_no_tail": {"EVAM_PP_ROI_TAIL": "1"},
    "roi_xcd": {"EVAM_PP_ROI_XCD": "1"},
    "rec_host": {"EVAM_PP_REC_DEVICE": "0"},
    "host_scalar": {"EVAM_PP_HOST_SIMD": "0"},
}


@pytest.mark.parametrize("family", sorted(FAMILY_ENVS))
def test_random_kernel_families(evam, O, coracle, gpu, family, monkeypatch):
    """random_case calls (EVAM_FUZZ_FAMILY_CASES each, default 12) on a handle created with one family switched off or
    one ROI-path option set: every output bit-exact against the oracle."""
    import torch

    for k, v in FAMILY_ENVS[family].items():
        monkeypatch.setenv(k, v)
    pp = evam.HipPreProcessor(device=0)  # knobs are read when the handle is created
    try:
        rng = np.random.default_rng(zlib.crc32(family.encode()))
        for n in range(int(os.environ.get("EVAM_FUZZ_FAMILY_CASES", "12"))):
            fmt, frames, shape, dtype, info, rois, offset, stride = random_case(evam, O, rng)
            tdt = torch.float32 if dtype == "f32" else torch.uint8
            got, _ = run_hip(evam, torch, upload(evam, frames, gpu), shape, tdt, info,
                             rois=[evam.Roi(*r) for r in rois] if rois else None, slot_offset=offset,
                             slot_stride=stride, pp=pp)
            ref, _ = run_oracle(O, coracle, frames, shape, dtype, info, rois=rois, slot_offset=offset,
                                slot_stride=stride)
            assert_same(got, ref, f"{family} case {n}: {fmt} {[(f.width, f.height) for f in frames]} -> {shape} "
                                  f"{dtype} {info} {'%d rois' % len(rois) if rois else 'frames'}")
    finally:
        pp.close()


@pytest.mark.parametrize("seed", range(int(os.environ.get("EVAM_FUZZ_SLOT_CASES", "24"))))
def test_random_slots_and_large_batches(evam, O, coracle, gpu, fuzz_pp, seed):
    """Random calls with an explicit output slot per item (evam_pp_run_slots: a random injective table into a larger
    tensor) and batches past one launch's 64 kernel-argument items: up to 70 one-size frames, or up to 150 ROIs over a
    few sources. Every written slot bit-exact against the oracle; every other slot untouched."""
    import torch

    rng = np.random.default_rng(50000 + seed)
    fmt = FORMATS[int(rng.integers(0, len(FORMATS)))]
    yuv = fmt in ("NV12", "I420")
    W, H = int(rng.integers(8, 500)), int(rng.integers(8, 300))
    if yuv:
        W, H = W + (W & 1), H + (H & 1)
    use_rois = rng.random() < 0.5
    n_src = int(rng.integers(1, 5)) if use_rois else int(rng.integers(60, 71))
    frames = [O.random_frame(rng, fc(O, fmt), W, H) for _ in range(n_src)]
    if use_rois:
        rois = []
        for _ in range(int(rng.integers(65, 151))):
            si = int(rng.integers(0, n_src))
            x, y = int(rng.integers(-10, W - 1)), int(rng.integers(-10, H - 1))
            w, h = int(rng.integers(1, W)), int(rng.integers(1, H))
            rois.append((si, x, y, max(w, 1 - x), max(h, 1 - y)))
        n_items = len(rois)
    else:
        rois, n_items = None, n_src
    DW, DH = int(rng.integers(1, 160)), int(rng.integers(1, 160))
    dtype = "f32" if rng.random() < 0.5 else "u8"
    kw = {"resize": ["no-aspect-ratio", "aspect-ratio"][int(rng.integers(0, 2))],
          "placement": "center" if rng.random() < 0.5 else "top_left", "fill": tuple(int(v) for v in rng.integers(0, 256, 3))}
    if dtype == "f32":
        kw["range"] = (0.0, 1.0)
    info = evam.PreProcInfo(**kw)
    batch = n_items + int(rng.integers(0, 40))
    slots = rng.permutation(batch)[:n_items].astype(np.int32)
    tdt = torch.float32 if dtype == "f32" else torch.uint8
    out = torch.full((batch, 3, DH, DW), 7, dtype=tdt, device=gpu)
    fuzz_pp.convert(upload(evam, frames, gpu), out, info, rois=[evam.Roi(*r) for r in rois] if rois else None,
                    slots=slots)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    # the oracle writes item i at slot_offset + i: one item at a time into its slot
    ref = np.full(got.shape, 7, dtype=got.dtype)
    items = rois if rois else [(i, 0, 0, 0, 0) for i in range(n_items)]
    one = (1, 3, DH, DW)
    for i, r in enumerate(items):
        part, _ = run_oracle(O, coracle, frames, one, dtype, info, rois=[r])
        ref[slots[i]] = part[0]
    assert_same(got, ref, f"seed {seed}: {fmt} {W}x{H} x{n_src} -> {DW}x{DH} {dtype} {kw} "
                          f"{'%d rois' % n_items if rois else '%d frames' % n_items} batch {batch}")


@pytest.mark.parametrize("seed", range(int(os.environ.get("EVAM_FUZZ_MIXED_CASES", "24"))))
def test_random_mixed_format_calls(evam, O, coracle, gpu, fuzz_pp, seed):
    """Random calls whose sources differ in format (one launch per format group, each group's ROI records in its own
    region of the call's record slot): 2-5 sources of random formats and sizes, full frames or up to 60 ROIs over all
    of them, every output bit-exact against the oracle."""
    import torch

    rng = np.random.default_rng(80000 + seed)
    frames = []
    for _ in range(int(rng.integers(2, 6))):
        fmt = FORMATS[int(rng.integers(0, len(FORMATS)))]
        W, H = int(rng.integers(2, 700)), int(rng.integers(2, 500))
        if fmt in ("NV12", "I420"):
            W, H = W + (W & 1), H + (H & 1)
        frames.append(O.random_frame(rng, fc(O, fmt), W, H))
    rois = None
    if rng.random() < 0.6:
        rois = []
        for _ in range(int(rng.integers(1, 61))):
            si = int(rng.integers(0, len(frames)))
            W, H = frames[si].width, frames[si].height
            x, y = int(rng.integers(-W // 4 - 1, W)), int(rng.integers(-H // 4 - 1, H))
            w, h = int(rng.integers(1, W + W // 4 + 1)), int(rng.integers(1, H + H // 4 + 1))
            rois.append((si, x, y, max(w, 1 - x), max(h, 1 - y)))
    n_items = len(rois) if rois else len(frames)
    DW, DH = int(rng.integers(1, 400)), int(rng.integers(1, 300))
    dtype = "f32" if rng.random() < 0.5 else "u8"
    mode = ["no-aspect-ratio", "aspect-ratio", "crop"][int(rng.integers(0, 3))]
    kw = {"resize": "aspect-ratio", "crop": "central"} if mode == "crop" else {"resize": mode}
    info = evam.PreProcInfo(placement="center" if rng.random() < 0.5 else "top_left",
                            color_space="RGB" if rng.random() < 0.5 else "BGR",
                            fill=tuple(int(v) for v in rng.integers(0, 256, 3)),
                            **({"range": (0.0, 1.0), "mean": (0.2, 0.3, 0.4), "std": (0.5, 0.6, 0.7)}
                               if dtype == "f32" else {}), **kw)
    shape = (n_items, 3, DH, DW)
    got, _ = run_hip(evam, torch, upload(evam, frames, gpu), shape, torch.float32 if dtype == "f32" else torch.uint8,
                     info, rois=[evam.Roi(*r) for r in rois] if rois else None, pp=fuzz_pp)
    ref, _ = run_oracle(O, coracle, frames, shape, dtype, info, rois=rois)
    assert_same(got, ref, f"seed {seed}: {[(f.fourcc, f.width, f.height) for f in frames]} -> {DW}x{DH} {dtype} {kw} "
                          f"{'%d rois' % n_items if rois else 'frames'}")


@pytest.mark.parametrize("seed", range(int(os.environ.get("EVAM_FUZZ_LARGE_CASES", "6"))))
def test_random_large_outputs(evam, O, coracle, gpu, fuzz_pp, seed):
    """Tensors past the ranges the other random tests draw from: 700 - 4096 columns and rows (identity sizes, 4K
    upscales, wide strips past the strip kernel's 2,048-column limit), full frames or a few ROIs, u8 or fp32."""
    import torch

    rng = np.random.default_rng(90000 + seed)
    fmt = FORMATS[int(rng.integers(0, len(FORMATS)))]
    W, H = int(rng.integers(64, 2000)), int(rng.integers(64, 1200))
    if fmt in ("NV12", "I420"):
        W, H = W + (W & 1), H + (H & 1)
    frames = [O.random_frame(rng, fc(O, fmt), W, H) for _ in range(int(rng.integers(1, 3)))]
    DW, DH = int(rng.integers(700, 4097)), int(rng.integers(700, 2200))
    if seed % 3 == 0:
        DW, DH = W, H  # identity size
    rois = None
    if rng.random() < 0.4:
        rois = [(int(rng.integers(0, len(frames))), int(rng.integers(0, W // 2)), int(rng.integers(0, H // 2)),
                 int(rng.integers(2, W // 2)), int(rng.integers(2, H // 2))) for _ in range(int(rng.integers(1, 4)))]
    dtype = "f32" if rng.random() < 0.4 else "u8"
    mode = ["no-aspect-ratio", "aspect-ratio", "crop"][int(rng.integers(0, 3))]
    kw = {"resize": "aspect-ratio", "crop": "central"} if mode == "crop" else {"resize": mode}
    info = evam.PreProcInfo(placement="center", fill=(1, 2, 3), **({"range": (0.0, 1.0)} if dtype == "f32" else {}),
                            **kw)
    n = len(rois) if rois else len(frames)
    shape = (n, 3, DH, DW)
    got, _ = run_hip(evam, torch, upload(evam, frames, gpu), shape, torch.float32 if dtype == "f32" else torch.uint8,
                     info, rois=[evam.Roi(*r) for r in rois] if rois else None, pp=fuzz_pp)
    ref, _ = run_oracle(O, coracle, frames, shape, dtype, info, rois=rois)
    assert_same(got, ref, f"seed {seed}: {fmt} {W}x{H} x{len(frames)} -> {DW}x{DH} {dtype} {kw} "
                          f"{'%d rois' % n if rois else 'frames'}")


@pytest.mark.parametrize("seed", range(int(os.environ.get("EVAM_FUZZ_INVALID_CASES", "24"))))
def test_random_invalid_calls(evam, O, coracle, gpu, fuzz_pp, seed):
    """A random valid call (random_case) broken in one way — an ROI outside its frame, a source index out of range, a
    slot past the tensor, a repeated explicit slot, a misaligned plane pitch, an odd 4:2:0 size: the call fails with
    the documented status before anything is written (the output keeps its fill), and the same handle then runs the
    unbroken call bit-exact."""
    import torch

    rng = np.random.default_rng(60000 + seed)
    fmt, frames, shape, dtype, info, rois, offset, stride = random_case(evam, O, rng)
    imgs = upload(evam, frames, gpu)
    n_items = len(rois) if rois else len(frames)
    kinds = ["empty_roi", "src_index", "slot_past_end", "misaligned_pitch"]
    if n_items >= 2:
        kinds.append("repeated_slot")
    if fmt in ("NV12", "I420"):
        kinds.append("odd_420")
    kind = kinds[int(rng.integers(0, len(kinds)))]
    bad_imgs, bad_rois = list(imgs), list(rois) if rois else [(i, 0, 0, 0, 0) for i in range(len(frames))]
    kw = {"slot_offset": offset, "slot_stride": stride}
    if kind == "empty_roi":  # the last item replaced: the item count (and so every slot) stays valid
        W, H = frames[0].width, frames[0].height
        bad_rois[-1] = (0, W + 5, H + 5, 4, 4)
    elif kind == "src_index":
        bad_rois[-1] = (len(frames), 0, 0, 0, 0)
    elif kind == "slot_past_end":
        kw["slot_offset"] = shape[0] - (n_items - 1) * stride  # the last item one slot past the end
    elif kind == "repeated_slot":
        kw = {"slots": np.array([0] * n_items, dtype=np.int32)}
    elif kind == "misaligned_pitch":
        im = imgs[0]
        p0 = im.planes[0]
        pitch = p0.shape[1] + 8  # >= the row bytes, not a multiple of 16
        q = torch.zeros((p0.shape[0], pitch), dtype=torch.uint8, device=gpu)
        bad_imgs[0] = evam.Image(im.fourcc, im.width, im.height, [q] + list(im.planes[1:]))
    elif kind == "odd_420":
        im = imgs[0]
        bad_imgs[0] = evam.Image(im.fourcc, im.width - 1, im.height, list(im.planes))
    want = {"empty_roi": -4, "src_index": -1, "slot_past_end": -1, "repeated_slot": -1, "misaligned_pitch": -3,
            "odd_420": -1}[kind]
    tdt = torch.float32 if dtype == "f32" else torch.uint8
    if kind in ("misaligned_pitch", "odd_420", "repeated_slot") and not rois:
        bad_rois = None  # a frame-list call
    out = torch.full(shape, 7, dtype=tdt, device=gpu)
    with pytest.raises(evam.PreProcError) as ei:
        fuzz_pp.convert(bad_imgs, out, info, rois=[evam.Roi(*r) for r in bad_rois] if bad_rois else None, **kw)
    torch.cuda.synchronize()
    assert ei.value.status == want, f"seed {seed} {kind}: {ei.value}"
    assert bool((out == 7).all()), f"seed {seed} {kind}: the failed call wrote into the output"
    got, _ = run_hip(evam, torch, imgs, shape, tdt, info, rois=[evam.Roi(*r) for r in rois] if rois else None,
                     slot_offset=offset, slot_stride=stride, pp=fuzz_pp)
    ref, _ = run_oracle(O, coracle, frames, shape, dtype, info, rois=rois, slot_offset=offset, slot_stride=stride)
    assert_same(got, ref, f"seed {seed}: the call after a {kind} failure")
