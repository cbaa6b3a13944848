"""GPU parity on the exact BASELINE workloads bench.py times, at full size, bit-exact vs the C oracle.

Each test builds its inputs with bench.py's own generators: the seeded device frames of
``bench.device_frames`` (copied back to the host for the oracle) and, for C3, the ``bench.seed_rois`` ROI
sets. So the numbers bench.py reports are quoted on launches whose outputs are checked here element by
element. Reference anchors: ``models_list/vehicle-detection-0202.json:3`` (C1/C2 default pre-proc),
``pipelines/object_classification/vehicle_attributes/pipeline.json:4-5`` (C3 gvaclassify ROIs),
``models_list/action-recognition-0001.json:3-13`` (C5 aspect-ratio + central crop).
"""
import numpy as np
import pytest

import bench
from test_gpu_parity import assert_same, info_lut

pytestmark = pytest.mark.gpu


def host_frames(O, imgs):
    """Host copies of bench's device frames (same bytes, same pitches) for the oracle."""
    return [O.HostFrame(im.fourcc, im.width, im.height, [p.cpu().numpy() for p in im.planes]) for im in imgs]


def oracle_items(O, coracle, frames, items, out_shape, dtype, info, slot=lambda i: i):
    ref = np.zeros(out_shape, np.float32 if dtype == "f32" else np.uint8)
    lut = (info_lut(O, info) if info.range is not None or info.mean is not None else O.np_norm_lut(0)) \
        if dtype == "f32" else None
    mode = info.resize_mode()
    placement = 1 if info.placement == "center" else 0
    for i, (si, x, y, w, h) in enumerate(items):
        coracle.preprocess_item(frames[si], (x, y, w, h), ref, slot(i), mode=mode, placement=placement,
                                color_rgb=info.color_space == "RGB", lut=lut, fill=info.fill)
    return ref


@pytest.mark.parametrize("shape", ["default", "band_nodd", "band_px2", "band_th16", "ahead64", "noprio", "wave"])
def test_c1_bench_batch(evam, O, coracle, gpu, shape, monkeypatch):
    """C1: 32 x 768x432 NV12 -> 32x3x512x512 u8, bench frames: the band kernel (default: six-column lanes;
    per-pixel taps; 2 pixels per lane; 16-row bands) and the wave kernel's REUSE path (EVAM_PP_WAVE=2)."""
    import torch

    for k, v in {"default": {}, "band_nodd": {"EVAM_PP_BAND_DD": "0"}, "band_px2": {"EVAM_PP_BAND_PX": "2"},
                 "band_th16": {"EVAM_PP_STRIP_TH": "16"},
                 "ahead64": {"EVAM_PP_BAND_AHEAD": "64"}, "noprio": {"EVAM_PP_PRIO": "0"},
                 "wave": {"EVAM_PP_WAVE": "2"}}[shape].items():
        monkeypatch.setenv(k, v)

    wl = bench.WORKLOADS["c1"]
    imgs = bench.device_frames(evam, torch, wl, 32, gpu, seed=1234)
    info = bench.make_info(evam, wl)
    out = torch.full((32, 3, 512, 512), 7, dtype=torch.uint8, device=gpu)
    pp = evam.HipPreProcessor(device=0)
    pp.convert(imgs, out, info)
    torch.cuda.synchronize()
    ref = oracle_items(O, coracle, host_frames(O, imgs), [(i, 0, 0, 0, 0) for i in range(32)], out.shape, "u8", info)
    assert_same(out.cpu().numpy(), ref, "C1 bench batch")
    pp.close()


@pytest.mark.parametrize("frames,family", [(1, "WAVE"), (4, "WAVE"), (8, "BAND")])
def test_c1_small_batches(evam, O, coracle, gpu, frames, family):
    """C1 at the reference's own batch (1 frame per launch, pipelines/object_detection/vehicle/pipeline.json:5) and
    other small batches: launches with fewer band rows than the band kernel's wave target run on the wave kernel
    (faster there, profiles/r04i_c1_small_batch_ab.txt), larger ones on the band kernel; both bit-exact."""
    import torch

    wl = bench.WORKLOADS["c1"]
    imgs = bench.device_frames(evam, torch, wl, frames, gpu, seed=77)
    info = bench.make_info(evam, wl)
    out = torch.full((frames, 3, 512, 512), 7, dtype=torch.uint8, device=gpu)
    pp = evam.HipPreProcessor(device=0)
    pp.convert(imgs, out, info)
    torch.cuda.synchronize()
    N = evam.native
    assert pp.stats().kernels == getattr(N, "KERNEL_" + family), pp.stats().kernels
    ref = oracle_items(O, coracle, host_frames(O, imgs), [(i, 0, 0, 0, 0) for i in range(frames)], out.shape, "u8", info)
    assert_same(out.cpu().numpy(), ref, f"C1 batch {frames}")
    pp.close()


# kernel shapes forced on the full-size workloads: the default choice (the strip kernel for C2 / C4 / C5),
# the strip kernel with one row per DMA instruction (unpaired taps) and other tile heights, and the staged kernel's
# pipeline shapes
STAGED_SHAPES = {"default": {},
                 "strip_unpaired": {"EVAM_PP_STRIP_PAIR": "0"},
                 "strip_th32": {"EVAM_PP_STRIP_TH": "32"},
                 "strip_px1": {"EVAM_PP_STRIP_PX": "1"},
                 "strip_px1_unpaired": {"EVAM_PP_STRIP_PX": "1", "EVAM_PP_STRIP_PAIR": "0"},
                 "staged": {"EVAM_PP_STRIP": "0"},
                 "r2": {"EVAM_PP_STRIP": "0", "EVAM_PP_STAGE_R": "2", "EVAM_PP_NSEGX": "4"},
                 "r1": {"EVAM_PP_STRIP": "0", "EVAM_PP_STAGE_R": "1", "EVAM_PP_NSEGX": "4"}}


@pytest.mark.parametrize("shape", sorted(STAGED_SHAPES))
def test_c2_bench_batch(evam, O, coracle, gpu, shape, monkeypatch):
    """C2 headline: 32 distinct 1080p NV12 frames (pitch 1920) -> 32x3x512x512 fp32 normalised, through the
    strip kernel (default, every ring depth, tall tiles) and every staged-kernel pipeline shape."""
    import torch

    for k, v in STAGED_SHAPES[shape].items():
        monkeypatch.setenv(k, v)

    wl = bench.WORKLOADS["c2"]
    imgs = bench.device_frames(evam, torch, wl, 32, gpu, seed=1234)
    assert imgs[0].pitches == [1920, 1920]
    info = bench.make_info(evam, wl)
    out = torch.full((32, 3, 512, 512), 7, dtype=torch.float32, device=gpu)
    pp = evam.HipPreProcessor(device=0)
    pp.convert(imgs, out, info)
    torch.cuda.synchronize()
    ref = oracle_items(O, coracle, host_frames(O, imgs), [(i, 0, 0, 0, 0) for i in range(32)], out.shape, "f32", info)
    assert_same(out.cpu().numpy(), ref, "C2 bench batch")
    pp.close()


@pytest.mark.parametrize("kernel", ["roi_tail1", "roi", "roi_noprio", "roi_unsorted", "roi_pinned", "roi_xcd"])
@pytest.mark.parametrize("seed", [0, 3])
def test_c3_bench_roi_set(evam, O, coracle, gpu, seed, kernel, monkeypatch):
    """C3: bench.py's seeded ROI set (50 per frame, w 24..400, h 24..300) on 32 bench 1080p NV12 frames ->
    1600x3x72x72 fp32 through the ROI kernel, with and without its tail split (EVAM_PP_ROI_TAIL: the 64 ROIs beyond 6
    per CU as row tiles), without progress-based priority (EVAM_PP_PRIO=0), without the largest-bytes pre-order and
    the snake deal over the CUs (EVAM_PP_ROI_SORT=0 EVAM_PP_ROI_SNAKE=0), with the records in pinned host memory
    instead of host-written device memory (EVAM_PP_REC_DEVICE=0) and with each frame's ROIs dealt to one XCD
    (EVAM_PP_ROI_XCD=1)."""
    import torch

    if kernel == "roi_pinned":
        monkeypatch.setenv("EVAM_PP_REC_DEVICE", "0")
        kernel = "roi"
    if kernel == "roi_xcd":  # each frame's ROIs dealt to one XCD (EVAM_PP_ROI_XCD=1)
        monkeypatch.setenv("EVAM_PP_ROI_XCD", "1")
        kernel = "roi"
    if kernel.endswith("_noprio"):
        monkeypatch.setenv("EVAM_PP_PRIO", "0")
        kernel = kernel[:-7]
    if kernel == "roi_unsorted":  # call order before the sort by row groups, bands dealt in one direction
        monkeypatch.setenv("EVAM_PP_ROI_SORT", "0")
        monkeypatch.setenv("EVAM_PP_ROI_SNAKE", "0")
    monkeypatch.setenv("EVAM_PP_ROI_TAIL", "1" if kernel == "roi_tail1" else "4")

    wl = bench.WORKLOADS["c3"]
    imgs = bench.device_frames(evam, torch, wl, 32, gpu, seed=1234)
    rois = bench.seed_rois(wl["rois"], 32, *wl["src"], seed=seed)
    assert len(rois) == 1600
    info = bench.make_info(evam, wl)
    out = torch.full((1600, 3, 72, 72), 7, dtype=torch.float32, device=gpu)
    pp = evam.HipPreProcessor(device=0)
    pp.convert(imgs, out, info, rois=evam.RoiBatch(np.array(rois, dtype=np.int32)))
    torch.cuda.synchronize()
    N = evam.native
    assert pp.stats().kernels == N.KERNEL_ROI
    ref = oracle_items(O, coracle, host_frames(O, imgs), rois, out.shape, "f32", info)
    assert_same(out.cpu().numpy(), ref, f"C3 bench ROI set seed {seed} {kernel}")
    pp.close()


@pytest.mark.parametrize("placement", ["top_left", "center"])
@pytest.mark.parametrize("shape", ["default", "strip_unpaired", "strip_th32", "strip_px1", "staged", "r2"])
def test_c4_random_4k_letterbox(evam, O, coracle, gpu, placement, shape, monkeypatch):
    """C4: random (not constant) 3840x2160 NV12 bench frames letterboxed to 640x640 fp32: every 6x gather
    (column taps 6dx+2, weights 1024/1024) on the real 4K pitch is checked, in both placements."""
    import torch

    for k, v in STAGED_SHAPES[shape].items():
        monkeypatch.setenv(k, v)
    wl = bench.WORKLOADS["c4"]
    imgs = bench.device_frames(evam, torch, wl, 2, gpu, seed=1234)
    info = bench.make_info(evam, wl)
    info.placement = placement
    out = torch.full((2, 3, 640, 640), 7, dtype=torch.float32, device=gpu)
    pp = evam.HipPreProcessor(device=0)
    xf = pp.convert(imgs, out, info, want_transform=True)
    torch.cuda.synchronize()
    assert (xf[0].resized_w, xf[0].resized_h, xf[0].pad_y) == (640, 360, 140 if placement == "center" else 0)
    ref = oracle_items(O, coracle, host_frames(O, imgs), [(0, 0, 0, 0, 0), (1, 0, 0, 0, 0)], out.shape, "f32", info)
    assert_same(out.cpu().numpy(), ref, f"C4 4K letterbox {placement}")
    pp.close()


@pytest.mark.parametrize("shape", ["default", "strip_unpaired", "strip_px1", "staged"])
def test_c5_ring_step(evam, O, coracle, gpu, shape, monkeypatch):
    """C5: a 32-stream clip-ring step (1080p NV12 -> aspect(max) 398x224 -> central crop 224x224 fp32 into
    slot t % 16 of a [32, 16, 3, 224, 224] ring), two steps with different frames and slots."""
    import torch

    for k, v in STAGED_SHAPES[shape].items():
        monkeypatch.setenv(k, v)
    wl = bench.WORKLOADS["c5"]
    info = bench.make_info(evam, wl)
    ring = torch.full((32 * 16, 3, 224, 224), 7, dtype=torch.float32, device=gpu)
    pp = evam.HipPreProcessor(device=0)
    for t in (0, 17):
        imgs = bench.device_frames(evam, torch, wl, 32, gpu, seed=1234 + t)
        pp.convert(imgs, ring, info, slot_offset=t % 16, slot_stride=16)
        torch.cuda.synchronize()
        slots = [s * 16 + t % 16 for s in range(32)]
        got = ring[slots].cpu().numpy()
        ref = oracle_items(O, coracle, host_frames(O, imgs), [(s, 0, 0, 0, 0) for s in range(32)],
                           (32, 3, 224, 224), "f32", info)
        assert_same(got, ref, f"C5 ring step t={t}")
    # slots no step wrote keep their initial value
    untouched = [s * 16 + 5 for s in range(32)]
    assert (ring[untouched] == 7).all().item()
    pp.close()


@pytest.mark.parametrize("variant", ["strip", "strip_unpaired", "wave"])
def test_c5_bgrx_ring_step(evam, O, coracle, gpu, variant, monkeypatch):
    """C5 with BGRx sources (bench.py c5_bgrx: 32 x 768x432 BGRx -> aspect(max) -> central crop 224x224 fp32 into
    ring slot t % 16): the strip kernel's packed-format path (the default), and the wave kernel it replaced."""
    import torch

    monkeypatch.setenv("EVAM_PP_STRIP", "0" if variant == "wave" else "1")
    if variant == "strip_unpaired":
        monkeypatch.setenv("EVAM_PP_STRIP_PAIR", "0")
    N = evam.native
    wl = bench.WORKLOADS["c5_bgrx"]
    info = bench.make_info(evam, wl)
    ring = torch.full((32 * 16, 3, 224, 224), 7, dtype=torch.float32, device=gpu)
    pp = evam.HipPreProcessor(device=0)
    t = 3
    imgs = bench.device_frames(evam, torch, wl, 32, gpu, seed=4321)
    pp.convert(imgs, ring, info, slot_offset=t, slot_stride=16)
    torch.cuda.synchronize()
    want = N.KERNEL_WAVE if variant == "wave" else N.KERNEL_STRIP
    assert pp.stats().kernels == want, (variant, pp.stats().kernels)
    got = ring[[s * 16 + t for s in range(32)]].cpu().numpy()
    ref = oracle_items(O, coracle, host_frames(O, imgs), [(s, 0, 0, 0, 0) for s in range(32)],
                       (32, 3, 224, 224), "f32", info)
    assert_same(got, ref, f"C5 BGRx ring step {variant}")
    pp.close()


@pytest.mark.parametrize("n_streams", [2, 3])
@pytest.mark.parametrize("config", ["c5", "c2"])
def test_inflight_two_streams_bit_equal(evam, gpu, config, n_streams):
    """bench.py --inflight N (default 3): successive launches rotate over N handles bound to N HIP streams (their
    outputs are independent, so the next launches' ramps overlap launch t's tail). The tensors equal one-at-a-time
    launches on one stream bit for bit (C5: four ring steps into one [32,16,...] clip ring; C2: four batches)."""
    import torch

    wl = bench.WORKLOADS[config]
    info = bench.make_info(evam, wl)
    sets = [evam.ImageBatch(bench.device_frames(evam, torch, wl, 32, gpu, seed=77 + k)) for k in range(2)]
    DW, DH = wl["dst"]
    ring = wl.get("ring")
    shape = (32 * ring, 3, DH, DW) if ring else (32, 3, DH, DW)

    def run(pps, streams):
        outs = [torch.full(shape, 7.0, device=gpu) for _ in range(1 if ring else 4)]
        for t in range(4):
            with torch.cuda.stream(streams[t % len(streams)]):
                if ring:
                    pps[t % len(pps)].convert(sets[t % 2], outs[0], info, slot_offset=t, slot_stride=ring)
                else:
                    pps[t % len(pps)].convert(sets[t % 2], outs[t], info)
        torch.cuda.synchronize()
        return [o.cpu() for o in outs]

    serial = run([evam.HipPreProcessor(device=0)], [torch.cuda.current_stream(gpu)])
    streams = [torch.cuda.Stream(gpu) for _ in range(n_streams)]
    pps = [evam.HipPreProcessor(device=0, stream=s) for s in streams]
    two = run(pps, streams)
    for a, b in zip(serial, two):
        assert torch.equal(a.view(torch.int32), b.view(torch.int32))
    for p in pps:
        p.close()


@pytest.mark.parametrize("rec_device", ["1", "0"])
def test_c3_roi_ring_full_queue(evam, gpu, rec_device, monkeypatch):
    """The ROI record ring under a full queue: 48 back-to-back C3-size calls (1,600 ROIs
    each, a different seeded ROI set every call, a different output tensor every call) with no host work or sync
    between them, so the 16 record slots wrap three times while the GPU still runs earlier calls and every slot is
    rewritten behind its fence. Records in host-written device memory (default) and in pinned host memory. Every
    output equals the same call run alone and synchronised, bit for bit (that single-call result is pinned against the
    oracle by test_c3_bench_roi_set)."""
    import torch

    monkeypatch.setenv("EVAM_PP_REC_DEVICE", rec_device)
    wl = bench.WORKLOADS["c3"]
    batch = evam.ImageBatch(bench.device_frames(evam, torch, wl, 32, gpu, seed=1234))
    info = bench.make_info(evam, wl)
    n_calls = 48
    sets = [evam.RoiBatch(np.array(bench.seed_rois(wl["rois"], 32, *wl["src"], seed=500 + k), dtype=np.int32))
            for k in range(n_calls)]
    assert all(len(s) == 1600 for s in sets)
    pp = evam.HipPreProcessor(device=0)
    outs = [torch.full((1600, 3, 72, 72), 7.0, device=gpu) for _ in range(n_calls)]
    torch.cuda.synchronize()
    for k in range(n_calls):
        pp.convert(batch, outs[k], info, rois=sets[k])
    torch.cuda.synchronize()
    assert pp.stats().kernels == evam.native.KERNEL_ROI
    ref = torch.full((1600, 3, 72, 72), 7.0, device=gpu)
    for k in range(n_calls):
        pp.convert(batch, ref, info, rois=sets[k])
        torch.cuda.synchronize()
        assert torch.equal(outs[k].view(torch.int32), ref.view(torch.int32)), f"call {k} (rec_device={rec_device})"
    pp.close()
