"""Host->device feed: pinned ring + copy stream, parity with the oracle per batch."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("fmt,depth", [("NV12", 2), ("I420", 3), ("BGRX", 2)])
def test_feed_batches_match_oracle(evam, O, coracle, gpu, fmt, depth):
    import torch

    fc = {"NV12": O.NV12, "I420": O.I420, "BGRX": O.BGRX}[fmt]
    W, H, B, DW, DH = 200, 120, 3, 96, 64
    feed = evam.feed.HostFeed(fc, W, H, batch=B, depth=depth)
    pp = evam.HipPreProcessor(device=0)
    info = evam.PreProcInfo(range=(0.0, 1.0), mean=(0.5, 0.4, 0.3), std=(0.2, 0.25, 0.3))
    lut = O.np_norm_lut(3, (0.0, 1.0), (0.5, 0.4, 0.3), (0.2, 0.25, 0.3))
    rng = np.random.default_rng(11)
    outs, refs = [], []
    for step in range(2 * depth + 1):                       # wraps the ring at least twice
        frames = [O.random_frame(rng, fc, W, H) for _ in range(B)]
        k = feed.acquire()
        if step % 2:
            feed.fill(k, frames)
        else:                                               # decoder-writes-into-pinned path
            for i, f in enumerate(frames):
                for dst, src in zip(feed.host_planes(k)[i], f.planes):
                    dst[:, :src.shape[1]] = src
        feed.submit(k)
        out = torch.empty((B, 3, DH, DW), dtype=torch.float32, device=gpu)
        pp.convert(feed.batch(k), out, info)
        feed.release(k)
        outs.append(out)
        ref = np.zeros((B, 3, DH, DW), np.float32)
        for i, f in enumerate(frames):
            coracle.preprocess_item(f, None, ref, i, lut=lut)
        refs.append(ref)
    torch.cuda.synchronize()
    pp.close()
    for step, (o, r) in enumerate(zip(outs, refs)):
        assert np.array_equal(o.cpu().numpy().view(np.uint32), r.view(np.uint32)), f"step {step}"


def test_feed_rejects_oversize_batch(evam, O, gpu):
    feed = evam.feed.HostFeed("NV12", 64, 48, batch=1, depth=2)
    with pytest.raises(ValueError):
        feed.fill(feed.acquire(), [O.random_frame(np.random.default_rng(0), O.NV12, 64, 48)] * 2)


@pytest.mark.parametrize("fmt,resize,src,dst", [("NV12", "aspect-ratio", (384, 216), (64, 64)),
                                                ("I420", "no-aspect-ratio", (200, 120), (40, 20)),
                                                ("NV12", "crop", (320, 192), (48, 48)),
                                                ("NV12", "crop", (192, 320), (48, 48)),   # vertical crop, top > 0
                                                ("I420", "aspect-ratio", (200, 360), (40, 40)),
                                                ("BGRX", "no-aspect-ratio", (120, 96), (30, 24))])
def test_feed_touched_rows_only(evam, O, coracle, gpu, fmt, resize, src, dst):
    """set_geometry: only the rows the resize reads cross PCIe (strided 2-D copies); the device slots start
    poisoned (0xA5), so a kernel reading any row the plan skipped would break parity with the oracle."""
    import torch

    fc = {"NV12": O.NV12, "I420": O.I420, "BGRX": O.BGRX}[fmt]
    (W, H), (DW, DH), B = src, dst, 2
    kw = {"resize": "aspect-ratio", "crop": "central"} if resize == "crop" else {"resize": resize}
    info = evam.PreProcInfo(range=(0.0, 1.0), **kw)
    feed = evam.feed.HostFeed(fc, W, H, batch=B, depth=2)
    feed.set_geometry(DW, DH, info)
    for d in feed.dev:
        d.fill_(0xA5)
    assert feed.strided and feed.bytes_per_batch < B * feed.frame_bytes
    pp = evam.HipPreProcessor(device=0)
    lut = O.np_norm_lut(1, (0.0, 1.0))
    rng = np.random.default_rng(5)
    mode = info.resize_mode()
    for step in range(3):
        frames = [O.random_frame(rng, fc, W, H) for _ in range(B)]
        k = feed.acquire()
        feed.fill(k, frames)
        feed.submit(k)
        out = torch.empty((B, 3, DH, DW), dtype=torch.float32, device=gpu)
        pp.convert(feed.batch(k), out, info)
        feed.release(k)
        torch.cuda.synchronize()
        ref = np.zeros((B, 3, DH, DW), np.float32)
        for i, f in enumerate(frames):
            coracle.preprocess_item(f, None, ref, i, mode=mode, lut=lut)
        assert np.array_equal(out.cpu().numpy().view(np.uint32), ref.view(np.uint32)), f"step {step}"
    pp.close()


@pytest.mark.parametrize("seed", range(int(os.environ.get("EVAM_FUZZ_FEED_CASES", "12"))))
def test_feed_touched_rows_random(evam, O, coracle, gpu, seed):
    """Random geometries through set_geometry's touched-row feed: format, frame and tensor sizes, the three resize
    modes, placement, batch; the device slots start poisoned (0xA5), so a row the plan skipped but a kernel reads
    breaks parity with the oracle."""
    import torch

    rng = np.random.default_rng(9000 + seed)
    fmt = ["NV12", "I420", "BGRX"][int(rng.integers(0, 3))]
    fc = {"NV12": O.NV12, "I420": O.I420, "BGRX": O.BGRX}[fmt]
    W, H = int(rng.integers(8, 900)), int(rng.integers(8, 700))
    if fmt != "BGRX":
        W, H = W + (W & 1), H + (H & 1)
    DW, DH, B = int(rng.integers(1, 300)), int(rng.integers(1, 300)), int(rng.integers(1, 5))
    mode = ["no-aspect-ratio", "aspect-ratio", "crop"][int(rng.integers(0, 3))]
    kw = {"resize": "aspect-ratio", "crop": "central"} if mode == "crop" else {"resize": mode}
    info = evam.PreProcInfo(range=(0.0, 1.0), placement="center" if rng.random() < 0.5 else "top_left",
                            fill=(3, 130, 250), **kw)
    feed = evam.feed.HostFeed(fc, W, H, batch=B, depth=2)
    feed.set_geometry(DW, DH, info)
    for d in feed.dev:
        d.fill_(0xA5)
    pp = evam.HipPreProcessor(device=0)
    try:
        for step in range(2):
            frames = [O.random_frame(rng, fc, W, H) for _ in range(B)]
            k = feed.acquire()
            feed.fill(k, frames)
            feed.submit(k)
            out = torch.empty((B, 3, DH, DW), dtype=torch.float32, device=gpu)
            pp.convert(feed.batch(k), out, info)
            feed.release(k)
            torch.cuda.synchronize()
            ref, _ = _oracle_batch(O, coracle, frames, (B, 3, DH, DW), info)
            assert np.array_equal(out.cpu().numpy().view(np.uint32), ref.view(np.uint32)), \
                f"seed {seed} step {step}: {fmt} {W}x{H} -> {DW}x{DH} {kw} B {B}"
    finally:
        pp.close()


def _oracle_batch(O, coracle, frames, shape, info):
    ref = np.zeros(shape, np.float32)
    lut = O.np_norm_lut(1, (0.0, 1.0))
    geoms = [coracle.preprocess_item(f, None, ref, i, mode=info.resize_mode(),
                                     placement=1 if info.placement == "center" else 0, lut=lut, fill=info.fill)
             for i, f in enumerate(frames)]
    return ref, geoms
