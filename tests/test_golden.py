"""Committed golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py).

These are oracle-generated regression vectors, so parity is unpinned (see make_golden.py). The CPU legs
check that both oracle restatements still reproduce them bit for bit. The GPU leg checks the HIP path
through the C ABI against the same bytes.
"""
import glob
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

import make_golden as G  # noqa: E402

CASES = sorted(glob.glob(os.path.join(HERE, "golden", "*.npz")))
IDS = [os.path.basename(p)[:-4] for p in CASES]


def test_fixture_set_complete():
    assert set(IDS) == set(G.CASES), "regenerate with tests/golden/make_golden.py"


def _bitwise_equal(a, b):
    return a.shape == b.shape and a.dtype == b.dtype and np.array_equal(a.view(np.uint8), b.view(np.uint8))


@pytest.mark.parametrize("path", CASES, ids=IDS)
def test_c_oracle_reproduces(path, coracle):
    meta, frames, expected = G.load_case(path)
    got = G.compute(frames, meta["items"], meta["info"], tuple(meta["dst"]), meta["dtype"], coracle)
    assert _bitwise_equal(got, expected)


@pytest.mark.parametrize("path", CASES, ids=IDS)
def test_numpy_oracle_reproduces(path, O):
    meta, frames, expected = G.load_case(path)
    DW, DH = meta["dst"]
    mode, placement, rgb, lut, fill = G.oracle_args(meta["info"])
    items = meta["items"] or [(i, 0, 0, 0, 0) for i in range(len(frames))]
    for k, (fi, x, y, w, h) in enumerate(items):
        ref = O.np_preprocess_item(frames[fi], (x, y, w, h), DW, DH, mode=mode, placement=placement,
                                   color_rgb=rgb, lut=lut if meta["dtype"] == "f32" else None, fill=fill)
        assert _bitwise_equal(ref, expected[k]), f"item {k}"


@pytest.mark.gpu
@pytest.mark.parametrize("path", CASES, ids=IDS)
def test_hip_matches_golden(path, evam, gpu):
    import torch

    meta, frames, expected = G.load_case(path)
    imgs = [evam.Image.from_host(f.fourcc, f.width, f.height, f.planes, device=gpu) for f in frames]
    info = evam.PreProcInfo(**{k: (tuple(v) if isinstance(v, list) else v) for k, v in meta["info"].items()})
    rois = [evam.Roi(*r) for r in meta["items"]] if meta["items"] else None
    out = torch.full(expected.shape, 7, dtype=torch.float32 if meta["dtype"] == "f32" else torch.uint8,
                     device=gpu)
    pp = evam.HipPreProcessor(device=0)
    pp.convert(imgs, out, info, rois=rois)
    torch.cuda.synchronize()
    pp.close()
    assert _bitwise_equal(out.cpu().numpy(), expected)
