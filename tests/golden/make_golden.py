#!/usr/bin/env python3
"""Regenerate the golden pre-processing fixtures in this directory.

    python tests/golden/make_golden.py

PARITY UNPINNED: the reference ships no tests or golden vectors for this path.
Its arithmetic lives in OpenCV 4.5 / DL Streamer 2022.1, and neither is present here. So these
fixtures come from this repository's CPU restatement (oracle/). They are produced by the C oracle,
and the script checks that the independent numpy restatement agrees bit for bit. They pin the
oracle and the HIP path against regressions. They are not a reference output.

Each case is one ``<name>.npz`` (no pickles), holding:
- ``meta``: a JSON string with frames, items, pre-processing info, output shape and dtype;
- ``f<i>_p<j>``: the planes of frame i;
- ``expected``: the output tensor.

The cases follow the model-proc configurations named in SURVEY.md §3 / BASELINE.json configs. They
are scaled down so the pure-numpy leg finishes in seconds.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle as O  # noqa: E402

IMAGENET_BGR = dict(range=(0.0, 1.0), mean=(0.406, 0.456, 0.485), std=(0.225, 0.224, 0.229))

# name: (frames [(fourcc, W, H, pattern)], items [(frame, x, y, w, h)] or None, info, (DW, DH), dtype)
CASES = {
    # gvadetect, C2 family: NV12 full frame -> square fp32, range [0,1] + mean/std
    "nv12_detect_f32": ([("NV12", 96, 54, "uniform"), ("NV12", 96, 54, "gradient")], None,
                        dict(IMAGENET_BGR), (64, 64), "f32"),
    # C1 family: NV12 -> u8 BGR planar, upscale
    "nv12_upscale_u8": ([("NV12", 48, 28, "gradient")], None, {}, (80, 80), "u8"),
    # gvaclassify, C3 family: ROIs incl. odd coordinates, partially outside, tiny; RGB + range only
    "i420_roi_classify_f32": ([("I420", 160, 90, "uniform")],
                              [(0, 10, 11, 33, 21), (0, 141, 70, 40, 40), (0, -5, -7, 20, 17),
                               (0, 0, 0, 0, 0), (0, 77, 3, 3, 80)],
                              dict(color_space="RGB", range=(0.0, 1.0)), (24, 24), "f32"),
    # YOLO-style letterbox, centred, fill 114
    "bgrx_letterbox_center_u8": ([("BGRX", 120, 68, "gradient")], None,
                                 dict(resize="aspect-ratio", placement="center", fill=(114, 114, 114)),
                                 (64, 64), "u8"),
    # action-recognition, C5 family: aspect(max) + central crop
    "nv12_aspect_central_crop_f32": ([("NV12", 128, 72, "uniform")], None,
                                     dict(resize="aspect-ratio", crop="central", range=(0.0, 255.0),
                                          mean=(110.0, 120.0, 130.0), std=(58.0, 57.0, 59.0)),
                                     (48, 48), "f32"),
    # packed BGR, identity size and 2x downscale (OpenCV's INTER_AREA special case)
    "bgr_identity_u8": ([("BGR", 40, 30, "uniform")], None, {}, (40, 30), "u8"),
    "bgr_half_u8": ([("BGR", 40, 30, "uniform")], None, {}, (20, 15), "u8"),
    # top-left letterbox of a portrait NV12 ROI with per-channel fill
    "nv12_roi_letterbox_u8": ([("NV12", 64, 64, "gradient")], [(0, 6, 2, 18, 50), (0, 30, 40, 30, 10)],
                              dict(resize="aspect-ratio", fill=(1, 2, 3)), (32, 32), "u8"),
    # SURVEY.md §8c size/ratio grid: 64x48 and 66x50 4:2:0 (odd chroma edge), BGRx 40x30;
    # resize ratios < 1, 1, 2 (INTER_AREA special case), ~3.75 and 6
    "nv12_64x48_ratio1_u8": ([("NV12", 64, 48, "uniform")], None, {}, (64, 48), "u8"),
    "nv12_64x48_ratio2_u8": ([("NV12", 64, 48, "uniform")], None, {}, (32, 24), "u8"),
    "i420_66x50_ratio3p75_u8": ([("I420", 66, 50, "uniform")], None, {}, (18, 13), "u8"),
    "nv12_66x50_ratio6_f32": ([("NV12", 66, 50, "gradient")], None, dict(IMAGENET_BGR), (11, 8), "f32"),
    "i420_64x48_upscale_f32": ([("I420", 64, 48, "gradient")], None, dict(range=(-1.0, 1.0)), (150, 112), "f32"),
    "bgrx_40x30_rois_u8": ([("BGRX", 40, 30, "uniform")],
                           [(0, 0, 0, 40, 30), (0, 39, 29, 5, 5), (0, 3, 5, 7, 9), (0, 20, -3, 30, 12)],
                           {}, (16, 16), "u8"),
}

FOURCC = {"NV12": O.NV12, "I420": O.I420, "BGRX": O.BGRX, "BGR": O.BGR}


def oracle_args(info: dict):
    resize = info.get("resize", "no-aspect-ratio")
    mode = 0 if resize != "aspect-ratio" else (2 if info.get("crop") == "central" else 1)
    placement = 1 if info.get("placement") == "center" else 0
    rgb = info.get("color_space") == "RGB"
    flags = (1 if "range" in info else 0) | (2 if ("mean" in info or "std" in info) else 0)
    lut = O.np_norm_lut(flags, info.get("range", (0.0, 255.0)), info.get("mean", (0, 0, 0)),
                        info.get("std", (1, 1, 1)))
    return mode, placement, rgb, lut, tuple(info.get("fill", (0, 0, 0)))


def compute(frames, items, info, dst, dtype, c):
    """Expected output through the C oracle, cross-checked against the numpy restatement."""
    DW, DH = dst
    items = items or [(i, 0, 0, 0, 0) for i in range(len(frames))]
    mode, placement, rgb, lut, fill = oracle_args(info)
    out = np.zeros((len(items), 3, DH, DW), np.float32 if dtype == "f32" else np.uint8)
    for k, (fi, x, y, w, h) in enumerate(items):
        c.preprocess_item(frames[fi], (x, y, w, h), out, k, mode=mode, placement=placement, color_rgb=rgb,
                          lut=lut if dtype == "f32" else None, fill=fill)
        ref = O.np_preprocess_item(frames[fi], (x, y, w, h), DW, DH, mode=mode, placement=placement,
                                   color_rgb=rgb, lut=lut if dtype == "f32" else None, fill=fill)
        if not np.array_equal(out[k].view(np.uint8), ref.view(np.uint8)):
            raise SystemExit(f"C and numpy oracles disagree on item {k}")
    return out


def load_case(path: str):
    """(meta, frames [HostFrame], expected) from one fixture file. Used by the tests too."""
    with np.load(path, allow_pickle=False) as z:
        meta = json.loads(str(z["meta"]))
        frames = []
        for i, f in enumerate(meta["frames"]):
            planes = [z[f"f{i}_p{j}"] for j in range(f["n_planes"])]
            frames.append(O.HostFrame(FOURCC[f["fourcc"]], f["width"], f["height"], planes))
        expected = z["expected"]
    return meta, frames, expected


def main():
    O.build_c_oracle()
    c = O.COracle()
    for idx, (name, (fspecs, items, info, dst, dtype)) in enumerate(sorted(CASES.items())):
        rng = np.random.default_rng(1000 + idx)
        frames = [O.random_frame(rng, FOURCC[fc], w, h, pattern=pat) for fc, w, h, pat in fspecs]
        expected = compute(frames, items, info, dst, dtype, c)
        meta = dict(name=name, dtype=dtype, dst=list(dst), info=info,
                    items=[list(r) for r in items] if items else None,
                    frames=[dict(fourcc=fc, width=w, height=h, n_planes=len(fr.planes))
                            for (fc, w, h, _), fr in zip(fspecs, frames)],
                    generator="oracle/evam_oracle.c (C) == oracle/oracle.py (numpy); parity unpinned")
        arrays = {f"f{i}_p{j}": p for i, fr in enumerate(frames) for j, p in enumerate(fr.planes)}
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), meta=np.array(json.dumps(meta)),
                            expected=expected, **arrays)
        print(f"{name}: {expected.shape} {expected.dtype}")


if __name__ == "__main__":
    main()
