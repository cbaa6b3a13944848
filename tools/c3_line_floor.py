#!/usr/bin/env python3
"""C3 read-traffic floors (CPU only): algorithmic bytes vs the 128-B lines a per-ROI staging reads vs the per-frame
union of those lines (what a design sharing lines between overlapping ROIs of one frame would read), over
bench.py's four seeded ROI sets."""
import sys, numpy as np
import os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench
W, H, DW, DH = 1920, 1080, 72, 72
def rows_used(y0, ch):
    # OpenCV INTER_LINEAR row table: sy = floor((dy+0.5)*s-0.5), taps sy, sy+1 clamped
    s = ch / DH
    r = set()
    for dy in range(DH):
        fy = (dy + 0.5) * s - 0.5
        sy = int(np.floor(fy))
        for t in (sy, sy + 1):
            r.add(y0 + min(max(t, 0), ch - 1))
    return r
tot_alg = tot_lines = tot_union = 0
for seed in range(4):
    rois = bench.seed_rois(50, 32, W, H, seed=seed)
    per_frame = {}
    alg = lines = 0
    for f, x, y, w, h in rois:
        ry = rows_used(y, h)
        rc = {r >> 1 for r in ry}
        # luma: bytes x..x+w-1 ; chroma NV12: bytes 2*(x>>1) .. 2*((x+w-1)>>1)+1
        lx0, lx1 = x, x + w - 1
        cx0, cx1 = 2 * (x >> 1), 2 * ((x + w - 1) >> 1) + 1
        alg += len(ry) * w + len(rc) * (cx1 - cx0 + 1)
        nl_y = (lx1 // 128 - lx0 // 128 + 1); nl_c = (cx1 // 128 - cx0 // 128 + 1)
        lines += (len(ry) * nl_y + len(rc) * nl_c) * 128
        s = per_frame.setdefault(f, set())
        for r in ry:
            for l in range(lx0 // 128, lx1 // 128 + 1): s.add(("y", r, l))
        for r in rc:
            for l in range(cx0 // 128, cx1 // 128 + 1): s.add(("c", r, l))
    union = sum(len(s) for s in per_frame.values()) * 128
    print(f"seed {seed}: algorithmic reads {alg/1e6:.1f} MB, per-ROI 128-B lines {lines/1e6:.1f} MB ({lines/alg:.2f}x), "
          f"per-frame union of lines {union/1e6:.1f} MB ({union/alg:.2f}x)")
