#!/usr/bin/env python3
"""Per-workgroup timeline of one ROI-kernel launch (diagnostic; needs the trace build).

Build:  tools/build_variant.sh trace "-DEVAM_PP_TRACE=1"      (ab/libevam_pp_trace.so)
Run:    EVAM_PP_LIB=$PWD/ab/libevam_pp_trace.so python tools/roi_timeline.py [--config c3]

Runs bench.py's own workload (pooled frame sets, a new ROI set per step), then reads the stamps the
kernel wrote for the last launch: entry, after the record read + geometry, after the setup (tables,
per-lane state, first DMA issued), end of the row-group loop, on the 100 MHz constant clock (10 ns).
Prints phase distributions, the tail, how loop time scales with the ROI's row groups, and per-XCD end
times, as one JSON object.
"""
import argparse
import ctypes
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--steps", type=int, default=40)
    a = ap.parse_args()
    if "trace" not in os.environ.get("EVAM_PP_LIB", ""):
        raise SystemExit("set EVAM_PP_LIB to the -DEVAM_PP_TRACE build (ab/libevam_pp_trace.so)")
    import torch

    import bench

    evam = importlib.import_module("edge-video-analytics-microservice_amd")
    wl = bench.WORKLOADS[a.config]
    dev = torch.device("cuda:0")
    n = wl["frames"]
    info = bench.make_info(evam, wl)
    DW, DH = wl["dst"]
    rois = [evam.RoiBatch(np.array(bench.seed_rois(wl["rois"], n, *wl["src"], seed=k), dtype=np.int32))
            for k in range(bench.ROI_SETS)]
    sets = [evam.ImageBatch(bench.device_frames(evam, torch, wl, n, dev, seed=1234 + 7919 * k)) for k in range(5)]
    outs = [torch.empty((len(rois[0]), 3, DH, DW), dtype=torch.float32, device=dev) for _ in range(5)]
    pp = evam.HipPreProcessor(device=0)
    lib = evam.native.load_library()
    lib.evam_pp_debug_trace.argtypes = [ctypes.c_void_p, ctypes.c_int]
    for t in range(a.steps):
        if t == a.steps - 1:  # clear, then trace the last launch only
            torch.cuda.synchronize()
            lib.evam_pp_debug_trace(None, 0)
        pp.convert(sets[t % 5], outs[t % 5], info, rois=rois[t % len(rois)])
    torch.cuda.synchronize()
    cap = 4096
    buf = (ctypes.c_ulonglong * (12 * cap))()
    rc = lib.evam_pp_debug_trace(ctypes.cast(buf, ctypes.c_void_p), cap)
    if rc:
        raise SystemExit(f"evam_pp_debug_trace: {rc}")
    tr = np.frombuffer(buf, dtype=np.uint64).reshape(cap, 12)
    tr = tr[tr[:, 3] != 0]  # the traced launch's workgroups
    nwg = len(tr)
    t0 = tr[:, 0].astype(np.int64).min()
    t = (tr[:, :4].astype(np.int64) - t0) * 10 / 1000.0  # us from the first workgroup's entry
    s8, s9, s10 = ((tr[:, k].astype(np.int64) - t0) * 10 / 1000.0 for k in (8, 9, 10))
    cw, ch = (tr[:, 4] & 0xFFFFFFFF).astype(int), (tr[:, 4] >> 32).astype(int)
    ng, R = (tr[:, 5] & 0xFFFFFFFF).astype(int), (tr[:, 5] >> 32).astype(int)
    xcc = (tr[:, 6] & 0xFFFFFFFF).astype(int)
    nY = (tr[:, 7] & 0xFFFFFFFF).astype(int)

    def dist(v):
        q = np.percentile(v, [0, 10, 50, 90, 100])
        return [round(float(x), 2) for x in q]

    loop = t[:, 3] - t[:, 2]
    per_group = loop / np.maximum(ng, 1)
    end = t[:, 3]
    order = np.argsort(end)
    res = {
        "config": a.config, "workgroups": int(nwg),
        "phase_us_p0_p10_p50_p90_p100": {
            "entry": dist(t[:, 0]), "record+geometry": dist(t[:, 1] - t[:, 0]),
            "setup": dist(t[:, 2] - t[:, 1]), "loop": dist(loop), "end": dist(end),
            "setup: row table + LUT barrier": dist(s8 - t[:, 1]), "setup: column table barrier": dist(s9 - s8),
            "setup: per-lane state": dist(t[:, 2] - s9), "loop: group 0 DMA wait + barrier": dist(s10 - t[:, 2])},
        "groups_per_roi": dist(ng), "rows_per_group": dist(R), "us_per_group": dist(per_group),
        "last_10_to_finish": [{"end": round(float(end[i]), 2), "cw": int(cw[i]), "ch": int(ch[i]),
                               "groups": int(ng[i]), "R": int(R[i]), "nY": int(nY[i]),
                               "entry": round(float(t[i, 0]), 2), "loop": round(float(loop[i]), 2)}
                              for i in order[-10:]],
        "end_by_xcc": {int(x): round(float(end[xcc == x].max()), 2) for x in sorted(set(xcc.tolist()))},
        "active_workgroups_by_us": [int(((t[:, 0] <= u) & (end > u)).sum()) for u in range(0, int(end.max()) + 2, 2)],
    }
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
