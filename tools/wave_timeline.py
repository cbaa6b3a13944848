#!/usr/bin/env python3
"""Per-wave timeline of one strip- or band-kernel launch (diagnostic; needs the trace build).

Build:  tools/build_variant.sh trace "-DEVAM_PP_TRACE=1"      (ab/libevam_pp_trace.so)
Run:    EVAM_PP_LIB=ab/libevam_pp_trace.so EVAM_PP_DIAGNOSTIC_BUILD_OK=1 python tools/wave_timeline.py --config c2

Runs bench.py's own workload (pooled frame sets, device-resident), then reads the stamps every wave of the
last launch wrote on the 100 MHz constant clock (10 ns): entry, first DMA issued, LUT barrier passed, first
row's DMA landed, end (last stores retired). The band kernel (C1) stamps its first row's landing as both the
LUT barrier and the landing, and its workgroups hold two waves (the dispatch rank assumes four). Prints phase distributions, the active waves over time and
per-XCD end times, as one JSON object.
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
SLOTS = 12  # kTraceSlots of the trace build


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=["c1", "c2", "c4", "c5"])  # C3: tools/roi_timeline.py
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
    ring = wl.get("ring")
    info = bench.make_info(evam, wl)
    DW, DH = wl["dst"]
    sets = [evam.ImageBatch(bench.device_frames(evam, torch, wl, n, dev, seed=1234 + 7919 * k)) for k in range(5)]
    dt = torch.float32 if wl["dtype"] == "f32" else torch.uint8
    nout = n * (ring or 1)
    outs = [torch.empty((nout, 3, DH, DW), dtype=dt, device=dev) for _ in range(1 if ring else 5)]
    pp = evam.HipPreProcessor(device=0)
    lib = evam.native.load_library()
    lib.evam_pp_debug_trace.argtypes = [ctypes.c_void_p, ctypes.c_int]
    for t in range(a.steps):
        if t == a.steps - 1:  # clear, then trace the last launch only
            torch.cuda.synchronize()
            lib.evam_pp_debug_trace(None, 0)
        if ring:
            pp.convert(sets[t % 5], outs[0], info, slot_offset=t % ring, slot_stride=ring)
        else:
            pp.convert(sets[t % 5], outs[t % 5], info)
    torch.cuda.synchronize()
    cap = 16384
    buf = (ctypes.c_ulonglong * (SLOTS * cap))()
    rc = lib.evam_pp_debug_trace(ctypes.cast(buf, ctypes.c_void_p), cap)
    if rc:
        raise SystemExit(f"evam_pp_debug_trace: {rc}")
    tr = np.frombuffer(buf, dtype=np.uint64).reshape(cap, SLOTS)
    tr = tr[tr[:, 4] != 0]  # live waves of the traced launch
    t0 = tr[:, 0].astype(np.int64).min()
    t = (tr[:, :5].astype(np.int64) - t0) * 10 / 1000.0  # us from the first wave's entry
    rows = (tr[:, 5] >> 48).astype(int)
    idx = np.nonzero(np.frombuffer(buf, dtype=np.uint64).reshape(cap, SLOTS)[:, 4] != 0)[0]
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    rank = (idx // 4) // n_cu  # workgroups of 4 waves (C2 / C4 / C5 strip tiles)
    xcc = (tr[:, 6] & 0xFFFFFFFF).astype(int)

    def dist(v):
        q = np.percentile(v, [0, 10, 50, 90, 100])
        return [round(float(x), 2) for x in q]

    end = t[:, 4]
    loop = t[:, 4] - t[:, 3]
    res = {
        "config": a.config, "waves": int(len(tr)), "rows_per_wave": dist(rows),
        "phase_us_p0_p10_p50_p90_p100": {
            "entry": dist(t[:, 0]),
            "entry -> first DMA issued": dist(t[:, 1] - t[:, 0]),
            "first DMA issued -> LUT barrier": dist(t[:, 2] - t[:, 1]),
            "LUT barrier -> first row landed": dist(t[:, 3] - t[:, 2]),
            "first row landed -> end": dist(loop),
            "first row landed (absolute)": dist(t[:, 3]),
            "end (absolute)": dist(end)},
        "us_per_row_after_first": dist(loop / np.maximum(rows, 1)),
        "end_by_xcc": {int(x): round(float(end[xcc == x].max()), 2) for x in sorted(set(xcc.tolist()))},
        # dispatch-order rank of the wave's workgroup on its CU (linear workgroup index // CUs): the older
        # waves of a SIMD win its issue arbitration (MI355X_MICROARCH.md, Two waves per SIMD, item 2)
        "end_by_dispatch_rank": {int(r): dist(end[rank == r]) for r in sorted(set(rank.tolist()))},
        "us_per_row_by_dispatch_rank": {int(r): dist((loop / np.maximum(rows, 1))[rank == r])
                                        for r in sorted(set(rank.tolist()))},
        "active_waves_by_us": [int(((t[:, 0] <= u) & (end > u)).sum()) for u in np.arange(0, float(end.max()) + 1, 1.0)],
    }
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
