#!/usr/bin/env python3
"""Host-side cost of the pipeline-server path per frame, on CPU: PipelineServer's device runner with the HIP
pre-processor replaced by a stub that does the host part of a real call (ImageBatch marshalling, the slot table) but
launches nothing, so the rate printed is the ceiling the Python layer puts on `bench.py --via pipeline`.

    python tools/pipeline_host_profile.py [--config c5|c2] [--streams 32] [--frames 4096] [--profile]
"""
import argparse
import cProfile
import json
import os
import pstats
import queue
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c5", choices=["c2", "c5"])
    ap.add_argument("--streams", type=int, default=32)
    ap.add_argument("--frames", type=int, default=4096)
    ap.add_argument("--hub-batch", type=int, default=256)
    ap.add_argument("--stream-batch", type=int, default=16)
    ap.add_argument("--profile", action="store_true")
    args = ap.parse_args()

    import numpy as np
    import torch

    import __graft_entry__ as g
    import bench

    evam = g.import_package()
    ps, pre = evam.pipeline_server, evam.preproc

    class HostOnlyPP:
        def __init__(self, device=0, stream=None):
            pass

        def convert(self, srcs, out, info=None, rois=None, slot_offset=0, slot_stride=1, want_transform=False,
                    slots=None):
            b = srcs if isinstance(srcs, pre.ImageBatch) else pre.ImageBatch(srcs)
            if slots is not None:
                np.ascontiguousarray(slots, dtype=np.int32)
            if want_transform:
                return [None] * len(b)

        def close(self):
            pass

    pre.HipPreProcessor = HostOnlyPP
    ps.ClipRing._page = lambda self: torch.zeros((self.ROWS * 16, 3, 2, 2))
    ps._InferenceStage._tensor = lambda self, n: torch.zeros((n, 3, 2, 2))
    wl = bench.WORKLOADS[args.config]
    action = bool(wl.get("ring"))
    tmp = tempfile.mkdtemp(prefix="evam_hostprof_")
    kind, net = ("action_recognition", "bench_action") if action else ("object_detection", "bench_detector")
    pdir = os.path.join(tmp, "pipelines", kind, "bench")
    os.makedirs(pdir)
    json.dump(bench.ACTION_TEMPLATE if action else bench.PIPE_TEMPLATE, open(os.path.join(pdir, "pipeline.json"), "w"))
    mdir = os.path.join(tmp, "models", net, "1")
    os.makedirs(os.path.join(mdir, "FP32"))
    open(os.path.join(mdir, "FP32", f"{net}.xml"), "w").write(bench.IR_STUB.format(w=2, h=2))
    json.dump({"input_preproc": [{"format": "image", "params": {"resize": "aspect-ratio", "crop": "central"}}]
               if action else []}, open(os.path.join(mdir, f"{net}.json"), "w"))
    empty = torch.full((1, 1, 7), -1.0)
    ps.PipelineServer.start({"pipeline_dir": os.path.join(tmp, "pipelines"), "model_dir": os.path.join(tmp, "models"),
                             "batch_max": args.hub_batch, "batch_target": args.hub_batch, "batch_wait_ms": 1.0})
    ps.PipelineServer.register_model(f"{net}/1", ps.InferenceModel(lambda t: empty.expand(t.shape[0], 1, 7), (2, 2)))
    fc = pre.FOURCC_BY_NAME["NV12"]
    planes = [torch.zeros((1080, 1920), dtype=torch.uint8), torch.zeros((540, 1920), dtype=torch.uint8)]
    pool = [pre.Image(fc, 1920, 1080, planes) for _ in range(64)]
    S, F = args.streams, args.frames
    qs = []
    for k in range(S):
        q = queue.Queue()
        for t in range(F):
            q.put(pool[(k + t) % len(pool)])
        q.put(None)
        qs.append(q)
    prof = cProfile.Profile() if args.profile else None
    if prof:  # the work runs on the device runner's thread: profile that thread's loop
        loop = ps.DeviceRunner._loop

        def profiled(self):
            prof.enable()
            try:
                loop(self)
            finally:
                prof.disable()

        ps.DeviceRunner._loop = profiled
    t0 = time.perf_counter()
    pipes = []
    for k in range(S):
        p = ps.PipelineServer.pipeline(kind, "bench")
        p.start(source={"type": "application", "input": qs[k]}, destination={},
                parameters={("action-properties" if action else "detection-properties"): {"batch-size": args.stream_batch}})
        pipes.append(p)
    for p in pipes:
        assert p.wait(600)["state"] == "COMPLETED"
    el = time.perf_counter() - t0
    ps.PipelineServer.stop()
    print(json.dumps({"config": args.config, "frames": S * F, "host_only_frames_per_s": round(S * F / el, 1),
                      "us_per_frame": round(el / (S * F) * 1e6, 3)}))
    if prof:
        pstats.Stats(prof).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
