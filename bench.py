#!/usr/bin/env python3
"""Benchmark of the EVAM pre-process hot path on MI355X (BASELINE.json metric).

Default workload (BASELINE.json configs[1], "C2"): a batch of 32 synthetic 1920x1080 NV12 frames,
device-resident, -> 32x3x512x512 fp32 NCHW normalised (range [0,1], ImageNet mean/std in BGR order),
one fused kernel launch per step, three steps in flight on three handles / HIP streams (the shape
PipelineServer's device runner runs by default; `--inflight 1` times one launch at a time, and every
line carries that one-at-a-time kernel figure as roofline.single_launch). Other configs (--config
c1|c3|c4|c5) are the remaining BASELINE workloads; the driver's headline line is c2.

    python bench.py [--gpus N --steps K --warmup W] [--config c2] [--no-cpu-baseline]

Multi-GPU: one process per GPU; camera streams are partitioned s mod G, every rank runs its own batch
(weak scaling), no collective touches the hot loop; after the timed region one all_reduce(MAX) of the
elapsed time and one all_gather of per-rank stats run over RCCL. `bench.py --gpus N` started without a
launcher starts the N ranks itself (the environment torch.distributed.run would set); under torchrun
(`--nproc-per-node N ... bench.py --gpus N`) each rank runs directly.

HBM-honest by default: every step reads a different set of frames and writes a different output
tensor, from a pool whose footprint is >= 3x the 256 MiB Infinity Cache (MI355X_MICROARCH.md: a buffer
stays on-die only while everything touched between two of its uses fits in ~256 MiB), so the timed
launches stream from HBM, not from the die-level cache. `--pool 1` re-reads one resident set (the
round-1 mode); its numbers are reported as the secondary `roofline.resident` field either way.

Output: ONE JSON line from rank 0 with value = frames/s over all ranks, plus `roofline` (algorithmic
bytes per launch / mean launch time from HIP events on the launch stream) and `cpu_baseline` (the C
oracle, OpenMP on the host cores, on a bounded sample — rank 0 at N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
# VALU issue ceiling in wave64 instructions/s: 256 CUs x 4 SIMDs, one wave-instruction per 2 cycles per SIMD
# (32 lanes/cycle), 2.4 GHz max clock (MI355X_MICROARCH.md, Wave scheduling / chip parameters)
VALU_PEAK_GINST = 256 * 4 * 2.4e9 / 2 / 1e9
VALU_BOUND_CONFIGS = ("c1",)  # u8 output: a fifth of C2's bytes for the same pixels, integer-issue bound
METRIC = "pre-processed frames/sec (1080p NV12→512² NCHW fp32) 1–8 GPU; % HBM peak"
BGR_MEAN = (0.406, 0.456, 0.485)
BGR_STD = (0.225, 0.224, 0.229)
ROI_SETS = 4  # C3: distinct seeded ROI sets cycled step by step
MALL_BYTES = 256 * 2**20  # MI355X Infinity Cache (die-level L3)

WORKLOADS = {
    "c1": dict(desc="C1: 768x432 NV12 -> 512x512 u8 BGR NCHW (no normalisation)", fourcc="NV12", src=(768, 432),
               frames=32, dst=(512, 512), dtype="u8", norm=False, mode="no-aspect-ratio"),
    "c2": dict(desc="C2: 32x 1920x1080 NV12 (pitch 1920, device-resident) -> 32x3x512x512 fp32 NCHW, "
                    "range [0,1] + mean/std", fourcc="NV12", src=(1920, 1080), frames=32, dst=(512, 512),
               dtype="f32", norm=True, mode="no-aspect-ratio"),
    "c3": dict(desc="C3: 32x 1080p NV12 frames x 50 ROIs (w 24..400, h 24..300; a new seeded set every step, "
                    "4 sets cycled) -> 1600x3x72x72 fp32",
               fourcc="NV12", src=(1920, 1080), frames=32, dst=(72, 72), dtype="f32", norm=True,
               mode="no-aspect-ratio", rois=50),
    "c4": dict(desc="C4: 64 streams x 3840x2160 NV12 -> 640x640 fp32 letterbox (640x360 + fill)", fourcc="NV12",
               src=(3840, 2160), frames=64, dst=(640, 640), dtype="f32", norm=True, mode="aspect-ratio"),
    "c5": dict(desc="C5: 32 streams x 1080p NV12 -> aspect(max) 398x224 -> central crop 224x224 fp32, "
                    "slot t%16 of a [32,16,3,224,224] clip ring", fourcc="NV12", src=(1920, 1080), frames=32,
               dst=(224, 224), dtype="f32", norm=False, mode="aspect-ratio", crop="central", ring=16),
}
# Format and batch variants of the configs: I420 is avdec_h264's output, i.e. the CPU
# decodebin path of pipelines/object_detection/vehicle/pipeline.json:4; BGRx is the action-recognition
# template's input (pipelines/action_recognition/general/pipeline.json:3, videoconvert ! BGRx) at the
# reference run's 768x432 (charts/README.md:117-119); C1 at batch 1 is the reference run's own shape
# (one stream, gvadetect at its default batch, pipelines/object_detection/vehicle/pipeline.json:5).
WORKLOADS.update({
    "c1_i420": dict(WORKLOADS["c1"], desc="C1/I420: 768x432 I420 -> 512x512 u8 BGR NCHW", fourcc="I420"),
    "c2_i420": dict(WORKLOADS["c2"], desc="C2/I420: 32x 1920x1080 I420 -> 32x3x512x512 fp32 NCHW, range [0,1] + "
                                          "mean/std", fourcc="I420"),
    "c5_bgrx": dict(WORKLOADS["c5"], desc="C5/BGRx: 32 streams x 768x432 BGRx -> aspect(max) 398x224 -> central crop "
                                          "224x224 fp32, slot t%16 of a [32,16,3,224,224] clip ring", fourcc="BGRX",
                    src=(768, 432)),
    "c1_b1": dict(WORKLOADS["c1"], desc="C1 batch 1: one 768x432 NV12 frame -> 1x3x512x512 u8 per launch (latency)",
                  frames=1),
})


def seed_rois(n_per_frame, n_frames, W, H, seed=0):
    rng = np.random.default_rng(seed)
    rois = []
    for f in range(n_frames):
        for _ in range(n_per_frame):
            w = int(rng.integers(24, 401))
            h = int(rng.integers(24, 301))
            x = int(rng.integers(0, W - w + 1))
            y = int(rng.integers(0, H - h + 1))
            rois.append((f, x, y, w, h))
    return rois


def make_info(evam, wl):
    kw = {}
    if wl["norm"]:
        kw.update(range=(0.0, 1.0), mean=BGR_MEAN, std=BGR_STD)
    if wl["mode"] == "aspect-ratio":
        kw.update(resize="aspect-ratio", crop=wl.get("crop"))
    return evam.PreProcInfo(**kw)


def device_frames(evam, torch, wl, n, device, seed):
    """n synthetic frames, i.i.d. uniform bytes from a seeded device generator (one surface each)."""
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    fc = evam.preproc.FOURCC_BY_NAME[wl["fourcc"]]
    W, H = wl["src"]
    imgs = []
    for _ in range(n):
        planes = [torch.randint(0, 256, (r, p), dtype=torch.uint8, device=device, generator=gen)
                  for r, p in evam.plane_layout(fc, W, H, pitch_align=16)]
        imgs.append(evam.Image(fc, W, H, planes))
    return imgs


def pool_sets(step_bytes: int, want: int) -> int:
    """Frame / output sets cycled by the timed loop: enough that the pool is >= 3x the Infinity Cache."""
    if want > 0:
        return want
    return max(1, min(64, -(-3 * MALL_BYTES // max(step_bytes, 1))))


def cpu_baseline(wl, budget_s: float):
    """Time the CPU baseline on the host cores: oracle/evam_cpu_fast.c, the oracle's exact arithmetic
    (byte-identical, tests/test_oracle.py::test_cpu_fast_matches_oracle) organised like OpenCV's optimised
    CPU path — one OpenMP region over (item, row stripe) tasks of the whole batch, each source row converted
    and horizontally resized once, AVX2 auto-vectorised loops. It converts only the source rows the resize
    reads, where the reference's cvtColor converts the whole crop, so it is an upper bound of the
    reference's CPU rate. The batch reads distinct frames (up to 256 MB of them), like the GPU pool."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # checker / baseline only

    O.build_c_oracle()
    c = O.COracle()
    cores = len(os.sched_getaffinity(0))
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit():
        cores = min(cores, int(env))
    c.set_num_threads(cores)
    rng = np.random.default_rng(0)
    fc = {"NV12": O.NV12, "I420": O.I420, "BGRX": O.BGRX, "BGR": O.BGR}[wl["fourcc"]]
    W, H = wl["src"]
    fbytes = W * H * 3 // 2 if wl["fourcc"] in ("NV12", "I420") else W * H * 4
    n = max(1, min(wl["frames"], (256 << 20) // max(1, fbytes)))
    frames = [O.random_frame(rng, fc, W, H) for _ in range(n)]
    DW, DH = wl["dst"]
    f32 = wl["dtype"] == "f32"
    lut = O.np_norm_lut(3, (0.0, 1.0), BGR_MEAN, BGR_STD) if wl["norm"] else O.np_norm_lut(0)
    mode = {"no-aspect-ratio": 0, "aspect-ratio": 2 if wl.get("crop") else 1}[wl["mode"]]
    rois = seed_rois(wl["rois"], n, W, H) if wl.get("rois") else None
    batch = O.FastBatch(c, frames, rois)
    out = np.zeros((len(rois) if rois else n, 3, DH, DW), np.float32 if f32 else np.uint8)
    batch.run(out, mode=mode, lut=lut if f32 else None)  # warm-up: page in the output, thread pool
    done = 0
    t0 = time.perf_counter()
    while True:
        batch.run(out, mode=mode, lut=lut if f32 else None)
        done += n
        el = time.perf_counter() - t0
        if el >= budget_s and done >= 2 * n:
            break
    items = f" ({len(rois)} ROIs)" if rois else ""
    return {"value": round(done / el, 3), "unit": "frames/s", "cores": cores, "kind": "port",
            "sample": f"{done} frames of {wl['desc'].split(':')[0]} in batches of {n} distinct frames{items} "
                      f"through oracle/evam_cpu_fast.c (oracle arithmetic, OpenCV-style row cache, AVX2, "
                      f"OpenMP {cores} threads; converts only rows the resize reads: an upper bound of the "
                      f"reference's full-crop cvtColor path) in {el:.1f} s"}


def load_pmc_traffic(config_name: str, n_frames_per_launch: int, pool: int):
    """HBM bytes per launch from the committed rocprofv3 PMC summary of this exact workload (same frames
    per launch and the same pool of cycled sets: a resident set's FETCH_SIZE counts Infinity-Cache hits)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    try:
        d = json.load(open(path))
        e = d.get(config_name)
        if e and e.get("frames_per_launch") == n_frames_per_launch and e.get("pool_sets", 1) == pool:
            return e.get("hbm_bytes_per_launch")
    except Exception:
        return None
    return None


PIPE_TEMPLATE = {
    "type": "GStreamer",
    "template": ["{auto_source} ! decodebin",
                 " ! gvadetect model={models[bench_detector][1][network]} name=detection",
                 " ! gvametaconvert name=metaconvert ! appsink name=appsink"],
    "description": "bench: full-frame detection pre-processing through the pipeline-server counterpart",
    "parameters": {"type": "object", "properties": {
        "detection-properties": {"element": {"name": "detection", "format": "element-properties"}}}},
}
ACTION_TEMPLATE = {
    "type": "GStreamer",
    "template": ["{auto_source} ! decodebin",
                 " ! gvaactionrecognitionbin enc-model={models[bench_action][1][network]} "
                 "model-proc={models[bench_action][1][proc]} name=action",
                 " ! gvametaconvert name=metaconvert ! appsink name=appsink"],
    "description": "bench: action-recognition encoder pre-processing (clip ring, no decoder) through the "
                   "pipeline-server counterpart",
    "parameters": {"type": "object", "properties": {
        "action-properties": {"element": {"name": "action", "format": "element-properties"}}}},
}
IR_STUB = ('<?xml version="1.0"?><net name="bench_detector" version="11"><layers><layer id="0" name="data" '
           'type="Parameter" version="opset1"><data shape="1,3,{h},{w}" element_type="f32"/></layer></layers></net>')


def via_pipeline(args, evam, torch, wl, device_index):
    """C2 frames through PipelineServer: `streams` application-source pipelines on one device, each fed
    `frames` device-resident frames; the per-device batching hub coalesces them into batched launches.
    The registered detector returns no detections, so the line measures pre-processing plus the pipeline
    machinery (queues, per-frame results, hub hand-off), not a model."""
    import queue
    import tempfile

    ps = evam.pipeline_server
    action = bool(wl.get("ring"))
    tmp = tempfile.mkdtemp(prefix="evam_bench_")
    kind, net = ("action_recognition", "bench_action") if action else ("object_detection", "bench_detector")
    pdir = os.path.join(tmp, "pipelines", kind, "bench")
    os.makedirs(pdir)
    json.dump(ACTION_TEMPLATE if action else PIPE_TEMPLATE, open(os.path.join(pdir, "pipeline.json"), "w"))
    DW, DH = wl["dst"]
    mdir = os.path.join(tmp, "models", net, "1")
    os.makedirs(os.path.join(mdir, "FP32"))
    open(os.path.join(mdir, "FP32", f"{net}.xml"), "w").write(IR_STUB.format(w=DW, h=DH))
    params = {}
    if wl["norm"]:
        params.update(range=[0.0, 1.0], mean=list(BGR_MEAN), std=list(BGR_STD))
    if wl["mode"] == "aspect-ratio":
        params.update(resize="aspect-ratio", **({"crop": wl["crop"]} if wl.get("crop") else {}))
    proc = {"input_preproc": [{"format": "image", "params": params}] if params else []}
    json.dump(proc, open(os.path.join(mdir, f"{net}.json"), "w"))
    empty = torch.full((1, 1, 7), -1.0)

    def detector(t):
        return empty.expand(t.shape[0], 1, 7)

    S, F = args.streams, args.frames_per_stream
    ps.PipelineServer.start({"pipeline_dir": os.path.join(tmp, "pipelines"), "model_dir": os.path.join(tmp, "models"),
                             "device": device_index, "batch_max": args.hub_batch, "batch_wait_ms": 1.0,
                             "batch_target": args.hub_batch, "runner": args.runner,
                             "inflight": args.runner_inflight})
    # C5: the encoder is never called (no dec-model: the stage only fills the clip ring, as bench.py's direct line)
    ps.PipelineServer.register_model(f"{net}/1", ps.InferenceModel(detector, (DW, DH), name="bench"))
    # distinct frames: at least 2 per stream and >= 3x the Infinity Cache, as the direct leg's pool
    W, H = wl["src"]
    n_pool = max(2 * S, -(-3 * MALL_BYTES // (W * H * 3 // 2)))
    pool = device_frames(evam, torch, wl, n_pool, torch.device(f"cuda:{device_index}"), seed=99)

    def run(frames_per_stream):
        qs, pipes = [], []
        for k in range(S):
            q = queue.Queue()
            for t in range(frames_per_stream):
                q.put(pool[(k + t * S) % len(pool)])
            q.put(None)
            qs.append(q)
        t0 = time.perf_counter()
        for k in range(S):
            p = ps.PipelineServer.pipeline(kind, "bench")
            p.start(source={"type": "application", "input": qs[k]}, destination={},
                    parameters={("action-properties" if action else "detection-properties"):
                                {"batch-size": args.stream_batch}})
            pipes.append(p)
        for p in pipes:
            st = p.wait(600)
            if st["state"] != "COMPLETED":
                raise RuntimeError(f"pipeline ended {st}")
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    run(max(2, args.stream_batch))  # warm-up: hub thread, handles, CUDA context
    ps.PipelineServer.hub().batches.clear()
    el = run(F)
    sizes = [b[1] for b in ps.PipelineServer.hub().batches]
    ps.PipelineServer.stop()
    return {"value": round(S * F / el, 1), "elapsed_s": round(el, 4), "streams": S, "frames_per_stream": F,
            "stream_batch_size": args.stream_batch, "runner": args.runner, "runner_inflight": args.runner_inflight,
            "pool_frames": n_pool,
            "hub_launches": len(sizes),
            "mean_frames_per_launch": round(float(np.mean(sizes)), 2) if sizes else 0.0}


def rank_envs(n: int, base: dict, port: int) -> list[dict]:
    """The environment torch.distributed.run gives each of n ranks on one node (one process per GPU,
    streams s mod n), for `bench.py --gpus n` started without a launcher."""
    envs = []
    for r in range(n):
        e = dict(base)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0",
                 ROLE_RANK=str(r), ROLE_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                 TORCHELASTIC_RUN_ID="evam-bench")
        envs.append(e)
    return envs


def launch_ranks(n: int, backend: str) -> int:
    """Start n rank processes of this script (one per GPU) and wait for them; rank 0 prints the aggregated line.
    Returns the exit status: non-zero if any rank failed (the others are then terminated). With RCCL ("nccl") each
    rank needs its own device, so fewer visible devices than n is an error, never a silent one-rank run. Runs before
    this process touches the GPU (torch.cuda.device_count() does not initialise it on this image)."""
    import socket
    import subprocess

    import torch

    if backend == "nccl":
        have = torch.cuda.device_count()
        if have < n:
            print(f"bench.py --gpus {n}: only {have} visible GPU(s); one rank per GPU needs {n} "
                  "(EVAM_BENCH_BACKEND=gloo rehearses several ranks on one GPU)", file=sys.stderr)
            return 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, os.path.abspath(__file__), *sys.argv[1:]]
    procs = [subprocess.Popen(cmd, env=e) for e in rank_envs(n, os.environ, port)]
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                print(f"bench.py --gpus {n}: rank {procs.index(p)} exited with {code}; stopping the others",
                      file=sys.stderr)
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc


def load_pmc_valu(config_name: str, n_frames_per_launch: int, pool: int):
    """Wave-level VALU instructions per launch from the committed rocprofv3 PMC summary, if any."""
    path = os.path.join(ROOT, "profiles", "pmc_valu.json")
    try:
        e = json.load(open(path)).get(config_name)
        if e and e.get("frames_per_launch") == n_frames_per_launch and e.get("pool_sets", 1) == pool:
            return int(e["valu_insts_per_launch"])
    except Exception:
        return None
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--config", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--frames", type=int, default=0, help="frames per rank per step (default: workload's)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--feed", choices=["device", "host"], default="device",
                    help="host: frames start in pinned host memory and cross PCIe every step (SURVEY §8 f3); "
                         "reported as a separate PCIe-inclusive line, never the headline value")
    ap.add_argument("--feed-rows", choices=["touched", "all"], default="touched",
                    help="--feed host: copy only the source rows the resize reads (default) or whole frames")
    ap.add_argument("--cpu-budget", type=float, default=12.0, help="seconds of CPU-baseline work")
    ap.add_argument("--pool", type=int, default=0,
                    help="frame/output sets cycled step by step (0: auto, >= 3x the 256 MiB Infinity Cache; "
                         "1: one resident set)")
    ap.add_argument("--resident-steps", type=int, default=200,
                    help="extra steps on one resident set, reported as roofline.resident (0: skip)")
    ap.add_argument("--via", choices=["direct", "pipeline"], default="direct",
                    help="pipeline: drive the workload's frames through PipelineServer (application-source "
                         "pipelines, one per stream, batched across streams by the per-device hub); reported "
                         "as its own line next to the direct kernel rate")
    ap.add_argument("--streams", type=int, default=32, help="--via pipeline: pipelines (streams)")
    ap.add_argument("--frames-per-stream", type=int, default=16384, help="--via pipeline: frames per stream")
    ap.add_argument("--stream-batch", type=int, default=16, help="--via pipeline: gvadetect batch-size per stream")
    ap.add_argument("--hub-batch", type=int, default=256, help="--via pipeline: max frames per hub launch")
    ap.add_argument("--inflight", type=int, default=3,
                    help="launches in flight: step t runs on handle/stream t mod N (independent outputs), so the next "
                         "launches' ramps overlap launch t's tail, timed by wall clock. The default 3 is the shape the "
                         "product runs (PipelineServer's device runner, server option inflight=3); the one-launch-at-"
                         "a-time kernel figure is reported next to it as roofline.single_launch either way")
    ap.add_argument("--runner-inflight", type=int, default=3,
                    help="--via pipeline: ticks the device runner keeps in flight (server option inflight)")
    ap.add_argument("--runner", choices=["device", "threads"], default="device",
                    help="--via pipeline: one runner thread per device (default) or one thread per pipeline")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `bench.py --gpus N` without a launcher: start the N ranks here (before anything touches the GPU)
        sys.exit(launch_ranks(args.gpus, os.environ.get("EVAM_BENCH_BACKEND", "nccl")))
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")

    import torch
    import torch.distributed as dist
    import __graft_entry__ as g

    evam = g.import_package()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU with --nproc-per-node "
                         f"{args.gpus} (or run bench.py --gpus {args.gpus} without a launcher)")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # EVAM_BENCH_BACKEND=gloo: rehearse the multi-process path with more ranks than GPUs (ranks share
    # devices round-robin; the post-run exchange goes over gloo on CPU tensors). Default: RCCL.
    backend = os.environ.get("EVAM_BENCH_BACKEND", "nccl")
    if backend == "gloo":
        local = local % max(1, torch.cuda.device_count())
    # EVAM_BENCH_PG=1: a process group even for one rank, so a one-GPU box runs the RCCL reduction path
    # (init, all_reduce MAX, all_gather on device tensors) that the driver's multi-GPU runs take
    pg = world > 1 or os.environ.get("EVAM_BENCH_PG") == "1"
    if pg:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group(backend)
    device = torch.device(f"cuda:{local}")
    torch.cuda.set_device(device)

    wl = WORKLOADS[args.config]
    if args.via == "pipeline":
        if world > 1 or wl.get("rois"):
            raise SystemExit("--via pipeline is wired for one process and the full-frame configs (c1, c2, c4, c5)")
        r = via_pipeline(args, evam, torch, wl, local)
        print(json.dumps({
            "metric": f"{METRIC} [{args.config}, via PipelineServer]", "value": r["value"], "unit": "frames/s",
            "n_gpus": 1, "higher_is_better": True, "dtype": "u8" if wl["dtype"] == "u8" else "u8->f32",
            "data": "synthetic device-resident frames through application sources; null detector",
            "config": {"workload": wl["desc"], **r,
                       "path": (("one runner thread per device: bulk ingest of every stream's queue -> "
                                 "gvaactionrecognitionbin stage -> one evam_pp_run_slots per tick over all streams' "
                                 "new frames into the shared [32,16,3,H,W] clip ring (no decoder) -> per-frame results")
                                if args.runner == "device" and wl.get("ring") else
                                "one runner thread per device: bulk ingest of every stream's queue -> gvadetect "
                                "stage -> one evam_pp_run per tick over all streams -> model -> per-frame results"
                                if args.runner == "device" else
                                "Pipeline thread per stream -> gvadetect stage -> per-device BatchHub -> one "
                                "evam_pp_run per tick -> model -> per-frame results")}}), flush=True)
        return
    n = args.frames or wl["frames"]
    strong = args.config == "c4" and world > 1 and not args.frames
    if strong:  # C4 is a fixed set of 64 streams, partitioned s mod G (strong split)
        n = len(evam.streams.streams_for_rank(wl["frames"], world, rank))
    info = make_info(evam, wl)
    DW, DH = wl["dst"]
    roi_sets = None
    if wl.get("rois"):
        # A new detection result every step: ROI sets cycle through ROI_SETS seeds, so every call
        # re-plans and re-uploads its descriptors (nothing is cached across steps).
        roi_sets = [evam.RoiBatch(np.array(seed_rois(wl["rois"], n, *wl["src"], seed=k), dtype=np.int32))
                    for k in range(ROI_SETS)]
    n_items = len(roi_sets[0]) if roi_sets is not None else n
    ring = wl.get("ring")
    out_n = n * ring if ring else n_items
    dtype = torch.float32 if wl["dtype"] == "f32" else torch.uint8
    esz = 4 if wl["dtype"] == "f32" else 1
    fc = evam.preproc.FOURCC_BY_NAME[wl["fourcc"]]
    in_bytes = n * sum(r * p for r, p in evam.plane_layout(fc, *wl["src"], pitch_align=16))
    out_step = n_items * 3 * DH * DW * esz  # output bytes one step writes
    # Pool: P frame sets and (full-tensor outputs) P output tensors, one of each per step, so a buffer is
    # touched again only after the whole pool went by. The clip ring already spreads its writes over
    # 16 slots, so it keeps one tensor.
    P = 1 if args.feed == "host" else pool_sets(in_bytes + out_step, args.pool)
    batches = [evam.ImageBatch(device_frames(evam, torch, wl, n, device, seed=1234 + rank + 7919 * k))
               for k in range(P)]
    n_out = 1 if ring else P
    outs = [torch.empty((out_n, 3, DH, DW), dtype=dtype, device=device) for _ in range(n_out)]
    pool_bytes = P * in_bytes + n_out * out_n * 3 * DH * DW * esz
    if args.inflight > 1:  # one handle per stream; the streams run side by side
        inflight_streams = [torch.cuda.Stream(device) for _ in range(args.inflight)]
        pps = [evam.HipPreProcessor(device=local, stream=st) for st in inflight_streams]
    else:
        pps = [evam.HipPreProcessor(device=local)]
    pp = pps[0]

    feed = None
    if args.feed == "host":
        if roi_sets is not None or ring:
            raise SystemExit("--feed host is wired for full-frame batches (c1, c2, c4)")
        feed = evam.feed.HostFeed(evam.preproc.FOURCC_BY_NAME[wl["fourcc"]], *wl["src"], batch=n, depth=3,
                                  device=local)
        if args.feed_rows == "touched":  # only the source rows the resize reads cross PCIe
            feed.set_geometry(DW, DH, info)
        frng = np.random.default_rng(1234 + rank)
        for hb in feed.host:   # stands in for a decoder writing into the pinned ring
            hb.numpy()[:] = frng.integers(0, 256, hb.numel(), dtype=np.uint8)

    def step(t, k=None, inflight=False):
        """One launch; k = pool set (default: set t mod P, so consecutive steps touch different sets).
        inflight: on handle t mod --inflight (its own stream)."""
        k = t % P if k is None else k
        out = outs[k % n_out]
        slot = t % len(pps) if inflight else 0
        pp = pps[slot]
        if feed is not None:
            # the copy wait and the consumed mark go on the stream the handle launches on
            st = inflight_streams[slot] if len(pps) > 1 else None
            j = feed.acquire()
            feed.submit(j)
            pp.convert(feed.batch(j, stream=st), out, info)
            feed.release(j, stream=st)
            return
        if ring:
            pp.convert(batches[k], out, info, slot_offset=t % ring, slot_stride=ring)
        else:
            pp.convert(batches[k], out, info, rois=roi_sets[t % ROI_SETS] if roi_sets else None)

    # algorithmic bytes per launch, from the library's own accounting
    pp.set_option(evam.native.OPT_STATS, 1)
    acc = []
    for t in range(ROI_SETS if roi_sets else 1):
        step(t)
        st = pp.stats()
        acc.append(int(st.src_bytes + st.dst_bytes))
    torch.cuda.synchronize()
    alg_bytes = int(round(sum(acc) / len(acc)))  # mean over the ROI sets a run cycles through
    pp.set_option(evam.native.OPT_STATS, 0)

    inflight = len(pps) > 1
    for t in range(args.warmup):
        step(t, inflight=inflight)
    stream = inflight_streams[0] if len(pps) > 1 else torch.cuda.current_stream(device)  # where pps[0] launches
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    if pg:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    # Launch-time events: e0 goes on the stream after step 0's launch, so e0 -> e1 spans launches 1 .. K-1 back
    # to back. Recorded before step 0, e0 also timed the idle GPU while the host enqueued step 0 (~20 us after
    # the synchronize: ~1 us per step of a 20-step run, profiles/r03y_bench_lines.txt). The wall clock (value)
    # still covers all K steps.
    ev_from = 1 if args.steps > 1 else 0
    if ev_from == 0:
        e0.record(stream)
    for t in range(args.steps):
        step(t, inflight=inflight)
        if t == 0 and ev_from == 1:
            e0.record(stream)
    t_submit = time.perf_counter() - t0  # host time to enqueue the K steps (≈ wall when host-bound)
    e1.record(stream)
    torch.cuda.synchronize()
    if pg:
        dist.barrier()
    wall = time.perf_counter() - t0
    kern_ms = e0.elapsed_time(e1) / (args.steps - ev_from)  # one launch per step
    if inflight:  # launches overlap on several streams: the launch rate is the wall-clock step
        kern_ms = wall / args.steps * 1e3
    # One launch at a time (the kernel-quality figure, comparable with a rocprof kernel average): back-to-back launches
    # of the same pooled workload on ONE handle and stream, HIP events on that stream from the end of the first launch
    # to the end of the last. Without launches in flight this is the timed loop's own event figure.
    if inflight:
        n_single = max(args.steps, 100)
        for t in range(10):
            step(t)
        s0 = torch.cuda.Event(enable_timing=True)
        s1 = torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        for t in range(n_single):
            step(t)
            if t == 0:
                s0.record(stream)
        s1.record(stream)
        torch.cuda.synchronize()
        single_ms, single_n = s0.elapsed_time(s1) / (n_single - 1), n_single - 1
    else:
        single_ms, single_n = kern_ms, args.steps - ev_from
    # Per-launch spread (median, p10 / p90), measured after the timed region: one event
    # pair around each of up to 200 extra steps, so the timed loop above carries no per-step events.
    n_dist = min(args.steps, 200)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n_dist)]
    for t, (a, b) in enumerate(evs):
        a.record(stream)
        step(t)
        b.record(stream)
    torch.cuda.synchronize()
    per = np.sort(np.array([a.elapsed_time(b) for a, b in evs])) if n_dist else np.zeros(1)
    pct = {q: round(float(np.percentile(per, q)), 5) for q in (10, 50, 90)}
    # Latency of one batch on an idle device: host enqueue -> kernel done, synchronised per step (the shape a
    # single camera stream sees; the throughput loop above keeps the device busy instead).
    n_lat = min(args.steps, 200)
    lat = []
    for t in range(n_lat):
        torch.cuda.synchronize()
        s0 = time.perf_counter()
        step(t)
        torch.cuda.synchronize()
        lat.append(time.perf_counter() - s0)
    lat_ms = np.array(lat) * 1e3 if lat else np.zeros(1)
    latency = {"items": n_items, "steps": n_lat,
               "ms_p10_p50_p90": [round(float(np.percentile(lat_ms, q)), 4) for q in (10, 50, 90)],
               "note": "host enqueue to kernel completion per launch, device idle before each"}
    # Host cost of one call, unthrottled: 12 calls enqueued back to back after a synchronize. That is fewer than
    # the pinned ROI-record ring's 16 slots, so no call waits for the GPU. host_submit_ms_per_step (the timed loop)
    # includes those waits: once the host runs 16 calls ahead of a GPU-bound stream, each call waits for the
    # kernel of 16 calls ago, and host_submit approaches ms_per_step however cheap the call is.
    host_us = None
    if feed is None:
        runs = []
        for _ in range(20):
            torch.cuda.synchronize()
            s0 = time.perf_counter()
            for t in range(12):
                step(t)
            runs.append((time.perf_counter() - s0) / 12)
        torch.cuda.synchronize()
        host_us = round(float(np.median(runs)) * 1e6, 2)
    # Secondary: the same launches re-reading ONE set (frames and output resident in the Infinity Cache
    # when they fit), for comparison with the pooled headline.
    resident = None
    if args.resident_steps > 0 and feed is None:
        for t in range(20):
            step(t, k=0)
        r0 = torch.cuda.Event(enable_timing=True)
        r1 = torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        r0.record(stream)
        for t in range(args.resident_steps):
            step(t, k=0)
        r1.record(stream)
        torch.cuda.synchronize()
        res_ms = r0.elapsed_time(r1) / args.resident_steps
        res_gbs = alg_bytes / (res_ms * 1e-3) / 1e9
        resident = {"achieved": round(res_gbs, 1), "frac": round(res_gbs / HBM_PEAK_GBS, 4),
                    "mean_launch_ms": round(res_ms, 5), "steps": args.resident_steps,
                    "set_bytes": in_bytes + out_n * 3 * DH * DW * esz}
    tot = evam.streams.reduce_run(wall, n * args.steps, alg_bytes * args.steps,
                                  device=device if pg and backend == "nccl" else None,
                                  device_key=evam.streams.device_key(local))
    wall_max = tot.elapsed_max_s
    value = tot.frames / wall_max
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    traffic = load_pmc_traffic(args.config, n, P)

    if rank == 0:
        res = {
            "metric": (METRIC if args.config == "c2" else f"{METRIC} [{args.config}]")
                      + (" [host feed, PCIe-inclusive]" if feed is not None else ""),
            "value": round(value, 1),
            "unit": "frames/s",
            # RCCL: one rank per GPU by construction (it refuses two ranks on one device); a gloo rehearsal may put
            # several ranks on one GPU, counted once by device_key
            "n_gpus": world if (pg and backend == "nccl") else tot.devices,
            "ranks": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall_max / args.steps * 1e3, 4),
            "host_submit_ms_per_step": round(t_submit / args.steps * 1e3, 4),
            "host_us_per_call": host_us,  # unthrottled host cost of one call (see above)
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "u8" if wl["dtype"] == "u8" else "u8->f32",
            "data": "synthetic (seeded uniform u8 planes generated on device; no video decode)",
            "config": {"workload": wl["desc"], "frames_per_gpu_per_step": n, "items_per_launch": n_items,
                       "src": f"{wl['src'][0]}x{wl['src'][1]} {wl['fourcc']}", "dst": f"{DW}x{DH}",
                       "pool_sets": P, "pool_bytes": pool_bytes,
                       "pool": "each step reads a different frame set and writes a different output tensor; "
                               "pool >= 3x the 256 MiB Infinity Cache" if P > 1 else "one resident set",
                       "launches_in_flight": len(pps),
                       "launch": (f"step t on handle t mod {len(pps)}, each bound to its own HIP stream (PipelineServer's "
                                  f"device runner, inflight={len(pps)}): launch t+1's ramp overlaps launch t's tail"
                                  if inflight else "one handle, one HIP stream, launches back to back"),
                       "parallelism": f"streams s mod {world}, one process per GPU, no hot-loop collective"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "algorithmic_bytes_per_launch": alg_bytes, "mean_launch_ms": round(kern_ms, 5),
                         "event_launches": args.steps - ev_from,
                         "timing": (f"algorithmic bytes of one step / wall-clock step time, {len(pps)} launches in "
                                    "flight on separate streams (kernels overlap: a rocprof kernel average is longer "
                                    "than the step; the one-at-a-time kernel figure is single_launch)"
                                    if inflight else "HIP events on the launch stream"),
                         "single_launch": {
                             "achieved": round(alg_bytes / (single_ms * 1e-3) / 1e9, 1),
                             "frac": round(alg_bytes / (single_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                             "mean_launch_ms": round(single_ms, 5), "launches": single_n,
                             "timing": "HIP events on one handle's stream, launches back to back, one at a time "
                                       "(compare with the rocprof kernel average of a one-stream run)"},
                         "launch_ms_p10_p50_p90": [pct[10], pct[50], pct[90]], "resident": resident},
            "latency": latency,
        }
        valu = load_pmc_valu(args.config, n, P) if args.config in VALU_BOUND_CONFIGS else None
        if valu:
            # integer-issue-bound workload: the roofline that bounds it is the VALU issue rate; the HBM
            # figures stay as a secondary block
            r = res["roofline"]
            hbm = {k: r[k] for k in ("achieved", "peak", "unit", "frac", "traffic")}
            g = valu / (kern_ms * 1e-3) / 1e9
            g1 = valu / (single_ms * 1e-3) / 1e9
            res["roofline"] = {"bound": "valu", "achieved": round(g, 1), "peak": VALU_PEAK_GINST,
                               "unit": "G wave64-VALU-inst/s", "frac": round(g / VALU_PEAK_GINST, 4),
                               "traffic": r["traffic"], "valu_insts_per_launch": valu, "hbm": hbm,
                               **{k: r[k] for k in ("algorithmic_bytes_per_launch", "mean_launch_ms", "event_launches",
                                                    "timing", "launch_ms_p10_p50_p90", "resident")},
                               "single_launch": dict(r["single_launch"], achieved=round(g1, 1),
                                                     frac=round(g1 / VALU_PEAK_GINST, 4),
                                                     hbm_frac=r["single_launch"]["frac"])}
        if feed is not None:
            res["h2d"] = {"bytes_per_step": feed.bytes_per_batch, "frame_bytes": feed.frame_bytes,
                          "rows": args.feed_rows,
                          "copy": "strided" if feed.strided else "contiguous",
                          "GBps": round(feed.bytes_per_batch * args.steps / wall_max / 1e9, 2),
                          "note": "frames copied from pinned host memory every step on a copy stream, overlapped "
                                  "with the kernel (depth-3 ring; rows=touched: only the source rows the resize "
                                  "reads, as strided 2-D copies unless they cover >= 85% of the frame); "
                                  "roofline.mean_launch_ms includes copy waits"}
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(wl, args.cpu_budget)
        else:
            res["cpu_baseline"] = None
        print(json.dumps(res), flush=True)
    for h in pps:
        h.close()
    if pg:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
