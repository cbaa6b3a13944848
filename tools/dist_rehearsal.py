#!/usr/bin/env python3
"""One rank of a multi-process pre-processing run (streams partitioned s mod G).

Launched once per rank (torchrun, or tests/test_dist_gpu.py's subprocesses) with RANK / WORLD_SIZE /
MASTER_ADDR / MASTER_PORT in the environment. Every rank pre-processes the streams it owns of a fixed
stream set through its own HipPreProcessor on its own device (LOCAL_RANK mod the visible devices, so
several ranks may share one GPU in a rehearsal), writes its outputs keyed by stream id, and joins the
post-run reduction (streams.reduce_run) over gloo. Nothing crosses ranks on the data path.

    python tools/dist_rehearsal.py --config c2 --streams 8 --out /tmp/rank.npz
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=["c2", "c4", "c5"])
    ap.add_argument("--streams", type=int, default=8)
    ap.add_argument("--out", required=True)
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    import __graft_entry__ as g
    import bench

    evam = g.import_package()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank))) % max(1, torch.cuda.device_count())
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    device = torch.device(f"cuda:{local}")
    torch.cuda.set_device(device)

    wl = bench.WORKLOADS[args.config]
    mine = evam.streams.streams_for_rank(args.streams, world, rank)
    DW, DH = wl["dst"]
    ring = wl.get("ring")
    pp = evam.HipPreProcessor(device=local)
    pp.set_option(evam.native.OPT_STATS, 1)
    info = bench.make_info(evam, wl)
    # C5: each owned stream keeps its own 16-slot clip ring on this rank (rings partitioned over ranks); the
    # rehearsal runs steps t = 0, 1 and 17 (slot 1 written twice: the later frame wins), every step's
    # frame a function of (stream, t) only, so any partition sees the same bytes
    steps = (0, 1, 17) if ring else (0,)
    out = torch.full((len(mine) * (ring or 1), 3, DH, DW), 7.0, dtype=torch.float32, device=device)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    alg = 0
    for t in steps:
        imgs = [bench.device_frames(evam, torch, wl, 1, device, seed=100 + s + 1000 * t)[0] for s in mine]
        if mine:
            if ring:
                pp.convert(imgs, out, info, slot_offset=t % ring, slot_stride=ring)
            else:
                pp.convert(imgs, out, info)
            st = pp.stats()
            alg += int(st.src_bytes + st.dst_bytes)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    tot = evam.streams.reduce_run(elapsed, len(mine) * len(steps), alg, device_key=evam.streams.device_key(local))
    np.savez(args.out, streams=np.array(mine, dtype=np.int64), out=out.cpu().numpy())
    print(json.dumps({"rank": rank, "world": tot.world, "frames": tot.frames, "alg_bytes": tot.alg_bytes,
                      "per_rank_frames": tot.per_rank_frames, "elapsed_max_s": tot.elapsed_max_s,
                      "my_streams": mine, "device": local, "devices": tot.devices, "ring": ring or 1}),
          flush=True)
    pp.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
