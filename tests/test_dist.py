"""Multi-GPU layout on CPU: stream partition (s mod G) and the post-run reduction over gloo, world 2."""
import os
import socket

import pytest


def test_partition_disjoint_and_complete(evam):
    S = evam.streams
    for world in (1, 2, 3, 8):
        for n in (0, 1, 7, 64):
            parts = [S.streams_for_rank(n, world, r) for r in range(world)]
            flat = sorted(s for p in parts for s in p)
            assert flat == list(range(n))
            for r, p in enumerate(parts):
                assert all(S.owner(s, world) == r for s in p)
    assert S.local_batch(list("abcdefg"), 3, 1) == ["b", "e"]
    with pytest.raises(ValueError):
        S.streams_for_rank(4, 2, 2)


def test_reduce_run_single_process(evam):
    t = evam.streams.reduce_run(0.5, 32, 1000)
    assert (t.world, t.frames, t.alg_bytes, t.devices) == (1, 32, 1000, 1)
    assert t.frames_per_s == 64.0


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import torch.distributed as dist

    import __graft_entry__ as g

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        evam = g.import_package()
        streams = evam.streams.streams_for_rank(64, world, rank)
        # per-rank "work": 32 frames of this rank's streams, elapsed differs per rank
        t = evam.streams.reduce_run(elapsed_s=1.0 + rank, frames=len(streams), alg_bytes=100 * len(streams),
                                    device_key=evam.streams.device_key(rank))
        # two ranks on one device (a rehearsal): counted as one GPU
        shared = evam.streams.reduce_run(1.0, 1, 1, device_key=evam.streams.device_key(0))
        q.put((rank, t.world, t.elapsed_max_s, t.frames, t.alg_bytes, t.per_rank_frames, t.devices, shared.devices))
    finally:
        dist.destroy_process_group()


def test_reduce_run_gloo_world2():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = sorted(q.get(timeout=10) for _ in range(2))
    for rank, world, el, frames, nbytes, per, devs, shared_devs in res:
        assert world == 2
        assert devs == 2 and shared_devs == 1
        assert el == 2.0                 # max over ranks
        assert frames == 64 and nbytes == 6400
        assert per == [32, 32]


def test_bench_rank_envs():
    """bench.py --gpus N without a launcher: the environment of each rank is torchrun's (RANK = LOCAL_RANK = r,
    WORLD_SIZE = N, one rendezvous on 127.0.0.1)."""
    import bench

    envs = bench.rank_envs(4, {"PATH": "/bin", "RANK": "9"}, 29999)
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert {e["WORLD_SIZE"] for e in envs} == {"4"} and {e["LOCAL_WORLD_SIZE"] for e in envs} == {"4"}
    assert {(e["MASTER_ADDR"], e["MASTER_PORT"]) for e in envs} == {("127.0.0.1", "29999")}
    assert all(e["PATH"] == "/bin" for e in envs)


def test_bench_gpus_without_devices_exits_nonzero():
    """--gpus 2 under RCCL with fewer visible GPUs than ranks (none here) exits non-zero before any rank starts."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "EVAM_BENCH_BACKEND")}
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2"], env=env, capture_output=True,
                       text=True, timeout=120)
    assert p.returncode == 2 and "visible GPU" in p.stderr and not p.stdout.strip()
