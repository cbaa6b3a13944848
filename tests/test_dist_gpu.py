"""Multi-rank rehearsal on one GPU: two worker processes share cuda:0 over
gloo, each pre-processes its ``s mod 2`` streams of a fixed 8-stream set, and every rank's tensors must
equal a single-process run of the same streams bit for bit; the post-run reduction totals must add up.
The workers are plain child processes (tools/dist_rehearsal.py), as torchrun would start them."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tools", "dist_rehearsal.py")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(world, config, tmp_path, streams=8):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        out = str(tmp_path / f"{config}_w{world}_r{r}.npz")
        procs.append((subprocess.Popen([sys.executable, WORKER, "--config", config, "--streams", str(streams),
                                        "--out", out], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                       text=True), out))
    res = []
    for p, out in procs:
        try:
            so, se = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q, _ in procs:
                q.kill()
            raise
        assert p.returncode == 0, se[-2000:]
        meta = json.loads(so.strip().splitlines()[-1])
        d = np.load(out)
        res.append((meta, d["streams"], d["out"]))
    return res


@pytest.mark.parametrize("config", ["c2", "c4", "c5"])
def test_two_ranks_match_single_process(gpu, tmp_path, config):
    """C2 / C4 frames and C5 clip rings (each stream's 16-slot ring lives on its owner rank)."""
    single = _run(1, config, tmp_path)
    (meta1, s1, out1), = single
    ring = meta1["ring"]
    steps = 3 if ring > 1 else 1
    assert list(s1) == list(range(8)) and meta1["frames"] == 8 * steps
    assert meta1["devices"] == 1
    by_stream = {int(s): out1[i * ring:(i + 1) * ring] for i, s in enumerate(s1)}
    two = _run(2, config, tmp_path)
    seen = []
    for meta, streams, out in two:
        assert meta["world"] == 2 and meta["devices"] == 1       # two ranks, one physical GPU
        assert meta["frames"] == 8 * steps and meta["per_rank_frames"] == [4 * steps, 4 * steps]
        assert meta["alg_bytes"] == meta1["alg_bytes"]           # summed over ranks == single process
        assert list(streams) == list(range(meta["rank"], 8, 2))  # s mod 2 ownership
        for i, s in enumerate(streams):
            a, b = out[i * ring:(i + 1) * ring], by_stream[int(s)]
            assert (a.view(np.uint32) == b.view(np.uint32)).all(), f"{config} stream {s} rank {meta['rank']}"
            seen.append(int(s))
    assert sorted(seen) == list(range(8))
    if ring > 1:  # slots no step wrote keep their initial value; slots 0 and 1 were written
        r = by_stream[0]
        assert (r[5] == 7.0).all() and not (r[0] == 7.0).all() and not (r[1] == 7.0).all()


def test_bench_rccl_reduction_path_one_rank(gpu, tmp_path):
    """bench.py's multi-GPU reduction on RCCL (backend "nccl": init_process_group with the device, barrier, all_reduce MAX
    of the elapsed time, all_gather of the per-rank totals on device tensors), run as one rank on this one-GPU box
    (EVAM_BENCH_PG=1): the path the driver's 2/4/8-GPU runs take, short of the inter-GPU transport."""
    port = _free_port()
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
               EVAM_BENCH_PG="1")
    env.pop("EVAM_BENCH_BACKEND", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "10", "--warmup", "3",
                        "--no-cpu-baseline", "--resident-steps", "0"], env=env, capture_output=True, text=True,
                       timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    d = json.loads(p.stdout.strip().splitlines()[-1])
    assert d["n_gpus"] == 1 and d["ranks"] == 1 and d["value"] > 0


def _bench_env(**kw):
    env = dict(os.environ, **kw)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "EVAM_BENCH_PG"):
        env.pop(k, None)
    return env


def test_bench_gpus2_launches_two_ranks(gpu):
    """`bench.py --gpus 2` with no launcher starts two ranks itself. On this one-GPU box the gloo
    rehearsal shares the device: rank 0's line reports both ranks and the frames of both."""
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "10", "--warmup", "3",
                        "--no-cpu-baseline", "--resident-steps", "0"], env=_bench_env(EVAM_BENCH_BACKEND="gloo"),
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.strip().splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]  # rank 0 prints the one line
    d = json.loads(lines[0])
    assert d["ranks"] == 2 and d["n_gpus"] == 1 and d["value"] > 0
    assert d["config"]["frames_per_gpu_per_step"] == 32


def test_bench_gpus2_rccl_refuses_one_gpu(gpu):
    """Under RCCL each rank needs its own GPU: --gpus 2 on a one-GPU box exits non-zero, never times one rank."""
    import torch

    if torch.cuda.device_count() >= 2:
        pytest.skip("more than one GPU visible")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "10", "--warmup", "3",
                        "--no-cpu-baseline"], env=_bench_env(), capture_output=True, text=True, timeout=120)
    assert p.returncode != 0
    assert "visible GPU" in p.stderr and not p.stdout.strip()
