"""Multi-GPU layout of the pre-process path: camera streams partitioned across GPUs.

The reference runs one GStreamer pipeline per stream (`evas/manager.py:127-141` starts one pipeline
per configured source), and pre-processing has no data dependency between streams. Scaling
out is therefore a partition, not a collective:
- stream ``s`` is owned by rank ``s mod G``, with one process per GPU (``torchrun``);
- each rank batches the frames of the streams it owns into one ``evam_pp_run`` launch.

Nothing crosses ranks on the data path. The only exchange is one ``all_reduce(MAX)`` of elapsed
time and one ``all_gather`` of per-rank counters after a timed region (``reduce_run``). It works
on any ``torch.distributed`` backend: RCCL on the GPU box, ``gloo`` in the CPU tests.
"""
from __future__ import annotations

from dataclasses import dataclass


def owner(stream: int, world: int) -> int:
    """Rank that pre-processes ``stream`` (``s mod G``)."""
    if world <= 0 or stream < 0:
        raise ValueError("stream must be >= 0 and world >= 1")
    return stream % world


def streams_for_rank(n_streams: int, world: int, rank: int) -> list[int]:
    """Streams owned by ``rank`` of ``world``: ``rank, rank+G, rank+2G, ...``."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    return list(range(rank, n_streams, world))


def local_batch(frames_by_stream, world: int, rank: int) -> list:
    """This rank's frames, in stream order, from a list indexed by stream id."""
    return [frames_by_stream[s] for s in streams_for_rank(len(frames_by_stream), world, rank)]


def device_key(local_device: int) -> int:
    """Identity of a physical device across ranks (ranks that share a GPU in a rehearsal share a key): the
    machine (``/etc/machine-id``, else the hostname — containers may share one) and the device's PCI location
    (bus / device / domain from the HIP properties when a GPU is visible, else the local index)."""
    import socket
    import zlib

    host = socket.gethostname()
    try:
        with open("/etc/machine-id") as f:
            host = f.read().strip() + "/" + host
    except OSError:
        pass
    loc = f"idx{int(local_device)}"
    try:
        import torch

        if torch.cuda.is_available() and int(local_device) < torch.cuda.device_count():
            pr = torch.cuda.get_device_properties(int(local_device))
            loc = "pci{}:{}:{}".format(*(getattr(pr, k, -1) for k in ("pci_domain_id", "pci_bus_id", "pci_device_id")))
    except Exception:  # noqa: BLE001 — identity only; the index is the fallback
        pass
    return zlib.crc32(f"{host}|{loc}".encode()) & 0x7FFFFFFFFFFF


@dataclass
class RunTotals:
    world: int
    elapsed_max_s: float      # slowest rank's elapsed time
    frames: int               # frames processed by all ranks
    alg_bytes: int            # algorithmic bytes moved by all ranks
    per_rank_frames: list
    devices: int = 1          # distinct physical devices over the ranks (device_key), not the rank count

    @property
    def frames_per_s(self) -> float:
        return self.frames / self.elapsed_max_s if self.elapsed_max_s > 0 else 0.0


def reduce_run(elapsed_s: float, frames: int, alg_bytes: int, device=None, device_key: int = 0) -> RunTotals:
    """Combine one timed region across ranks: max elapsed, summed counters, distinct devices.

    Call it on every rank after the timed region. It is never used inside the hot loop. With
    ``torch.distributed`` uninitialised (a single process), it returns this process's numbers.
    ``device`` is where the small exchange tensors live: a CUDA device for RCCL, CPU for gloo.
    ``device_key``: this rank's physical device (``device_key()``); ranks sharing a GPU count once.
    """
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return RunTotals(1, float(elapsed_s), int(frames), int(alg_bytes), [int(frames)], 1)
    world = dist.get_world_size()
    el = torch.tensor([float(elapsed_s)], dtype=torch.float64, device=device)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    mine = torch.tensor([int(frames), int(alg_bytes), int(device_key)], dtype=torch.int64, device=device)
    allst = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allst, mine)
    per = [int(t[0].item()) for t in allst]
    devs = len({int(t[2].item()) for t in allst})
    return RunTotals(world, float(el.item()), sum(per), sum(int(t[1].item()) for t in allst), per, devs)
