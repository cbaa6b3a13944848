"""Host->device frame feed.

Decode stays upstream on the reference path (``decodebin``, ``pipelines/*/pipeline.json:3``). A
CPU decoder hands over frames in host memory, so they must cross PCIe before the kernel can read
them. ``HostFeed`` is a ring of ``depth`` batch slots. Each slot has:
- a pinned host buffer that the decoder writes into (``host_planes``, or ``fill`` to copy in);
- a device buffer of the same layout, laid out as ``batch`` frames back to back, each frame's
  planes at ``plane_layout`` pitches.

One slot moves as ONE ``hipMemcpyAsync`` on a dedicated copy stream. That copy overlaps the
pre-process kernel of the previous slot on the compute stream, with events in both directions:
- ``copied[k]``: the compute stream waits on it before the kernel reads slot k;
- ``consumed[k]``: the copy stream waits on it before it overwrites the device side of slot k.

The host blocks only when it reuses a pinned slot whose copy has not finished yet.

Per step::

    k = feed.acquire()                 # waits until slot k's pinned buffer is free
    feed.fill(k, frames)               # or decode straight into feed.host_planes(k)
    feed.submit(k)                     # H2D on the copy stream
    pp.convert(feed.batch(k), out, info)   # batch() makes the compute stream wait for the copy
    feed.release(k)                    # the kernel that read slot k is enqueued
"""
from __future__ import annotations

import numpy as np

from .preproc import FOURCC_BY_NAME, Image, ImageBatch, plane_layout


class HostFeed:
    def __init__(self, fourcc, width: int, height: int, batch: int, depth: int = 3, device: int = 0,
                 pitch_align: int = 64):
        import torch

        if depth < 2:
            raise ValueError("depth must be >= 2 to overlap copies with kernels")
        self.torch = torch
        self.fourcc = FOURCC_BY_NAME[fourcc] if isinstance(fourcc, str) else int(fourcc)
        self.width, self.height, self.n, self.depth = width, height, batch, depth
        self.device = torch.device(f"cuda:{device}")
        self.layout = plane_layout(self.fourcc, width, height, pitch_align)
        self.frame_bytes = sum(r * p for r, p in self.layout)
        nbytes = batch * self.frame_bytes
        self.host = [torch.empty(nbytes, dtype=torch.uint8, pin_memory=True) for _ in range(depth)]
        self.dev = [torch.empty(nbytes, dtype=torch.uint8, device=self.device) for _ in range(depth)]
        self.copy_stream = torch.cuda.Stream(self.device)
        self.copied = [torch.cuda.Event() for _ in range(depth)]
        self.consumed = [torch.cuda.Event() for _ in range(depth)]
        self._submitted = [False] * depth
        self._used = [False] * depth
        self._next = 0
        self._batches = [ImageBatch([self._image(self.dev[k], i) for i in range(batch)]) for k in range(depth)]
        self._host_views = [[self._planes(self.host[k].numpy(), i) for i in range(batch)] for k in range(depth)]

    @property
    def bytes_per_batch(self) -> int:
        return self.n * self.frame_bytes

    def _planes(self, buf, i):
        out, off = [], i * self.frame_bytes
        for r, p in self.layout:
            out.append(buf[off:off + r * p].reshape(r, p))
            off += r * p
        return out

    def _image(self, dev, i):
        return Image(self.fourcc, self.width, self.height, self._planes(dev, i))

    def host_planes(self, k: int):
        """Writable pinned numpy views ``[frame][plane] -> (rows, pitch)`` of slot ``k``."""
        return self._host_views[k]

    def acquire(self) -> int:
        """Next slot. Blocks until the previous H2D copy out of its pinned buffer has finished."""
        k = self._next
        self._next = (k + 1) % self.depth
        if self._submitted[k]:
            self.copied[k].synchronize()
            self._submitted[k] = False
        return k

    def fill(self, k: int, frames):
        """Copy host frames (objects with ``.planes`` or dicts with ``"planes"``) into slot ``k``."""
        if len(frames) > self.n:
            raise ValueError(f"{len(frames)} frames > batch {self.n}")
        for i, f in enumerate(frames):
            planes = f["planes"] if isinstance(f, dict) else f.planes
            for dst, src in zip(self._host_views[k][i], planes):
                src = np.asarray(src)
                rows, w = min(dst.shape[0], src.shape[0]), min(dst.shape[1], src.shape[1])
                dst[:rows, :w] = src[:rows, :w]

    def submit(self, k: int):
        """Enqueue slot ``k``'s H2D copy on the copy stream, after the last kernel that read it."""
        torch = self.torch
        with torch.cuda.stream(self.copy_stream):
            if self._used[k]:
                self.copy_stream.wait_event(self.consumed[k])
            self.dev[k].copy_(self.host[k], non_blocking=True)
            self.copied[k].record(self.copy_stream)
        self._submitted[k] = True

    def batch(self, k: int, stream=None) -> ImageBatch:
        """Slot ``k``'s device frames. The compute stream (default: current) waits for the copy."""
        s = stream or self.torch.cuda.current_stream(self.device)
        s.wait_event(self.copied[k])
        return self._batches[k]

    def release(self, k: int, stream=None):
        """Mark slot ``k`` consumed once the work enqueued so far on the compute stream completes."""
        s = stream or self.torch.cuda.current_stream(self.device)
        self.consumed[k].record(s)
        self._used[k] = True

    def synchronize(self):
        self.copy_stream.synchronize()
