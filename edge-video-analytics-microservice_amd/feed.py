"""Host->device frame feed.

Decode stays upstream on the reference path (``decodebin``, ``pipelines/*/pipeline.json:3``). A
CPU decoder hands over frames in host memory, so they must cross PCIe before the kernel can read
them. ``HostFeed`` is a ring of ``depth`` batch slots. Each slot has:
- a pinned host buffer that the decoder writes into (``host_planes``, or ``fill`` to copy in);
- a device buffer of the same layout, laid out as ``batch`` frames back to back, each frame's
  planes at ``plane_layout`` pitches.

One slot moves on a dedicated copy stream: by default as ONE ``hipMemcpyAsync`` of the whole batch; after
``set_geometry`` (the pre-processing the batch will get) only the source rows the resize reads cross PCIe —
the row table's touched luma rows and their chroma rows, as strided ``hipMemcpy2DAsync`` runs per frame and
plane (C4: 720 of 2,160 luma rows, a third of every frame), unless they cover >= 85% of the frame (C2), where
the one contiguous copy is faster. The kernels read exactly those rows, so the
rows left stale on the device are never used. The copies overlap the pre-process kernel of the previous
slot on the compute stream, with events in both directions:
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

import ctypes

from . import _native as N
from .preproc import FOURCC_BY_NAME, Image, ImageBatch, plane_layout

_HIP = None


def _hip():
    """The HIP runtime the process already loaded (torch's, which libevam_pp.so is bound to: ``_native``), for
    hipMemcpy2DAsync. Opened by its mapped path with RTLD_NOLOAD, so a name lookup can never load a second HIP
    runtime (``/opt/rocm``'s) whose streams and pointers would not be torch's; more than one mapped runtime, or
    none, raises."""
    global _HIP
    if _HIP is None:
        import os

        import torch  # noqa: F401 — loads the HIP runtime torch was built against

        N.load_library()
        with open("/proc/self/maps") as f:
            paths = {ln.split(None, 5)[5].strip() for ln in f
                     if len(ln.split(None, 5)) == 6 and os.path.basename(ln.split(None, 5)[5].strip())
                     .startswith("libamdhip64.so")}
        if len(paths) != 1:
            raise RuntimeError(f"expected exactly one loaded HIP runtime (libamdhip64.so), found {sorted(paths)}")
        lib = ctypes.CDLL(paths.pop(), mode=os.RTLD_NOLOAD | os.RTLD_LOCAL)
        lib.hipMemcpy2DAsync.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                                         ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
        lib.hipMemcpy2DAsync.restype = ctypes.c_int
        _HIP = lib
    return _HIP


def resized_height(W: int, H: int, DW: int, DH: int, mode: int) -> tuple[int, int]:
    """(resized height, first visible resized row) of a full frame (roi_geometry in csrc/evam_geom.h; SURVEY.md
    §8 a6): mode 0 no-aspect, 1 aspect-ratio letterbox, 2 aspect-ratio + central crop."""
    if mode == 0:
        return DH, 0
    sx, sy = DW / W, DH / H
    x_dom = (sx <= sy) if mode == 1 else (sx >= sy)
    rh = int(H * sx) if x_dom else DH
    rh = max(rh, 1)
    if mode == 1:
        return min(rh, DH), 0
    rh = max(rh, DH)
    return rh, (rh - DH) // 2


def touched_rows(fourcc: int, W: int, H: int, DW: int, DH: int, mode: int) -> list[list[int]]:
    """Source rows per plane that pre-processing a full W x H frame to DW x DH reads: the OpenCV row table's two
    taps of every visible output row (the library's own evam_pp_linear_table), and for 4:2:0 the chroma rows
    r >> 1 of those. Packed formats: one plane."""
    rh, top = resized_height(W, H, DW, DH, mode)
    lib = N.load_library()
    ofs = (ctypes.c_int32 * rh)()
    c0 = (ctypes.c_int16 * rh)()
    c1 = (ctypes.c_int16 * rh)()
    N.check(lib, lib.evam_pp_linear_table(H, rh, 0, ofs, c0, c1))
    rows = set()
    for dy in range(top, min(rh, top + DH)):
        s = ofs[dy]
        rows.add(min(max(s, 0), H - 1))
        rows.add(min(max(s + 1, 0), H - 1))
    luma = sorted(rows)
    if fourcc in (FOURCC_BY_NAME["NV12"], FOURCC_BY_NAME["I420"]):
        chroma = sorted({r >> 1 for r in luma})
        return [luma, chroma] + ([chroma] if fourcc == FOURCC_BY_NAME["I420"] else [])
    return [luma]


def copy_runs(rows: list[int], max_cmds: int = 8) -> list[tuple[int, int, int, int]]:
    """Strided copy commands (first row, rows per run, row stride between runs, runs) covering `rows`:
    consecutive rows form runs, runs of equal length at a constant stride merge into one strided command.
    More than `max_cmds` commands: one command over the whole span instead (e.g. 1080 -> 512 reads 1,024 of
    1,080 rows in irregular runs)."""
    if not rows:
        return []
    runs, a = [], rows[0]
    for p, q in zip(rows, rows[1:] + [None]):
        if q != p + 1:
            runs.append((a, p - a + 1))
            a = q
    cmds = []
    for start, length in runs:
        if cmds:
            s0, l0, st, k = cmds[-1]
            stride = start - (s0 + (k - 1) * st) if k > 1 else start - s0
            if length == l0 and (k == 1 or stride == st):
                cmds[-1] = (s0, l0, stride, k + 1)
                continue
        cmds.append((start, length, length, 1))
    if len(cmds) > max_cmds:
        return [(rows[0], rows[-1] - rows[0] + 1, rows[-1] - rows[0] + 1, 1)]
    return cmds


class HostFeed:
    whole_copy_fraction = 0.85  # touched bytes / frame bytes at or above which one contiguous copy is used

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
        self._plan = None  # per plane: (plane byte offset in a frame, pitch, copy commands); None: whole batch

    def set_geometry(self, out_w: int, out_h: int, info=None):
        """Copy only the source rows that pre-processing every frame to out_w x out_h with `info`
        (PreProcInfo; default no-aspect-ratio) reads. Full-frame items only (ROI batches read rows this plan
        does not know)."""
        mode = info.resize_mode() if info is not None else 0
        rows = touched_rows(self.fourcc, self.width, self.height, out_w, out_h, mode)
        plan, off = [], 0
        for (r, p), pr in zip(self.layout, rows):
            plan.append((off, p, copy_runs(pr)))
            off += r * p
        self.rows_per_plane = [len(r) for r in rows]
        planned = sum(p * l * k for _, p, cmds in plan for _, l, _, k in cmds)
        # Strided copies pay per command: when they would move most of the frame anyway (C2: 1080 -> 512 reads
        # 1,024 of 1,080 rows, one span per plane), one contiguous copy of the batch is faster (55 vs 42 GB/s,
        # profiles/r04k_ab_lines.txt)
        self._plan = None if planned >= self.whole_copy_fraction * self.frame_bytes else plan

    @property
    def strided(self) -> bool:
        """True when submit() copies only the planned rows (strided 2-D copies), False for one contiguous copy."""
        return self._plan is not None

    @property
    def bytes_per_batch(self) -> int:
        """Bytes one submit() moves over PCIe."""
        if self._plan is None:
            return self.n * self.frame_bytes
        return self.n * sum(p * l * k for _, p, cmds in self._plan for _, l, _, k in cmds)

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
            if self._plan is None:
                self.dev[k].copy_(self.host[k], non_blocking=True)
            else:
                hip, st = _hip(), ctypes.c_void_p(self.copy_stream.cuda_stream)
                hb, db = self.host[k].data_ptr(), self.dev[k].data_ptr()
                for i in range(self.n):
                    fo = i * self.frame_bytes
                    for off, pitch, cmds in self._plan:
                        for r0, length, stride, runs in cmds:
                            o = fo + off + r0 * pitch
                            # runs of `length` rows, `stride` rows apart: one 2-D copy (width = the run's bytes)
                            rc = hip.hipMemcpy2DAsync(db + o, stride * pitch, hb + o, stride * pitch, length * pitch,
                                                      runs, 1, st)  # 1: hipMemcpyHostToDevice
                            if rc != 0:
                                raise RuntimeError(f"hipMemcpy2DAsync failed ({rc})")
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
