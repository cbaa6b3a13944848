"""Host-side mirror of DL Streamer's pre-processor interface, backed by the HIP kernels.

Reference interface (third party, DL Streamer 2022.1, selected by EVAM's pipeline templates
``pipelines/object_detection/vehicle/pipeline.json:5``,
``pipelines/object_classification/vehicle_attributes/pipeline.json:4-5``,
``pipelines/action_recognition/general/pipeline.json:3-4``):

* ``Image`` — DLS ``InferenceBackend::Image`` (format, width, height, planes, stride, rect);
* ``PreProcInfo`` — DLS ``InputImageLayerDesc`` built from a model-proc ``input_preproc`` entry
  (``models_list/vehicle-detection-0202.json:3`` = defaults, ``models_list/action-recognition-0001.json:3-13``
  = BGR + aspect-ratio + central crop);
* ``Transform`` — DLS ``ImageTransformationParams`` (scale / crop / padding for post-proc);
* ``HipPreProcessor.convert`` — DLS ``ImagePreprocessor::Convert`` batched over frames and ROIs.
  Failures raise :class:`PreProcError` (DLS throws ``std::runtime_error``).

There is no CPU fallback: if ``libevam_pp.so`` is missing the constructor raises.
"""
from __future__ import annotations

import ctypes
import weakref
from collections.abc import Sequence as _SequenceABC
from dataclasses import dataclass, field
from typing import Iterable, Sequence

from . import _native as N
from ._native import PreProcError  # noqa: F401  (re-export)

FOURCC_BY_NAME = {"NV12": N.FOURCC_NV12, "I420": N.FOURCC_I420, "BGRX": N.FOURCC_BGRX,
                  "BGRA": N.FOURCC_BGRA, "BGR": N.FOURCC_BGR}
NAME_BY_FOURCC = {v: k for k, v in FOURCC_BY_NAME.items()}


def plane_layout(fourcc: int, width: int, height: int, pitch_align: int = 64):
    """[(rows, pitch)] for each plane of a frame; pitches rounded up to ``pitch_align`` bytes."""
    al = lambda n: (n + pitch_align - 1) // pitch_align * pitch_align  # noqa: E731
    if fourcc == N.FOURCC_NV12:
        return [(height, al(width)), (height // 2, al(width))]
    if fourcc == N.FOURCC_I420:
        return [(height, al(width)), (height // 2, al(width // 2)), (height // 2, al(width // 2))]
    bpp = 3 if fourcc == N.FOURCC_BGR else 4
    return [(height, al(width * bpp))]


@dataclass
class Image:
    """A decoded frame resident in device memory (DLS ``Image``). ``planes`` are 2-D uint8 torch
    tensors of shape (rows, pitch); the tensors keep the memory alive."""

    fourcc: int
    width: int
    height: int
    planes: list = field(default_factory=list)
    _c: N.EvamImage | None = field(default=None, repr=False, compare=False)
    _cb: bytes | None = field(default=None, repr=False, compare=False)

    @property
    def pitches(self):
        return [int(p.stride(0)) for p in self.planes]

    def to_c(self) -> N.EvamImage:
        if self._c is None:
            c = N.EvamImage()
            c.fourcc, c.width, c.height = self.fourcc, self.width, self.height
            for i, p in enumerate(self.planes):
                c.pitch[i] = int(p.stride(0))
                c.planes[i] = int(p.data_ptr())
            self._c = c
        return self._c

    def c_bytes(self) -> bytes:
        """The packed ``evam_image`` (cached: an ImageBatch joins these instead of copying structs)."""
        if self._cb is None:
            self._cb = bytes(self.to_c())
        return self._cb

    @classmethod
    def alloc(cls, fourcc: int | str, width: int, height: int, device="cuda", pitch_align: int = 64):
        import torch

        fc = FOURCC_BY_NAME[fourcc] if isinstance(fourcc, str) else fourcc
        planes = [torch.empty((r, p), dtype=torch.uint8, device=device) for r, p in
                  plane_layout(fc, width, height, pitch_align)]
        return cls(fc, width, height, planes)

    @classmethod
    def from_host(cls, fourcc: int, width: int, height: int, host_planes: Sequence, device="cuda"):
        """Upload 2-D numpy planes (rows, pitch) to the device (the host->device feed)."""
        import torch

        planes = [torch.from_numpy(p).to(device) for p in host_planes]
        return cls(fourcc, width, height, planes)


class ImageBatch:
    """A list of Images marshalled once into the C array that evam_pp_run takes (keeps per-call
    host overhead flat for a fixed frame pool)."""

    def __init__(self, images: Sequence[Image]):
        self.images = list(images)
        # one join of cached packed structs: ~0.02 us per image instead of ~0.8 us for a ctypes
        # struct-by-struct array constructor (the pipeline hub marshals hundreds of frames per launch)
        self.c_array = (N.EvamImage * len(self.images)).from_buffer_copy(
            b"".join([im.c_bytes() for im in self.images]))

    def __len__(self):
        return len(self.images)


@dataclass(frozen=True)
class Roi:
    """A region of ``srcs[src_index]`` (DLS region of interest, gvaclassify)."""

    src_index: int
    x: int
    y: int
    w: int
    h: int


class RoiBatch:
    """ROIs marshalled once into the ``evam_roi`` array that evam_pp_run takes.

    Backed by a contiguous ``int32 [n, 5]`` numpy array (src_index, x, y, w, h), which has the layout
    of ``evam_roi[n]``: a detector's output converted with numpy is handed to the library without a
    per-ROI Python loop (a gvaclassify batch is ~50 ROIs per frame)."""

    def __init__(self, rois):
        import numpy as np

        if isinstance(rois, np.ndarray):
            a = rois
        else:
            a = np.array([(r.src_index, r.x, r.y, r.w, r.h) if isinstance(r, Roi) else tuple(r) for r in rois])
            if a.size == 0:
                a = np.zeros((0, 5), np.int32)
        # evam_roi is int32: refuse silent truncation (floats) and wrap-around (out-of-range int64)
        if a.dtype != np.int32:
            if a.size and not np.issubdtype(a.dtype, np.integer):
                raise PreProcError(N.ERR_INVALID_ARG, f"ROI array must hold integers, got dtype {a.dtype}")
            if a.size and (a.min() < -2**31 or a.max() > 2**31 - 1):
                raise PreProcError(N.ERR_INVALID_ARG, "ROI values outside the int32 range")
        self.array = np.ascontiguousarray(a, dtype=np.int32)
        if self.array.ndim == 1 and self.array.size == 0:
            self.array = self.array.reshape(0, 5)
        if self.array.ndim != 2 or self.array.shape[1] != 5:
            raise PreProcError(N.ERR_INVALID_ARG, f"ROI array must be [n, 5] int32, got {self.array.shape}")
        self.c_ptr = self.array.ctypes.data_as(ctypes.POINTER(N.EvamRoi))

    def __len__(self):
        return int(self.array.shape[0])


@dataclass
class PreProcInfo:
    """Model input pre-processing description (DLS ``InputImageLayerDesc`` from a model-proc)."""

    resize: str = "no-aspect-ratio"     # "no" | "no-aspect-ratio" | "aspect-ratio"
    crop: str | None = None             # None | "central"
    color_space: str = "BGR"            # "BGR" | "RGB"
    range: tuple | None = None          # (min, max)
    mean: tuple | None = None           # per output channel
    std: tuple | None = None            # per output channel
    placement: str = "top_left"         # letterbox placement: "top_left" | "center"
    fill: tuple = (0, 0, 0)             # u8 pad value per output channel

    @classmethod
    def from_model_proc(cls, entry: dict | None) -> "PreProcInfo":
        """From one ``input_preproc`` entry of a DLS model-proc json (``{"format": "image", "params": {...}}``)."""
        if not entry:
            return cls()
        params = entry.get("params", entry)
        info = cls()
        if "resize" in params:
            info.resize = params["resize"]
        if "crop" in params:
            info.crop = params["crop"]
        if "color_space" in params:
            info.color_space = params["color_space"]
        if "range" in params:
            info.range = tuple(float(v) for v in params["range"])
        if "mean" in params:
            info.mean = tuple(float(v) for v in params["mean"])
        if "std" in params:
            info.std = tuple(float(v) for v in params["std"])
        if "padding" in params:
            pad = params["padding"]
            if "fill_value" in pad:
                fv = pad["fill_value"]
                info.fill = tuple(int(v) for v in (fv if isinstance(fv, (list, tuple)) else [fv] * 3))
        return info

    def cache_key(self, out_dtype: int):
        """Hashable value of every field that reaches the C struct (lists are normalised to tuples)."""
        t = lambda v: tuple(v) if isinstance(v, list) else v  # noqa: E731
        return (self.resize, self.crop, self.color_space, t(self.range), t(self.mean), t(self.std),
                self.placement, t(self.fill), out_dtype)

    def resize_mode(self) -> int:
        if self.resize in ("no", "no-aspect-ratio", None):
            if self.crop not in (None, "", "none"):
                raise PreProcError(N.ERR_UNSUPPORTED, f"crop={self.crop!r} requires resize=aspect-ratio")
            return N.RESIZE_NO_ASPECT
        if self.resize == "aspect-ratio":
            if self.crop in (None, "", "none"):
                return N.RESIZE_ASPECT
            if self.crop == "central":
                return N.RESIZE_ASPECT_CROP
            raise PreProcError(N.ERR_UNSUPPORTED, f"crop={self.crop!r} is not supported (central only)")
        raise PreProcError(N.ERR_UNSUPPORTED, f"resize={self.resize!r} is not supported")

    def to_c(self, out_dtype: int) -> N.EvamPreproc:
        c = N.EvamPreproc()
        c.resize_mode = self.resize_mode()
        c.placement = N.PLACE_CENTER if self.placement == "center" else N.PLACE_TOP_LEFT
        if self.color_space not in ("BGR", "RGB"):
            raise PreProcError(N.ERR_UNSUPPORTED, f"color_space={self.color_space!r} is not supported")
        c.color_order = N.COLOR_RGB if self.color_space == "RGB" else N.COLOR_BGR
        c.out_dtype = out_dtype
        flags = 0
        c.range[0], c.range[1] = (0.0, 255.0)
        if self.range is not None:
            flags |= N.NORM_RANGE
            c.range[0], c.range[1] = self.range
        mean = self.mean or (0.0, 0.0, 0.0)
        std = self.std or (1.0, 1.0, 1.0)
        if self.mean is not None or self.std is not None:
            flags |= N.NORM_MEAN_STD
        for i in range(3):
            c.mean[i] = mean[i]
            c.std[i] = std[i]
            c.fill[i] = int(self.fill[i])
        c.norm_flags = flags
        return c


@dataclass
class Transform:
    """DLS ``ImageTransformationParams`` for one item: maps source pixels to tensor pixels."""

    scale_x: float
    scale_y: float
    crop_x: int
    crop_y: int
    crop_w: int
    crop_h: int
    pad_x: int
    pad_y: int
    resized_w: int
    resized_h: int

    def tensor_to_source(self, u: float, v: float):
        """Inverse mapping of a tensor coordinate back to source-frame coordinates (for boxes)."""
        return ((u - self.pad_x) / self.scale_x + self.crop_x, (v - self.pad_y) / self.scale_y + self.crop_y)


class Transforms(_SequenceABC):
    """The per-item transforms of one call, built on access (a detection batch needs the transform only
    of the frames that produced detections)."""

    __slots__ = ("_xf",)

    def __init__(self, xf):
        self._xf = xf

    def __len__(self):
        return len(self._xf)

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[k] for k in range(*i.indices(len(self)))]
        x = self._xf[i]
        return Transform(x.scale_x, x.scale_y, x.crop_x, x.crop_y, x.crop_w, x.crop_h, x.pad_x, x.pad_y,
                         x.resized_w, x.resized_h)


class HipPreProcessor:
    """The ``pre-process-backend=hip`` implementation: one handle per (device, stream-thread)."""

    backend_name = "hip"

    def __init__(self, device: int = 0, stream=None):
        import torch

        self._lib = N.load_library()
        self.device = int(device)
        self._torch = torch
        self._follow_torch_stream = stream is None
        if not torch.cuda.is_available():
            raise PreProcError(N.ERR_NO_DEVICE, "no HIP device visible (the HIP backend has no CPU fallback)")
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        self._stream_ptr = int(getattr(s, "cuda_stream", s) or 0)
        h = ctypes.c_void_p()
        N.check(self._lib, self._lib.evam_pp_create(self.device, ctypes.c_void_p(self._stream_ptr),
                                                     ctypes.byref(h)))
        self._h = h
        self._cfg_cache: dict = {}
        self._last_cfg = None  # (info, dtype code, its fields, byref of the C struct) of the last call
        self._tdesc: dict = {}  # id(output tensor) -> (weakref, version, data_ptr, evam_tensor, dtype code, byref)
        self._default_info = PreProcInfo()
        self._run = self._lib.evam_pp_run
        raw = getattr(torch._C, "_cuda_getCurrentRawStream", None)
        self._raw_stream = raw if raw is not None else (
            lambda d: torch.cuda.current_stream(d).cuda_stream)

    # -- lifecycle ------------------------------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            self._lib.evam_pp_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # -- options ---------------------------------------------------------------------------------
    def set_option(self, option: int, value: int):
        N.check(self._lib, self._lib.evam_pp_set_option(self._h, option, int(value)))

    def stats(self) -> N.EvamStats:
        st = N.EvamStats()
        N.check(self._lib, self._lib.evam_pp_get_stats(self._h, ctypes.byref(st)))
        return st

    def sync(self):
        N.check(self._lib, self._lib.evam_pp_sync(self._h))

    def _bind_stream(self):
        if self._follow_torch_stream:
            s = int(self._raw_stream(self.device) or 0)
            if s != self._stream_ptr:
                N.check(self._lib, self._lib.evam_pp_set_stream(self._h, ctypes.c_void_p(s)))
                self._stream_ptr = s

    def _tensor_desc(self, out, slot_offset: int, slot_stride: int):
        """``byref`` of the validated evam_tensor for ``out``, and its dtype code. Cached per output tensor (a stage
        packs into the same inference blob every call; a runner or a bench cycles through a few): the same tensor
        object at the same version (``resize_`` / ``set_`` / ``as_strided_`` bump it) and storage has the shape,
        dtype, device and layout it was checked with, so they are not read again (~1 us per call)."""
        e = self._tdesc.get(id(out))
        if e is None or e[0]() is not out or e[1] != out._version or e[2] != out.data_ptr():
            e = self._tensor_entry(out)
        t = e[3]
        if t.slot_offset != slot_offset or t.slot_stride != slot_stride:
            t.slot_offset, t.slot_stride = int(slot_offset), int(slot_stride)
        return e[5], e[4]

    def _tensor_entry(self, out):
        torch = self._torch
        if out.dim() != 4 or out.shape[1] != 3 or not out.is_contiguous():
            raise PreProcError(N.ERR_INVALID_ARG, f"out must be a contiguous [N,3,H,W] tensor, got {tuple(out.shape)}")
        if out.dtype == torch.uint8:
            dt = N.DTYPE_U8
        elif out.dtype == torch.float32:
            dt = N.DTYPE_F32
        else:
            raise PreProcError(N.ERR_UNSUPPORTED, f"out dtype {out.dtype} is not supported (uint8, float32)")
        if out.device.type != "cuda" or (out.device.index or 0) != self.device:
            raise PreProcError(N.ERR_INVALID_ARG, f"out must live on cuda:{self.device}, got {out.device}")
        t = N.EvamTensor()
        t.data = out.data_ptr()
        t.n, t.c, t.h, t.w = (int(v) for v in out.shape)
        e = (weakref.ref(out), out._version, t.data, t, dt, ctypes.byref(t))
        if len(self._tdesc) >= 16:
            self._tdesc.clear()
        self._tdesc[id(out)] = e
        return e

    # -- the hot path ------------------------------------------------------------------------------
    def convert(self, srcs, out, info: PreProcInfo | None = None, rois: Iterable | None = None,
                slot_offset: int = 0, slot_stride: int = 1, want_transform: bool = False, slots=None):
        """Pre-process ``srcs`` (or ``rois`` of them) into ``out`` ([N,3,H,W] uint8/float32, device).

        ``srcs``: an :class:`ImageBatch` (marshalled once) or a sequence of :class:`Image`.
        ``rois``: a :class:`RoiBatch`, an ``int32 [n, 5]`` array or a sequence of :class:`Roi`.
        Item i goes to slot ``slot_offset + i * slot_stride`` of ``out``, or to ``slots[i]`` when ``slots`` (one
        distinct slot per item, ``evam_pp_run_slots``) is given.
        Returns a list of :class:`Transform` when ``want_transform`` (``"lazy"``: a :class:`Transforms`
        sequence that builds each on access). Asynchronous on the current
        torch stream of ``self.device`` (or the stream given at construction).
        """
        info = info or self._default_info
        batch = srcs if isinstance(srcs, ImageBatch) else ImageBatch(srcs)
        tref, dt = self._tensor_desc(out, slot_offset, slot_stride)
        lc = self._last_cfg
        if lc is not None and lc[0] is info and lc[1] == dt and lc[2] == info.__dict__:
            cached = lc[3]  # the last call's info object, every field as it was (~1.3 us of key building saved)
        else:
            # keyed on the field values (PreProcInfo is mutable; a field changed after a call must not reuse
            # a stale struct), bounded so callers building a new info per call cannot grow it without limit
            key = info.cache_key(dt)
            cached = self._cfg_cache.get(key)
            if cached is None:
                if len(self._cfg_cache) >= 64:
                    self._cfg_cache.clear()
                cached = ctypes.byref(info.to_c(dt))
                self._cfg_cache[key] = cached
            # snapshot of the fields for the identity check above; a list field can change in place, so an info
            # holding one takes the keyed path every call
            d = info.__dict__
            self._last_cfg = None if any(v.__class__ is list for v in d.values()) else (info, dt, dict(d), cached)
        if rois is not None:
            rb = rois if isinstance(rois, RoiBatch) else RoiBatch(rois)
            n_items = len(rb)
            if n_items == 0:
                raise PreProcError(N.ERR_INVALID_ARG, "rois is empty")
            items_p = rb.c_ptr
        else:
            n_items = len(batch)
            items_p = None
        xf = (N.EvamTransform * n_items)() if want_transform else None
        self._bind_stream()
        if slots is not None:
            import numpy as np

            sl = np.ascontiguousarray(slots, dtype=np.int32)
            if sl.shape != (n_items,):
                raise PreProcError(N.ERR_INVALID_ARG, f"slots must hold one slot per item ({n_items}), got {sl.shape}")
            rc = self._lib.evam_pp_run_slots(self._h, batch.c_array, len(batch), items_p, n_items, cached,
                                             tref, sl.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), xf)
        else:
            rc = self._run(self._h, batch.c_array, len(batch), items_p, n_items, cached, tref, xf)
        if rc:
            N.check(self._lib, rc)
        if not want_transform:
            return None
        return Transforms(xf) if want_transform == "lazy" else list(Transforms(xf))


# Backend registry keyed by the DL Streamer element property value `pre-process-backend`.
_BACKENDS = {"hip": HipPreProcessor}
REFERENCE_ONLY_BACKENDS = ("opencv", "ie", "vaapi", "vaapi-surface-sharing")


def create_preprocessor(backend: str = "hip", **kw):
    """Instantiate the pre-processor selected by a ``pre-process-backend`` property value."""
    if backend in _BACKENDS:
        return _BACKENDS[backend](**kw)
    if backend in REFERENCE_ONLY_BACKENDS:
        raise PreProcError(N.ERR_UNSUPPORTED,
                           f"pre-process-backend={backend!r} is the reference DL Streamer CPU/VA path; "
                           "this build provides 'hip'")
    raise PreProcError(N.ERR_INVALID_ARG, f"unknown pre-process-backend {backend!r}")
