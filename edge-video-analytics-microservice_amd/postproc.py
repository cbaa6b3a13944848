"""Post-processing after the pre-process path.

Detections are mapped back to frame coordinates through the per-item ``evam_transform``, which the HIP
path exports (§8 a11). Results are emitted in the two JSON shapes the reference publishes:

- ``gvametaconvert`` JSON. The reference sample output is at ``charts/README.md:117-119``:
  ``objects[].detection.bounding_box``, ``x, y, w, h``, ``roi_type``, ``resolution``, ``source``,
  ``timestamp``.
- The EVAM publisher metadata (``evas/publisher.py:183-230``): ``height``, ``width``, ``channels``,
  ``caps``, ``img_handle``, and ``gva_meta[]`` with ``x, y, height, width, object_id, tensor[]``.

Pixel rectangles follow DL Streamer's region-of-interest rule [3P]:
``x = floor(x_min * W + 0.5)`` and ``w = floor((x_max - x_min) * W + 0.5)``, on boxes clipped to
[0, 1]. All three sample rows of ``charts/README.md`` pin this rule
(``tests/test_pipeline_server.py::test_readme_metadata_rows``, fixture ``tests/golden/readme_metadata.jsonl``).
"""
from __future__ import annotations

import json
import math
from dataclasses import dataclass, field

import numpy as np


@dataclass
class Tensor:
    """One inference result attached to a region (DLS ``GVA::Tensor``)."""

    name: str
    confidence: float
    label_id: int
    label: str | None = None
    is_detection: bool = False
    model: str | None = None


@dataclass
class Region:
    """A region of interest in frame pixels, plus its normalized box (DLS ``RegionOfInterest``)."""

    x: int
    y: int
    w: int
    h: int
    bbox: tuple                      # (x_min, y_min, x_max, y_max), normalized to the frame
    label: str
    label_id: int
    confidence: float
    object_id: int = 0
    tensors: list = field(default_factory=list)


class FrameResult:
    """Inference results of one frame: regions, messages and frame-level tensors (e.g. action recognition).

    The three lists are created on first access: the pipeline layer makes one FrameResult per frame, and
    most frames of a detection stream never get a region (three eager lists per frame made the young-object
    collections of a 32-stream run measurably slower)."""

    __slots__ = ("width", "height", "timestamp", "source", "_regions", "_messages", "_tensors")

    def __init__(self, width: int, height: int, timestamp: int = 0, source: str | None = None,
                 regions: list | None = None, messages: list | None = None, tensors: list | None = None):
        self.width = width
        self.height = height
        self.timestamp = timestamp   # ns
        self.source = source
        self._regions = regions
        self._messages = messages
        self._tensors = tensors

    @property
    def regions(self) -> list:
        if self._regions is None:
            self._regions = []
        return self._regions

    @property
    def messages(self) -> list:
        if self._messages is None:
            self._messages = []
        return self._messages

    @property
    def tensors(self) -> list:
        if self._tensors is None:
            self._tensors = []
        return self._tensors

    def __repr__(self):
        return (f"FrameResult(width={self.width}, height={self.height}, timestamp={self.timestamp}, "
                f"source={self.source!r}, regions={self.regions!r}, messages={self.messages!r}, "
                f"tensors={self.tensors!r})")


def roi_rect(bbox, width: int, height: int):
    """Pixel rect (x, y, w, h) of a normalized box, clipped to [0, 1] first."""
    x0, y0, x1, y1 = (min(max(float(v), 0.0), 1.0) for v in bbox)
    return (int(math.floor(x0 * width + 0.5)), int(math.floor(y0 * height + 0.5)),
            int(math.floor((x1 - x0) * width + 0.5)), int(math.floor((y1 - y0) * height + 0.5)))


def is_identity(xf, frame_w: int, frame_h: int, tensor_w: int, tensor_h: int) -> bool:
    """True when the item was a plain full-frame resize, so tensor-normalized == frame-normalized."""
    return (xf is None or (xf.pad_x == 0 and xf.pad_y == 0 and xf.crop_x == 0 and xf.crop_y == 0
                           and xf.crop_w == frame_w and xf.crop_h == frame_h
                           and xf.resized_w == tensor_w and xf.resized_h == tensor_h))


def tensor_box_to_frame(box, xf, frame_w: int, frame_h: int, tensor_w: int, tensor_h: int):
    """Normalized tensor box -> normalized frame box through the item's transform.

    Inverse of the mapping in ``include/evam_pp.h`` (``evam_transform``). For a plain full-frame
    resize the box passes through unchanged, as in DLS, which only corrects aspect-ratio/crop items.
    """
    if is_identity(xf, frame_w, frame_h, tensor_w, tensor_h):
        return tuple(min(max(float(v), 0.0), 1.0) for v in box)
    x0, y0 = xf.tensor_to_source(float(box[0]) * tensor_w, float(box[1]) * tensor_h)
    x1, y1 = xf.tensor_to_source(float(box[2]) * tensor_w, float(box[3]) * tensor_h)
    return tuple(min(max(v, 0.0), 1.0) for v in (x0 / frame_w, y0 / frame_h, x1 / frame_w, y1 / frame_h))


def parse_ssd(raw, threshold: float):
    """Rows of an SSD ``DetectionOutput`` blob ``[..., 7]`` = (image_id, label, conf, x0, y0, x1, y1).

    Returns (image_id, label_id, confidence, box) with confidence >= threshold. Parsing stops at the
    first ``image_id < 0`` terminator, per the OpenVINO DetectionOutput convention.
    """
    a = np.asarray(raw, dtype=np.float32).reshape(-1, 7)
    out = []
    for row in a:
        if row[0] < 0:
            break
        if row[2] >= threshold:
            out.append((int(row[0]), int(row[1]), float(row[2]), tuple(float(v) for v in row[3:7])))
    return out


def parse_ssd_batch(raw, threshold: float):
    """``parse_ssd`` over a whole ``[N, K, 7]`` batch at once: per item, the rows before its first
    ``image_id < 0`` terminator with confidence >= threshold. Items without detections cost no Python
    loop (a batched detector's output is parsed in one vectorised pass)."""
    a = np.asarray(raw, dtype=np.float32)
    a = a.reshape(a.shape[0], -1, 7)
    live = np.cumsum(a[:, :, 0] < 0, axis=1) == 0          # rows before the terminator
    keep = live & (a[:, :, 2] >= threshold)
    out = [[] for _ in range(a.shape[0])]
    for i in np.flatnonzero(keep.any(axis=1)):
        for row in a[i][keep[i]]:
            out[i].append((int(row[0]), int(row[1]), float(row[2]), tuple(float(v) for v in row[3:7])))
    return out


def detections_to_regions(dets, xf, frame_w, frame_h, tensor_w, tensor_h, labels=None, model=None):
    """Parsed detections of one item -> frame ``Region``s."""
    regions = []
    for _, label_id, conf, box in dets:
        bb = tensor_box_to_frame(box, xf, frame_w, frame_h, tensor_w, tensor_h)
        x, y, w, h = roi_rect(bb, frame_w, frame_h)
        label = labels[label_id] if labels and 0 <= label_id < len(labels) else str(label_id)
        t = Tensor("detection", conf, label_id, label, is_detection=True, model=model)
        regions.append(Region(x, y, w, h, bb, label, label_id, conf, tensors=[t]))
    return regions


def classify(logits, labels=None, method: str = "max", name: str = "classification", model=None):
    """One ``tensor_to_label`` converter over a ``[N, C]`` output -> a ``Tensor`` per item."""
    a = np.asarray(logits, dtype=np.float64).reshape(len(logits), -1)
    if method == "softmax":
        e = np.exp(a - a.max(axis=1, keepdims=True))
        a = e / e.sum(axis=1, keepdims=True)
    ids = a.argmax(axis=1)
    return [Tensor(name, float(a[i, k]), int(k), labels[k] if labels and k < len(labels) else str(int(k)),
                   model=model) for i, k in enumerate(ids)]


def gvametaconvert(fr: FrameResult) -> dict:
    """The gvametaconvert JSON of one frame (``charts/README.md:117-119`` shape)."""
    objs = []
    for r in fr.regions:
        o = {"x": r.x, "y": r.y, "w": r.w, "h": r.h, "roi_type": r.label}
        for t in r.tensors:
            if t.is_detection:
                o["detection"] = {"bounding_box": {"x_min": r.bbox[0], "y_min": r.bbox[1],
                                                   "x_max": r.bbox[2], "y_max": r.bbox[3]},
                                  "confidence": t.confidence, "label": t.label, "label_id": t.label_id}
            else:
                o[t.name] = {"label": t.label, "label_id": t.label_id, "confidence": t.confidence}
        if r.object_id:
            o["id"] = r.object_id
        objs.append(o)
    d = {"resolution": {"height": fr.height, "width": fr.width}, "timestamp": fr.timestamp}
    if objs:
        d["objects"] = objs
    if fr.source is not None:
        d["source"] = fr.source
    for t in fr.tensors:
        d.setdefault("tensors", []).append({"name": t.name, "label": t.label, "label_id": t.label_id,
                                            "confidence": t.confidence})
    return d


def gvametaconvert_json(fr: FrameResult) -> str:
    return json.dumps(gvametaconvert(fr), sort_keys=True, separators=(",", ":"))


def publisher_meta(fr: FrameResult, caps: str = "", img_handle: str = "") -> dict:
    """The EVAM publisher's per-frame metadata dict (``evas/publisher.py:183-230``)."""
    meta = {"height": fr.height, "width": fr.width, "channels": 3, "caps": caps, "img_handle": img_handle}
    for m in fr.messages:
        meta.update(json.loads(m) if isinstance(m, str) else m)
    gva = []
    for r in fr.regions:
        tens = []
        for t in r.tensors:
            tm = {"name": t.name, "confidence": t.confidence, "label_id": t.label_id}
            if not t.is_detection:
                tm["label"] = t.label
            tens.append(tm)
        gva.append({"x": r.x, "y": r.y, "height": r.h, "width": r.w, "object_id": r.object_id, "tensor": tens})
    meta["gva_meta"] = gva
    return meta
