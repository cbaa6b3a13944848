"""Pipeline-server counterpart: the direct caller of the pre-process path.

EVAM drives pipelines through the DL Streamer Pipeline Server API (``evas/manager.py:100-155``):

    PipelineServer.start({'log_level': ..., 'ignore_init_errors': True})
    pipeline = PipelineServer.pipeline(name, version)
    pipeline.start(source=src, destination=dest, parameters=model_params)
    PipelineServer.wait();  PipelineServer.stop()

This module exposes the same API over the reference's own ``pipelines/<name>/<version>/pipeline.json``
templates. Loading a template covers:
- ``{models[alias][version][network|proc]}`` and ``{env[VAR]}`` are resolved;
- the launch string is parsed into elements;
- the request's ``parameters`` are validated against the template schema and mapped onto element
  properties. All schema forms of SURVEY.md §8b are handled:
  - ``"element": "<name>"``;
  - ``{"name", "property"}``;
  - a list of those (fan-out);
  - ``{"name", "format": "element-properties"}`` (dict passthrough);
  - ``"format": "json"``;
  - defaults, including ``{env[VAR]}``.

The inference elements are ``gvadetect``, ``gvaclassify`` and ``gvaactionrecognitionbin``; each one
with ``pre-process-backend=hip`` runs on the HIP path (``hip`` is also the default when the property is
absent). Each element:
1. gates and selects its stream's work on the pipeline's thread (``inference-interval``, ``object-class``,
   ``reclassify-interval``);
2. hands it to the device's :class:`BatchHub`, which coalesces the requests of every pipeline with an
   interchangeable element into ONE batched pre-processing launch and one model call per tick (bounded
   by a unit count and a latency budget) — the reference runs one pipeline per stream and never batches
   across them (``evas/manager.py:127-141``);
3. runs the registered model (a torch callable: OpenVINO is not part of this stack);
4. post-processes (``postproc.py``: transform-mapped boxes, ``tensor_to_label``, gvametaconvert JSON).

Decode stays upstream. An ``application`` source delivers decoded frames:
device ``Image``s, or host planes uploaded on arrival.
"""
from __future__ import annotations

import collections
import contextlib
import gc
import itertools
import json
import operator
import os
import queue
import re
import shlex
import threading
import time
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field

from . import _native as N
from . import postproc as P
from ._native import PreProcError
from .preproc import Image

_WIDTH, _HEIGHT = operator.attrgetter("width"), operator.attrgetter("height")
INFERENCE_ELEMENTS = ("gvadetect", "gvaclassify", "gvaactionrecognitionbin", "gvainference")
HIP_BACKENDS = ("hip",)
# backends DL Streamer 2022.1 accepts that only the reference implements
REFERENCE_ONLY_BACKENDS = ("ie", "opencv", "vaapi", "vaapi-surface-sharing")


# ------------------------------------------------------------------------------------------------
# Template handling
# ------------------------------------------------------------------------------------------------
@dataclass
class Element:
    """One element of a GStreamer launch string: ``factory prop=value ...`` or a caps filter."""

    factory: str
    properties: dict = field(default_factory=dict)
    caps: str | None = None

    @property
    def name(self) -> str | None:
        return self.properties.get("name")


class _Fmt(dict):
    """str.format mapping that leaves unknown top-level fields (e.g. {auto_source}) in place."""

    def __missing__(self, key):
        return "{" + key + "}"


class _EnvLookup:
    def __getitem__(self, key):
        return os.environ.get(key, "")


def resolve_template(template, models: dict, extra: dict | None = None) -> str:
    """Join a template (str or list of str) and substitute ``{models[..]..}``, ``{env[..]}`` and extras."""
    text = "".join(template) if isinstance(template, (list, tuple)) else str(template)

    def sub(m):
        expr = m.group(1)
        root = expr.split("[", 1)[0]
        if root == "models":
            keys = re.findall(r"\[([^\]]+)\]", expr)
            node = models
            for k in keys:
                if not isinstance(node, dict) or k not in node:
                    raise KeyError(f"model reference {{{expr}}} not found")
                node = node[k]
            return str(node)
        if root == "env":
            return os.environ.get(re.findall(r"\[([^\]]+)\]", expr)[0], "")
        if extra is not None and expr in extra:
            return str(extra[expr])
        return m.group(0)

    return re.sub(r"\{([A-Za-z_][^{}]*)\}", sub, text)


def parse_launch(text: str) -> list[Element]:
    """Split a gst-launch string on ``!`` into elements; ``key=value`` tokens become properties."""
    elems = []
    for part in text.split("!"):
        part = part.strip()
        if not part:
            continue
        toks = shlex.split(part)
        head = toks[0]
        if "/" in head and "=" not in head.split(",", 1)[0]:     # caps filter, e.g. video/x-raw,format=BGRx
            elems.append(Element("capsfilter", {}, caps=part))
            continue
        props = {}
        for t in toks[1:]:
            if "=" in t:
                k, v = t.split("=", 1)
                props[k] = v
        elems.append(Element(head, props))
    return elems


def _type_ok(value, typ) -> bool:
    if typ is None:
        return True
    if isinstance(typ, list):
        return any(_type_ok(value, t) for t in typ)
    return {"string": lambda v: isinstance(v, str),
            "integer": lambda v: isinstance(v, int) and not isinstance(v, bool),
            "number": lambda v: isinstance(v, (int, float)) and not isinstance(v, bool),
            "boolean": lambda v: isinstance(v, bool),
            "object": lambda v: isinstance(v, dict),
            "array": lambda v: isinstance(v, list)}.get(typ, lambda v: True)(value)


def _expand_default(value):
    """``{env[VAR]}`` defaults: the variable's value, or None (property left unset) if it is empty."""
    if isinstance(value, str):
        m = re.fullmatch(r"\{env\[([^\]]+)\]\}", value)
        if m:
            return os.environ.get(m.group(1)) or None
    return value


def apply_parameters(elements: list[Element], schema: dict | None, parameters: dict | None) -> dict:
    """Validate ``parameters`` against the template schema and set element properties.

    Returns the effective parameter dict (request values plus defaults). Raises ValueError for an
    unknown parameter or a type mismatch, as the reference's schema validation does.
    """
    props = (schema or {}).get("properties", {})
    parameters = dict(parameters or {})
    unknown = sorted(set(parameters) - set(props))
    if unknown:
        raise ValueError(f"unknown pipeline parameter(s): {unknown}")
    by_name = {e.name: e for e in elements if e.name}
    effective = {}
    for key, spec in props.items():
        if key in parameters:
            value = parameters[key]
            if not _type_ok(value, spec.get("type")):
                raise ValueError(f"parameter {key!r}: expected {spec.get('type')}, got {type(value).__name__}")
            if "enum" in spec and value not in spec["enum"]:
                raise ValueError(f"parameter {key!r}: {value!r} not in {spec['enum']}")
        elif "default" in spec:
            value = _expand_default(spec["default"])
            if value is None:
                continue
        else:
            continue
        effective[key] = value
        targets = spec.get("element")
        if targets is None:
            continue
        for tgt in targets if isinstance(targets, list) else [targets]:
            if isinstance(tgt, str):
                tgt = {"name": tgt}
            el = by_name.get(tgt["name"])
            if el is None:
                raise ValueError(f"parameter {key!r} targets unknown element {tgt['name']!r}")
            fmt = tgt.get("format")
            if fmt == "element-properties":
                if not isinstance(value, dict):
                    raise ValueError(f"parameter {key!r}: element-properties needs an object")
                for k, v in value.items():
                    el.properties[k] = v
            elif fmt == "json":
                el.properties[tgt.get("property", key)] = json.dumps(value)
            else:
                el.properties[tgt.get("property", key)] = value
    return effective


# ------------------------------------------------------------------------------------------------
# Models
# ------------------------------------------------------------------------------------------------
@dataclass
class InferenceModel:
    """A model bound to a network path: a torch callable over the pre-processed NCHW batch.

    ``fn(tensor) -> output``: for detection, an SSD ``DetectionOutput`` blob ``[N, K, 7]`` (boxes
    normalized to the input tensor). For classification, a dict ``{layer_name: [N, C]}`` or one
    ``[N, C]`` tensor. ``input_size`` is ``(W, H)``. Labels and pre-processing come from the
    model-proc (``models_list/*.json``).
    """

    fn: object
    input_size: tuple
    model_proc: dict | None = None
    out_dtype: str = "f32"
    name: str | None = None

    def preproc_info(self, overrides: dict | None = None):
        from .preproc import PreProcInfo

        entry = None
        if self.model_proc:
            for e in self.model_proc.get("input_preproc", []):
                if e.get("format", "image") == "image":
                    entry = e
                    break
        info = PreProcInfo.from_model_proc(entry)
        for k, v in (overrides or {}).items():
            setattr(info, k, v)
        return info

    def postprocs(self):
        return list((self.model_proc or {}).get("output_postproc", []))


def ir_input_size(xml_path: str):
    """(W, H) of an OpenVINO IR's first image input (``<layer type="Parameter">`` NCHW shape)."""
    root = ET.parse(xml_path).getroot()
    for layer in root.iter("layer"):
        if layer.get("type") == "Parameter":
            data = layer.find("data")
            shape = data.get("shape") if data is not None else None
            if shape:
                dims = [int(d) for d in shape.split(",")]
            else:
                dims = [int(d.text) for d in layer.find("output").find("port").findall("dim")]
            if len(dims) == 4:
                return dims[3], dims[2]
    raise ValueError(f"{xml_path}: no 4-D input layer")


def scan_models(model_dir: str, precisions=("FP32", "FP16", "INT8")) -> dict:
    """``{alias: {version: {"network": xml, "proc": json, "<precision>": xml}}}`` from a model tree.

    Layout as the reference's model downloader writes it (``tools/model_downloader``):
    ``<model_dir>/<alias>/<version>/<precision>/<model>.xml`` plus an optional ``<model>.json`` proc.
    """
    models: dict = {}
    if not model_dir or not os.path.isdir(model_dir):
        return models
    for alias in sorted(os.listdir(model_dir)):
        adir = os.path.join(model_dir, alias)
        if not os.path.isdir(adir):
            continue
        for version in sorted(os.listdir(adir)):
            vdir = os.path.join(adir, version)
            if not os.path.isdir(vdir):
                continue
            entry = {}
            for f in sorted(os.listdir(vdir)):
                p = os.path.join(vdir, f)
                if f.endswith(".json"):
                    entry["proc"] = p
                elif os.path.isdir(p):
                    xml = [x for x in sorted(os.listdir(p)) if x.endswith(".xml")]
                    if xml:
                        entry[f] = os.path.join(p, xml[0])
            for prec in precisions:
                if prec in entry:
                    entry["network"] = entry[prec]
                    break
            if entry:
                models.setdefault(alias, {})[version] = entry
    return models


# ------------------------------------------------------------------------------------------------
# Stages
# ------------------------------------------------------------------------------------------------
def _backend_of(el: Element) -> str:
    b = str(el.properties.get("pre-process-backend", "hip"))
    if b in HIP_BACKENDS:
        return b
    if b in REFERENCE_ONLY_BACKENDS:
        raise PreProcError(N.ERR_UNSUPPORTED, f"{el.name or el.factory}: pre-process-backend={b!r} is the "
                                              "reference's CPU/VA path; this build provides 'hip'")
    raise PreProcError(N.ERR_UNSUPPORTED, f"{el.name or el.factory}: unknown pre-process-backend {b!r}")


def roi_inside(x: int, y: int, w: int, h: int, W: int, H: int) -> bool:
    """True when a detected box has a non-empty intersection with its W x H frame.

    Boxes that fail are skipped by gvaclassify stages: for ``evam_roi`` a rect with ``w <= 0`` or
    ``h <= 0`` means "the whole frame", and a rect that clips to nothing is an error for the whole call.
    """
    if w <= 0 or h <= 0:
        return False
    return min(x + w, W) - max(x, 0) > 0 and min(y + h, H) - max(y, 0) > 0


class _Request:
    """One pipeline's share of a hub batch: its items, and an event the pipeline thread waits on."""

    __slots__ = ("stage", "items", "units", "t0", "done", "error")

    def __init__(self, stage, items, units, event=True):
        self.stage = stage
        self.items = items
        self.units = units
        self.t0 = time.perf_counter()
        self.done = threading.Event() if event else None
        self.error = None



def _bind_thread_device(device: int) -> None:
    """Make ``device`` the calling thread's current HIP device, so a model call on a runner / hub thread
    allocates and launches on the GPU whose pipelines it serves (``devices`` option), not on GPU 0."""
    import torch

    if torch.cuda.is_available() and int(device) < torch.cuda.device_count():
        torch.cuda.set_device(int(device))

class BatchHub:
    """Per-device batching hub: one ``evam_pp_run`` (and one model call) per stage key per tick, over the
    frames / ROIs of every pipeline the device owns.

    The reference runs one GStreamer pipeline per camera stream (``evas/manager.py:127-141``) and each
    inference element batches only its own stream's frames (``batch-size``). On a GPU that leaves the
    launch nearly empty: one 1080p frame is ~1 us of HBM work against a ~5 us launch floor. The hub
    coalesces the requests of all pipelines whose inference elements are interchangeable (same model,
    same pre-processing, same element properties: ``stage.hub_key()``) into one batch, bounded by
    ``max_batch`` units (frames, or ROIs for gvaclassify) and a latency budget ``max_wait_s`` after the
    oldest pending request; ``target`` flushes as soon as that many units are pending. Every pipeline
    thread blocks only on its own request, so a slow stream never holds up a tick beyond the budget.
    """

    def __init__(self, device: int, max_batch: int = 64, max_wait_s: float = 0.002, target: int | None = None,
                 drain_timeout_s: float = 2.0, inflight: int = 1):
        self.device = int(device)
        # ticks the device runner keeps in flight: tick t runs on handle / stream t mod inflight, so the next ticks'
        # launch ramps overlap tick t's tail (server default 3: C2 through the runner 865 k -> 920 k f/s against 2,
        # 4 slower, C1 / C4 / C5 equal within noise; profiles/r06f_pipeline_inflight.txt)
        self.inflight = max(1, int(inflight))
        self.drain_timeout_s = float(drain_timeout_s)  # runner shutdown: how long held-back results may wait
        self.max_batch = max(1, int(max_batch))
        self.max_wait_s = float(max_wait_s)
        self.target = int(target) if target else None
        self._pending: dict = {}
        self._units: dict = {}          # pending units per key
        self._cv = threading.Condition()
        self._stop = False
        self._pps: dict = {}            # slot -> pre-processing handle (bound to the slot's stream)
        self._rings: dict = {}          # action stage hub key -> ClipRing shared by the device's action streams
        self._streams: list | None = None
        self.batches: list = []        # (key, units, requests) per executed batch (inspection / tests)
        self._thread = threading.Thread(target=self._loop, name=f"evam-hub-{device}", daemon=True)
        self._thread.start()

    def stream(self, slot: int = 0):
        """Slot's torch stream (None: one tick at a time, or no GPU: the thread's current stream)."""
        if self.inflight == 1:
            return None
        if self._streams is None:
            import torch

            self._streams = ([torch.cuda.Stream(self.device) for _ in range(self.inflight)]
                             if torch.cuda.is_available() else [None] * self.inflight)
        return self._streams[slot % self.inflight]

    def stream_ctx(self, slot: int = 0):
        s = self.stream(slot)
        if s is None:
            return contextlib.nullcontext()
        import torch

        return torch.cuda.stream(s)

    def pp(self, slot: int = 0):
        """Slot's pre-processing handle. With several ticks in flight each slot owns a handle bound to its own
        stream: a handle that followed the current stream would order every stream switch behind the previous
        stream's work (evam_pp_set_stream), and the ticks could not overlap."""
        h = self._pps.get(slot)
        if h is None:
            from .preproc import HipPreProcessor

            s = self.stream(slot)
            h = self._pps[slot] = HipPreProcessor(device=self.device) if s is None else \
                HipPreProcessor(device=self.device, stream=s)
        return h

    def clip_ring(self, key, size, device: int):
        """The ClipRing of action streams whose stages share ``key`` (one model and pre-processing) on this device."""
        r = self._rings.get(key)
        if r is None:
            r = self._rings[key] = ClipRing(device, size)
        return r

    def submit(self, stage, items, units: int):
        """Queue ``items`` of ``stage`` and block until the batch holding them ran (re-raises its error)."""
        if units <= 0:
            return
        req = _Request(stage, items, units)
        key = stage.hub_key()
        with self._cv:
            if self._stop:
                raise RuntimeError("batch hub is closed")
            q = self._pending.setdefault(key, [])
            q.append(req)
            n = self._units.get(key, 0) + units
            self._units[key] = n
            # wake the hub only when it has something new to decide: a first request (its deadline
            # starts) or a full batch; other submits would wake it just to go back to sleep
            if len(q) == 1 or n >= (self.target or self.max_batch):
                self._cv.notify()
        req.done.wait()
        if req.error is not None:
            raise req.error

    def _ready(self, now):
        """(key, requests) to run now, or (None, wait seconds)."""
        wait = None
        for key, reqs in self._pending.items():
            units = self._units[key]
            if units >= (self.target or self.max_batch) or now - reqs[0].t0 >= self.max_wait_s:
                take, n = [], 0
                while reqs and (not take or n + reqs[0].units <= self.max_batch):
                    n += reqs[0].units
                    take.append(reqs.pop(0))
                self._units[key] = units - n
                if not reqs:
                    del self._pending[key]
                    del self._units[key]
                return key, take
            left = self.max_wait_s - (now - reqs[0].t0)
            wait = left if wait is None else min(wait, left)
        return None, wait

    def _loop(self):
        _bind_thread_device(self.device)
        while True:
            with self._cv:
                while True:
                    if self._stop and not self._pending:
                        return
                    key, take = self._ready(time.perf_counter())
                    if key is not None:
                        break
                    self._cv.wait(timeout=take)
            try:
                # slot 0's handle launches on slot 0's stream: the model call must run on the same stream
                with self.stream_ctx(0):
                    s = self.stream(0)
                    if s is not None:
                        import torch

                        s.wait_stream(torch.cuda.default_stream(self.device))  # the application's frames
                    take[0].stage.run_batch(take, self.pp())
                self.batches.append((key, sum(r.units for r in take), len(take)))
                if len(self.batches) > 4096:
                    del self.batches[:2048]
            except BaseException as e:  # noqa: BLE001 — delivered to every waiting pipeline
                for r in take:
                    r.error = e
            for r in take:
                r.done.set()

    def close(self):
        with self._cv:
            self._stop = True
            self._cv.notify_all()
        self._thread.join(10)
        for h in self._pps.values():
            h.close()
        self._pps = {}
        self._rings = {}


class DeviceRunner:
    """Per-device pipeline runner (the default; server option ``runner``: ``"device"`` | ``"threads"``).

    One thread services every pipeline the device owns, the way one GStreamer main loop serves many
    pipelines in native code: it drains each application source in bulk, and once the ready frames of
    all pipelines reach the hub's ``target`` (or the oldest has waited ``max_wait_s``) it runs one tick —
    stage by stage, ONE ``evam_pp_run`` and one model call per interchangeable stage over every pipeline's
    frames (chunks of at most ``max_batch`` units), then each pipeline's per-stream bookkeeping and its
    destination. With one Python thread per stream instead (``"threads"``: 32 pipeline threads handing
    requests to the :class:`BatchHub` thread) the GIL hand-offs and per-frame queue calls bounded the
    pipeline layer at ~28 % of the kernel rate (``profiles/r02r_bench_via_pipeline*.json``).
    """

    def __init__(self, hub: "BatchHub"):
        self.hub = hub
        self._pipes: list = []
        self._draining: list = []  # ended pipelines whose destination still holds back results (queue full)
        self._ticks = 0            # ticks run; tick t uses the hub's slot t mod hub.inflight
        self._pending = collections.deque()  # ticks launched, not completed (at most hub.inflight - 1, oldest first)
        self._cv = threading.Condition()
        self._stop = False
        self._thread = threading.Thread(target=self._guarded_loop, name=f"evam-runner-{hub.device}", daemon=True)
        self._thread.start()

    def add(self, pipe):
        with self._cv:
            if self._stop:
                raise RuntimeError("device runner is closed")
            self._pipes.append(pipe)
            self._cv.notify()

    def close(self):
        with self._cv:
            self._stop = True
            self._cv.notify_all()
        self._thread.join(10)

    def _guarded_loop(self):
        """The runner thread. Whatever escapes the loop (a bug, not a stream's error: those fail only their
        own pipeline) fails every pipeline the runner still holds, so no ``wait()`` blocks on a dead thread."""
        try:
            _bind_thread_device(self.hub.device)
            self._loop()
        except BaseException as e:  # noqa: BLE001
            with self._cv:
                pipes, self._pipes = list(self._pipes), []
                draining, self._draining = list(self._draining), []
                self._stop = True
            for p in pipes + draining:
                ended = p in draining  # already ended (COMPLETED / ABORTED), only handing over held-back results
                if not ended:
                    try:
                        p._fail(e)
                    except Exception:  # noqa: BLE001 — the destination's own error; the pipeline ends either way
                        pass
                if p._out_backlog:
                    # no thread is left to hand the held-back results over: report them, never block wait(). The
                    # end-of-stream marker queued behind them is offered once more, so a consumer reading until None
                    # still ends when its queue has room; a pipeline that had ended keeps its state.
                    n = sum(1 for x in p._out_backlog if x is not None)
                    p._out_backlog.clear()
                    dst = p.destination.get("metadata", p.destination)
                    out = dst.get("output")
                    try:
                        if out is not None and hasattr(out, "put_nowait"):
                            out.put_nowait(None)
                    except Exception:  # noqa: BLE001 — a full queue: the marker cannot be delivered either
                        pass
                    p.error = f"{p.error or type(e).__name__ + ': ' + str(e)}; {n} result(s) undelivered"
                    if not ended:
                        p.state = p.ERROR
                p._done.set()

    def _drain(self):
        """Hand held-back results to destinations that have room again. A pipeline whose last result (the
        end-of-stream marker included) went out is complete: only then does its ``wait()`` return."""
        keep = []
        for p in self._draining:
            try:
                if not p._flush_out():
                    keep.append(p)
                    continue
            except Exception as e:  # noqa: BLE001 — the destination itself failed: nothing left to deliver to
                p.error, p.state = f"{type(e).__name__}: {e}", p.ERROR
                p._out_backlog.clear()
            p._done.set()
        self._draining = keep

    def _drain_at_shutdown(self, timeout_s: float):
        """Keep flushing held-back results for up to ``timeout_s``; a pipeline whose destination still cannot
        take them ends in ERROR with the number of undelivered results (never a silent drop)."""
        deadline = time.perf_counter() + timeout_s
        while self._draining and time.perf_counter() < deadline:
            self._drain()
            if self._draining:
                time.sleep(0.001)
        for p in self._draining:
            n = len(p._out_backlog)
            p.error = f"destination full at shutdown: {n} result(s) undelivered after {timeout_s:g} s"
            p.state = p.ERROR
            p._out_backlog.clear()
            p._done.set()
        self._draining = []

    def _finish(self, p, e=None):
        """End pipeline ``p`` (``e``: its error), isolated from the other pipelines of the device."""
        try:
            if e is not None:
                p._fail(e)
            else:
                p._end()
        except Exception as e2:  # noqa: BLE001 — a destination that raised on end of stream
            p.error, p.state = f"{type(e2).__name__}: {e2}", p.ERROR
            p._done.set()
        if p._out_backlog:
            self._draining.append(p)

    def _loop(self):
        hub = self.hub
        idle = 0.0005
        while True:
            with self._cv:
                while not self._pipes and not self._draining and not self._stop:
                    self._cv.wait()
                stopping = self._stop and not self._pipes
                pipes = list(self._pipes)
            if stopping:
                self._complete_pending()
                self._drain_at_shutdown(self.hub.drain_timeout_s)
                return
            if self._draining:
                self._drain()
            ready, oldest, total, done = [], None, 0, []
            for p in pipes:
                if p._out_backlog:
                    try:
                        p._flush_out()
                    except Exception as e:  # noqa: BLE001
                        self._finish(p, e)
                        done.append(p)
                        continue
                    if len(p._out_backlog) >= p._out_limit and not p._stop.is_set():
                        # backpressure: a destination that does not keep up stops its own stream (no ingest,
                        # no tick), like a blocking push in a native pipeline; the other streams go on
                        continue
                try:
                    p._ingest()
                except Exception as e:  # noqa: BLE001 — reported through status(), as the reference does
                    self._finish(p, e)
                    done.append(p)
                    continue
                n = len(p._pend) - p._head
                if p._stop.is_set() or (p._eos and not n):
                    # its results still in flight (the pending tick) go out before its end of stream
                    self._complete_pending()
                    self._finish(p)
                    done.append(p)
                elif n >= p._batch or p._eos:
                    ready.append(p)
                    total += n
                    oldest = p._pend_t0 if oldest is None else min(oldest, p._pend_t0)
            if done:
                with self._cv:
                    self._pipes = [p for p in self._pipes if p not in done]
            if not ready:
                self._complete_pending()
                time.sleep(idle)
                continue
            if total < (hub.target or 1) and time.perf_counter() - oldest < hub.max_wait_s:
                self._complete_pending()
                time.sleep(idle)
                continue
            # about max_batch frames per tick, in whole batch-size multiples per pipeline
            share = max(1, hub.max_batch // len(ready))
            work = []
            for p in ready:
                n = len(p._pend) - p._head
                k = max(p._batch, share // p._batch * p._batch)
                k = min(k, n) if p._eos else min(k, n // p._batch * p._batch)
                work.append((p, p._pend[p._head:p._head + k]))
                p._head += k  # a read index, not del [:k]: a stream's backlog is taken in O(k) per tick
                if p._head >= 4096 and 2 * p._head >= len(p._pend):
                    del p._pend[:p._head]
                    p._head = 0
                p._pend_t0 = time.perf_counter()
            self._tick(work)

    def _tick(self, work):
        """Run the stage chains of `work` [(pipeline, frames)] stage by stage, batched across pipelines, on the
        hub's next slot (handle and stream). With ``hub.inflight`` > 1 a batch whose stage ends every chain in it
        and can launch without completing (``launch_batch``: detection, action recognition) is only enqueued here;
        its completion, the pipelines' bookkeeping and the tick's results wait until ``hub.inflight`` - 1 later ticks
        have been launched, so the next ticks' kernels overlap this one's tail. Ticks complete in launch order, so
        every stream's results keep their order."""
        hub = self.hub
        slot = self._ticks % hub.inflight
        self._ticks += 1
        failed = set()
        deferred = []  # (completion, chunk)
        errors = []    # (pipeline, error) of this tick: reported after the previous tick's results went out

        def fail(p, e):
            failed.add(p)
            errors.append((p, e))

        with hub.stream_ctx(slot):
            s = hub.stream(slot)
            if s is not None:
                import torch

                # the application's frames were written on its own (default) stream
                s.wait_stream(torch.cuda.default_stream(hub.device))
            depth = max(len(p.stages) for p, _ in work)
            for k in range(depth):
                groups: dict = {}
                for p, items in work:
                    if p in failed or k >= len(p.stages) or not items:
                        continue
                    st = p.stages[k]
                    try:
                        if not st.batchable:
                            st.process(items)
                            continue
                        w, units = st.prepare(items)
                    except Exception as e:  # noqa: BLE001
                        fail(p, e)
                        continue
                    if units > 0:
                        groups.setdefault(st.hub_key(), []).append((p, _Request(st, w, units, event=False)))
                for key, reqs in groups.items():
                    i = 0
                    while i < len(reqs):  # chunks of at most max_batch units (at least one request)
                        j, n = i, 0
                        while j < len(reqs) and (j == i or n + reqs[j][1].units <= hub.max_batch):
                            n += reqs[j][1].units
                            j += 1
                        chunk = reqs[i:j]
                        i = j
                        stage = chunk[0][1].stage
                        defer = (hub.inflight > 1 and hasattr(stage, "launch_batch")
                                 and all(k == len(p.stages) - 1 for p, _ in chunk))
                        try:
                            if defer:
                                deferred.append((stage.launch_batch([r for _, r in chunk], hub.pp(slot)), chunk))
                            else:
                                stage.run_batch([r for _, r in chunk], hub.pp(slot))
                            hub.batches.append((key, n, len(chunk)))
                            if len(hub.batches) > 4096:
                                del hub.batches[:2048]
                        except Exception as e:  # noqa: BLE001 — delivered to every pipeline of the batch
                            for p, _ in chunk:
                                fail(p, e)
                            continue
                        if not defer:
                            self._finish_batch(chunk, failed, fail)
        tick = (slot, deferred, work, failed)
        if errors or not deferred:
            # a stream's earlier results (the pending ticks) precede its error and this tick's results
            self._complete_pending()
        for p, e in errors:
            self._finish(p, e)
        if errors:
            # out of the runner now, not when this tick completes: a deferred tick may stay pending, and the
            # loop must not ingest or schedule a stream whose end-of-stream marker is already out
            self._drop({p for p, _ in errors})
        if deferred:
            # up to hub.inflight ticks launched: complete the oldest beyond inflight - 1 pending (in launch order), so
            # the next tick's launch goes out while the others still run
            self._pending.append(tick)
            while len(self._pending) > max(1, hub.inflight - 1):
                self._complete(self._pending.popleft())
        else:
            self._complete(tick)

    def _finish_batch(self, chunk, failed, fail=None):
        for p, r in chunk:
            if p not in failed:
                try:
                    r.stage.finish(r.items)
                except Exception as e:  # noqa: BLE001 — this stream's bookkeeping only
                    if fail is not None:
                        fail(p, e)
                    else:
                        self._finish(p, e)
                        failed.add(p)

    def _complete(self, tick):
        """Complete a tick: its deferred batches (model output to the host, per-stream bookkeeping), then every
        stream's results of the tick to its destination."""
        slot, deferred, work, failed = tick
        if deferred:
            with self.hub.stream_ctx(slot):
                for done, chunk in deferred:
                    try:
                        done()
                    except Exception as e:  # noqa: BLE001 — delivered to every pipeline of the batch
                        for p, _ in chunk:
                            self._finish(p, e)
                            failed.add(p)
                        continue
                    self._finish_batch(chunk, failed)
        for p, items in work:
            if p not in failed:
                try:
                    p._emit_all(items)
                except Exception as e:  # noqa: BLE001 — this stream's destination only
                    self._finish(p, e)
                    failed.add(p)
        if failed:
            self._drop(failed)

    def _drop(self, pipes):
        with self._cv:
            self._pipes = [p for p in self._pipes if p not in pipes]

    def _complete_pending(self):
        while self._pending:
            self._complete(self._pending.popleft())


class _InferenceStage:
    """Common part of gvadetect / gvaclassify: interval gating, model lookup, HIP pre-processing.

    ``process(items)`` runs on the pipeline's own thread: it gates and selects the work of this stream,
    then hands it to the server's per-device :class:`BatchHub`, which executes ``run_batch`` for the
    requests of all pipelines sharing ``hub_key()``.
    """

    def __init__(self, el: Element, server, device: int, slot: int = 0):
        self.el = el
        self.backend = _backend_of(el)
        self.device = device
        self.slot = slot  # the pipeline's logical device: its BatchHub / DeviceRunner
        self.server = server
        net = el.properties.get("model") or el.properties.get("enc-model")
        self.model = server.model_for(net, device)
        if self.model is None:
            raise RuntimeError(f"{el.name or el.factory}: no model registered for {net!r} "
                               "(PipelineServer.register_model)")
        mp = el.properties.get("model-proc")
        if mp and self.model.model_proc is None and os.path.exists(mp):
            self.model.model_proc = json.load(open(mp))
        self.interval = int(el.properties.get("inference-interval", 1))
        self.threshold = float(el.properties.get("threshold", 0.5))
        self.batch_size = int(el.properties.get("batch-size", 1))
        self._pp = None
        self.info = self.model.preproc_info()

    def out_dtype(self) -> int:
        return N.DTYPE_F32 if self.model.out_dtype == "f32" else N.DTYPE_U8

    # A stage's work for one stream: prepare (gating / selection, on the caller's thread) -> run_batch over the
    # requests of every interchangeable stage (one launch) -> finish (per-stream bookkeeping).
    batchable = True

    def prepare(self, items):
        raise NotImplementedError

    def finish(self, work):
        pass

    def process(self, items):
        """Thread runner: gate, hand the work to the device's BatchHub (blocks until its batch ran), finish."""
        work, units = self.prepare(items)
        self.server.hub(self.slot).submit(self, work, units)
        self.finish(work)

    def hub_key(self):
        """Stages with equal keys are interchangeable: their requests run as one batch (computed once: the
        element's model, pre-processing and properties are fixed for the pipeline's life)."""
        k = self.__dict__.get("_hub_key")
        if k is None:
            k = self._hub_key = self._make_hub_key()
        return k

    def _make_hub_key(self):
        return (self.el.factory, id(self.model), self.info.cache_key(self.out_dtype()), self.threshold)

    def pp(self):
        if self._pp is None:
            from .preproc import HipPreProcessor

            self._pp = HipPreProcessor(device=self.device)
        return self._pp

    def close(self):
        if self._pp is not None:
            self._pp.close()
            self._pp = None

    def _tensor(self, n):
        import torch

        W, H = self.model.input_size
        dt = torch.float32 if self.model.out_dtype == "f32" else torch.uint8
        return torch.empty((n, 3, H, W), dtype=dt, device=f"cuda:{self.device}")


class DetectStage(_InferenceStage):
    def prepare(self, items):
        """items: list of (frame_index, Image, FrameResult) -> (the frames to infer, units)."""
        run = [it for it in items if it[0] % self.interval == 0] if self.interval > 1 else items
        return run, len(run)

    def launch_batch(self, reqs, pp):
        """Enqueue one launch over the frames of every request and the model call on it; returns the completion
        (the model output's copy to the host, the detections attached to the frames). The device runner calls it
        after the next tick's launch when it keeps several ticks in flight."""
        run = [it for r in reqs for it in r.items]
        out = self._tensor(len(run))
        xfs = pp.convert([img for _, img, _ in run], out, self.info, want_transform="lazy")
        raw = self.model.fn(out)

        def complete():
            r = raw.detach().float().cpu().numpy() if hasattr(raw, "detach") else raw
            W, H = self.model.input_size
            labels = None
            for pp_ in self.model.postprocs():
                labels = pp_.get("labels", labels)
            for k, dets in enumerate(P.parse_ssd_batch(r, self.threshold)):
                if dets:
                    _, img, fr = run[k]
                    fr.regions.extend(P.detections_to_regions(dets, xfs[k], img.width, img.height, W, H, labels,
                                                              model=self.model.name))
        complete.out = out  # the tensor the kernel writes stays alive until its batch completes
        return complete

    def run_batch(self, reqs, pp):
        """One launch over the frames of every request, completed before returning."""
        self.launch_batch(reqs, pp)()


class ClassifyStage(_InferenceStage):
    """gvaclassify: the regions of each frame whose label matches ``object-class``, batched across pipelines.

    ``reclassify-interval`` (``pipelines/object_classification/vehicle_attributes/pipeline.json:68-71``):
    as in DL Streamer, it applies to tracked objects (regions with a non-zero ``object_id``, from gvatrack):
    such an object is classified again only every N-th frame of its stream, and in between its last
    results are attached again. Untracked regions (object_id 0) are classified on every gated frame.
    """

    def __init__(self, el, server, device, slot=0):
        super().__init__(el, server, device, slot)
        oc = el.properties.get("object-class")
        self.object_class = set(str(oc).split(",")) if oc else None
        self.reclassify = max(1, int(el.properties.get("reclassify-interval", 1)))
        self._cache: dict = {}   # object_id -> (frame index classified at, tensors)
        self._deferred: list = []  # (region, region of an earlier frame of this call it takes results from)

    def _make_hub_key(self):
        oc = tuple(sorted(self.object_class)) if self.object_class else None
        return super()._make_hub_key() + (oc,)

    def prepare(self, items):
        work = []          # (frame_index, Image, [regions to classify])
        sched = {}         # object_id -> (frame index, region) classified by this call
        self._deferred = []
        for fi, img, fr in items:
            if fi % self.interval:
                continue
            todo = []
            for r in fr.regions:
                if self.object_class is not None and r.label not in self.object_class:
                    continue
                if not roi_inside(r.x, r.y, r.w, r.h, img.width, img.height):
                    continue  # degenerate box: the C ABI would read w/h <= 0 as "full frame"
                if r.object_id and self.reclassify > 1:
                    hit = self._cache.get(r.object_id)
                    if hit is not None and fi - hit[0] < self.reclassify:
                        r.tensors.extend(hit[1])
                        continue
                    # an earlier frame of this same call classifies the object: its results, once run
                    s = sched.get(r.object_id)
                    if s is not None and fi - s[0] < self.reclassify:
                        self._deferred.append((r, s[1]))
                        continue
                    sched[r.object_id] = (fi, r)
                todo.append(r)
            if todo:
                work.append((fi, img, todo))
        return work, sum(len(t) for _, _, t in work)

    def finish(self, work):
        if self.reclassify > 1:
            for fi, _, todo in work:
                for r in todo:
                    if r.object_id:
                        self._cache[r.object_id] = (fi, [t for t in r.tensors if t.model == self.model.name])
            for r, src in self._deferred:
                r.tensors.extend(t for t in src.tensors if t.model == self.model.name)
            self._deferred = []
            if len(self._cache) > 65536:
                self._cache.clear()

    def run_batch(self, reqs, pp):
        """One ROI launch over the regions of every request (hub thread)."""
        import numpy as np

        frames, rois, owners = [], [], []
        for req in reqs:
            for _, img, todo in req.items:
                idx = len(frames)
                frames.append(img)
                for r in todo:
                    rois.append((idx, r.x, r.y, r.w, r.h))
                    owners.append(r)
        if not rois:
            return
        from .preproc import RoiBatch

        out = self._tensor(len(rois))
        pp.convert(frames, out, self.info, rois=RoiBatch(np.asarray(rois, dtype=np.int32)))
        res = self.model.fn(out)
        posts = self.model.postprocs() or [{}]
        if not isinstance(res, dict):
            res = {posts[0].get("layer_name", "classification"): res}
        for pp_ in posts:
            layer = pp_.get("layer_name") or next(iter(res))
            logits = res[layer]
            logits = logits.detach().float().cpu().numpy() if hasattr(logits, "detach") else logits
            name = pp_.get("attribute_name", layer)
            tens = P.classify(logits, pp_.get("labels"), pp_.get("method", "max"), name, model=self.model.name)
            for r, t in zip(owners, tens):
                r.tensors.append(t)


_SECOND = operator.itemgetter(1)  # the Image of a (frame_index, Image, FrameResult) work item


class ClipRing:
    """The clip ring of one action model on one device, shared by every action stream the device serves
    (BASELINE configs[4]: 16-frame 224x224 clip stacking, batched across streams).

    Pages of ``[ROWS * 16, 3, H, W]`` fp32 (``ROWS`` streams of 16 slots: the ``[S, 16, 3, H, W]`` layout of
    bench.py's C5 line); a stream owns one row and writes its frame ``t`` at slot ``row * 16 + t % 16``, so the row
    always holds its 16 most recent pre-processed frames. ``event`` marks the last launch that used the ring: ticks
    run on alternating streams (``inflight``), and the next tick's launch waits for it before it overwrites slots.
    """

    ROWS = 32

    def __init__(self, device: int, size):
        self.device = int(device)
        self.W, self.H = size
        self.pages: list = []
        self.free: list = []
        self.event = None

    def acquire(self):
        """A free (page, row); a new page when every row is taken."""
        if not self.free:
            p = len(self.pages)
            self.pages.append(self._page())
            self.free = [(p, r) for r in range(self.ROWS - 1, -1, -1)]
        return self.free.pop()

    def _page(self):
        import torch

        return torch.zeros((self.ROWS * ActionRecognitionStage.CLIP, 3, self.H, self.W), dtype=torch.float32,
                           device=f"cuda:{self.device}")

    def release(self, pr):
        self.free.append(pr)

    def enter(self):
        """Order this tick's launches (on the current stream) behind the last tick that used the ring."""
        if self.event is not None:
            import torch

            torch.cuda.current_stream(self.device).wait_event(self.event)

    def leave(self):
        """Mark the end of this tick's use of the ring on the current stream."""
        if self.pages and self.pages[0].is_cuda:
            import torch

            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
            self.event = ev


class ActionRecognitionStage(_InferenceStage):
    """gvaactionrecognitionbin (``pipelines/action_recognition/general/pipeline.json:3-4``): the encoder's
    pre-processing (model-proc ``resize: aspect-ratio`` + ``crop: central``,
    ``models_list/action-recognition-0001.json:3-13``) into a 16-slot clip ring per stream, batched across streams.

    Every stream of the device owns a row of the model's shared :class:`ClipRing`; one ``evam_pp_run_slots`` per
    tick writes the new frames of ALL action streams, each at its own slot ``row * 16 + t % 16`` (streams need not be
    in step). A launch covers up to 16 consecutive frames of every stream; with a decoder it ends at the first frame
    whose window is due, so no slot a due window reads is overwritten before the window is taken.

    Inference follows the reference element: the encoder runs once per frame (on the frames each launch wrote, batched
    across streams) and the decoder on the window of the stream's last 16 embeddings, oldest first, on every
    ``inference-interval``-th frame once 16 frames have arrived. Without a decoder (``dec-model`` unset) the stage
    only fills the ring.
    """

    CLIP = 16

    def __init__(self, el, server, device, slot=0):
        super().__init__(el, server, device, slot)
        self.t = 0           # frames of this stream written so far
        self._row = None     # (page, row) in the device's ClipRing
        self.last_row = None
        self._emb = collections.deque(maxlen=self.CLIP)  # the stream's last 16 encoder outputs (device rows)
        dec = el.properties.get("dec-model")
        self.decoder = server.model_for(dec, device) if dec else None
        mp = el.properties.get("model-proc")
        self.dec_proc = json.load(open(mp)) if mp and os.path.exists(mp) else None
        if self.dec_proc:  # the decoder's model-proc carries the encoder's input_preproc too
            self.info = InferenceModel(None, self.model.input_size, self.dec_proc).preproc_info()

    def _make_hub_key(self):
        return super()._make_hub_key() + ("clip", id(self.decoder) if self.decoder is not None else None)

    def out_dtype(self) -> int:
        return N.DTYPE_F32

    def ring(self) -> ClipRing:
        return self.server.hub(self.slot).clip_ring(self.hub_key(), self.model.input_size, self.device)

    def ring_row(self):
        """This stream's 16 ring slots ``[16, 3, H, W]`` (slot k holds frame t with t % 16 == k), or None."""
        pr = self._row if self._row is not None else self.last_row
        if pr is None:
            return None
        p, r = pr
        return self.ring().pages[p][r * self.CLIP:(r + 1) * self.CLIP]

    def prepare(self, items):
        return items, len(items)

    def close(self):
        if self._row is not None:
            self.last_row = self._row  # inspection (tests): the row keeps its frames until another stream takes it
            self.ring().release(self._row)
            self._row = None
        super().close()

    def _due(self, req, j) -> bool:
        return (self.decoder is not None and self.t + j + 1 >= self.CLIP
                and req.items[j][0] % self.interval == 0)

    def launch_batch(self, reqs, pp):
        """Enqueue the launches over every request's frames (and, with a decoder, the encoder / decoder calls);
        returns the completion that attaches the decoded actions to the frames."""
        import numpy as np
        import torch

        C = self.CLIP
        ring = self.ring()
        for r in reqs:
            if r.stage._row is None:
                r.stage._row = ring.acquire()
        ring.enter()
        dec = self.decoder
        lens = [len(r.items) for r in reqs]
        kmax = max(lens)
        windows = []  # (FrameResult, logits) of due frames
        pos = 0
        while pos < kmax:
            end = min(kmax, pos + C)
            if dec is not None:
                for j in range(pos, end):  # the launch ends with the first frame whose window is due
                    if any(j < n and r.stage._due(r, j) for r, n in zip(reqs, lens)):
                        end = j + 1
                        break
            by_page: dict = {}
            for r, n in zip(reqs, lens):
                j1 = min(end, n)
                if j1 <= pos:
                    continue
                st = r.stage
                p, row = st._row
                imgs, sl, owners = by_page.setdefault(p, ([], [], []))
                imgs.extend(map(_SECOND, r.items[pos:j1]))
                sl.append((row * C, st.t + pos, j1 - pos))
                owners.append((r, pos, j1))
            for p, (imgs, sl, owners) in by_page.items():
                # slot of frame j of a request: row * 16 + (t + j) % 16, for all requests in a few array operations
                base, ph, k = np.array(sl, dtype=np.int64).T
                first = np.repeat(np.cumsum(k) - k, k)
                slots = (np.repeat(base, k) + (np.repeat(ph, k) + np.arange(len(imgs)) - first) % C).astype(np.int32)
                page = ring.pages[p]
                pp.convert(imgs, page, self.info, slots=slots)
                if dec is None:
                    continue
                emb = self.model.fn(page.index_select(0, torch.from_numpy(slots).to(page.device, torch.int64)))
                k = 0
                for r, j0, j1 in owners:
                    st = r.stage
                    for j in range(j0, j1):
                        st._emb.append(emb[k])
                        k += 1
                        if st._due(r, j):
                            windows.append((r.items[j][2], dec.fn(torch.stack(tuple(st._emb)))))
            pos = end
        for r, n in zip(reqs, lens):
            r.stage.t += n
        ring.leave()

        def complete():
            if not windows:
                return
            logits = torch.cat([lg.reshape(1, -1) if hasattr(lg, "reshape") else torch.as_tensor(lg).reshape(1, -1)
                                for _, lg in windows]).detach().float().cpu().numpy()
            post = (self.dec_proc or {}).get("output_postproc", [{}])[0]
            tens = P.classify(logits, post.get("labels"), post.get("method", "softmax"),
                              post.get("attribute_name", "action"), model=dec.name)
            for (fr, _), t in zip(windows, tens):
                fr.tensors.append(t)

        return complete

    def run_batch(self, reqs, pp):
        self.launch_batch(reqs, pp)()


STAGES = {"gvadetect": DetectStage, "gvaclassify": ClassifyStage, "gvainference": DetectStage,
          "gvaactionrecognitionbin": ActionRecognitionStage}


# ------------------------------------------------------------------------------------------------
# Pipelines
# ------------------------------------------------------------------------------------------------
@dataclass
class PipelineDefinition:
    name: str
    version: str
    path: str
    type: str
    template: object
    description: str = ""
    parameters: dict = field(default_factory=dict)

    @classmethod
    def load(cls, path: str, name: str, version: str) -> "PipelineDefinition":
        d = json.load(open(path))
        return cls(name, version, path, d.get("type", "GStreamer"), d.get("template", ""),
                   d.get("description", ""), d.get("parameters", {}))


class Pipeline:
    """One pipeline instance (``PipelineServer.pipeline(name, version)``)."""

    QUEUED, RUNNING, COMPLETED, ERROR, ABORTED = "QUEUED", "RUNNING", "COMPLETED", "ERROR", "ABORTED"
    kIngest = 1024  # device runner: most frames of one stream ingested and not yet run

    def __init__(self, server: "_Server", definition: PipelineDefinition, instance_id: int):
        self.server = server
        self.definition = definition
        self.id = instance_id
        self.state = self.QUEUED
        self.error = None
        self.elements: list[Element] = []
        self.parameters: dict = {}
        self.stages: list = []
        self.frames = 0
        self.start_time = None
        self.end_time = None
        self._thread = None
        self._stop = threading.Event()
        # device-runner state (DeviceRunner): frames ingested and not yet run, end of stream, completion
        self._pend: list = []
        self._head = 0  # frames before it are taken
        self._pend_t0 = 0.0
        self._eos = False
        self._batch = 1
        self._done = threading.Event()
        self._ended = False  # end of stream (or error) delivered: nothing of this stream may follow its marker
        self._runner = False
        self._out_backlog = collections.deque()  # runner mode: results a full destination queue could not take
        self._out_limit = 1  # held-back results at which the runner stops ingesting / running this stream
        # logical device: pipeline k of the server runs on devices[(k - 1) mod G] (streams partitioned over GPUs)
        self.slot = server.slot_for(instance_id)
        self.device = server.devices[self.slot]

    # -- construction ------------------------------------------------------------------------
    def build(self, source=None, parameters=None):
        src = source or {}
        auto = {"uri": "urisourcebin uri={}".format(src.get("uri", "")),
                "application": "appsrc name=source", "gst": src.get("element", "")}.get(src.get("type"),
                                                                                       "appsrc name=source")
        text = resolve_template(self.definition.template, self.server.models, {"auto_source": auto})
        self.elements = parse_launch(text)
        self.parameters = apply_parameters(self.elements, self.definition.parameters, parameters)
        for el in self.elements:
            if "model" in el.properties and "model-proc" not in el.properties:
                proc = self.server.proc_for(el.properties["model"])
                if proc:
                    el.properties["model-proc"] = proc
        return self

    def element(self, name: str) -> Element | None:
        return next((e for e in self.elements if e.name == name), None)

    def backends(self) -> dict:
        """{element name: pre-process backend} for the inference elements."""
        return {(e.name or e.factory): _backend_of(e) for e in self.elements if e.factory in INFERENCE_ELEMENTS}

    # -- execution ---------------------------------------------------------------------------
    def start(self, source=None, destination=None, parameters=None):
        """Build the element graph, instantiate the HIP stages, and run the frame loop in a thread."""
        self.build(source, parameters)
        self.stages = [STAGES[e.factory](e, self.server, self.device, self.slot)
                       for e in self.elements if e.factory in STAGES]
        self.source = source or {}
        self.destination = destination or {}
        self.state = self.RUNNING
        self.start_time = time.time()
        if self.server.options.get("runner", "device") == "threads":
            self._thread = threading.Thread(target=self._run, name=f"pipeline-{self.id}", daemon=True)
            self._thread.start()
        else:
            self._runner = True
            self._batch = max([getattr(s, "batch_size", 1) for s in self.stages] + [1])
            dst = self.destination.get("metadata", self.destination)
            self._out_limit = max(1, self._batch, int(getattr(dst.get("output"), "maxsize", 0) or 0))
            self._pend_t0 = time.perf_counter()
            self.server.runner(self.slot).add(self)
        return self.id

    # -- device-runner side (called on the DeviceRunner thread only) ----------------------------------
    def _ingest(self):
        """Move whatever the source holds now into ``_pend`` as (frame_index, Image, FrameResult), without
        blocking: an application queue is drained in one step under its lock, not item by item."""
        if self._eos:
            return
        src = self.source
        kind = src.get("type")
        # At most kIngest frames ahead of the runner per stream: the rest stays in the application's queue
        # (bounded buffering; a backlog of hundreds of thousands of live records made the collector's
        # full passes grow with it).
        backlog = len(self._pend) - self._head
        if backlog > self.kIngest // 4:  # refill in large steps, not a few frames per tick
            return
        room = self.kIngest - backlog
        if kind == "application":
            q = src.get("input")
            if type(q) is queue.Queue:  # FIFO deque inside; subclasses (LIFO, priority, custom _get) go item by item
                with q.mutex:
                    d = q.queue
                    if len(d) <= room:
                        got = list(d)
                        d.clear()
                    else:
                        got = [d.popleft() for _ in range(room)]
                    q.not_full.notify_all()
            else:
                got = []
                while len(got) < room:
                    try:
                        got.append(q.get_nowait())
                    except queue.Empty:
                        break
        elif kind == "frames":
            frames = src.get("frames", [])
            got = list(frames[self.frames:self.frames + room])
            if self.frames + len(got) >= len(frames):
                got.append(None)
        else:
            raise PreProcError(N.ERR_UNSUPPORTED, f"source type {kind!r}: decode is upstream of this build; use an "
                                                  "'application' source of decoded frames")
        if not got:
            return
        types = set(map(type, got))  # C-level scan (Image.__eq__ would run per item for `None in got`)
        if type(None) in types:      # end of stream
            got = got[:next(i for i, x in enumerate(got) if x is None)]
            self._eos = True
            types = set(map(type, got))
        if not got:
            return
        if len(self._pend) == self._head:
            self._pend.clear()
            self._head = 0
            self._pend_t0 = time.perf_counter()
        base, uri, FR = self.frames, self.source.get("uri"), P.FrameResult
        if types == {Image}:
            n = len(got)
            idx = range(base, base + n)
            frs = map(FR, map(_WIDTH, got), map(_HEIGHT, got), idx, itertools.repeat(uri, n))
            self._pend.extend(zip(idx, got, frs))
        else:
            for k, item in enumerate(got):
                img = self._as_image(item)
                ts = int(item.get("timestamp", 0)) if isinstance(item, dict) else base + k
                self._pend.append((base + k, img, FR(img.width, img.height, timestamp=ts, source=uri)))
        self.frames += len(got)

    def _emit_all(self, items):
        if self._ended:  # results of a tick completed after the stream failed: never after its end marker
            return
        dst = self.destination.get("metadata", self.destination)
        if dst.get("output") is None:
            return
        for _, img, fr in items:
            self._emit(fr, img)

    def _fail(self, e):
        self.error = f"{type(e).__name__}: {e}"
        self.state = self.ERROR
        self._end()

    def _end(self):
        if self._ended or self._done.is_set():
            return
        self._ended = True
        if self.state == self.RUNNING:
            self.state = self.ABORTED if self._stop.is_set() else self.COMPLETED
        for st in self.stages:
            st.close()
        self.end_time = time.time()
        dst = self.destination.get("metadata", self.destination)
        if dst.get("output") is not None:
            self._put(dst["output"], None)
        if not self._out_backlog:
            # otherwise complete once the device runner has handed the held-back results (and the end-of-stream
            # marker) to the destination (DeviceRunner._drain), so wait() never returns ahead of them
            self._done.set()

    def _frames(self):
        src = self.source
        if src.get("type") == "application":
            q = src.get("input")
            while not self._stop.is_set():
                try:
                    item = q.get(timeout=0.1)
                except queue.Empty:
                    continue
                # then whatever is already queued, without blocking again: one wake-up per burst of
                # frames rather than per frame (the pipeline threads of all streams share the GIL)
                burst = [item]
                while item is not None and len(burst) < 64:
                    try:
                        item = q.get_nowait()
                    except queue.Empty:
                        break
                    burst.append(item)
                for item in burst:
                    if item is None:        # end of stream
                        return
                    yield item
        elif src.get("type") == "frames":
            yield from src.get("frames", [])
        else:
            raise PreProcError(N.ERR_UNSUPPORTED, f"source type {src.get('type')!r}: decode is upstream of this "
                                                  "build; use an 'application' source of decoded frames")

    def _as_image(self, item):
        if isinstance(item, Image):
            return item
        if isinstance(item, dict):         # host frame {fourcc, width, height, planes}
            return Image.from_host(item["fourcc"], item["width"], item["height"], item["planes"],
                                   device=f"cuda:{self.device}")
        raise TypeError(f"unsupported frame object {type(item).__name__}")

    def _emit(self, fr: P.FrameResult, img):
        dst = self.destination.get("metadata", self.destination)
        out = dst.get("output")
        mode = dst.get("mode", "frames")
        if out is None:
            return
        item = (img, fr) if mode == "frames" else P.gvametaconvert_json(fr)
        if self._runner:
            self._put(out, item)
        else:
            out.put(item)  # threads mode: a full queue blocks this stream's own thread only

    def _put(self, out, item):
        """Runner mode: never block the device's shared runner on one stream's destination. A full bounded
        queue keeps the results (in order) in this pipeline's backlog; the runner retries them."""
        if not self._runner or not hasattr(out, "put_nowait"):
            out.put(item)
            return
        if self._out_backlog:  # keep the order: behind what is already held back
            self._out_backlog.append(item)
            self._flush_out()
            return
        try:
            out.put_nowait(item)
        except queue.Full:
            self._out_backlog.append(item)

    def _flush_out(self) -> bool:
        """Move backlog results into the destination while it has room; True when none are left."""
        dst = self.destination.get("metadata", self.destination)
        out = dst.get("output")
        b = self._out_backlog
        while b:
            try:
                out.put_nowait(b[0])
            except queue.Full:
                return False
            b.popleft()
        return True

    def _run(self):
        try:
            batch = max([getattr(s, "batch_size", 1) for s in self.stages] + [1])
            pend = []
            for item in self._frames():
                img = self._as_image(item)
                ts = int(item.get("timestamp", 0)) if isinstance(item, dict) else self.frames
                fr = P.FrameResult(img.width, img.height, timestamp=ts, source=self.source.get("uri"))
                pend.append((self.frames, img, fr))
                self.frames += 1
                if len(pend) >= batch:
                    self._flush(pend)
                    pend = []
                if self._stop.is_set():
                    break
            if pend:
                self._flush(pend)
            self.state = self.ABORTED if self._stop.is_set() else self.COMPLETED
        except Exception as e:  # noqa: BLE001 — reported through status(), as the reference does
            self.error = f"{type(e).__name__}: {e}"
            self.state = self.ERROR
        finally:
            for s in self.stages:
                s.close()
            self.end_time = time.time()
            dst = self.destination.get("metadata", self.destination)
            if dst.get("output") is not None:
                dst["output"].put(None)

    def _flush(self, pend):
        for s in self.stages:
            s.process(pend)
        for _, img, fr in pend:
            self._emit(fr, img)

    def stop(self):
        self._stop.set()
        return self.status()

    def wait(self, timeout=None):
        if self._runner:
            self._done.wait(timeout)
        elif self._thread is not None:
            self._thread.join(timeout)
        return self.status()

    def status(self) -> dict:
        el = ((self.end_time or time.time()) - self.start_time) if self.start_time else 0.0
        return {"id": self.id, "state": self.state, "avg_fps": self.frames / el if el > 0 else 0.0,
                "elapsed_time": el, "start_time": self.start_time, "message": self.error}


class _Server:
    """State behind the ``PipelineServer`` facade (one per process, like the reference's)."""

    def __init__(self):
        self.options: dict = {}
        self.definitions: dict = {}
        self.models: dict = {}
        self.registry: dict = {}      # network or alias/version -> model serving every device
        self.registry_dev: dict = {}  # (network or alias/version, device) -> model bound to that device
        self.instances: list[Pipeline] = []
        self.started = False
        self.device = 0
        self.devices = [0]      # logical devices: pipeline k runs on devices[(k - 1) % len(devices)]
        self._hubs: dict = {}    # logical device -> BatchHub
        self._runners: dict = {}  # logical device -> DeviceRunner
        self._gc_saved = None
        self._hub_lock = threading.Lock()

    def slot_for(self, instance_id: int) -> int:
        """Logical device of pipeline instance ``instance_id`` (1-based): streams s -> GPU s mod G
        (SURVEY.md §8e), the same partition bench.py and streams.py apply across ranks."""
        return (int(instance_id) - 1) % len(self.devices)

    def hub(self, slot: int = 0) -> BatchHub:
        """The batching hub of logical device ``slot`` (created on first use; options ``batch_max``,
        ``batch_wait_ms``, ``batch_target``). Each one owns its own pre-processing handle and stream."""
        with self._hub_lock:
            h = self._hubs.get(slot)
            if h is None:
                o = self.options
                h = self._hubs[slot] = BatchHub(self.devices[slot], max_batch=int(o.get("batch_max", 64)),
                                                max_wait_s=float(o.get("batch_wait_ms", 2.0)) / 1e3,
                                                target=o.get("batch_target"),
                                                drain_timeout_s=float(o.get("drain_timeout_ms", 2000.0)) / 1e3,
                                                inflight=int(o.get("inflight", 3)))
            return h

    def runner(self, slot: int = 0) -> DeviceRunner:
        """The pipeline runner of logical device ``slot`` (created on first use; it batches through that
        device's hub)."""
        hub = self.hub(slot)
        with self._hub_lock:
            if not self._runners and self._gc_saved is None:
                self._gc_saved = (gc.get_threshold(), False)
                if self.options.get("gc_freeze", True):
                    # The heap built so far (torch, models, templates) leaves the collector's generations:
                    # the runner makes a few short-lived objects per frame, and every young collection that
                    # escalated would otherwise rescan it (2x the per-frame cost at 32 streams).
                    gc.freeze()
                    self._gc_saved = (self._gc_saved[0], True)
                gct = self.options.get("gc_threshold", (20000, 100, 1000))
                if gct:
                    # Per-frame records die by reference count, never in cycles; collecting them every 700
                    # allocations (the default) cost as much as the rest of the runner at 32 streams.
                    gc.set_threshold(*gct)
            r = self._runners.get(slot)
            if r is None:
                r = self._runners[slot] = DeviceRunner(hub)
            return r

    def close_hub(self):
        with self._hub_lock:
            for r in self._runners.values():
                r.close()
            self._runners = {}
            if self._gc_saved is not None:  # the process's collector settings, as before the runners
                thresholds, frozen = self._gc_saved
                gc.set_threshold(*thresholds)
                if frozen:
                    gc.unfreeze()
                self._gc_saved = None
            for h in self._hubs.values():
                h.close()
            self._hubs = {}

    def start(self, options=None):
        o = dict(options or {})
        self.options = o
        self.device = int(o.get("device", os.environ.get("EVAM_HIP_DEVICE", 0)))
        devs = o.get("devices")
        if devs is None and os.environ.get("EVAM_HIP_DEVICES"):
            devs = [int(x) for x in os.environ["EVAM_HIP_DEVICES"].split(",") if x.strip()]
        self.devices = [int(d) for d in devs] if devs else [self.device]
        if not self.devices:
            raise ValueError("PipelineServer.start: 'devices' must name at least one device")
        self.device = self.devices[0]
        pdir = o.get("pipeline_dir") or os.environ.get("PIPELINE_DIR", "pipelines")
        mdir = o.get("model_dir") or os.environ.get("MODEL_DIR", "models")
        self.models = scan_models(mdir)
        self.definitions = {}
        errors = []
        if os.path.isdir(pdir):
            for name in sorted(os.listdir(pdir)):
                ndir = os.path.join(pdir, name)
                if not os.path.isdir(ndir):
                    continue
                for version in sorted(os.listdir(ndir)):
                    path = os.path.join(ndir, version, "pipeline.json")
                    if os.path.exists(path):
                        try:
                            self.definitions.setdefault(name, {})[version] = PipelineDefinition.load(path, name, version)
                        except (OSError, ValueError) as e:
                            errors.append(f"{path}: {e}")
        elif not o.get("ignore_init_errors", False):
            raise FileNotFoundError(f"pipeline directory {pdir!r} not found")
        if errors and not o.get("ignore_init_errors", False):
            raise ValueError("; ".join(errors))
        self.started = True

    def model_for(self, network, device=None):
        """The model bound to ``network`` (a path or an ``alias/version`` key) for ``device``: a registration for
        that device first, then a device-independent one."""
        if network is None:
            return None
        m = re.search(r"([^/]+)/([^/]+)/[^/]+/[^/]+\.xml$", str(network))
        keys = [network] + ([f"{m.group(1)}/{m.group(2)}"] if m else [])
        for k in keys:
            if device is not None and (k, int(device)) in self.registry_dev:
                return self.registry_dev[(k, int(device))]
        for k in keys:
            if k in self.registry:
                return self.registry[k]
        return None

    def proc_for(self, network):
        for alias, versions in self.models.items():
            for version, e in versions.items():
                if network in e.values() and "proc" in e:
                    return e["proc"]
        return None


_SERVER = _Server()


class PipelineServer:
    """Facade with the reference's class-level API (``evas/manager.py:100-155``)."""

    @staticmethod
    def start(options=None):
        _SERVER.start(options)

    @staticmethod
    def pipelines():
        return [{"name": d.name, "version": d.version, "type": d.type, "description": d.description,
                 "parameters": d.parameters}
                for vs in _SERVER.definitions.values() for d in vs.values()]

    @staticmethod
    def pipeline(name, version):
        d = _SERVER.definitions.get(name, {}).get(str(version))
        if d is None:
            return None
        p = Pipeline(_SERVER, d, len(_SERVER.instances) + 1)
        _SERVER.instances.append(p)
        return p

    @staticmethod
    def pipeline_instances():
        return list(_SERVER.instances)

    @staticmethod
    def register_model(network_or_key: str, model: InferenceModel, device: int | None = None):
        """Bind a model to a network path or an ``alias/version`` key (replaces OpenVINO loading).

        ``device``: the model serves only the pipelines placed on that logical device (option ``devices``: its
        weights live on that GPU); register one per device. Without it the model serves every device, and its
        ``fn`` receives each device's input tensors (it must accept any of them); it also replaces the per-device
        registrations of that key, so the latest registration wins everywhere until a device is bound again."""
        if device is None:
            _SERVER.registry[network_or_key] = model
            for k in [k for k in _SERVER.registry_dev if k[0] == network_or_key]:
                del _SERVER.registry_dev[k]
        else:
            _SERVER.registry_dev[(network_or_key, int(device))] = model

    @staticmethod
    def models():
        return _SERVER.models

    @staticmethod
    def wait(timeout=None):
        for p in list(_SERVER.instances):
            p.wait(timeout)

    @staticmethod
    def stop():
        for p in list(_SERVER.instances):
            p.stop()
        for p in list(_SERVER.instances):
            p.wait(5.0)
        _SERVER.instances.clear()
        _SERVER.close_hub()
        _SERVER.started = False

    @staticmethod
    def hub(slot: int = 0):
        """The batching hub of logical device ``slot`` (inspection: ``hub().batches``)."""
        return _SERVER.hub(slot)

    @staticmethod
    def devices():
        """The logical devices pipelines are partitioned over (option ``devices``; default ``[device]``)."""
        return list(_SERVER.devices)
