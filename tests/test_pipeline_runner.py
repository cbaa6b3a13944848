"""The per-device pipeline runner (pipeline_server.DeviceRunner) on CPU: the HIP pre-processor is replaced by
a recording stub (the kernels are covered by the GPU suites), so these tests check the runner's own logic —
bulk ingest of application queues, batch-size gating and end of stream, one launch per interchangeable
stage across pipelines bounded by batch_max, per-stream stage order, destinations, errors, stop — in the
`"device"` runner and, for the same scenario, the `"threads"` runner (per-pipeline threads + BatchHub)."""
import json
import queue
import time

import pytest
import torch

from test_pipeline_server import PIPES, make_model_tree


class StubPP:
    """Records every convert call; returns lazily built identity transforms like HipPreProcessor."""

    calls = []
    slot_calls = []

    def __init__(self, device=0, stream=None):
        pass

    def convert(self, srcs, out, info=None, rois=None, slot_offset=0, slot_stride=1, want_transform=False, slots=None):
        n_src = len(srcs)
        n_roi = None if rois is None else len(rois)
        StubPP.calls.append((n_src, n_roi, tuple(out.shape)))
        if slots is not None:
            StubPP.slot_calls.append([int(v) for v in slots])
        if want_transform:
            return [None] * n_src

    def close(self):
        pass


@pytest.fixture
def stubbed(evam, monkeypatch, tmp_path):
    ps = evam.pipeline_server
    pre = evam.preproc
    monkeypatch.setattr(pre, "HipPreProcessor", StubPP)
    monkeypatch.setattr(ps._InferenceStage, "_tensor",
                        lambda self, n: torch.zeros((n, 3, self.model.input_size[1], self.model.input_size[0])))
    StubPP.calls = []
    StubPP.slot_calls = []
    mdir = make_model_tree(str(tmp_path / "models"), {
        "det_alias": {"det_ver": (64, 64, {"input_preproc": [], "output_postproc": [{"labels": ["bg", "car"]}]})},
        "cls_alias": {"cls_ver": (24, 24, {"input_preproc": [],
                                           "output_postproc": [{"layer_name": "color", "attribute_name": "color",
                                                                "labels": ["dark", "light"], "method": "max"}]})}})
    yield ps, pre, mdir
    ps.PipelineServer.stop()


def frames(pre, n, w=64, h=48):
    planes = [torch.zeros((h, w), dtype=torch.uint8), torch.zeros((h // 2, w), dtype=torch.uint8)]
    return [pre.Image(pre.FOURCC_BY_NAME["NV12"], w, h, planes) for _ in range(n)]


def register(ps, det_every=2, fail=False):
    def detector(t):
        if fail:
            raise RuntimeError("model failed")
        n = t.shape[0]
        out = torch.full((n, 1, 7), -1.0)
        out[::det_every, 0] = torch.tensor([0, 1, 0.9, 0.25, 0.25, 0.5, 0.75])   # a car on every det_every-th
        return out

    ps.PipelineServer.register_model("det_alias/det_ver", ps.InferenceModel(detector, (64, 64), name="det"))
    ps.PipelineServer.register_model("cls_alias/cls_ver", ps.InferenceModel(
        lambda t: {"color": torch.stack([torch.zeros(t.shape[0]), torch.ones(t.shape[0])], 1)}, (24, 24),
        name="cls"))


@pytest.mark.parametrize("runner", ["device", "threads"])
def test_runner_batches_across_pipelines(stubbed, runner):
    ps, pre, mdir = stubbed
    ps.PipelineServer.start({"pipeline_dir": PIPES, "model_dir": mdir, "runner": runner, "batch_max": 8,
                             "batch_wait_ms": 200, "batch_target": 8})
    register(ps)
    counts = [5, 3, 7, 1]  # frames per stream; batch-size 2 leaves a remainder flushed at end of stream
    pipes, outs = [], []
    for k, n in enumerate(counts):
        qin, qout = queue.Queue(), queue.Queue()
        for im in frames(pre, n):
            qin.put(im)
        qin.put(None)
        p = ps.PipelineServer.pipeline("detect_classify", "hip")
        p.start(source={"type": "application", "input": qin},
                destination={"metadata": {"type": "application", "output": qout, "mode": "json"}},
                parameters={"detection-properties": {"batch-size": 2}})
        pipes.append(p)
        outs.append(qout)
    for p in pipes:
        st = p.wait(60)
        assert st["state"] == "COMPLETED", st
    n_objects = 0
    for n, q in zip(counts, outs):
        lines = []
        while (x := q.get(timeout=5)) is not None:
            lines.append(json.loads(x))
        assert len(lines) == n
        for i, d in enumerate(lines):
            objs = d.get("objects", [])
            # frame i of a batch of 2 gets a car when its index in the launch is even; every car is classified
            assert all("color" in o and o["color"]["label"] == "light" for o in objs)
            n_objects += len(objs)
    det = [c for c in StubPP.calls if c[1] is None]
    cls = [c for c in StubPP.calls if c[1] is not None]
    assert sum(c[0] for c in det) == sum(counts)           # every frame pre-processed exactly once
    assert all(c[0] <= 8 for c in det)                       # batch_max frames per launch
    assert len(det) < sum(counts)                            # frames of several streams share launches
    assert n_objects > 0 and sum(c[1] for c in cls) == n_objects  # every car classified once
    hub = ps.PipelineServer.hub()
    assert any(b[2] > 1 for b in hub.batches)                # a launch served more than one pipeline


def test_runner_model_error_marks_pipelines(stubbed):
    ps, pre, mdir = stubbed
    ps.PipelineServer.start({"pipeline_dir": PIPES, "model_dir": mdir})
    register(ps, fail=True)
    qin = queue.Queue()
    for im in frames(pre, 3):
        qin.put(im)
    qin.put(None)
    p = ps.PipelineServer.pipeline("detect_classify", "hip")
    p.start(source={"type": "application", "input": qin}, destination={})
    st = p.wait(60)
    assert st["state"] == "ERROR" and "model failed" in st["message"]


def test_runner_stop_and_frames_source(stubbed):
    ps, pre, mdir = stubbed
    ps.PipelineServer.start({"pipeline_dir": PIPES, "model_dir": mdir})
    register(ps, det_every=1)
    # a "frames" source: the list is the whole stream
    qout = queue.Queue()
    p = ps.PipelineServer.pipeline("detect_classify", "hip")
    p.start(source={"type": "frames", "frames": frames(pre, 4)},
            destination={"metadata": {"output": qout, "mode": "frames"}})
    assert p.wait(60)["state"] == "COMPLETED"
    got = []
    while (x := qout.get(timeout=5)) is not None:
        got.append(x)
    assert len(got) == 4 and all(len(fr.regions) == 1 for _, fr in got)
    # an application source that never ends: stop() aborts it
    qin = queue.Queue()
    for im in frames(pre, 2):
        qin.put(im)
    p2 = ps.PipelineServer.pipeline("detect_classify", "hip")
    p2.start(source={"type": "application", "input": qin}, destination={})
    p2.stop()
    assert p2.wait(30)["state"] == "ABORTED"
    assert p2.status()["elapsed_time"] >= 0


def test_frame_result_lists_are_lazy(evam):
    P = evam.postproc
    fr = P.FrameResult(10, 20)
    assert fr._regions is None and fr.regions == [] and fr._regions == []
    fr.tensors.append(1)
    assert fr.tensors == [1] and P.FrameResult(1, 2, regions=[5]).regions == [5]
    assert json.loads(P.gvametaconvert_json(P.FrameResult(4, 4, timestamp=7)))["timestamp"] == 7


def test_runner_restores_collector_settings(stubbed):
    """The device runner raises the collector thresholds and freezes the startup heap while it serves;
    PipelineServer.stop() gives the process its own settings back."""
    import gc

    ps, pre, mdir = stubbed
    before = gc.get_threshold()
    ps.PipelineServer.start({"pipeline_dir": PIPES, "model_dir": mdir})
    register(ps)
    qin = queue.Queue()
    for im in frames(pre, 2):
        qin.put(im)
    qin.put(None)
    p = ps.PipelineServer.pipeline("detect_classify", "hip")
    p.start(source={"type": "application", "input": qin}, destination={})
    assert p.wait(30)["state"] == "COMPLETED"
    assert gc.get_threshold() == (20000, 100, 1000) and gc.get_freeze_count() > 0
    ps.PipelineServer.stop()
    assert gc.get_threshold() == before and gc.get_freeze_count() == 0


class _BadOut:
    """A destination whose put fails (a consumer's bug)."""

    def put(self, item):
        raise OSError("destination gone")

    def put_nowait(self, item):
        raise OSError("destination gone")


def _start(ps, pre, n, out, batch=2):
    qin = queue.Queue()
    for im in frames(pre, n):
        qin.put(im)
    qin.put(None)
    p = ps.PipelineServer.pipeline("detect_classify", "hip")
    p.start(source={"type": "application", "input": qin},
            destination={"metadata": {"type": "application", "output": out, "mode": "json"}},
            parameters={"detection-properties": {"batch-size": batch}})
    return p


def _drain(q, timeout=10):
    got = []
    while (x := q.get(timeout=timeout)) is not None:
        got.append(x)
    return got


def test_runner_isolates_a_failing_destination(stubbed):
    """an exception from one pipeline's destination fails that pipeline only; the device's other
    pipelines (same runner thread, same launches) complete and deliver every frame."""
    ps, pre, mdir = stubbed
    ps.PipelineServer.start({"pipeline_dir": PIPES, "model_dir": mdir, "batch_max": 8, "batch_target": 4})
    register(ps)
    good_q = queue.Queue()
    bad = _start(ps, pre, 6, _BadOut())
    good = _start(ps, pre, 6, good_q)
    assert bad.wait(30)["state"] == "ERROR" and "destination gone" in bad.status()["message"]
    assert good.wait(30)["state"] == "COMPLETED"
    assert len(_drain(good_q)) == 6


def test_runner_full_destination_does_not_stall_others(stubbed):
    """A bounded destination queue nobody reads must not block the runner that serves every stream of the
    device: its results wait in that pipeline's backlog (in order) while the other streams complete."""
    ps, pre, mdir = stubbed
    ps.PipelineServer.start({"pipeline_dir": PIPES, "model_dir": mdir, "batch_max": 8, "batch_target": 4})
    register(ps)
    slow_q, fast_q = queue.Queue(maxsize=1), queue.Queue()
    slow = _start(ps, pre, 9, slow_q)
    fast = _start(ps, pre, 9, fast_q)
    assert fast.wait(30)["state"] == "COMPLETED"
    assert len(_drain(fast_q)) == 9
    assert not slow._done.is_set()  # its results are still held back: not complete yet
    got = _drain(slow_q)  # the runner hands the held-back results over as the queue empties
    assert [json.loads(x)["timestamp"] for x in got] == list(range(9))
    assert slow.wait(30)["state"] == "COMPLETED"


def test_runner_backpressure_bounds_the_backlog(stubbed):
    """a consumer that never reads stops its own stream (no ingest, no tick) once its held-back
    results reach the destination's size; the backlog stays bounded while the other streams complete, and every
    result arrives, in order, once the consumer reads."""
    import time

    ps, pre, mdir = stubbed
    ps.PipelineServer.start({"pipeline_dir": PIPES, "model_dir": mdir, "batch_max": 8, "batch_target": 4,
                             "batch_wait_ms": 1})
    register(ps)
    slow_q, fast_q = queue.Queue(maxsize=2), queue.Queue()
    slow = _start(ps, pre, 400, slow_q)
    fast = _start(ps, pre, 64, fast_q)
    assert fast.wait(30)["state"] == "COMPLETED"
    assert len(_drain(fast_q)) == 64
    time.sleep(0.2)  # the runner keeps polling the stalled stream
    assert slow._out_limit == 2
    assert len(slow._out_backlog) <= slow._out_limit + 8   # at most one tick past the limit
    assert slow.frames - 2 - len(slow._out_backlog) <= 1024  # ingested ahead: bounded by kIngest, not 400 results
    got = _drain(slow_q)
    assert [json.loads(x)["timestamp"] for x in got] == list(range(400))
    assert slow.wait(30)["state"] == "COMPLETED"


def test_runner_wait_then_stop_delivers_everything(stubbed):
    """wait() returns only once every result and the end-of-stream marker are in the destination, so
    stop() right after it loses nothing, even while the consumer lags behind a small queue."""
    import threading
    import time

    ps, pre, mdir = stubbed
    ps.PipelineServer.start({"pipeline_dir": PIPES, "model_dir": mdir, "batch_max": 8, "batch_target": 4})
    register(ps)
    q = queue.Queue(maxsize=3)
    got = []

    def consumer():
        while True:
            x = q.get(timeout=30)
            if x is None:
                got.append(None)
                return
            got.append(json.loads(x)["timestamp"])
            time.sleep(0.002)

    th = threading.Thread(target=consumer)
    th.start()
    p = _start(ps, pre, 40, q)
    assert p.wait(60)["state"] == "COMPLETED"
    ps.PipelineServer.stop()
    th.join(30)
    assert got == list(range(40)) + [None]


def test_runner_shutdown_reports_undelivered_results(stubbed):
    """at shutdown, results a destination still cannot take after drain_timeout_ms are reported (the
    pipeline ends in ERROR with the count), never dropped silently."""
    ps, pre, mdir = stubbed
    ps.PipelineServer.start({"pipeline_dir": PIPES, "model_dir": mdir, "batch_max": 8, "batch_target": 4,
                             "drain_timeout_ms": 100})
    register(ps)
    q = queue.Queue(maxsize=2)
    p = _start(ps, pre, 12, q)
    import time

    t0 = time.time()
    while len(p._out_backlog) < 1 and time.time() - t0 < 30:
        time.sleep(0.01)
    ps.PipelineServer.stop()
    st = p.status()
    assert st["state"] == "ERROR" and "undelivered" in st["message"], st
    assert p._done.is_set()


def test_models_bind_per_device(stubbed):
    """with devices=[0, 1] a model registered for a device serves only the pipelines placed there; a
    device-independent registration remains the fallback."""
    ps, pre, mdir = stubbed
    ps.PipelineServer.start({"pipeline_dir": PIPES, "model_dir": mdir, "devices": [0, 1], "batch_max": 8,
                             "batch_target": 4, "batch_wait_ms": 50})
    register(ps)  # the device-independent classifier (and a detector every device could use)
    seen = {0: 0, 1: 0}

    def det_on(dev):
        def fn(t):
            seen[dev] += t.shape[0]
            return torch.full((t.shape[0], 1, 7), -1.0)
        return ps.InferenceModel(fn, (64, 64), name="det")

    for dev in (0, 1):
        ps.PipelineServer.register_model("det_alias/det_ver", det_on(dev), device=dev)
    outs = [queue.Queue() for _ in range(4)]
    pipes = [_start(ps, pre, 6, q) for q in outs]
    for p, q in zip(pipes, outs):
        assert p.wait(30)["state"] == "COMPLETED"
        assert len(_drain(q)) == 6
    assert seen == {0: 12, 1: 12}
    assert pipes[0].stages[0].model is not pipes[1].stages[0].model
    assert pipes[0].stages[0].model is pipes[2].stages[0].model
    assert pipes[0].stages[1].model is pipes[1].stages[1].model  # the classifier: one registration for both


def test_runner_partitions_streams_over_devices(stubbed):
    """Option ``devices``: pipeline k runs on devices[(k - 1) mod G] with that logical device's own hub and
    runner (streams partitioned over GPUs); the default stays one device (manager.py's call)."""
    ps, pre, mdir = stubbed
    ps.PipelineServer.start({"pipeline_dir": PIPES, "model_dir": mdir, "devices": [0, 1], "batch_max": 8,
                             "batch_target": 4, "batch_wait_ms": 100})
    register(ps)
    outs = [queue.Queue() for _ in range(4)]
    pipes = [_start(ps, pre, 4, q) for q in outs]
    assert [p.slot for p in pipes] == [0, 1, 0, 1] and [p.device for p in pipes] == [0, 1, 0, 1]
    assert ps.PipelineServer.devices() == [0, 1]
    for p, q in zip(pipes, outs):
        assert p.wait(30)["state"] == "COMPLETED"
        assert len(_drain(q)) == 4
    for slot in (0, 1):
        b = ps.PipelineServer.hub(slot).batches
        assert sum(x[1] for x in b if x[0][0] == "gvadetect") == 8   # two streams of 4 frames each
    assert ps.PipelineServer.hub(0) is not ps.PipelineServer.hub(1)


def test_runner_survives_an_internal_error(stubbed, monkeypatch):
    """Whatever escapes the runner loop fails every pipeline it holds (their wait() returns) instead of
    leaving them RUNNING behind a dead thread."""
    ps, pre, mdir = stubbed
    ps.PipelineServer.start({"pipeline_dir": PIPES, "model_dir": mdir})
    register(ps)

    def boom(self, work):
        raise RuntimeError("runner bug")

    monkeypatch.setattr(ps.DeviceRunner, "_tick", boom)
    p = _start(ps, pre, 4, queue.Queue())
    st = p.wait(30)
    assert st["state"] == "ERROR" and "runner bug" in st["message"]


def test_runner_keeps_two_ticks_in_flight(stubbed, monkeypatch):
    """with inflight 2 (3 is the default since round 6) the device runner launches tick t+1 before it
    completes tick t
    (model output to the host, detections, results), on the hub's alternate slot; ticks still complete in launch
    order and every stream's results are those of inflight 1, in order, end-of-stream marker last."""
    ps, pre, mdir = stubbed
    events = []
    orig = ps.DetectStage.launch_batch

    def launch(self, reqs, pp):
        tick = len([e for e in events if e[0] == "launch"])
        events.append(("launch", tick, id(pp)))
        done = orig(self, reqs, pp)

        def complete():
            events.append(("complete", tick))
            done()
        return complete

    monkeypatch.setattr(ps.DetectStage, "launch_batch", launch)

    def run(inflight, counts=(9, 6, 11)):
        events.clear()
        ps.PipelineServer.start({"pipeline_dir": PIPES, "model_dir": mdir, "batch_max": 4, "batch_target": 4,
                                 "batch_wait_ms": 200, "inflight": inflight})
        register(ps, det_every=1)  # a car in every frame: the results do not depend on how ticks group frames
        outs, pipes = [], []
        for k, n in enumerate(counts):
            qin, qout = queue.Queue(), queue.Queue()
            for im in frames(pre, n):
                qin.put(im)
            qin.put(None)
            p = ps.PipelineServer.pipeline("detect", "hip")
            p.start(source={"type": "application", "input": qin},
                    destination={"metadata": {"type": "application", "output": qout, "mode": "json"}},
                    parameters={"detection-properties": {"batch-size": 2}})
            pipes.append(p)
            outs.append(qout)
        for p in pipes:
            assert p.wait(60)["state"] == "COMPLETED"
        got = [[json.loads(x) for x in _drain(q)] for q in outs]
        ps.PipelineServer.stop()
        return got, list(events)

    one, ev1 = run(1)
    two, ev2 = run(2)
    assert [len(g) for g in one] == [9, 6, 11]
    assert one == two
    # inflight 1: every batch completes before the next launches
    assert all(ev1[i][0] == "launch" and ev1[i + 1] == ("complete", ev1[i][1]) for i in range(0, len(ev1), 2))
    # inflight 2: some tick launches before its predecessor completes; completions keep launch order, and
    # consecutive ticks alternate between the hub's two handles
    order = [e[1] for e in ev2 if e[0] == "complete"]
    assert order == sorted(order) and len(order) == len([e for e in ev2 if e[0] == "launch"])
    pos = {(e[0], e[1]): i for i, e in enumerate(ev2)}
    assert any(pos[("launch", t + 1)] < pos[("complete", t)] for t in range(len(order) - 1))
    handles = [e[2] for e in ev2 if e[0] == "launch"]
    assert len(set(handles)) == 2
    # inflight 3: three ticks launched before the oldest completes (two pending), on three handles, same results
    long_counts = (40, 30, 50)
    three, ev3 = run(3, long_counts)
    assert three == run(1, long_counts)[0] and [len(g) for g in three] == list(long_counts)
    three, ev3 = run(3, long_counts)
    order = [e[1] for e in ev3 if e[0] == "complete"]
    assert order == sorted(order) and len(order) == len([e for e in ev3 if e[0] == "launch"])
    pos = {(e[0], e[1]): i for i, e in enumerate(ev3)}
    # a batch still pending while batches on both other handles were launched after it
    hid = {e[1]: e[2] for e in ev3 if e[0] == "launch"}
    assert any(len({hid[u] for u in hid if u > t and pos[("launch", u)] < pos[("complete", t)]} - {hid[t]}) == 2
               for t in order)
    assert len(set(hid.values())) == 3


@pytest.mark.parametrize("inflight", [1, 2])
def test_runner_error_follows_earlier_results(stubbed, inflight):
    """A stream whose model fails in a later tick first receives every result of the ticks before it, then its end of
    stream, in that order, also while a tick is still in flight (inflight 2: the failing tick's error waits for the
    previous tick's completion)."""
    ps, pre, mdir = stubbed
    ps.PipelineServer.start({"pipeline_dir": PIPES, "model_dir": mdir, "batch_max": 2, "batch_target": 2,
                             "batch_wait_ms": 200, "inflight": inflight})
    n_calls = [0]

    def detector(t):
        n_calls[0] += 1
        if n_calls[0] == 2:
            raise RuntimeError("model failed on the second batch")
        return torch.full((t.shape[0], 1, 7), -1.0)

    ps.PipelineServer.register_model("det_alias/det_ver", ps.InferenceModel(detector, (64, 64), name="det"))
    qin, qout = queue.Queue(), queue.Queue()
    for im in frames(pre, 6):
        qin.put(im)
    qin.put(None)
    p = ps.PipelineServer.pipeline("detect", "hip")
    p.start(source={"type": "application", "input": qin},
            destination={"metadata": {"type": "application", "output": qout, "mode": "json"}},
            parameters={"detection-properties": {"batch-size": 2}})
    st = p.wait(30)
    assert st["state"] == "ERROR" and "second batch" in st.get("message", ""), st
    got = _drain(qout)
    assert len(got) == 2  # the first batch's two frames, then the end-of-stream marker


def test_runner_failed_stream_gets_nothing_after_its_marker(stubbed):
    """stream A fails in tick t (its pre-processing prepare raises) while stream B's detection batch of the
    same tick is deferred (inflight 2), so tick t stays pending. A must leave the runner at once: no later tick may
    ingest or run its frames, and nothing may reach A's destination after its end-of-stream marker."""
    import time

    ps, pre, mdir = stubbed
    ps.PipelineServer.start({"pipeline_dir": PIPES, "model_dir": mdir, "batch_max": 4, "batch_target": 4,
                             "batch_wait_ms": 500, "inflight": 2})
    register(ps, det_every=1)
    qa, qb, outa, outb = queue.Queue(), queue.Queue(), queue.Queue(), queue.Queue()
    pa, pb = (ps.PipelineServer.pipeline("detect", "hip") for _ in range(2))
    for p, qin, qout in ((pa, qa, outa), (pb, qb, outb)):
        p.start(source={"type": "application", "input": qin},
                destination={"metadata": {"type": "application", "output": qout, "mode": "json"}},
                parameters={"detection-properties": {"batch-size": 2}})
    st = pa.stages[0]
    orig, calls = st.prepare, [0]

    def prepare(items):
        calls[0] += 1
        if calls[0] == 2:
            raise RuntimeError("prepare failed on A's second tick")
        return orig(items)

    st.prepare = prepare
    for qin in (qa, qb):
        for im in frames(pre, 8):
            qin.put(im)
        qin.put(None)
    assert pb.wait(30)["state"] == "COMPLETED"
    sa = pa.wait(30)
    assert sa["state"] == "ERROR" and "second tick" in sa.get("message", ""), sa
    assert len(_drain(outb)) == 8
    got = _drain(outa)
    time.sleep(0.1)
    assert len(got) == 2 and outa.empty()  # the first tick's frames, the marker, and nothing after it
    assert calls[0] == 2                   # no tick ran A's frames after it failed


def test_runner_death_with_held_back_results(stubbed, monkeypatch):
    """a runner thread that dies while a pipeline holds results back for a full bounded destination
    still ends that pipeline: wait() returns, in ERROR, with the undelivered results counted (no thread is left
    to hand them over)."""
    import time

    ps, pre, mdir = stubbed
    ps.PipelineServer.start({"pipeline_dir": PIPES, "model_dir": mdir, "batch_max": 8, "batch_target": 2})
    register(ps)
    q = queue.Queue(maxsize=1)
    p = _start(ps, pre, 12, q)
    t0 = time.time()
    while len(p._out_backlog) < 1 and time.time() - t0 < 30:
        time.sleep(0.01)
    assert p._out_backlog

    def boom(self):
        raise RuntimeError("runner bug")

    monkeypatch.setattr(ps.DeviceRunner, "_complete_pending", boom)
    st = p.wait(30)
    assert p._done.is_set(), "wait() timed out behind a dead runner"
    assert st["state"] == "ERROR" and "runner bug" in st["message"] and "undelivered" in st["message"], st


def test_runner_death_while_draining_keeps_state(stubbed, monkeypatch):
    """a pipeline that had already ended (COMPLETED) and was only handing held-back results to a full
    destination keeps its state when the runner thread dies; it reports the undelivered results (the end-of-stream
    marker not counted) and wait() returns."""
    import time

    ps, pre, mdir = stubbed
    ps.PipelineServer.start({"pipeline_dir": PIPES, "model_dir": mdir, "batch_max": 64, "batch_target": 12})
    register(ps)
    q = queue.Queue(maxsize=1)
    p = _start(ps, pre, 12, q, batch=12)  # one tick runs the whole stream, then its end of stream
    t0 = time.time()
    while p.state != "COMPLETED" and time.time() - t0 < 30:
        time.sleep(0.01)
    assert p.state == "COMPLETED" and p._out_backlog and not p._done.is_set()

    def boom(self):
        raise RuntimeError("runner bug")

    monkeypatch.setattr(ps.DeviceRunner, "_drain", boom)
    st = p.wait(30)
    assert p._done.is_set(), "wait() timed out behind a dead runner"
    assert st["state"] == "COMPLETED" and "runner bug" in st["message"] and "undelivered" in st["message"], st
    n = int(st["message"].split("; ")[-1].split()[0])
    assert n == 12 - 1  # twelve results, one of them delivered (the queue holds it); the marker is not a result


@pytest.mark.parametrize("runner", ["device", "threads"])
def test_action_stage_shared_ring_slots(stubbed, runner, monkeypatch):
    """gvaactionrecognitionbin batched across streams (CPU, stubbed pre-processor, ring pages on the host): each launch
    gives every item its own slot (evam_pp_run_slots), each stream's frames go to row * 16 + t % 16 in frame order,
    launches are shared by the streams, a launch ends at the first frame whose window is due, and every frame from a
    stream's 16th on gets its action."""
    ps, pre, _ = stubbed
    monkeypatch.setattr(ps.ClipRing, "_page", lambda self: torch.zeros((self.ROWS * 16, 3, self.H, self.W)))
    mdir = make_model_tree(str(stubbed[2]) + "_ar", {
        "ar": {"enc": (32, 32, None),
               "dec": (32, 32, {"input_preproc": [{"format": "image", "params": {"resize": "aspect-ratio",
                                                                                 "crop": "central"}}],
                                "output_postproc": [{"attribute_name": "action", "method": "softmax",
                                                     "labels": ["a", "b", "c"]}]})}})
    ps.PipelineServer.start({"pipeline_dir": PIPES, "model_dir": mdir, "runner": runner, "batch_max": 64,
                             "batch_wait_ms": 50, "batch_target": 64})
    ps.PipelineServer.register_model("ar/enc", ps.InferenceModel(lambda x: x.mean(dim=(2, 3)), (32, 32)))
    ps.PipelineServer.register_model("ar/dec", ps.InferenceModel(lambda w: w.mean(0, keepdim=True), (32, 32)))
    counts, batches = [20, 17, 33, 16, 5], [1, 2, 3, 4, 1]
    pipes, outs, ins = [], [], []
    for n, b in zip(counts, batches):
        qin, qout = queue.Queue(), queue.Queue()
        for f in frames(pre, n):
            qin.put(f)
        p = ps.PipelineServer.pipeline("action", "general")
        p.start(source={"type": "application", "input": qin}, destination={"metadata": {"output": qout, "mode": "json"}},
                parameters={"ar-properties": {"batch-size": b}})
        pipes.append(p)
        outs.append(qout)
        ins.append(qin)
    deadline = time.time() + 30  # end of stream once every stream holds its ring row: rows are not reused below
    while any(p.stages[0]._row is None for p in pipes) and time.time() < deadline:
        time.sleep(0.005)
    for q in ins:
        q.put(None)
    for p in pipes:
        assert p.wait(30)["state"] == "COMPLETED"
    for call in StubPP.slot_calls:
        assert len(set(call)) == len(call)  # no two items of a launch share a slot
    seq = {}
    for call in StubPP.slot_calls:
        for v in call:
            seq.setdefault(v // 16, []).append(v % 16)
    rows = [p.stages[0].last_row[1] for p in pipes]
    assert len(set(rows)) == len(rows)
    for n, row in zip(counts, rows):
        assert seq[row] == [t % 16 for t in range(n)]
    assert len(StubPP.slot_calls) < sum(counts)
    for n, q in zip(counts, outs):
        res = []
        while (x := q.get(timeout=5)) is not None:
            res.append(json.loads(x))
        assert len(res) == n
        assert all("tensors" not in d for d in res[:15]) and all("tensors" in d for d in res[15:])
