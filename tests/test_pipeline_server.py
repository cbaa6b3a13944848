"""Pipeline-server counterpart and post-proc mapping (f2).

The CPU legs cover:
- template resolution, launch parsing and parameter schema forms (test templates under
  tests/pipelines);
- backend selection;
- the README metadata golden rows;
- optionally, the reference's own templates (only when /root/reference is present, i.e. in the build
  container; never on the GPU box).

The GPU leg runs the end-to-end loop: HIP pre-processing feeds synthetic torch models, and
postproc maps the results to JSON.
"""
import json
import os
import queue
import time

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
PIPES = os.path.join(HERE, "pipelines")
REF_PIPES = "/root/reference/pipelines"

IR_XML = """<?xml version="1.0"?>
<net name="{name}" version="11"><layers>
<layer id="0" name="data" type="Parameter" version="opset1"><data shape="1,3,{h},{w}" element_type="f32"/>
<output><port id="0" precision="FP32"><dim>1</dim><dim>3</dim><dim>{h}</dim><dim>{w}</dim></port></output></layer>
</layers></net>"""


def make_model_tree(root, spec):
    """spec: {alias: {version: (w, h, proc_dict_or_None)}} -> model_dir with FP32/FP16 IR stubs."""
    for alias, vs in spec.items():
        for version, (w, h, proc) in vs.items():
            for prec in ("FP16", "FP32"):
                d = os.path.join(root, alias, version, prec)
                os.makedirs(d, exist_ok=True)
                with open(os.path.join(d, f"{alias}-{version}.xml"), "w") as f:
                    f.write(IR_XML.format(name=alias, w=w, h=h))
            if proc is not None:
                with open(os.path.join(root, alias, version, f"{alias}-{version}.json"), "w") as f:
                    json.dump(proc, f)
    return root


@pytest.fixture
def ps(evam):
    return evam.pipeline_server


@pytest.fixture
def model_dir(tmp_path):
    return make_model_tree(str(tmp_path / "models"), {
        "det_alias": {"det_ver": (64, 64, {"json_schema_version": "2.0.0", "input_preproc": [],
                                           "output_postproc": [{"labels": ["bg", "car", "person"]}]})},
        "cls_alias": {"cls_ver": (24, 24, {"input_preproc": [{"format": "image", "params": {"color_space": "RGB",
                                                                                           "range": [0, 1]}}],
                                           "output_postproc": [{"layer_name": "color", "attribute_name": "color",
                                                                "labels": ["dark", "light"], "method": "max"}]})},
        "ar": {"enc": (32, 32, None),
               "dec": (32, 32, {"input_preproc": [{"format": "image", "params": {"resize": "aspect-ratio",
                                                                                 "crop": "central"}}],
                                "output_postproc": [{"attribute_name": "action", "method": "softmax",
                                                     "labels": ["a", "b", "c"]}]})},
    })


def test_launch_parsing(ps):
    els = ps.parse_launch('appsrc name=source ! decodebin ! videoconvert ! video/x-raw,format=BGRx '
                          '! gvadetect model=/m/a.xml name=detection threshold=0.4 ! appsink name="sink x"')
    assert [e.factory for e in els] == ["appsrc", "decodebin", "videoconvert", "capsfilter", "gvadetect", "appsink"]
    assert els[3].caps == "video/x-raw,format=BGRx"
    assert els[4].properties == {"model": "/m/a.xml", "name": "detection", "threshold": "0.4"}
    assert els[5].name == "sink x"


def test_model_tree_and_ir_shape(ps, model_dir):
    models = ps.scan_models(model_dir)
    e = models["det_alias"]["det_ver"]
    assert e["network"] == e["FP32"] and e["network"].endswith("FP32/det_alias-det_ver.xml")
    assert e["proc"].endswith(".json")
    assert ps.ir_input_size(e["network"]) == (64, 64)
    assert "proc" not in models["ar"]["enc"]


def test_parameter_schema_forms(ps, model_dir, monkeypatch):
    monkeypatch.setenv("EVAM_TEST_DET_DEVICE", "GPU")
    ps.PipelineServer.start({"pipeline_dir": PIPES, "model_dir": model_dir})
    p = ps.PipelineServer.pipeline("detect_classify", "hip")
    p.build({"type": "application"}, {"detection-properties": {"pre-process-backend": "hip", "nireq": 4},
                                      "inference-interval": 3, "detection-threshold": 0.25})
    det, cls = p.element("det"), p.element("cls")
    assert det.properties["pre-process-backend"] == "hip" and det.properties["nireq"] == 4      # passthrough
    assert det.properties["inference-interval"] == 3 and cls.properties["inference-interval"] == 3  # fan-out
    assert det.properties["threshold"] == 0.25                                                   # renamed
    assert det.properties["device"] == "GPU"                                                     # {env[..]} default
    assert cls.properties["object-class"] == "car"                                               # plain default
    assert det.properties["model"].endswith("det_alias/det_ver/FP32/det_alias-det_ver.xml")
    assert det.properties["model-proc"].endswith("det_alias-det_ver.json")                      # auto model-proc
    assert p.elements[0].factory == "appsrc"                                                     # {auto_source}
    assert p.backends() == {"det": "hip", "cls": "hip"}

    monkeypatch.delenv("EVAM_TEST_DET_DEVICE")
    q = ps.PipelineServer.pipeline("detect_classify", "hip").build({"type": "application"}, {})
    assert "device" not in q.element("det").properties       # unset env default leaves the property alone

    z = ps.PipelineServer.pipeline("zone", "count").build({"type": "application"},
                                                          {"zones": [{"name": "A", "polygon": [[0, 0], [1, 1]]}]})
    assert json.loads(z.element("zone").properties["kwarg"]) == [{"name": "A", "polygon": [[0, 0], [1, 1]]}]

    with pytest.raises(ValueError):
        ps.PipelineServer.pipeline("detect_classify", "hip").build({}, {"no-such-param": 1})
    with pytest.raises(ValueError):
        ps.PipelineServer.pipeline("detect_classify", "hip").build({}, {"inference-interval": "3"})
    with pytest.raises(ValueError):
        ps.PipelineServer.pipeline("zone", "count").build({}, {"mode": "other"})
    assert ps.PipelineServer.pipeline("nope", "1") is None
    names = {(d["name"], d["version"]) for d in ps.PipelineServer.pipelines()}
    assert names == {("detect_classify", "hip"), ("detect", "hip"), ("action", "general"), ("zone", "count")}
    ps.PipelineServer.stop()


def test_backend_selection(ps, evam, model_dir):
    ps.PipelineServer.start({"pipeline_dir": PIPES, "model_dir": model_dir})
    for backend in ("opencv", "ie", "vaapi"):
        p = ps.PipelineServer.pipeline("detect_classify", "hip").build(
            {"type": "application"}, {"detection-properties": {"pre-process-backend": backend}})
        with pytest.raises(evam.PreProcError) as ei:
            p.backends()
        assert ei.value.status == evam.native.ERR_UNSUPPORTED
    p = ps.PipelineServer.pipeline("detect_classify", "hip").build({"type": "application"}, {})
    assert p.backends() == {"det": "hip", "cls": "hip"}     # hip is the default in this build
    ps.PipelineServer.stop()


@pytest.mark.skipif(not os.path.isdir(REF_PIPES), reason="reference templates only in the build container")
def test_reference_templates_resolve(ps):
    """Every reference pipeline.json resolves, parses and accepts the hip backend selection."""
    import tempfile

    with tempfile.TemporaryDirectory() as td:
        spec = {}
        for name in os.listdir(REF_PIPES):
            for version in os.listdir(os.path.join(REF_PIPES, name)):
                text = open(os.path.join(REF_PIPES, name, version, "pipeline.json")).read()
                import re

                for a, v in re.findall(r"\{models\[([^\]]+)\]\[([^\]]+)\]", text):
                    spec.setdefault(a, {})[v] = (64, 64, {"input_preproc": []})
        make_model_tree(td, spec)
        ps.PipelineServer.start({"pipeline_dir": REF_PIPES, "model_dir": td})
        defs = ps.PipelineServer.pipelines()
        assert len(defs) >= 10
        n_inference = 0
        for d in defs:
            p = ps.PipelineServer.pipeline(d["name"], d["version"])
            params = {}
            for key, s in d["parameters"].get("properties", {}).items():
                el = s.get("element")
                if isinstance(el, dict) and el.get("format") == "element-properties":
                    params[key] = {"pre-process-backend": "hip"}
            p.build({"type": "uri", "uri": "file:///x.mp4"}, params)
            assert p.elements[0].factory == "urisourcebin"
            b = p.backends()
            n_inference += len(b)
            assert all(v == "hip" for v in b.values())
        assert n_inference >= 10
        ps.PipelineServer.stop()


# ---- post-proc mapping (f2) ---------------------------------------------------------------------
def test_readme_metadata_rows(evam):
    """charts/README.md:117-119 sample rows: pixel rects from normalized boxes, and the exact JSON."""
    P = evam.postproc
    for line in open(os.path.join(HERE, "golden", "readme_metadata.jsonl")):
        ref = json.loads(line)
        W, H = ref["resolution"]["width"], ref["resolution"]["height"]
        fr = P.FrameResult(W, H, timestamp=ref["timestamp"], source=ref["source"])
        for o in ref["objects"]:
            d = o["detection"]
            bb = d["bounding_box"]
            box = (bb["x_min"], bb["y_min"], bb["x_max"], bb["y_max"])
            assert P.roi_rect(box, W, H) == (o["x"], o["y"], o["w"], o["h"])
            t = P.Tensor("detection", d["confidence"], d["label_id"], d["label"], is_detection=True)
            fr.regions.append(P.Region(*P.roi_rect(box, W, H), box, d["label"], d["label_id"], d["confidence"],
                                       tensors=[t]))
        assert P.gvametaconvert_json(fr) == line.strip()
        pm = P.publisher_meta(fr, caps="video/x-raw", img_handle="h")
        assert pm["gva_meta"][0]["tensor"][0] == {"name": "detection", "confidence": d["confidence"],
                                                  "label_id": d["label_id"]}
        assert (pm["width"], pm["height"], pm["channels"]) == (W, H, 3)


def test_transform_mapping_letterbox(evam):
    P = evam.postproc
    # 1920x1080 -> 640x640 top-left letterbox: resized 640x360, scale 1/3
    xf = evam.Transform(640 / 1920, 360 / 1080, 0, 0, 1920, 1080, 0, 0, 640, 360)
    box_t = (0.25, 0.25, 0.5, 0.5)               # tensor-normalized
    bb = P.tensor_box_to_frame(box_t, xf, 1920, 1080, 640, 640)
    assert np.allclose(bb, (0.25, 160 / 360, 0.5, 320 / 360))
    # centred placement: pad_y = 140
    xf = evam.Transform(1 / 3, 1 / 3, 0, 0, 1920, 1080, 0, 140, 640, 360)
    bb = P.tensor_box_to_frame((0.0, 140 / 640, 1.0, 500 / 640), xf, 1920, 1080, 640, 640)
    assert np.allclose(bb, (0.0, 0.0, 1.0, 1.0))
    # identity full-frame resize passes through unchanged (and clipped)
    xf = evam.Transform(512 / 1920, 512 / 1080, 0, 0, 1920, 1080, 0, 0, 512, 512)
    assert P.tensor_box_to_frame((0.1, -0.2, 1.3, 0.7), xf, 1920, 1080, 512, 512) == (0.1, 0.0, 1.0, 0.7)


def test_parse_ssd_and_classify(evam):
    P = evam.postproc
    raw = np.array([[0, 1, 0.9, .1, .1, .2, .2], [0, 2, 0.3, .1, .1, .2, .2], [-1, 0, 0, 0, 0, 0, 0],
                    [0, 1, 0.99, 0, 0, 1, 1]], np.float32)
    d = P.parse_ssd(raw, 0.5)
    assert len(d) == 1 and d[0][1] == 1 and abs(d[0][2] - 0.9) < 1e-6
    t = P.classify(np.array([[1.0, 3.0], [5.0, 2.0]]), ["a", "b"], "softmax", "color")
    assert [x.label for x in t] == ["b", "a"] and abs(t[0].confidence - 1 / (1 + np.exp(-2))) < 1e-12


# ---- end to end on the GPU ---------------------------------------------------------------------
@pytest.mark.gpu
def test_end_to_end_detect_classify(ps, evam, model_dir, gpu, O):
    import torch

    calls = {"det": [], "cls": []}

    def detector(t):
        calls["det"].append(tuple(t.shape))
        n = t.shape[0]
        out = torch.full((n, 3, 7), -1.0)
        out[:, 0] = torch.tensor([0, 1, 0.9, 0.25, 0.25, 0.5, 0.75])     # car
        out[:, 1] = torch.tensor([0, 2, 0.8, 0.0, 0.0, 0.1, 0.1])        # person (not classified)
        return out

    def classifier(t):
        calls["cls"].append(tuple(t.shape))
        m = t.mean(dim=(1, 2, 3))
        return {"color": torch.stack([1 - m, m], 1)}

    ps.PipelineServer.start({"pipeline_dir": PIPES, "model_dir": model_dir})
    ps.PipelineServer.register_model("det_alias/det_ver", ps.InferenceModel(detector, (64, 64), name="det"))
    ps.PipelineServer.register_model("cls_alias/cls_ver", ps.InferenceModel(classifier, (24, 24), name="cls"))
    qin, qout = queue.Queue(), queue.Queue()
    rng = np.random.default_rng(3)
    frames = [O.random_frame(rng, O.NV12, 320, 180) for _ in range(3)]
    for f in frames:
        qin.put({"fourcc": f.fourcc, "width": f.width, "height": f.height, "planes": f.planes})
    qin.put(None)
    p = ps.PipelineServer.pipeline("detect_classify", "hip")
    p.start(source={"type": "application", "input": qin},
            destination={"metadata": {"type": "application", "output": qout, "mode": "json"}},
            parameters={"detection-properties": {"pre-process-backend": "hip"}})
    st = p.wait(60)
    assert st["state"] == "COMPLETED", st
    lines = []
    while True:
        x = qout.get(timeout=5)
        if x is None:
            break
        lines.append(json.loads(x))
    assert len(lines) == 3
    # the device runner coalesces a stream's queued frames (batch-size multiples) into one launch
    assert sum(c[0] for c in calls["det"]) == 3 and all(c[1:] == (3, 64, 64) for c in calls["det"])
    assert sum(c[0] for c in calls["cls"]) == 3 and all(c[1:] == (3, 24, 24) for c in calls["cls"])
    for d in lines:
        car, person = d["objects"]
        assert (car["x"], car["y"], car["w"], car["h"]) == (80, 45, 80, 90)
        assert car["roi_type"] == "car" and "color" in car and "color" not in person
        assert car["color"]["label"] in ("dark", "light")
    ps.PipelineServer.stop()


@pytest.mark.gpu
def test_end_to_end_action_ring(ps, evam, model_dir, gpu, O):
    """gvaactionrecognitionbin: each frame is pre-processed into the stream's clip-ring slot t % 16, the encoder runs
    once per frame (on the frames of each launch) and the decoder on the window of the last 16 embeddings, oldest
    first, from the 16th frame on (the reference element's encoder / decoder split)."""
    import torch

    enc_in, enc_out, dec_in = [], [], []

    def encoder(x):                             # [n, 3, 32, 32] -> [n, 3]
        enc_in.append(x.clone())
        e = x.mean(dim=(2, 3))
        enc_out.append(e.clone())
        return e

    def decoder(window):                        # [16, 3] -> [1, 3]
        dec_in.append(window.clone())
        return window.mean(0, keepdim=True)

    ps.PipelineServer.start({"pipeline_dir": PIPES, "model_dir": model_dir})
    ps.PipelineServer.register_model("ar/enc", ps.InferenceModel(encoder, (32, 32)))
    ps.PipelineServer.register_model("ar/dec", ps.InferenceModel(decoder, (32, 32)))
    rng = np.random.default_rng(5)
    frames = [O.random_frame(rng, O.BGRX, 96, 54) for _ in range(18)]
    src = {"type": "frames", "frames": [{"fourcc": f.fourcc, "width": f.width, "height": f.height,
                                          "planes": f.planes} for f in frames]}
    qout = queue.Queue()
    p = ps.PipelineServer.pipeline("action", "general")
    p.start(source=src, destination={"metadata": {"output": qout, "mode": "json"}})
    assert p.wait(60)["state"] == "COMPLETED"
    out = []
    while (x := qout.get(timeout=5)) is not None:
        out.append(json.loads(x))
    assert len(out) == 18
    assert all("tensors" not in d for d in out[:15]) and all("tensors" in d for d in out[15:])
    # every frame reached the encoder once, in order, aspect+central-cropped 96x54 -> 57x32 -> 32x32, bit-exact
    ref = np.zeros((18, 3, 32, 32), np.float32)
    c = O.COracle()
    for i in range(18):
        c.preprocess_item(frames[i], None, ref, i, mode=2, lut=O.np_norm_lut(0))
    got = torch.cat(enc_in).cpu().numpy()
    assert got.shape == ref.shape and np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    # the decoder saw frames 0..15, 1..16, 2..17 (oldest first)
    emb = torch.cat(enc_out)
    assert len(dec_in) == 3
    for k, w in enumerate(dec_in):
        assert torch.equal(w, emb[k:k + 16])
    # the ring row holds the last 16 frames at slot t % 16
    row = p.stages[0].ring_row().cpu().numpy()
    for t in range(2, 18):
        assert np.array_equal(row[t % 16], ref[t])
    ps.PipelineServer.stop()


@pytest.mark.gpu
@pytest.mark.parametrize("runner", ["device", "threads"])
def test_action_streams_batched_staggered(ps, evam, model_dir, gpu, O, runner):
    """32 action pipelines on one device, at different batch sizes and lengths so their frame counters are out of
    step: every frame of every stream lands bit-exact in its stream's ring slot (checked as the
    encoder reads it, and in the rows' final contents), launches are shared across streams, and every decoder window
    is one stream's last 16 frames in order."""
    import torch

    S = 32
    enc_in, enc_out, dec_in = [], [], []

    def encoder(x):
        enc_in.append(x.clone())
        e = x.flatten(1).double().sum(1, keepdim=True).float()  # [n, 1] per-frame signature
        e = torch.cat([e, x[:, :, 0, :4].flatten(1)], 1)          # plus raw pixels: unique per frame
        enc_out.append(e.clone())
        return e

    def decoder(window):
        dec_in.append(window.clone())
        return torch.zeros((1, 3), device=window.device)

    ps.PipelineServer.start({"pipeline_dir": PIPES, "model_dir": model_dir, "runner": runner, "batch_max": 256})
    ps.PipelineServer.register_model("ar/enc", ps.InferenceModel(encoder, (32, 32)))
    ps.PipelineServer.register_model("ar/dec", ps.InferenceModel(decoder, (32, 32)))
    rng = np.random.default_rng(77)
    W, H = 160, 90
    n_frames = [18 + (7 * s) % 13 for s in range(S)]
    batches = [1 + s % 4 for s in range(S)]
    frames = [[O.random_frame(rng, O.NV12, W, H) for _ in range(n_frames[s])] for s in range(S)]
    c = O.COracle()
    ref = {}
    for s in range(S):
        r = np.zeros((n_frames[s], 3, 32, 32), np.float32)
        for t, f in enumerate(frames[s]):
            c.preprocess_item(f, None, r, t, mode=2, lut=O.np_norm_lut(0))
        ref[s] = r
    by_bytes = {ref[s][t].tobytes(): (s, t) for s in range(S) for t in range(n_frames[s])}
    assert len(by_bytes) == sum(n_frames)
    qs, pipes = [], []
    for s in range(S):
        q = queue.Queue()
        p = ps.PipelineServer.pipeline("action", "general")
        p.start(source={"type": "application", "input": q}, destination={},
                parameters={"ar-properties": {"batch-size": batches[s]}})
        qs.append(q)
        pipes.append(p)
    for s in range(S):
        for f in frames[s]:
            qs[s].put(evam.Image.from_host(f.fourcc, f.width, f.height, f.planes, device="cuda:0"))
    # end of stream only once every stream holds its ring row (an ended stream's row goes back to the free list),
    # so every row's final contents below belong to its own stream
    deadline = time.time() + 60
    while any(p.stages[0]._row is None for p in pipes) and time.time() < deadline:
        time.sleep(0.01)
    for q in qs:
        q.put(None)
    for p in pipes:
        assert p.wait(120)["state"] == "COMPLETED"
    # every written slot, as the encoder read it: each (stream, frame) exactly once, bit-exact, in stream order
    got = torch.cat(enc_in).cpu().numpy()
    ids = [by_bytes.get(g.tobytes()) for g in got]
    assert None not in ids, "a pre-processed frame matches no oracle frame"
    assert sorted(ids) == sorted((s, t) for s in range(S) for t in range(n_frames[s]))
    for s in range(S):
        assert [t for s2, t in ids if s2 == s] == list(range(n_frames[s]))
    assert len(enc_in) < sum(n_frames) / 2  # launches are shared across streams
    # every decoder window: one stream's frames c-16 .. c-1, oldest first
    emb = torch.cat(enc_out).cpu().numpy()
    row_of = {emb[i].tobytes(): ids[i] for i in range(len(ids))}
    wins = {s: [] for s in range(S)}
    for w in dec_in:
        ws = [row_of[r.tobytes()] for r in w.cpu().numpy()]
        s = ws[0][0]
        assert all(x[0] == s for x in ws) and [x[1] for x in ws] == list(range(ws[0][1], ws[0][1] + 16))
        wins[s].append(ws[-1][1])
    for s in range(S):
        assert wins[s] == list(range(15, n_frames[s]))
    # the rows' final contents: slot t % 16 holds frame t for the last 16 frames of every stream
    rows = set()
    for s, p in enumerate(pipes):
        st = p.stages[0]
        rows.add(st.last_row)
        row = st.ring_row().cpu().numpy()
        for t in range(n_frames[s] - 16, n_frames[s]):
            assert np.array_equal(row[t % 16].view(np.uint32), ref[s][t].view(np.uint32)), (s, t)
    assert len(rows) == S
    ps.PipelineServer.stop()


@pytest.mark.gpu
def test_runner_inflight_on_gpu_streams(ps, evam, model_dir, gpu, O):
    """Two ticks in flight on real HIP streams (the device runner's default): a detector that reads the
    pre-processed tensor on the GPU (per-frame mean -> confidence) gives every stream the same results, in the same
    order, as one tick at a time, and the per-frame means equal the oracle's pre-processing of that frame."""
    import torch

    rng = np.random.default_rng(23)
    frames = [O.random_frame(rng, O.NV12, 320, 180) for _ in range(3 * 7)]
    c = O.COracle()
    ref = np.zeros((len(frames), 3, 64, 64), np.float32)
    for i, f in enumerate(frames):
        c.preprocess_item(f, None, ref, i, lut=O.np_norm_lut(0))

    def detector(t):  # stays on the device until the runner copies the output back
        n = t.shape[0]
        out = torch.full((n, 1, 7), -1.0, device=t.device)
        out[:, 0, 0] = 0
        out[:, 0, 1] = 1
        out[:, 0, 2] = 0.6 + t.float().mean(dim=(1, 2, 3)) / 1000.0
        out[:, 0, 3:] = torch.tensor([0.25, 0.25, 0.5, 0.75], device=t.device)
        return out

    def run(inflight):
        ps.PipelineServer.start({"pipeline_dir": PIPES, "model_dir": model_dir, "inflight": inflight,
                                 "batch_target": 4, "batch_max": 4, "batch_wait_ms": 50})
        ps.PipelineServer.register_model("det_alias/det_ver", ps.InferenceModel(detector, (64, 64), name="det"))
        pipes, outs = [], []
        for k in range(3):
            qin, qout = queue.Queue(), queue.Queue()
            for f in frames[k::3]:
                qin.put({"fourcc": f.fourcc, "width": f.width, "height": f.height, "planes": f.planes})
            qin.put(None)
            p = ps.PipelineServer.pipeline("detect", "hip")
            p.start(source={"type": "application", "input": qin},
                    destination={"metadata": {"type": "application", "output": qout, "mode": "json"}},
                    parameters={"detection-properties": {"batch-size": 1}})
            pipes.append(p)
            outs.append(qout)
        for p in pipes:
            assert p.wait(120)["state"] == "COMPLETED"
        got = []
        for q in outs:
            rows = []
            while (x := q.get(timeout=5)) is not None:
                rows.append(json.loads(x))
            got.append(rows)
        ps.PipelineServer.stop()
        return got

    one, two = run(1), run(2)
    assert one == two and [len(g) for g in two] == [7, 7, 7]
    for k, rows in enumerate(two):
        for j, d in enumerate(rows):
            conf = d["objects"][0]["detection"]["confidence"]
            assert abs(conf - (0.6 + float(ref[k + 3 * j].mean()) / 1000.0)) < 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("runner", ["device", "threads"])
def test_hub_batches_across_pipelines(ps, evam, model_dir, gpu, O, runner):
    """Four application-source pipelines on one device: the batching hub runs ONE detection launch over the
    four streams' frames and ONE ROI launch over their vehicles per tick (the reference runs one pipeline
    per stream, evas/manager.py:127-141, and never batches across them), and every classifier input row is
    bit-exact with the oracle's pre-processing of that stream's ROI."""
    import torch

    calls, cls_inputs = [], []

    def detector(t):
        calls.append(("det", tuple(t.shape)))
        n = t.shape[0]
        out = torch.full((n, 3, 7), -1.0)
        out[:, 0] = torch.tensor([0, 1, 0.9, 0.25, 0.25, 0.5, 0.75])     # car
        out[:, 1] = torch.tensor([0, 2, 0.8, 0.0, 0.0, 0.1, 0.1])        # person (not classified)
        return out

    def classifier(t):
        calls.append(("cls", tuple(t.shape)))
        cls_inputs.append(t.detach().cpu().numpy().copy())
        m = t.mean(dim=(1, 2, 3))
        return {"color": torch.stack([1 - m, m], 1)}

    ps.PipelineServer.start({"pipeline_dir": PIPES, "model_dir": model_dir, "batch_target": 4,
                             "batch_wait_ms": 20000, "runner": runner})
    ps.PipelineServer.register_model("det_alias/det_ver", ps.InferenceModel(detector, (64, 64), name="det"))
    ps.PipelineServer.register_model("cls_alias/cls_ver", ps.InferenceModel(classifier, (24, 24), name="cls"))
    rng = np.random.default_rng(17)
    frames = [O.random_frame(rng, O.NV12, 320, 180) for _ in range(4)]
    pipes, outs = [], []
    for f in frames:
        qin, qout = queue.Queue(), queue.Queue()
        qin.put({"fourcc": f.fourcc, "width": f.width, "height": f.height, "planes": f.planes})
        qin.put(None)
        p = ps.PipelineServer.pipeline("detect_classify", "hip")
        p.start(source={"type": "application", "input": qin},
                destination={"metadata": {"type": "application", "output": qout, "mode": "json"}})
        pipes.append(p)
        outs.append(qout)
    for p in pipes:
        st = p.wait(120)
        assert st["state"] == "COMPLETED", st
    assert calls.count(("det", (4, 3, 64, 64))) == 1 and calls.count(("cls", (4, 3, 24, 24))) == 1, calls
    assert len(calls) == 2
    hub_batches = ps.PipelineServer.hub().batches
    assert sorted(b[1:] for b in hub_batches) == [(4, 4), (4, 4)]     # (units, requests) per launch
    # every classifier row is one stream's car ROI, pre-processed exactly as the oracle does
    info = ps.InferenceModel(None, (24, 24), json.load(open(os.path.join(
        model_dir, "cls_alias", "cls_ver", "cls_alias-cls_ver.json")))).preproc_info()
    c = O.COracle()
    ref = np.zeros((4, 3, 24, 24), np.float32)
    lut = O.np_norm_lut(1, info.range)
    for i, f in enumerate(frames):
        c.preprocess_item(f, (80, 45, 80, 90), ref, i, color_rgb=True, lut=lut)
    got = cls_inputs[0]
    matched = sorted(next(j for j in range(4) if np.array_equal(got[k], ref[j])) for k in range(4))
    assert matched == [0, 1, 2, 3]
    for q in outs:
        d = json.loads(q.get(timeout=5))
        car = d["objects"][0]
        assert (car["x"], car["y"], car["w"], car["h"]) == (80, 45, 80, 90) and "color" in car
    ps.PipelineServer.stop()


@pytest.mark.gpu
def test_streams_partitioned_over_devices(ps, evam, model_dir, gpu, O):
    """Option ``devices``: pipeline k runs on devices[(k - 1) mod G] (the reference starts one
    pipeline per source, evas/manager.py:129-141). Two logical devices on the one GPU of the box: pipelines
    1, 3 batch through hub 0 and 2, 4 through hub 1, each hub with its own pre-processing handle and stream,
    and every classifier input row is bit-exact with the oracle (so with a one-device run)."""
    import torch

    cls_inputs = []

    def detector(t):
        n = t.shape[0]
        out = torch.full((n, 3, 7), -1.0)
        out[:, 0] = torch.tensor([0, 1, 0.9, 0.25, 0.25, 0.5, 0.75])     # car
        return out

    def classifier(t):
        cls_inputs.append(t.detach().cpu().numpy().copy())
        m = t.mean(dim=(1, 2, 3))
        return {"color": torch.stack([1 - m, m], 1)}

    ps.PipelineServer.start({"pipeline_dir": PIPES, "model_dir": model_dir, "devices": [0, 0], "batch_target": 2,
                             "batch_wait_ms": 20000})
    assert ps.PipelineServer.devices() == [0, 0]
    ps.PipelineServer.register_model("det_alias/det_ver", ps.InferenceModel(detector, (64, 64), name="det"))
    ps.PipelineServer.register_model("cls_alias/cls_ver", ps.InferenceModel(classifier, (24, 24), name="cls"))
    rng = np.random.default_rng(29)
    frames = [O.random_frame(rng, O.NV12, 320, 180) for _ in range(4)]
    pipes = []
    for f in frames:
        qin = queue.Queue()
        qin.put({"fourcc": f.fourcc, "width": f.width, "height": f.height, "planes": f.planes})
        qin.put(None)
        p = ps.PipelineServer.pipeline("detect_classify", "hip")
        p.start(source={"type": "application", "input": qin},
                destination={"metadata": {"type": "application", "output": queue.Queue(), "mode": "json"}})
        pipes.append(p)
    assert [p.slot for p in pipes] == [0, 1, 0, 1] and [p.device for p in pipes] == [0, 0, 0, 0]
    for p in pipes:
        st = p.wait(120)
        assert st["state"] == "COMPLETED", st
    h0, h1 = ps.PipelineServer.hub(0), ps.PipelineServer.hub(1)
    assert h0 is not h1
    # each hub served its two streams: one 2-frame detection launch and one 2-ROI classification launch
    assert sorted(b[1:] for b in h0.batches) == [(2, 2), (2, 2)]
    assert sorted(b[1:] for b in h1.batches) == [(2, 2), (2, 2)]
    info = ps.InferenceModel(None, (24, 24), json.load(open(os.path.join(
        model_dir, "cls_alias", "cls_ver", "cls_alias-cls_ver.json")))).preproc_info()
    c = O.COracle()
    ref = np.zeros((4, 3, 24, 24), np.float32)
    for i, f in enumerate(frames):
        c.preprocess_item(f, (80, 45, 80, 90), ref, i, color_rgb=True, lut=O.np_norm_lut(1, info.range))
    rows = [r for t in cls_inputs for r in t]
    assert len(rows) == 4
    matched = sorted(next(j for j in range(4) if np.array_equal(r, ref[j])) for r in rows)
    assert matched == [0, 1, 2, 3]
    ps.PipelineServer.stop()


@pytest.mark.parametrize("per_call", [1, 7, 4])
def test_classify_reclassify_interval(ps, evam, per_call):
    """gvaclassify reclassify-interval (pipelines/object_classification/vehicle_attributes/pipeline.json:68-71):
    a tracked region (object_id != 0) is sent for classification only every N-th frame of its stream and gets
    its last results attached in between; untracked regions are classified every frame; degenerate boxes are
    never sent (the C ABI would read w/h <= 0 as the full frame). per_call: frames handed to one prepare()
    (the device runner passes a stream's whole batch): frames of one call that fall inside the interval of
    an earlier frame of the same call take that frame's results."""
    P = evam.postproc

    class FakeHub:
        def __init__(self):
            self.sent = []

        def submit(self, stage, items, units):
            for fi, img, todo in items:
                for r in todo:
                    self.sent.append((fi, r.object_id))
                    r.tensors.append(P.Tensor("color", 0.9, 1, "light", model="cls"))

    hub = FakeHub()

    class FakeServer:
        device = 0

        def model_for(self, net, device=None):
            return ps.InferenceModel(None, (24, 24), {"input_preproc": []}, name="cls")

        def hub(self, slot=0):
            return hub

    el = ps.Element("gvaclassify", {"model": "m.xml", "reclassify-interval": "3", "object-class": "car"})
    st = ps.ClassifyStage(el, FakeServer(), 0)

    class Img:
        width, height = 320, 180

    def region(oid, x=10, w=40, label="car"):
        return P.Region(x, 10, w, 30, (0, 0, 0.1, 0.1), label, 1, 0.9, object_id=oid)

    results, call = [], []
    for fi in range(7):
        fr = P.FrameResult(320, 180, regions=[region(5), region(0), region(6, label="person"), region(7, x=400),
                                             region(8, w=0)])
        call.append((fi, Img(), fr))
        results.append(fr)
        if len(call) == per_call or fi == 6:
            st.process(call)
            call = []
    tracked = [fi for fi, oid in hub.sent if oid == 5]
    untracked = [fi for fi, oid in hub.sent if oid == 0]
    assert tracked == [0, 3, 6] and untracked == list(range(7))
    assert {oid for _, oid in hub.sent} == {0, 5}                   # person, off-frame, zero-width: never sent
    for fr in results:
        assert len(fr.regions[0].tensors) == 1 and fr.regions[0].tensors[0].label == "light"
        assert fr.regions[2].tensors == [] and fr.regions[3].tensors == [] and fr.regions[4].tensors == []


def test_parse_ssd_batch_matches_per_item(evam):
    """The vectorised batch parse equals parse_ssd item by item (terminator, threshold, empty items)."""
    P = evam.postproc
    rng = np.random.default_rng(4)
    raw = rng.uniform(0, 1, size=(9, 6, 7)).astype(np.float32)
    raw[:, :, 0] = 0
    raw[1, 2, 0] = -1          # terminator mid-way
    raw[3, 0, 0] = -1          # empty item
    raw[5, :, 2] = 0.1         # all below threshold
    got = P.parse_ssd_batch(raw, 0.5)
    assert got == [P.parse_ssd(raw[i], 0.5) for i in range(9)]
    assert got[3] == [] and got[5] == []


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(3))
@pytest.mark.parametrize("runner", ["device", "threads"])
def test_end_to_end_random_detections_bit_exact(ps, evam, model_dir, gpu, O, coracle, runner, seed):
    """detect -> classify with random detections: every tensor the two models receive is checked bit for bit against
    the oracle. The detector's input is each full frame (64x64, BGR, no normalisation); the classifier's rows are the
    crops of the `car` detections, as the JSON reports them (x, y, w, h after the box mapping), in frame and object
    order (24x24, RGB, range [0, 1])."""
    import torch

    rng = np.random.default_rng(17 + 2 * seed + (runner == "threads"))
    n_frames, W, H = 24, 352, 198
    frames = [O.random_frame(rng, O.NV12, W, H, pattern="gradient" if k % 3 == 0 else "uniform")
              for k in range(n_frames)]
    boxes = []  # per frame: [label, conf, x0, y0, x1, y1] rows (normalised)
    for _ in range(n_frames):
        rows = []
        for _ in range(int(rng.integers(0, 9))):
            x0, y0 = rng.uniform(-0.1, 0.9, 2)
            x1, y1 = x0 + rng.uniform(0.01, 0.6), y0 + rng.uniform(0.01, 0.6)
            rows.append([float(rng.integers(1, 3)), 0.9, x0, y0, x1, y1])
        boxes.append(rows)
    det_in, cls_in = [], []
    seen = [0]

    def detector(t):
        det_in.append(t.detach().float().cpu().numpy().copy())
        n = t.shape[0]
        out = torch.full((n, 10, 7), -1.0)
        for i in range(n):
            for j, r in enumerate(boxes[seen[0] + i]):
                out[i, j] = torch.tensor([0.0] + r)
        seen[0] += n
        return out

    def classifier(t):
        cls_in.append(t.detach().float().cpu().numpy().copy())
        m = t.mean(dim=(1, 2, 3))
        return {"color": torch.stack([1 - m, m], 1)}

    ps.PipelineServer.start({"pipeline_dir": PIPES, "model_dir": model_dir, "runner": runner})
    try:
        ps.PipelineServer.register_model("det_alias/det_ver", ps.InferenceModel(detector, (64, 64), name="det"))
        ps.PipelineServer.register_model("cls_alias/cls_ver", ps.InferenceModel(classifier, (24, 24), name="cls"))
        qin, qout = queue.Queue(), queue.Queue()
        for f in frames:
            qin.put({"fourcc": f.fourcc, "width": f.width, "height": f.height, "planes": f.planes})
        qin.put(None)
        p = ps.PipelineServer.pipeline("detect_classify", "hip")
        p.start(source={"type": "application", "input": qin},
                destination={"metadata": {"type": "application", "output": qout, "mode": "json"}},
                parameters={"detection-properties": {"pre-process-backend": "hip"}})
        st = p.wait(60)
        assert st["state"] == "COMPLETED", st
        lines = []
        while True:
            x = qout.get(timeout=5)
            if x is None:
                break
            lines.append(json.loads(x))
    finally:
        ps.PipelineServer.stop()
    assert len(lines) == n_frames
    # detector input: every frame, in order
    got = np.concatenate(det_in)
    assert got.shape == (n_frames, 3, 64, 64)
    ref = np.zeros(got.shape, np.float32)
    lut0 = O.np_norm_lut(0)
    for i, f in enumerate(frames):
        coracle.preprocess_item(f, None, ref, i, lut=lut0)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), "detector input"
    # classifier input: the car crops the JSON reports, frame by frame
    crops = [(k, o["x"], o["y"], o["w"], o["h"]) for k, d in enumerate(lines) for o in d.get("objects", [])
             if "color" in o]
    n_car = sum(1 for rows in boxes for r in rows if r[0] == 1.0)
    assert crops and len(crops) <= n_car
    got = np.concatenate(cls_in) if cls_in else np.zeros((0, 3, 24, 24), np.float32)
    assert got.shape == (len(crops), 3, 24, 24)
    ref = np.zeros(got.shape, np.float32)
    lut1 = O.np_norm_lut(1, (0.0, 1.0))
    for i, (k, x, y, w, h) in enumerate(crops):
        coracle.preprocess_item(frames[k], (x, y, w, h), ref, i, color_rgb=True, lut=lut1)
    bad = [i for i in range(len(crops)) if not np.array_equal(got[i].view(np.uint32), ref[i].view(np.uint32))]
    assert not bad, f"classifier rows differ: {[(i, crops[i]) for i in bad[:5]]}"


def _fingerprint(row):
    """24-bit fingerprint of one model-input row (exact as a float32)."""
    import zlib

    return zlib.crc32(np.ascontiguousarray(row, dtype=np.float32).tobytes()) & 0xFFFFFF


def _box_of(fp):
    """A car box derived from a detector-input fingerprint (dyadic, so exact in float32)."""
    x0, y0 = (fp & 0xFF) / 512.0, ((fp >> 8) & 0xFF) / 512.0
    return x0, y0, x0 + 0.25 + ((fp >> 16) & 0x3F) / 256.0, y0 + 0.25


@pytest.mark.gpu
@pytest.mark.parametrize("runner,inflight", [("device", 3), ("device", 1), ("device", 4), ("threads", 1)])
def test_pipeline_soak_fingerprints(ps, evam, model_dir, gpu, O, coracle, runner, inflight):
    """Many detect -> classify streams at once (EVAM_SOAK_STREAMS x EVAM_SOAK_FRAMES, default 4 x 24), each stream its
    own frame size, batched across streams by the hub with 1, 3 (the default) or 4 ticks in flight. The detector answers each input row with a
    car box derived from a fingerprint of that row; the classifier answers with a fingerprint of its crop as the
    confidence. Every frame's JSON box must be the one its oracle detector input implies, and every crop's confidence
    the fingerprint of the oracle crop of the JSON rect: a frame or crop from another stream, slot or tick fails."""
    import torch

    S = int(os.environ.get("EVAM_SOAK_STREAMS", "4"))
    F = int(os.environ.get("EVAM_SOAK_FRAMES", "24"))
    rng = np.random.default_rng(31 + inflight + (runner == "threads"))
    sizes = [(2 * int(rng.integers(60, 400)), 2 * int(rng.integers(40, 250))) for _ in range(S)]
    frames = [[O.random_frame(rng, O.NV12, *sizes[s]) for _ in range(F)] for s in range(S)]

    def detector(t):
        a = t.detach().float().cpu().numpy()
        out = torch.full((a.shape[0], 2, 7), -1.0)
        for i in range(a.shape[0]):
            out[i, 0] = torch.tensor([0.0, 1.0, 0.9, *_box_of(_fingerprint(a[i]))])
        return out

    def classifier(t):
        a = t.detach().float().cpu().numpy()
        return {"color": torch.tensor([[float(_fingerprint(a[i])), -1.0] for i in range(a.shape[0])])}

    ps.PipelineServer.start({"pipeline_dir": PIPES, "model_dir": model_dir, "runner": runner, "inflight": inflight})
    outs = []
    try:
        ps.PipelineServer.register_model("det_alias/det_ver", ps.InferenceModel(detector, (64, 64), name="det"))
        ps.PipelineServer.register_model("cls_alias/cls_ver", ps.InferenceModel(classifier, (24, 24), name="cls"))
        pipes = []
        for s in range(S):
            qin, qout = queue.Queue(), queue.Queue()
            for f in frames[s]:
                qin.put({"fourcc": f.fourcc, "width": f.width, "height": f.height, "planes": f.planes})
            qin.put(None)
            p = ps.PipelineServer.pipeline("detect_classify", "hip")
            p.start(source={"type": "application", "input": qin},
                    destination={"metadata": {"type": "application", "output": qout, "mode": "json"}},
                    parameters={"detection-properties": {"pre-process-backend": "hip"}})
            pipes.append(p)
            outs.append(qout)
        for p in pipes:
            st = p.wait(120)
            assert st["state"] == "COMPLETED", st
    finally:
        ps.PipelineServer.stop()
    lut0, lut1 = O.np_norm_lut(0), O.np_norm_lut(1, (0.0, 1.0))
    n_crops = 0
    for s in range(S):
        lines = []
        while True:
            x = outs[s].get(timeout=5)
            if x is None:
                break
            lines.append(json.loads(x))
        assert len(lines) == F, (s, len(lines))
        for k, d in enumerate(lines):
            f = frames[s][k]
            det = np.zeros((1, 3, 64, 64), np.float32)
            coracle.preprocess_item(f, None, det, 0, lut=lut0)
            want = _box_of(_fingerprint(det[0]))
            (obj,) = d["objects"]
            bb = obj["detection"]["bounding_box"]
            got = (bb["x_min"], bb["y_min"], bb["x_max"], bb["y_max"])
            assert np.allclose(got, want, rtol=0, atol=1e-6), f"stream {s} frame {k}: detector input differs"
            if "color" not in obj:
                continue
            crop = np.zeros((1, 3, 24, 24), np.float32)
            coracle.preprocess_item(f, (obj["x"], obj["y"], obj["w"], obj["h"]), crop, 0, color_rgb=True, lut=lut1)
            assert obj["color"]["confidence"] == float(_fingerprint(crop[0])), f"stream {s} frame {k}: crop differs"
            n_crops += 1
    assert n_crops > S * F // 2
