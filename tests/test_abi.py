"""CPU tests of the C ABI boundary: the library loads, exports every symbol include/evam_pp.h declares,
struct layouts match the header, and the host-side error paths behave (no GPU compute calls)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "evam_pp.h")


def header_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char\*)\s+(evam_pp_\w+)\s*\(", src, re.M)))


def test_library_exports_every_declared_symbol(evam):
    lib = evam.load_library()
    declared = header_functions()
    assert declared, "no functions parsed from the header"
    assert set(declared) == set(evam.native.EXPORTED_SYMBOLS)
    for name in declared:
        assert hasattr(lib, name), f"{name} not exported"
    assert lib.evam_pp_abi_version() == evam.native.ABI_VERSION


def test_struct_sizes_match_header(evam):
    for cls, size in evam.native.STRUCT_SIZES.items():
        assert ctypes.sizeof(cls) == size, cls.__name__


def test_header_enums_match_python(evam):
    src = open(HEADER).read()
    vals = {k: int(v, 0) for k, v in re.findall(r"(EVAM_\w+)\s*=\s*(-?0x[0-9A-Fa-f]+|-?\d+)", src)}
    N = evam.native
    assert vals["EVAM_FOURCC_NV12"] == N.FOURCC_NV12 and vals["EVAM_FOURCC_I420"] == N.FOURCC_I420
    assert vals["EVAM_FOURCC_BGRX"] == N.FOURCC_BGRX and vals["EVAM_FOURCC_BGR"] == N.FOURCC_BGR
    assert vals["EVAM_PP_ERR_EMPTY_ROI"] == N.ERR_EMPTY_ROI and vals["EVAM_PP_ERR_ALIGNMENT"] == N.ERR_ALIGNMENT
    assert vals["EVAM_RESIZE_ASPECT_CROP"] == N.RESIZE_ASPECT_CROP
    # FourCC = a | b<<8 | c<<16 | d<<24 of the DL Streamer names
    for name, v in (("NV12", N.FOURCC_NV12), ("I420", N.FOURCC_I420), ("BGRX", N.FOURCC_BGRX)):
        assert v == int.from_bytes(name.encode(), "little")


def test_null_arguments_rejected(evam):
    lib = evam.load_library()
    assert lib.evam_pp_run(None, None, 0, None, 0, None, None, None) == evam.native.ERR_INVALID_ARG
    assert b"NULL" in lib.evam_pp_last_error()
    assert lib.evam_pp_run_slots(None, None, 0, None, 0, None, None, None, None) == evam.native.ERR_INVALID_ARG
    assert b"slots is NULL" in lib.evam_pp_last_error()
    assert lib.evam_pp_sync(None) == evam.native.ERR_INVALID_ARG
    assert lib.evam_pp_create(0, None, None) == evam.native.ERR_INVALID_ARG
    lib.evam_pp_destroy(None)  # no-op


def test_create_without_gpu_reports_no_device(evam):
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    lib = evam.load_library()
    h = ctypes.c_void_p()
    assert lib.evam_pp_create(0, None, ctypes.byref(h)) == evam.native.ERR_NO_DEVICE
    with pytest.raises(evam.PreProcError):
        evam.HipPreProcessor(device=0)


def test_model_proc_mapping(evam):
    """In-tree model-procs: vehicle-detection-0202 (input_preproc [] -> defaults) and
    action-recognition-0001 (BGR, resize aspect-ratio, crop central), restated inline
    (models_list/vehicle-detection-0202.json:3, models_list/action-recognition-0001.json:3-13)."""
    N = evam.native
    d = evam.PreProcInfo.from_model_proc(None)
    c = d.to_c(N.DTYPE_U8)
    assert (c.resize_mode, c.color_order, c.norm_flags) == (N.RESIZE_NO_ASPECT, N.COLOR_BGR, 0)
    a = evam.PreProcInfo.from_model_proc({"format": "image", "layer_name": "0",
                                          "params": {"color_space": "BGR", "resize": "aspect-ratio",
                                                     "crop": "central"}})
    assert a.to_c(N.DTYPE_F32).resize_mode == N.RESIZE_ASPECT_CROP
    n = evam.PreProcInfo.from_model_proc({"params": {"range": [0, 1], "mean": [0.1, 0.2, 0.3], "std": [1, 2, 3],
                                                     "color_space": "RGB"}})
    c = n.to_c(N.DTYPE_F32)
    assert c.norm_flags == 3 and c.color_order == N.COLOR_RGB and list(c.std) == [1.0, 2.0, 3.0]
    with pytest.raises(evam.PreProcError):
        evam.PreProcInfo(resize="aspect-ratio", crop="top_left").to_c(N.DTYPE_U8)
    with pytest.raises(evam.PreProcError):
        evam.PreProcInfo(color_space="GRAYSCALE").to_c(N.DTYPE_U8)


def test_backend_selection(evam):
    with pytest.raises(evam.PreProcError):
        evam.create_preprocessor("opencv")
    with pytest.raises(evam.PreProcError):
        evam.create_preprocessor("nonsense")


def test_transform_inverse(evam):
    t = evam.Transform(scale_x=640 / 3840, scale_y=360 / 2160, crop_x=0, crop_y=0, crop_w=3840, crop_h=2160,
                       pad_x=0, pad_y=140, resized_w=640, resized_h=360)
    x, y = t.tensor_to_source(320, 320)
    assert abs(x - 1920) < 1e-6 and abs(y - 1080) < 1e-6


def test_variant_library_override_is_confined(evam, monkeypatch, tmp_path):
    """EVAM_PP_LIB (A/B runs) loads only a tools/build_variant.sh build from <repo>/ab/; a stray setting
    pointing anywhere else is refused instead of silently replacing the product library."""
    from importlib import import_module

    native = import_module(evam.__name__ + "._native")
    stray = tmp_path / "libevam_pp_x.so"
    stray.write_bytes(b"")
    monkeypatch.setattr(native, "_LIB", None)
    monkeypatch.setenv("EVAM_PP_LIB", str(stray))
    with pytest.raises(RuntimeError, match="only variant builds"):
        native.load_library()
    monkeypatch.delenv("EVAM_PP_LIB")
    assert native.load_library() is not None


def test_library_has_no_undefined_kernel_symbols():
    """Every kernel the host code launches has its host-side stub in the library: a kernel whose stub clang did not
    emit loads lazily on CPU but fails at dlopen on the GPU box (round 5: a local struct inside a kernel template)."""
    import shutil
    import subprocess

    if shutil.which("nm") is None:
        pytest.skip("needs nm")
    lib = os.path.join(ROOT, "edge-video-analytics-microservice_amd", "libevam_pp.so")
    out = subprocess.run(["nm", "-D", "--undefined-only", lib], capture_output=True, text=True, check=True).stdout
    bad = [ln.split()[-1] for ln in out.splitlines() if "evam" in ln]
    assert not bad, bad


def test_convert_host_caches_follow_changes(evam):
    """HipPreProcessor.convert's per-call caches (no GPU: a recording stand-in for evam_pp_run, and the device check
    of the output tensor skipped): the evam_tensor of an output tensor is reused only while the tensor object, its
    version and storage are unchanged (resize_ re-validates), each of several output tensors keeps its own, and the
    C config follows every change of the PreProcInfo, in-place list edits included."""
    import torch

    native = evam.native
    P = evam.HipPreProcessor
    calls = []

    class Rec(P):
        def _tensor_entry(self, out):  # as the product's, minus the cuda-device check (CPU tensors here)
            t = native.EvamTensor()
            t.data = out.data_ptr()
            t.n, t.c, t.h, t.w = (int(v) for v in out.shape)
            dt = native.DTYPE_F32
            import weakref

            e = (weakref.ref(out), out._version, t.data, t, dt, ctypes.byref(t))
            self._tdesc[id(out)] = e
            return e

    def fake_run(h, arr, n_srcs, items, n_items, cfg, tref, xf):
        c, t = cfg._obj, tref._obj
        calls.append({"n": t.n, "data": t.data, "off": t.slot_offset, "stride": t.slot_stride,
                      "mean": tuple(c.mean), "t": id(t)})
        return 0

    pp = Rec.__new__(Rec)
    pp._torch, pp.device, pp._h = torch, 0, None
    pp._tdesc, pp._cfg_cache, pp._last_cfg = {}, {}, None
    pp._default_info = evam.PreProcInfo()
    pp._run, pp._bind_stream = fake_run, lambda: None
    batch = evam.ImageBatch.__new__(evam.ImageBatch)
    batch.images, batch.c_array = [None], (native.EvamImage * 1)()

    a, b = torch.empty(4, 3, 8, 8), torch.empty(6, 3, 8, 8)
    info = evam.PreProcInfo(mean=(1.0, 2.0, 3.0), std=(1.0, 1.0, 1.0))
    pp.convert(batch, a, info)
    pp.convert(batch, a, info, slot_offset=2)
    assert calls[-1]["t"] == calls[-2]["t"] and calls[-1]["off"] == 2 and calls[-1]["n"] == 4
    pp.convert(batch, b, info)
    pp.convert(batch, a, info)
    assert (calls[-2]["n"], calls[-1]["n"]) == (6, 4) and calls[-1]["data"] == a.data_ptr()
    a.resize_(2, 3, 8, 8)
    pp.convert(batch, a, info)
    assert calls[-1]["n"] == 2
    info.mean = (4.0, 5.0, 6.0)
    pp.convert(batch, a, info)
    assert calls[-1]["mean"] == (4.0, 5.0, 6.0)
    info.mean = [7.0, 8.0, 9.0]
    pp.convert(batch, a, info)
    info.mean[0] = 10.0
    pp.convert(batch, a, info)
    assert calls[-2]["mean"] == (7.0, 8.0, 9.0) and calls[-1]["mean"] == (10.0, 8.0, 9.0)
    other = evam.PreProcInfo(mean=(10.0, 8.0, 9.0), std=(1.0, 1.0, 1.0))
    pp.convert(batch, a, other)
    assert calls[-1]["mean"] == (10.0, 8.0, 9.0)
