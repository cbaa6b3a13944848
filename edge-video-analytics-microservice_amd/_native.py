"""ctypes binding of ``libevam_pp.so`` (the C ABI declared in ``include/evam_pp.h``).

The structures below mirror the header field-for-field; ``tests/test_abi.py`` checks their sizes
against the compiled library's expectations and that every declared symbol is exported.

``torch`` is imported before the library is loaded: the ROCm PyTorch wheel ships its own
``libamdhip64.so`` (SONAME ``libamdhip64.so.7``), and loading torch first makes the dynamic linker
bind this library to that same HIP runtime instead of a second copy from ``/opt/rocm``. Device
pointers and streams created by torch are then valid here.
"""
from __future__ import annotations

import ctypes
import os
import sys

LIB_NAME = "libevam_pp.so"
PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, LIB_NAME)

# evam_fourcc
FOURCC_NV12 = 0x3231564E
FOURCC_I420 = 0x30323449
FOURCC_BGRX = 0x58524742
FOURCC_BGRA = 0x41524742
FOURCC_BGR = 0x20524742

# evam_pp_status
OK = 0
ERR_INVALID_ARG = -1
ERR_UNSUPPORTED = -2
ERR_ALIGNMENT = -3
ERR_EMPTY_ROI = -4
ERR_HIP = -5
ERR_NO_DEVICE = -6
ERR_OOM = -7
STATUS_NAMES = {
    OK: "EVAM_PP_OK", ERR_INVALID_ARG: "EVAM_PP_ERR_INVALID_ARG", ERR_UNSUPPORTED: "EVAM_PP_ERR_UNSUPPORTED",
    ERR_ALIGNMENT: "EVAM_PP_ERR_ALIGNMENT", ERR_EMPTY_ROI: "EVAM_PP_ERR_EMPTY_ROI", ERR_HIP: "EVAM_PP_ERR_HIP",
    ERR_NO_DEVICE: "EVAM_PP_ERR_NO_DEVICE", ERR_OOM: "EVAM_PP_ERR_OOM",
}

RESIZE_NO_ASPECT, RESIZE_ASPECT, RESIZE_ASPECT_CROP = 0, 1, 2
PLACE_TOP_LEFT, PLACE_CENTER = 0, 1
COLOR_BGR, COLOR_RGB = 0, 1
DTYPE_U8, DTYPE_F32 = 0, 1
NORM_RANGE, NORM_MEAN_STD = 1, 2
OPT_STATS, OPT_TIMING = 1, 2

ABI_VERSION = 2  # 2: evam_pp_run_slots

# Every symbol include/evam_pp.h declares.
EXPORTED_SYMBOLS = (
    "evam_pp_create", "evam_pp_run", "evam_pp_run_slots", "evam_pp_sync", "evam_pp_set_stream", "evam_pp_set_option",
    "evam_pp_get_stats", "evam_pp_destroy", "evam_pp_last_error", "evam_pp_abi_version",
    "evam_pp_linear_table",
)

c_i32 = ctypes.c_int32


class EvamImage(ctypes.Structure):
    _fields_ = [("fourcc", c_i32), ("width", c_i32), ("height", c_i32), ("pitch", c_i32 * 3),
                ("planes", ctypes.c_void_p * 3)]


class EvamRoi(ctypes.Structure):
    _fields_ = [("src_index", c_i32), ("x", c_i32), ("y", c_i32), ("w", c_i32), ("h", c_i32)]


class EvamPreproc(ctypes.Structure):
    _fields_ = [("resize_mode", c_i32), ("placement", c_i32), ("color_order", c_i32), ("out_dtype", c_i32),
                ("norm_flags", c_i32), ("fill", ctypes.c_uint8 * 4), ("range", ctypes.c_float * 2),
                ("mean", ctypes.c_float * 3), ("std", ctypes.c_float * 3)]


class EvamTensor(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("n", c_i32), ("c", c_i32), ("h", c_i32), ("w", c_i32),
                ("slot_offset", c_i32), ("slot_stride", c_i32)]


class EvamTransform(ctypes.Structure):
    _fields_ = [("scale_x", ctypes.c_float), ("scale_y", ctypes.c_float), ("crop_x", c_i32), ("crop_y", c_i32),
                ("crop_w", c_i32), ("crop_h", c_i32), ("pad_x", c_i32), ("pad_y", c_i32),
                ("resized_w", c_i32), ("resized_h", c_i32)]


class EvamStats(ctypes.Structure):
    _fields_ = [("src_bytes", ctypes.c_int64), ("dst_bytes", ctypes.c_int64), ("n_items", c_i32),
                ("n_launches", c_i32), ("last_kernel_ms", ctypes.c_float), ("kernels", ctypes.c_uint32)]


# evam_pp_stats.kernels bits (include/evam_pp.h evam_kernel_family)
KERNEL_GENERIC, KERNEL_ROWS, KERNEL_STAGED, KERNEL_WAVE = 1, 2, 4, 8
KERNEL_STRIP, KERNEL_BAND, KERNEL_ROI = 16, 32, 64


STRUCT_SIZES = {EvamImage: 48, EvamRoi: 20, EvamPreproc: 56, EvamTensor: 32, EvamTransform: 40, EvamStats: 32}

_LIB = None


def _declare(lib: ctypes.CDLL) -> ctypes.CDLL:
    P = ctypes.POINTER
    vp = ctypes.c_void_p
    lib.evam_pp_create.argtypes = [ctypes.c_int, vp, P(vp)]
    lib.evam_pp_create.restype = ctypes.c_int
    lib.evam_pp_run.argtypes = [vp, P(EvamImage), ctypes.c_int, P(EvamRoi), ctypes.c_int, P(EvamPreproc),
                                P(EvamTensor), P(EvamTransform)]
    lib.evam_pp_run.restype = ctypes.c_int
    lib.evam_pp_run_slots.argtypes = [vp, P(EvamImage), ctypes.c_int, P(EvamRoi), ctypes.c_int, P(EvamPreproc),
                                      P(EvamTensor), P(c_i32), P(EvamTransform)]
    lib.evam_pp_run_slots.restype = ctypes.c_int
    lib.evam_pp_sync.argtypes = [vp]
    lib.evam_pp_sync.restype = ctypes.c_int
    lib.evam_pp_set_stream.argtypes = [vp, vp]
    lib.evam_pp_set_stream.restype = ctypes.c_int
    lib.evam_pp_set_option.argtypes = [vp, ctypes.c_int, ctypes.c_int]
    lib.evam_pp_set_option.restype = ctypes.c_int
    lib.evam_pp_get_stats.argtypes = [vp, P(EvamStats)]
    lib.evam_pp_get_stats.restype = ctypes.c_int
    lib.evam_pp_destroy.argtypes = [vp]
    lib.evam_pp_destroy.restype = None
    lib.evam_pp_last_error.argtypes = []
    lib.evam_pp_last_error.restype = ctypes.c_char_p
    lib.evam_pp_abi_version.argtypes = []
    lib.evam_pp_abi_version.restype = ctypes.c_int
    lib.evam_pp_linear_table.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, P(c_i32),
                                         P(ctypes.c_int16), P(ctypes.c_int16)]
    lib.evam_pp_linear_table.restype = ctypes.c_int
    return lib


def load_library(path: str | None = None) -> ctypes.CDLL:
    """Load the in-tree HIP library. Raises RuntimeError when it is missing — there is no fallback."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    import torch  # noqa: F401  (binds the library to torch's HIP runtime; see module docstring)

    p = path or LIB_PATH
    ab = os.environ.get("EVAM_PP_LIB")
    if path is None and ab:
        # A/B runs only: a variant of this library built by tools/build_variant.sh into <repo>/ab/. Anything
        # else is refused, and the swap is announced, so a stray setting cannot silently replace the product.
        ab_dir = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(LIB_PATH))), "ab")
        real = os.path.realpath(ab)
        if os.path.dirname(real) != os.path.realpath(ab_dir) or not os.path.basename(real).startswith("libevam_pp_"):
            raise RuntimeError(f"EVAM_PP_LIB={ab}: only variant builds in {ab_dir} (tools/build_variant.sh) are loaded")
        print(f"[evam_pp] EVAM_PP_LIB: loading the A/B variant {real}", file=sys.stderr)
        p = real
    if not os.path.exists(p):
        raise RuntimeError(
            f"{LIB_NAME} is not built at {p}: run `python -c 'import __graft_entry__ as g; g.build()'` "
            "(the HIP backend has no CPU fallback)")
    lib = _declare(ctypes.CDLL(p))
    if lib.evam_pp_abi_version() != ABI_VERSION:
        raise RuntimeError(f"{p}: ABI version {lib.evam_pp_abi_version()} != expected {ABI_VERSION}")
    if path is None:
        _LIB = lib
    return lib


class PreProcError(RuntimeError):
    """A failed evam_pp call; ``status`` is the evam_pp_status code (mirrors DLS throwing runtime_error)."""

    def __init__(self, status: int, message: str):
        self.status = status
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {message}")


def check(lib: ctypes.CDLL, rc: int) -> None:
    if rc != OK:
        raise PreProcError(rc, lib.evam_pp_last_error().decode(errors="replace"))
