"""MI355X-native pre-process backend for EVAM (Edge Video Analytics Microservice).

The directory name contains hyphens, so import it with importlib::

    import importlib
    evam = importlib.import_module("edge-video-analytics-microservice_amd")

After the first import the package is also reachable as ``evam_amd`` (``sys.modules`` alias).

Scope: decoded NV12/I420/BGRx/BGR frames -> colour conversion -> INTER_LINEAR /
letterbox / central-crop resize -> ROI crop-resize -> normalisation -> NCHW batch packing, as hand-written
HIP kernels for gfx950 behind the C ABI in ``include/evam_pp.h``.
"""
import sys as _sys

from ._native import PreProcError, load_library  # noqa: F401
from .preproc import (HipPreProcessor, Image, ImageBatch, PreProcInfo, Roi, RoiBatch, Transform,  # noqa: F401
                      create_preprocessor, plane_layout)
from . import _native as native  # noqa: F401
from . import streams  # noqa: F401
from . import postproc  # noqa: F401
from . import feed  # noqa: F401
from . import pipeline_server  # noqa: F401

_sys.modules.setdefault("evam_amd", _sys.modules[__name__])
