"""Host cost of one HipPreProcessor.convert() call (GPU box): a tiny workload so the GPU is idle and
the loop is host-bound. Prints microseconds per call for full-frame batches, a fixed ROI set and a
ROI set that changes every call (descriptor re-upload), and for the bare ctypes evam_pp_run call."""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import __graft_entry__ as g

    evam = g.import_package()
    dev = torch.device("cuda:0")
    imgs = [evam.Image.alloc("NV12", 64, 48, device=dev) for _ in range(32)]
    for im in imgs:
        for p in im.planes:
            p.fill_(77)
    batch = evam.ImageBatch(imgs)
    out = torch.empty((32, 3, 16, 16), dtype=torch.float32, device=dev)
    info = evam.PreProcInfo(range=(0.0, 1.0), mean=(0.4, 0.4, 0.4), std=(0.2, 0.2, 0.2))
    pp = evam.HipPreProcessor(device=0)
    rng = np.random.default_rng(0)
    roi_sets = []
    for k in range(4):
        a = np.zeros((1600, 5), np.int32)
        a[:, 0] = rng.integers(0, 32, 1600)
        a[:, 1] = rng.integers(0, 32, 1600)
        a[:, 2] = rng.integers(0, 24, 1600)
        a[:, 3] = rng.integers(8, 32, 1600)
        a[:, 4] = rng.integers(8, 24, 1600)
        roi_sets.append(evam.RoiBatch(a))
    out_roi = torch.empty((1600, 3, 16, 16), dtype=torch.float32, device=dev)

    def timeit(name, fn, n=2000):
        for i in range(50):
            fn(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(n):
            fn(i)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"{name:48s} {1e6 * (t1 - t0) / n:8.2f} us/call host, {1e6 * (t2 - t0) / n:8.2f} us/call incl. drain",
              flush=True)

    timeit("convert 32 full frames", lambda i: pp.convert(batch, out, info))
    timeit("convert 1600 ROIs (same set)", lambda i: pp.convert(batch, out_roi, info, rois=roi_sets[0]))
    timeit("convert 1600 ROIs (new set every call)", lambda i: pp.convert(batch, out_roi, info, rois=roi_sets[i % 4]))
    lib = pp._lib
    t = evam.native.EvamTensor()
    t.data = out.data_ptr()
    t.n, t.c, t.h, t.w, t.slot_offset, t.slot_stride = 32, 3, 16, 16, 0, 1
    cfg = info.to_c(evam.native.DTYPE_F32)
    tb, cb = ctypes.byref(t), ctypes.byref(cfg)
    timeit("bare evam_pp_run 32 full frames", lambda i: lib.evam_pp_run(pp._h, batch.c_array, 32, None, 32, cb, tb, None))
    pp.close()


if __name__ == "__main__":
    main()
