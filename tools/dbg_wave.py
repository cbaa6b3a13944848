"""Debug helper (GPU box): mismatch map of one wave-kernel case under several env variants."""
import os
import sys
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    import torch
    import __graft_entry__ as g
    import oracle as O
    from test_gpu_parity import run_hip, run_oracle, upload

    evam = g.import_package()
    fmt, src, dst, resize = O.I420, (768, 432), (512, 512), "no-aspect-ratio"
    rng = np.random.default_rng(zlib.crc32(repr(("I420", src, dst, resize)).encode()))
    frames = [O.random_frame(rng, fmt, src[0], src[1], pattern=p) for p in ("uniform", "gradient", "uniform")]
    c = O.COracle()
    for variant in sys.argv[1:] or ["base"]:
        for kv in variant.split(","):
            if "=" in kv:
                k, v = kv.split("=")
                os.environ[k] = v
        for dtype in ("u8", "f32"):
            info = evam.PreProcInfo(color_space="RGB", fill=(5, 50, 250), placement="center", resize=resize,
                                    **({"range": (0.0, 1.0), "mean": (0.1, 0.2, 0.3), "std": (0.3, 0.2, 0.1)}
                                       if dtype == "f32" else {}))
            shape = (3, 3, dst[1], dst[0])
            got, _ = run_hip(evam, torch, upload(evam, frames, "cuda:0"), shape,
                             torch.float32 if dtype == "f32" else torch.uint8, info)
            ref, _ = run_oracle(O, c, frames, shape, dtype, info)
            same = got.view(np.uint32) == ref.view(np.uint32) if dtype == "f32" else got == ref
            bad = np.argwhere(~same)
            print(variant, dtype, "mismatches", len(bad))
            if len(bad):
                rows = sorted(set((int(b[0]), int(b[2])) for b in bad))
                print("  (item,row):", rows[:40])
                cols = sorted(set(int(b[3]) for b in bad))
                print("  cols:", cols[:64])
                chans = sorted(set(int(b[1]) for b in bad))
                print("  chans:", chans)
                i = tuple(bad[0])
                print("  first", i, got[i], ref[i], hex(got.view(np.uint32)[i]) if dtype == "f32" else "")
        for kv in variant.split(","):
            if "=" in kv:
                os.environ.pop(kv.split("=")[0])


if __name__ == "__main__":
    main()
