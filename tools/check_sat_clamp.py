"""Exhaustive check of the saturating BT.601 clamp used by the HIP kernels (evam_pp.hip, hpass_sat).

For every (Y, U, V) byte triple and every channel, the kernel computes
    s   = min(y + term', 2^32 - 1)                (v_add_u32 clamp)
    c16 = max((s >> 16) - 61440, 0) & 0xFFF0      (v_pk_sub_u16 clamp, mask)
with y = max(Y, 16) * CY and term' = term + K + 2^32 - 2^28, and relies on
    c16 == 16 * clamp255((y + term + K) >> 20)   (OpenCV color_yuv)
and on 0 <= term' < 2^32 (no wrap in the 32-bit chroma term). Run: python tools/check_sat_clamp.py
"""
import numpy as np

CY, CUB, CUG, CVG, CVR = 1220542, 2116026, -409993, -852492, 1673527
HALF = 1 << 19
K = {"b": HALF - 128 * CUB - 16 * CY, "g": HALF - 128 * CVG - 128 * CUG - 16 * CY, "r": HALF - 128 * CVR - 16 * CY}
BIAS = (1 << 32) - (1 << 28)


def check() -> int:
    """Returns the number of mismatching (Y, U, V, channel) cases (0 = identity holds)."""
    U, V = [a.astype(np.int64) for a in np.meshgrid(np.arange(256), np.arange(256), indexing="ij")]
    terms = {"b": CUB * U, "g": CVG * V + CUG * U, "r": CVR * V}
    bad = 0
    for Y in range(256):
        y = max(Y, 16) * CY
        for ch, t in terms.items():
            tk = t + K[ch]
            tp = tk + BIAS
            assert tp.min() >= 0 and tp.max() < (1 << 32), ch
            s = np.minimum(y + tp, (1 << 32) - 1)
            c16 = np.maximum((s >> 16) - 61440, 0) & 0xFFF0
            bad += int((c16 != 16 * np.clip((y + tk) >> 20, 0, 255)).sum())
    return bad


if __name__ == "__main__":
    n = check()
    print("mismatches:", n)
    raise SystemExit(1 if n else 0)
