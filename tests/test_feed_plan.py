"""Host feed copy plan (CPU): the source rows a full-frame pre-process reads (feed.touched_rows, from the
library's own row table) and the strided copy commands that move them (feed.copy_runs)."""
import numpy as np
import pytest


def test_touched_rows_c4_is_a_third(evam, O):
    F = evam.feed
    rows = F.touched_rows(O.NV12, 3840, 2160, 640, 640, 1)  # C4: 1/6 scale, letterbox
    assert len(rows[0]) == 720 and len(rows[1]) == 360
    assert F.copy_runs(rows[0]) == [(2, 2, 6, 360)] and F.copy_runs(rows[1]) == [(1, 1, 3, 360)]


@pytest.mark.parametrize("src,dst,mode", [((1920, 1080), (512, 512), 0), ((3840, 2160), (640, 640), 1),
                                          ((1920, 1080), (224, 224), 2), ((768, 432), (512, 512), 0),
                                          ((640, 360), (72, 50), 1)])
def test_touched_rows_match_oracle_table(evam, O, coracle, src, dst, mode):
    """Luma rows = both clamped taps of every visible output row of the oracle's own y table."""
    F = evam.feed
    (W, H), (DW, DH) = src, dst
    rh, top = F.resized_height(W, H, DW, DH, mode)
    ofs, _, _ = coracle.linear_table(H, rh, False)
    want = sorted({min(max(int(s) + d, 0), H - 1) for s in ofs[top:top + DH] for d in (0, 1)})
    rows = F.touched_rows(O.NV12, W, H, DW, DH, mode)
    assert rows[0] == want and rows[1] == sorted({r >> 1 for r in want})


@pytest.mark.parametrize("seed", range(20))
def test_copy_runs_cover_rows(evam, seed):
    """Every row is copied; a strided plan copies nothing else (the bounding-span fallback may)."""
    F = evam.feed
    rng = np.random.default_rng(seed)
    rows = sorted(set(rng.integers(0, 400, int(rng.integers(1, 60))).tolist()))
    if seed % 3 == 0:  # periodic: runs of 2 every 5 rows
        rows = sorted({5 * k + d for k in range(40) for d in (1, 2)})
    cmds = F.copy_runs(rows)
    got = set()
    for r0, length, stride, runs in cmds:
        assert length <= stride
        for k in range(runs):
            got.update(range(r0 + k * stride, r0 + k * stride + length))
    assert set(rows) <= got
    if len(cmds) > 1 or cmds[0][3] > 1:
        assert got == set(rows)
    if seed % 3 == 0:
        assert cmds == [(1, 2, 5, 40)]


@pytest.mark.parametrize("src,dst,mode", [((192, 320), (48, 48), 2), ((1080, 1920), (224, 224), 2),
                                          ((320, 192), (48, 48), 2), ((200, 360), (40, 40), 1),
                                          ((3840, 2160), (640, 640), 1), ((64, 48), (16, 16), 0)])
def test_resized_height_matches_oracle_geometry(evam, O, src, dst, mode):
    """feed.resized_height (the rows the strided plan copies) against the oracle's own item geometry
    (rh and the central crop's row offset -oy), portrait sources with a vertical central crop included."""
    (W, H), (DW, DH) = src, dst
    g = O.item_geometry(O.NV12, W, H, 0, 0, 0, 0, mode, 0, DW, DH)
    rh, top = evam.feed.resized_height(W, H, DW, DH, mode)
    assert rh == g["rh"] and top == (-g["oy"] if mode == 2 else 0)
    if src == (192, 320):
        assert top == 16  # 320 * 48/192 = 80 resized rows, the middle 48 visible


@pytest.mark.parametrize("seed", range(40))
def test_touched_rows_random_geometries(evam, O, coracle, seed):
    """Random frame / tensor sizes and the three resize modes: resized_height against the oracle's item geometry, and
    touched_rows against both clamped taps of every visible row of the oracle's own row table (luma and 4:2:0 chroma
    rows)."""
    F = evam.feed
    rng = np.random.default_rng(700 + seed)
    W, H = 2 * int(rng.integers(1, 1200)), 2 * int(rng.integers(1, 1200))
    DW, DH, mode = int(rng.integers(1, 700)), int(rng.integers(1, 700)), int(rng.integers(0, 3))
    g = O.item_geometry(O.NV12, W, H, 0, 0, 0, 0, mode, 0, DW, DH)
    rh, top = F.resized_height(W, H, DW, DH, mode)
    assert rh == g["rh"] and top == (-g["oy"] if mode == 2 else 0), (W, H, DW, DH, mode)
    ofs, _, _ = coracle.linear_table(H, rh, False)
    want = sorted({min(max(int(s) + d, 0), H - 1) for s in ofs[top:top + DH] for d in (0, 1)})
    rows = F.touched_rows(O.NV12, W, H, DW, DH, mode)
    assert rows[0] == want and rows[1] == sorted({r >> 1 for r in want}), (W, H, DW, DH, mode)
