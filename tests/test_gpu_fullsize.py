"""Bit-exact parity at the BASELINE configs' full geometry and sample settings, including the
stratum wrap: the reference's frame f uses stratum (f % sq, f / sq % sq) (RayTracer.cpp:59-60), so
frames past sq^2 revisit the strata — the headline's frames 961-999 (spp 1000, sq 31), book 1's
484-499 (sq 22) and Cornell volume's 3969+ (sq 63).

Where the oracle would take minutes for a whole image it renders a band subset of rows (the GPU
renders the same partition), and where a late frame range matters it continues from the GPU's own
accumulation at frame k: the accumulation is a frame-ordered running sum (RayTracer.cpp:64), so
oracle(frames k..n | start = GPU(frames 0..k)) must equal GPU(frames 0..n) bit for bit.
"""
import numpy as np
import pytest

from conftest import scene_path
from helpers import SEED, gpu_render, oracle_render

pytestmark = pytest.mark.gpu

THREADS = 16  # the GPU box's CPU share


def _same(a, b):
    return np.array_equal(a.view(np.uint32), b.view(np.uint32))


def _check(name, w, h, spp, frames, **kw):
    part = {k: v for k, v in kw.items() if k in ("band_h", "rank", "world")}
    acc, rc, st, _ = gpu_render(name, w, h, spp, frames, **kw)
    o_acc, o_rc, o_cnt = oracle_render(name, w, h, spp, frames, forward=True, threads=THREADS, **part)
    assert st["overflow"] == 0
    np.testing.assert_array_equal(rc, o_rc)
    assert st["rays"] == o_cnt["rays"]
    mism = np.count_nonzero(acc.view(np.uint32) != o_acc.view(np.uint32))
    assert mism == 0, f"{mism} of {acc.size} floats differ"
    return acc, rc


def _check_continuation(name, w, h, spp, k, n, launch=None, **part):
    """GPU frames 0..n vs oracle frames k..n started from the GPU's accumulation at frame k.
    `launch`: GPU launch-shape settings (launch_frames / sample_budget) for both GPU renders."""
    from oracle.oracle import OracleScene
    launch = launch or {}
    a_k, rc_k, _, _ = gpu_render(name, w, h, spp, k, **part, **launch)
    a_n, rc_n, st_n, _ = gpu_render(name, w, h, spp, n, **part, **launch)
    o = OracleScene(scene_path(name), SEED)
    o_acc = a_k.copy()
    o_rc = np.zeros_like(rc_k)
    o.render(w, h, spp, n - k, frame_begin=k, accum=o_acc, ray_counts=o_rc, forward=True, threads=THREADS, **part)
    np.testing.assert_array_equal(rc_n - rc_k, o_rc)
    assert _same(a_n, o_acc)
    return st_n


def test_c1_cornell_400_at_64spp_full_image():
    """BASELINE configs[0]: cornell_box_original.json 400x400 @ 64 spp, the whole image."""
    _check("cornell_box_original", 400, 400, 64, 64)


def _check_recursive_order(name, w, h, spp, frames, acc, **part):
    """The north star's literal bar against the reference-shaped product order: the oracle's recursive
    RayColor (`emit + att * RayColor(...)`, RayTracer.cpp:20-45) on the same band and frames. The GPU
    multiplies the attenuations front to back, so the two differ only in the rounding of the product:
    per-pixel RMSE of clamp(accum / spp, 0, 1) (linear, per channel: SURVEY §8(d)) < 1e-3, and the
    largest relative difference of the accumulated sums < 1e-5 (both sides add non-negative samples
    in the same frame order, RayTracer.cpp:64)."""
    from helpers import rmse
    r_acc, _, _ = oracle_render(name, w, h, spp, frames, forward=False, threads=THREADS, **part)
    ga = np.clip(acc.astype(np.float64) / spp, 0.0, 1.0)
    ra = np.clip(r_acc.astype(np.float64) / spp, 0.0, 1.0)
    e = rmse(ga, ra)
    nz = r_acc != 0
    rel = float(np.max(np.abs(acc[nz].astype(np.float64) - r_acc[nz]) / np.abs(r_acc[nz].astype(np.float64))))
    assert np.array_equal(acc == 0, r_acc == 0)
    assert e < 1e-3, e
    assert rel < 1e-5, rel
    print(f"{name} {w}x{h} spp {spp}, {frames} frames {part}: RMSE vs the recursive order {e:.3g}, "
          f"max relative difference {rel:.3g}")


def test_c2_cornell_1024_all_1000_frames_band():
    """BASELINE configs[1] (the headline): 1024^2, spp 1000, every frame 0..999 (strata wrap at
    961), on rank 5 of a 32-way 16-row band split (32 rows x 1024): bit-identical to the oracle's
    front-to-back order, and within the north star's tolerance of its recursive (reference) order."""
    part = dict(band_h=16, rank=5, world=32)
    acc, _ = _check("cornell_box_original", 1024, 1024, 1000, 1000, **part)
    _check_recursive_order("cornell_box_original", 1024, 1024, 1000, 1000, acc, **part)


def test_c2_cornell_1024_whole_image_4_frames():
    """The whole 1024^2 headline image (every row, every pixel), frames 0..3 of the spp-1000
    stratification: bit-identical to the oracle, ray counts included (about 30 M rays)."""
    _check("cornell_box_original", 1024, 1024, 1000, 4)


def test_c3_book1_full_width_band_all_500_frames():
    """BASELINE configs[2]: book 1 at 1920x1080, spp 500 (sq 22: frames 484-499 wrap), a full-width
    band of 8 rows (rank 67 of 135)."""
    _check("final_render_book_1", 1920, 1080, 500, 500, band_h=8, rank=67, world=135)


def test_c4_cornell_volume_spp4000_first_frames():
    """BASELINE configs[3]: Cornell volume 1024^2 at spp 4000 (sq 63), 64 frames on 16 rows."""
    _check("cornell_box_volume", 1024, 1024, 4000, 64, band_h=16, rank=17, world=64)


def test_c4_cornell_volume_spp4000_across_sq2():
    """Frames 3950..3999 of spp 4000 cross sq^2 = 3969 (stratum (0, 0) again at 3969)."""
    _check_continuation("cornell_box_volume", 1024, 1024, 4000, 3950, 4000, band_h=8, rank=40, world=128)


def test_c5_book2_full_width_band():
    """BASELINE configs[4]: book 2 at 800x800, spp 10000 (sq 100), 24 frames on an 8-row band:
    bit-identical to the oracle's front-to-back order, and within the north star's tolerance of its
    recursive (reference) order."""
    part = dict(band_h=8, rank=50, world=100)
    acc, _ = _check("book2_final_scene_10000_samples", 800, 800, 10000, 24, **part)
    _check_recursive_order("book2_final_scene_10000_samples", 800, 800, 10000, 24, acc, **part)


@pytest.mark.parametrize("band_h", [1, 2, 4])
def test_c2_narrow_bands(band_h):
    """Row bands narrower than a work tile (tiles of 64x1, 32x2, 16x4 pixels): rank 5 of 8."""
    _check("cornell_box_original", 1024, 1024, 1000, 40, band_h=band_h, rank=5, world=8)


def test_c2_headline_last_frames_full_width():
    """The headline's wrap region on a wider band: frames 950..999 continued from the GPU."""
    _check_continuation("cornell_box_original", 1024, 1024, 1000, 950, 1000, band_h=64, rank=7, world=16)


@pytest.mark.parametrize("split", [0, 1, 3, 64])
def test_spp20_sq2_below_spp_frames_wrap(split):
    """spp 20: sq = 4, sq^2 = 16 < spp, so frames 16..19 (and 20..39) wrap; chunks of a split
    launch start mid-cycle."""
    acc, rc = _check("cornell_box_original", 72, 40, 20, 40, work_split=split)
    if split:
        acc0, _, _, _ = gpu_render("cornell_box_original", 72, 40, 20, 40, work_split=0)
        assert _same(acc, acc0)


def test_frames_beyond_sq2_in_several_launches():
    """spp 16 (sq 4), 40 frames as launches of 7 frames: launch boundaries inside the cycle."""
    _check("cornell_box_volume", 64, 48, 16, 40, launch_frames=7)


@pytest.mark.parametrize("name,w,h,spp,frames,part", [
    ("cornell_box_original", 72, 40, 20, 40, {}),                                  # frames past sq^2, 64-frame groups padded
    ("cornell_box_volume", 1024, 1024, 4000, 70, dict(band_h=8, rank=40, world=128)),  # a band, one padded group
    ("final_render_book_1", 64, 48, 16, 130, {}),                                  # defocus, 3 groups
])
def test_frame_tiles_forced(monkeypatch, name, w, h, spp, frames, part):
    """Frame tiles (a wave = one pixel x 64 one-frame chunks; book 2 runs them by default) forced on
    scenes that default to pixel tiles: the same bits as the oracle."""
    monkeypatch.setenv("RT2_FRAME_TILES", "1")
    _check(name, w, h, spp, frames, **part)


def test_frame_tiles_off_on_book2(monkeypatch):
    """Book 2 with frame tiles switched off (pixel tiles, 64-frame chunks) against the oracle."""
    monkeypatch.setenv("RT2_FRAME_TILES", "0")
    _check("book2_final_scene_10000_samples", 800, 800, 10000, 12, band_h=8, rank=50, world=100)


def _band_frame_bytes(w, h, band_h, rank, world):
    rows = sum(1 for y in range(h) if ((y // band_h) % world + (y // band_h) // world) % world == rank)
    return w * rows * 12


@pytest.mark.parametrize("boundary,how", [(2000, "launch_frames"), (1672, "sample_budget")])
def test_c5_book2_across_a_launch_boundary(boundary, how):
    """Book 2 (C5: 800x800 @ 10000 spp, frame tiles) across a launch boundary: the default 24 GiB
    sample budget (12 GiB per launch slot) cuts its one-GPU render into launches of 1672 frames
    (budget_frames rounded to octets); frames boundary-10 .. boundary+10 on a full-width band are
    continued by the oracle from the GPU's accumulation and must match bit for bit
    (RayTracer.cpp:55-70 renders every frame alike)."""
    part = dict(band_h=8, rank=50, world=100)
    launch = ({"launch_frames": boundary} if how == "launch_frames" else
              {"sample_budget": 2 * boundary * _band_frame_bytes(800, 800, **part)})
    st = _check_continuation("book2_final_scene_10000_samples", 800, 800, 10000, boundary - 10, boundary + 10,
                             launch=launch, **part)
    assert st["launches"] == 2


@pytest.mark.parametrize("boundary,how", [(1333, "launch_frames"), (1024, "sample_budget")])
def test_c4_cornell_volume_across_a_launch_boundary(boundary, how):
    """Cornell volume (C4: 1024^2 @ 4000 spp) across the bench's launch boundary (24 GiB budget, 12 GiB
    per slot: launches of 1024 frames) and an odd one (1333, launch_frames), continued by the oracle."""
    part = dict(band_h=8, rank=40, world=128)
    launch = ({"launch_frames": boundary} if how == "launch_frames" else
              {"sample_budget": 2 * boundary * _band_frame_bytes(1024, 1024, **part)})
    st = _check_continuation("cornell_box_volume", 1024, 1024, 4000, boundary - 10, boundary + 10, launch=launch,
                             **part)
    assert st["launches"] == 2
