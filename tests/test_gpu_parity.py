"""GPU parity: the gfx950 kernel (through the C ABI) against the CPU restatement (oracle/) on the same
seeded inputs.

Bar (BASELINE.json north star): per-pixel RMSE < 1e-3 on clamp(accum/spp, 0, 1) at matched seed.
Stronger checks held here:
  * rays per pixel are integers and must match EXACTLY (same RNG draws, same geometry decisions);
  * against the oracle's front-to-back product order (forward=True) the accumulation must be
    bit-identical; against the reference's recursive order the difference is rounding only.
"""
import numpy as np
import pytest

from helpers import gpu_render, oracle_render, rmse

pytestmark = pytest.mark.gpu

# (scene, w, h, spp setting, frames): small enough for the oracle to finish in seconds
CASES = [
    ("cornell_box_original", 64, 64, 16, 16),
    ("cornell_box_volume", 64, 64, 16, 8),
    ("final_render_book_1", 96, 54, 500, 4),
    ("book2_final_scene_10000_samples", 48, 48, 10000, 4),
    ("checker_test", 64, 48, 64, 8),
    ("perlin_spheres", 64, 48, 64, 8),
    ("cornell_box_scene_graph", 64, 64, 16, 8),
    ("cornell_box2", 64, 64, 16, 8),  # legacy schema: quads + boxes
    ("light_scene1", 64, 48, 16, 8),  # legacy schema: spheres + quads, textures
]


@pytest.mark.parametrize("name,w,h,spp,frames", CASES, ids=[c[0] for c in CASES])
def test_matched_seed_parity(have_gpu, name, w, h, spp, frames):
    acc, rc, st, _ = gpu_render(name, w, h, spp, frames)
    o_acc, o_rc, o_cnt = oracle_render(name, w, h, spp, frames, forward=True)
    assert st["overflow"] == 0
    # geometry + RNG decisions identical: exact ray counts per pixel
    np.testing.assert_array_equal(rc, o_rc)
    assert st["rays"] == o_cnt["rays"]
    # north-star bar on the displayed quantity
    e = rmse(np.clip(acc / frames, 0, 1), np.clip(o_acc / frames, 0, 1))
    assert e < 1e-3, e
    # bit-identical to the same-order restatement
    mism = np.count_nonzero(acc.view(np.uint32) != o_acc.view(np.uint32))
    assert mism == 0, f"{mism} of {acc.size} floats differ; max abs {np.abs(acc - o_acc).max()}"


@pytest.mark.parametrize("name", ["cornell_box_original", "book2_final_scene_10000_samples"])
def test_parity_vs_recursive_reference_order(have_gpu, name):
    w, h, spp, frames = 48, 48, 16, 8
    acc, rc, _, _ = gpu_render(name, w, h, spp, frames)
    o_acc, o_rc, _ = oracle_render(name, w, h, spp, frames, forward=False)
    np.testing.assert_array_equal(rc, o_rc)
    # only the rounding of the attenuation product differs
    rel = np.abs(acc - o_acc) / np.maximum(np.abs(o_acc), 1e-3)
    assert rel.max() < 1e-5, rel.max()
    assert rmse(np.clip(acc / frames, 0, 1), np.clip(o_acc / frames, 0, 1)) < 1e-6


def test_update_equals_render_and_chunking(have_gpu):
    a1, r1, _, _ = gpu_render("cornell_box_volume", 40, 40, 16, 7)
    a2, r2, _, _ = gpu_render("cornell_box_volume", 40, 40, 16, 7, updates=True)
    a3, r3, _, _ = gpu_render("cornell_box_volume", 40, 40, 16, 7, launch_frames=3)
    # every Update() launched at once (no queue), and a queue flushed every 2 frames
    a4, r4, s4, _ = gpu_render("cornell_box_volume", 40, 40, 16, 7, updates=True, lazy=0)
    a5, r5, s5, _ = gpu_render("cornell_box_volume", 40, 40, 16, 7, updates=True, lazy=2)
    assert np.array_equal(a1.view(np.uint32), a2.view(np.uint32))
    assert np.array_equal(a1.view(np.uint32), a3.view(np.uint32))
    assert np.array_equal(a1.view(np.uint32), a4.view(np.uint32))
    assert np.array_equal(a1.view(np.uint32), a5.view(np.uint32))
    assert np.array_equal(r1, r2) and np.array_equal(r1, r3) and np.array_equal(r1, r4) and np.array_equal(r1, r5)
    assert s4["launches"] == 7 and s5["launches"] == 4


@pytest.mark.parametrize("name", ["cornell_box_original", "final_render_book_1", "book2_final_scene_10000_samples"])
def test_work_split_is_invisible(have_gpu, name):
    # A pixel's frames cut into chunks rendered by different lanes (any chunk size, any wave batch,
    # several launches when the sample buffer is small) must sum to the same bits: samples are
    # accumulated in frame order after each launch (RayTracer.cpp:64).
    w, h, spp, frames = 72, 40, 64, 13
    base = gpu_render(name, w, h, spp, frames, work_split=0)
    o_acc, o_rc, _ = oracle_render(name, w, h, spp, frames, forward=True)
    assert np.array_equal(base[0].view(np.uint32), o_acc.view(np.uint32))
    assert np.array_equal(base[1], o_rc)
    frame_bytes = w * h * 12
    for kw in (dict(work_split=1), dict(work_split=100000), dict(work_split=64, batch_max=1),
               dict(work_split=64, batch_max=4096), dict(sample_budget=6 * frame_bytes),
               dict(sample_budget=1, work_split=5), dict(launch_frames=4, sample_budget=4 * frame_bytes)):
        acc, rc, st, px = gpu_render(name, w, h, spp, frames, **kw)
        assert np.array_equal(acc.view(np.uint32), base[0].view(np.uint32)), kw
        assert np.array_equal(rc, base[1]), kw
        assert np.array_equal(px, base[3]), kw
    # a larger image, where a small split gives multi-frame chunks of uneven length
    big = gpu_render(name, 256, 256, spp, frames, work_split=0)
    for split in (1, 2, 3):
        acc, rc, _, _ = gpu_render(name, 256, 256, spp, frames, work_split=split)
        assert np.array_equal(acc.view(np.uint32), big[0].view(np.uint32)), split
        assert np.array_equal(rc, big[1]), split


def test_row_band_partition_reassembles_bitwise(have_gpu):
    import raytrace2_amd as R
    w, h = 50, 45
    full, _, _, _ = gpu_render("cornell_box_original", w, h, 16, 4)
    parts = [gpu_render("cornell_box_original", w, h, 16, 4, band_h=8, rank=r, world=3)[0] for r in range(3)]
    assert sum(p.shape[0] for p in parts) == h
    img = R.assemble_bands(parts, h, 8)
    assert np.array_equal(img.view(np.uint32), full.view(np.uint32))


def test_pixels_are_tocolor_of_mean(have_gpu):
    frames = 5
    acc, _, _, px = gpu_render("cornell_box_original", 32, 32, 16, frames)
    c = np.clip(acc / np.float32(frames), 0, 1)
    expect = np.floor(c.astype(np.float64) * 255.999).astype(np.uint8)
    assert np.array_equal(px[..., :3], expect)
    assert np.all(px[..., 3] == 255)


@pytest.mark.parametrize("depth", [0, 1, 2])
def test_max_depth_edges(have_gpu, depth):
    acc, rc, _, _ = gpu_render("cornell_box_original", 32, 32, 16, 4, max_depth=depth)
    o_acc, o_rc, _ = oracle_render("cornell_box_original", 32, 32, 16, 4, max_depth=depth)
    np.testing.assert_array_equal(rc, o_rc)
    assert np.array_equal(acc.view(np.uint32), o_acc.view(np.uint32))
    if depth == 0:
        assert not acc.any() and not rc.any()


def test_full_size_rows_subset(have_gpu):
    """Config-2 geometry (1024x1024, spp setting 1000): a band subset of rows against the oracle."""
    w = h = 1024
    frames = 2
    acc, rc, st, _ = gpu_render("cornell_box_original", w, h, 1000, frames, band_h=16, rank=5, world=32)
    o_acc, o_rc, _ = oracle_render("cornell_box_original", w, h, 1000, frames, band_h=16, rank=5, world=32)
    np.testing.assert_array_equal(rc, o_rc)
    assert np.array_equal(acc.view(np.uint32), o_acc.view(np.uint32))


MODES = {"linear": {}, "stack_lds": {"RT2_NO_LINEAR": "1"}, "stack_global": {"RT2_NO_LINEAR": "1", "RT2_NO_LDS": "1"},
         "stack_hybrid": {"RT2_NO_LINEAR": "1", "RT2_FORCE_HYBRID": "1"},
         "stack_hybrid_top3": {"RT2_NO_LINEAR": "1", "RT2_FORCE_HYBRID": "1", "RT2_HYBRID_RECORDS": "6"}}


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("name,w,h,spp,frames", [c for c in CASES if c[0] != "book2_final_scene_10000_samples"],
                         ids=[c[0] for c in CASES if c[0] != "book2_final_scene_10000_samples"])
def test_every_traversal_mode_matches(have_gpu, monkeypatch, mode, name, w, h, spp, frames):
    """The threaded lockstep traversal and the stack traversal (scene in LDS, in global memory, or
    only the top of its BVH in LDS) visit nodes in the same per-lane order, so every mode is
    bit-identical to the oracle."""
    for k, v in MODES[mode].items():
        monkeypatch.setenv(k, v)
    acc, rc, st, _ = gpu_render(name, w, h, spp, min(frames, 4))
    o_acc, o_rc, _ = oracle_render(name, w, h, spp, min(frames, 4), forward=True)
    assert st["overflow"] == 0
    np.testing.assert_array_equal(rc, o_rc)
    assert np.array_equal(acc.view(np.uint32), o_acc.view(np.uint32))


@pytest.mark.parametrize("mode", ["linear", "stack_lds"])
def test_list_acceleration_matches_linear_child_loop(have_gpu, monkeypatch, mode):
    """Book 2's 1000-sphere HittableList (HittableList.cpp:8-22) through its exact acceleration tree
    gives bit-identical renders and ray counts to the reference's linear child loop, with far
    fewer sphere tests, in the threaded program (tree in pre-order, near child first) and in the
    stack traversal (near child first per ray)."""
    for k, v in MODES[mode].items():
        monkeypatch.setenv(k, v)
    name, w, h, spp, frames = "book2_final_scene_10000_samples", 200, 200, 10000, 4
    a1, r1, s1, _ = gpu_render(name, w, h, spp, frames, stats=True)
    monkeypatch.setenv("RT2_NO_LIST_ACCEL", "1")
    a2, r2, s2, _ = gpu_render(name, w, h, spp, frames, stats=True)
    assert s1["overflow"] == 0 and s2["overflow"] == 0
    np.testing.assert_array_equal(r1, r2)
    assert s1["rays"] == s2["rays"]
    mism = np.count_nonzero(a1.view(np.uint32) != a2.view(np.uint32))
    assert mism == 0, f"{mism} floats differ"
    assert s1["sphere_tests"] * 5 < s2["sphere_tests"], (s1["sphere_tests"], s2["sphere_tests"])


def test_book2_threaded_equals_stack(have_gpu, monkeypatch):
    """Book 2 (accelerated list, media, transforms, motion, noise) renders bit-identically in the
    threaded program and in the stack traversal, ray counts included."""
    args = ("book2_final_scene_10000_samples", 160, 160, 10000, 3)
    a1, r1, s1, _ = gpu_render(*args)
    monkeypatch.setenv("RT2_NO_LINEAR", "1")
    a2, r2, s2, _ = gpu_render(*args)
    assert s1["overflow"] == 0 and s2["overflow"] == 0
    np.testing.assert_array_equal(r1, r2)
    assert np.array_equal(a1.view(np.uint32), a2.view(np.uint32))


@pytest.mark.parametrize("name,w,h,spp,frames", [("final_render_book_1", 96, 54, 500, 4),
                                                 ("book2_final_scene_10000_samples", 120, 120, 10000, 3)])
def test_paired_bvh_steps_are_invisible(have_gpu, monkeypatch, name, w, h, spp, frames):
    """Paired BVH steps (compile.cpp: a step also tests its near child's box, with the tmax the
    child's own step would see) give bit-identical renders and ray counts to single-box steps, and
    every lane tests exactly the same boxes (equal box-test counts)."""
    a1, r1, s1, _ = gpu_render(name, w, h, spp, frames, stats=True)
    monkeypatch.setenv("RT2_BVH_PAIRS", "0")
    a2, r2, s2, _ = gpu_render(name, w, h, spp, frames, stats=True)
    assert s1["overflow"] == 0 and s2["overflow"] == 0
    np.testing.assert_array_equal(r1, r2)
    assert s1["rays"] == s2["rays"] and s1["bvh_tests"] == s2["bvh_tests"], (s1, s2)
    assert np.array_equal(a1.view(np.uint32), a2.view(np.uint32))


@pytest.mark.parametrize("mode", ["linear", "stack_global"])
def test_generated_stress_scene(have_gpu, tmp_path, monkeypatch, mode):
    """A scene from the authoring module (3000 random spheres, a 6 k-step threaded program; or the
    stack traversal over a global-memory scene) is bit-identical to the oracle too."""
    for k, v in MODES[mode].items():
        monkeypatch.setenv(k, v)
    import random
    from raytrace2_amd import authoring as A
    p = str(tmp_path / "field.json")
    A.sphere_field(3000, random.Random(1)).dump(p)
    acc, rc, st, _ = gpu_render(p, 64, 36, 64, 4)
    o_acc, o_rc, o_cnt = oracle_render(p, 64, 36, 64, 4, forward=True)
    assert st["overflow"] == 0
    np.testing.assert_array_equal(rc, o_rc)
    assert np.array_equal(acc.view(np.uint32), o_acc.view(np.uint32))


def test_progressive_loop_equals_updates(have_gpu):
    """ProgressiveLoop (frames per tick adapted to a time budget, pinned async Pixels() readback)
    ends bit-identical to the same number of Update() calls, and each tick's pixels are Pixels()
    of the frames done so far."""
    import raytrace2_amd as R
    from conftest import scene_path
    from raytrace2_amd.progressive import ProgressiveLoop
    w, h, frames = 96, 64, 23
    ref = gpu_render("cornell_box_volume", w, h, 64, frames, updates=True, counts=False)
    sc = R.Scene(scene_path("cornell_box_volume"), R.DEFAULT_SEED)
    tr = R.RayTracer(sc, 0)
    tr.set_seed(R.DEFAULT_SEED)
    tr.SetSamplesPerPixel(64)
    tr.OnResize((w, h))
    loop = ProgressiveLoop(tr, frames, budget_ms=0.05, first_frames=2)
    seen = []

    def on_tick(lp, px):
        assert np.array_equal(px, tr.Pixels())
        seen.append(lp.frames_done)

    loop.run(on_tick)
    assert seen[-1] == frames and len(seen) >= 2
    assert np.array_equal(tr.Accumulation().view(np.uint32), ref[0].view(np.uint32))
    assert tr.FrameIdx() == frames
    loop.close()
    tr.close()


@pytest.mark.parametrize("w,h", [(1, 1), (1, 7), (13, 1), (9, 9), (65, 3)])
def test_ragged_and_tiny_images(have_gpu, w, h):
    """Images smaller than one 8x8 tile or with partial edge tiles: edge lanes get no pixel, every
    real pixel is rendered once per frame, bit-identical to the oracle."""
    acc, rc, st, px = gpu_render("cornell_box_original", w, h, 16, 5)
    o_acc, o_rc, o_cnt = oracle_render("cornell_box_original", w, h, 16, 5, forward=True)
    assert acc.shape == (h, w, 3) and px.shape == (h, w, 4)
    np.testing.assert_array_equal(rc, o_rc)
    assert st["rays"] == o_cnt["rays"] and st["paths"] == w * h * 5
    assert np.array_equal(acc.view(np.uint32), o_acc.view(np.uint32))



@pytest.mark.parametrize("mode", ["linear", "stack_global"])
def test_axis_aligned_quad_shapes(have_gpu, tmp_path, monkeypatch, mode):
    """Axis-aligned quads in every orientation the compiler distinguishes (compile.cpp RectAAWords):
    rectangles with u along the plane's first or second axis (the threaded program's mirrored
    record), parallelograms (demoted to the axis-aligned test with division) and a sheared box under
    a transform, plus a smoke box: bit-identical to the oracle."""
    for k, v in MODES[mode].items():
        monkeypatch.setenv(k, v)
    from raytrace2_amd import authoring as A
    doc = A.SceneDoc()
    A._cornell_room(doc)
    A._cornell_camera(doc)
    white = doc.lambertian([0.73, 0.73, 0.73])
    blue = doc.lambertian([0.1, 0.2, 0.7])
    for q, u, v, m in (([100, 100, 300], [0, 0, 120], [150, 0, 0], blue),        # y plane, u along B
                       ([300, 40, 200], [120, 0, 0], [60, 0, 140], white),       # parallelogram
                       ([80, 200, 400], [0, 90, 30], [0, 0, 150], blue),         # x plane, sheared
                       ([250, 300, 500], [0, 100, 0], [140, 0, 0], white)):      # z plane, u along B
        doc.node(doc.quad(q, u, v, m))
    doc.node(doc.quad([0, 0, 0], [90, 0, 0], [30, 0, 90], white), xform=A.transform([330, 120, 150], [25, 0, 1, 0]))
    doc.node(doc.box([0, 0, 0], [100, 150, 100], 0, constant_medium=A.medium(0.02, [0.9, 0.9, 0.9])),
             xform=A.transform([160, 0, 120], [-30, 0, 1, 0]))
    p = str(tmp_path / "quads.json")
    doc.dump(p)
    acc, rc, st, _ = gpu_render(p, 64, 64, 16, 6)
    o_acc, o_rc, o_cnt = oracle_render(p, 64, 64, 16, 6, forward=True)
    assert st["overflow"] == 0
    np.testing.assert_array_equal(rc, o_rc)
    assert np.array_equal(acc.view(np.uint32), o_acc.view(np.uint32))
