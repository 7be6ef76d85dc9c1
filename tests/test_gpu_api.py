"""C-ABI error behaviour and host-side bookkeeping of a live tracer (needs the GPU): invalid
arguments return RT2_ERR_INVALID with a message and leave the tracer usable; FrameIdx counts queued
frames; Reset drops them."""
import numpy as np
import pytest

import raytrace2_amd as R
from conftest import scene_path
from raytrace2_amd._native import Rt2Error

pytestmark = pytest.mark.gpu


@pytest.fixture
def tracer(have_gpu):
    sc = R.Scene(scene_path("cornell_box_original"), R.DEFAULT_SEED)
    tr = R.RayTracer(sc, 0)
    tr.SetSamplesPerPixel(16)
    tr.OnResize((24, 16))
    yield tr
    tr.close()


@pytest.mark.parametrize("call", [
    lambda tr: setattr(tr, "max_depth", 70000),
    lambda tr: tr.OnResize((0, 5)),
    lambda tr: tr.OnResize((70000, 5)),
    lambda tr: tr.Render(-1),
    lambda tr: tr.SetSamplesPerPixel(0),
    lambda tr: tr.set_work_split(-1),
    lambda tr: tr.set_batch_max(0),
    lambda tr: tr.set_lazy_frames(-1),
    lambda tr: tr.set_partition(8, 3, 2),
])
def test_invalid_arguments_fail_loudly_and_keep_the_tracer(tracer, call):
    with pytest.raises(Rt2Error) as e:
        call(tracer)
    assert e.value.args and "rt2 error -1" in str(e.value)
    tracer.Render(2)
    assert tracer.FrameIdx() == 2 and np.isfinite(tracer.NonConvertedPixels()).all()


def test_camera_beyond_the_exact_range_fails_loudly(tracer):
    """The rectangle test is exact for ray origins within +-2^100 (compile.cpp RectAAWords): a camera
    whose rays would start beyond +-2^64 (capi.cpp CameraOriginsBounded) is refused at Render with
    RT2_ERR_INVALID, and the tracer renders again once the camera is back in range."""
    import dataclasses
    good = tracer.get_camera()
    tracer.set_camera(dataclasses.replace(good, center=(1e30, 278.0, -800.0)))
    with pytest.raises(Rt2Error) as e:
        tracer.Render(1)
    assert "2^64" in str(e.value)
    tracer.set_camera(good)
    tracer.Render(2)
    assert tracer.FrameIdx() == 2 and np.isfinite(tracer.NonConvertedPixels()).all()


def test_far_camera_renders_sphere_scenes_like_the_oracle():
    """the +-2^64 camera bound belongs to the tests that need it (QUADAA rectangles, box
    boundaries, transforms about y: CompiledScene::origins_bounded). A sphere-only scene renders a camera
    beyond it as the reference would (here every ray misses: the sphere test's squares overflow), bit for
    bit like the oracle."""
    from oracle.oracle import OracleScene
    name, w, h, spp, frames = "perlin_spheres", 24, 16, 4, 3
    sc = R.Scene(scene_path(name), R.DEFAULT_SEED)
    far = R.Camera((3e20, 2.0, 3.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 20.0, 0.0, 10.0)
    tr = R.RayTracer(sc, 0)
    tr.set_seed(R.DEFAULT_SEED)
    tr.SetSamplesPerPixel(spp)
    tr.OnResize((w, h))
    tr.camera = far
    tr.Render(frames)
    acc = tr.Accumulation()
    tr.close()
    o = OracleScene(scene_path(name), R.DEFAULT_SEED)
    o.set_camera(far.center, far.look_at, far.view_up, far.vfov, far.defocus_angle, far.focus_distance)
    o_acc, _, _ = o.render(w, h, spp, frames, forward=True)
    assert np.array_equal(acc.view(np.uint32), o_acc.view(np.uint32))


def test_queued_frames_and_reset(tracer):
    for _ in range(5):
        tracer.Update()
    assert tracer.FrameIdx() == 5 and tracer.stats()["launches"] == 1  # stats() launched the queue
    tracer.Update()
    tracer.Reset()  # drops the queued frame: nothing is launched for it
    assert tracer.FrameIdx() == 0 and tracer.stats()["launches"] == 1
    assert not tracer.Accumulation().any()
    tracer.Render(3)
    a = tracer.Accumulation()
    assert tracer.FrameIdx() == 3 and a.any()


def test_kernel_time_is_gpu_busy_time_not_queue_time(have_gpu):
    """with two launch slots, step i + 1's render is queued while step i's still
    holds the CUs; kernel_ms must count the time the GPU ran render launches (each launch timed by its
    own first-wave / last-wave clock, overlaps once), not the time a launch waited in its queue. Back
    to back renders (the bench's step shape, no host wait between them): kernel time <= wall time,
    the sum of the launches' own times >= their union, and the host never waited inside the loop."""
    import time
    sc = R.Scene(scene_path("cornell_box_original"), R.DEFAULT_SEED)
    tr = R.RayTracer(sc, 0)
    tr.SetSamplesPerPixel(1000)
    tr.OnResize((256, 256))
    tr.Render(100)
    tr.synchronize()
    tr.reset_stats()
    steps = 6
    t0 = time.perf_counter()
    for _ in range(steps):
        tr.Reset()
        tr.Render(1000)
        tr.flush()
    # (stats() synchronizes, and reports the host waits from before its own synchronization)
    waits_in_loop = tr.stats()["host_waits"]
    tr.synchronize()
    wall_ms = (time.perf_counter() - t0) * 1e3
    st = tr.stats()
    tr.close()
    assert st["launches"] == steps
    assert 0.0 < st["kernel_ms"] <= wall_ms * 1.001, (st["kernel_ms"], wall_ms)
    assert st["launch_ms_sum"] >= st["kernel_ms"] * 0.9999, (st["launch_ms_sum"], st["kernel_ms"])
    # consecutive launches overlap only in a launch's tail (about a millisecond)
    assert st["launch_ms_sum"] <= st["kernel_ms"] + 3.0 * steps, (st["launch_ms_sum"], st["kernel_ms"])
    # structural (no wall-clock ratio): the launch path blocked the host nowhere
    assert waits_in_loop == 0, waits_in_loop
    print(f"kernel {st['kernel_ms']:.1f} ms of {wall_ms:.1f} ms wall (informational)")
    # the two launch slots' sample buffers stay within the (total) sample budget (rt2.h)
    assert 0 < st["sample_buffer_bytes"] <= (24 << 30)
    assert st["sample_buffer_bytes"] == 2 * 1000 * 256 * 256 * 12
    assert st["device_bytes_peak"] >= st["sample_buffer_bytes"] + 256 * 256 * 16


@pytest.mark.parametrize("name,w,h,spp,frames", [("cornell_box_original", 64, 64, 1000, 6),
                                                 ("cornell_box_volume", 64, 64, 1000, 6),
                                                 ("book2_final_scene_10000_samples", 48, 48, 10000, 4)])
def test_box_level_test_certifies_and_changes_no_bit(have_gpu, monkeypatch, name, w, h, spp, frames):
    """The box-level test (boxaa.h; DESIGN.md §4 "Box-level test"): the compiler gives the scene's MakeBox
    runs and MakeBox medium boundaries a box record, the counting kernel reports that it certifies
    nearly every lane there (the rest run the six faces), and the accumulation equals, bit for bit, the
    render with the test switched off (RT2_BOX_AA=0 at scene load: plain six-face runs)."""
    def render(env):
        if env is None:
            monkeypatch.delenv("RT2_BOX_AA", raising=False)
        else:
            monkeypatch.setenv("RT2_BOX_AA", env)
        sc = R.Scene(scene_path(name), R.DEFAULT_SEED)
        tr = R.RayTracer(sc, 0)
        tr.set_seed(R.DEFAULT_SEED)
        tr.SetSamplesPerPixel(spp)
        tr.OnResize((w, h))
        tr.enable_stats(True)
        tr.Render(frames)
        acc = tr.Accumulation().copy()
        st = tr.stats()
        tr.close()
        return sc.info().box_steps, acc, st
    steps, acc, st = render(None)
    steps0, acc0, st0 = render("0")
    assert steps > 0 and steps0 == 0
    assert st["box_tests"] > 0 and st0["box_tests"] == 0
    assert st["box_certified"] >= 0.99 * st["box_tests"], (st["box_certified"], st["box_tests"])
    assert st["box_wave_runs"] <= 0.01 * st["box_wave_visits"], (st["box_wave_runs"], st["box_wave_visits"])
    assert st["rays"] == st0["rays"] and st["quad_tests"] == st0["quad_tests"]  # the reference's counts
    assert np.array_equal(acc.view(np.uint32), acc0.view(np.uint32))


def test_medium_box_far_away_matches_the_oracle(have_gpu):
    """The medium's box-boundary test (boxaa.h BoxAAPair) at distances where the second boundary query
    starts on the first hit itself: for t1 above 2^11, fl(t1 + 0.0001) = t1 (ConstantMedium.cpp:26-30), so
    the entry face answers both queries and the medium has zero thickness there. The Cornell volume seen
    from 6000 units away, bit-identical to the oracle (whose two queries run on the six faces)."""
    from oracle.oracle import OracleScene
    name, w, h, spp, frames = "cornell_box_volume", 24, 24, 4, 3
    sc = R.Scene(scene_path(name), R.DEFAULT_SEED)
    assert sc.info().box_steps == 2
    cam = R.Camera((278.0, 278.0, -6000.0), (278.0, 278.0, 0.0), (0.0, 1.0, 0.0), 6.0, 0.0, 10.0)
    tr = R.RayTracer(sc, 0)
    tr.set_seed(R.DEFAULT_SEED)
    tr.SetSamplesPerPixel(spp)
    tr.OnResize((w, h))
    tr.camera = cam
    tr.enable_stats(True)
    tr.Render(frames)
    acc = tr.Accumulation()
    st = tr.stats()
    tr.close()
    o = OracleScene(scene_path(name), R.DEFAULT_SEED)
    o.set_camera(cam.center, cam.look_at, cam.view_up, cam.vfov, cam.defocus_angle, cam.focus_distance)
    o_acc, _, _ = o.render(w, h, spp, frames, forward=True)
    assert st["box_certified"] > 0
    assert np.array_equal(acc.view(np.uint32), o_acc.view(np.uint32))
