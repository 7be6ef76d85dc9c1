"""The C++ drop-in boundary end to end: raytrace2_amd/lib/rt2_headless is the reference's headless
App::Run path (src/App.cpp:115-174, 243-248) compiled against include/rt2/RayTracer.hpp. Its PNG must
equal the one the Python mirror writes for the same scene, dims and samples, and LoadAppSettings must
drive it like the reference's settings.json."""
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, scene_path

pytestmark = pytest.mark.gpu
APP = os.path.join(ROOT, "raytrace2_amd", "lib", "rt2_headless")


def _run(args):
    r = subprocess.run([APP, *args], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def _python_png(name, w, h, spp, out):
    import raytrace2_amd as R
    sc = R.Scene(scene_path(name), R.DEFAULT_SEED)
    tr = R.RayTracer(sc, 0)
    tr.SetSamplesPerPixel(spp)
    tr.OnResize((w, h))
    for _ in range(spp):
        tr.Update(sc)
    R.WriteImage(tr.NonConvertedPixels(), w, h, out)
    tr.close()


@pytest.mark.parametrize("name", ["cornell_box_original", "cornell_box_volume"])
def test_headless_app_matches_python_mirror(have_gpu, tmp_path, name):
    a, b = str(tmp_path / "cpp.png"), str(tmp_path / "py.png")
    out = _run([scene_path(name), a, "--samples", "16", "--size", "96x64"])
    assert out["frames"] == 16 and out["launches"] == 1 and out["rays"] > 96 * 64 * 16
    _python_png(name, 96, 64, 16, b)
    assert open(a, "rb").read() == open(b, "rb").read()


def test_headless_app_multi_gpu_path(have_gpu, tmp_path):
    """rt2::RayTracer(scene, 0, n_gpus) over rt2_tracer_create_multi (RCCL, one GPU on the test box):
    the same PNG as the one-GPU path."""
    a, b = str(tmp_path / "multi.png"), str(tmp_path / "one.png")
    out = _run([scene_path("cornell_box_original"), a, "--samples", "12", "--size", "80x72", "--gpus", "1"])
    assert out["gpus"] == 1 and out["frames"] == 12
    _run([scene_path("cornell_box_original"), b, "--samples", "12", "--size", "80x72"])
    assert open(a, "rb").read() == open(b, "rb").read()


def test_headless_app_reads_settings(have_gpu, tmp_path):
    st = tmp_path / "settings.json"
    st.write_text(json.dumps({"render_once": True, "save_after_render_once": True, "num_samples": 9,
                              "max_depth": 3, "render_window": False}))
    out = _run([scene_path("cornell_box_original"), str(tmp_path / "s.png"), "--settings", str(st), "--size", "40x30"])
    assert out["frames"] == 9 and (out["width"], out["height"]) == (40, 30)
    from PIL import Image
    img = np.asarray(Image.open(str(tmp_path / "s.png")))
    assert img.shape[:2] == (30, 40) and img.max() > 0
