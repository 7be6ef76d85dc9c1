"""The drop-in boundary: librt2.so loads, exports every function include/rt2.h declares, and
reports errors through status codes + rt2_last_error (never aborts). No GPU compute here."""
import ctypes
import os
import subprocess

import pytest

import raytrace2_amd as R
from conftest import ROOT, scene_path


def test_every_declared_symbol_is_exported():
    names = R.declared_symbols()
    assert len(names) >= 40
    missing = [n for n in names if not hasattr(R.lib, n)]
    assert not missing
    # and nothing else with the rt2_ prefix is exported by accident (nm -D)
    out = subprocess.run(["nm", "-D", "--defined-only", R._native.LIB_PATH], capture_output=True, text=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T rt2_" in l}
    assert exported == set(names)


def test_header_is_plain_c():
    # the header compiles as C99 with no HIP/torch includes
    src = os.path.join(ROOT, "include", "rt2.h")
    r = subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-fsyntax-only", "-x", "c", src],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    import re
    txt = open(src).read()
    assert set(re.findall(r"#include\s*<([^>]+)>", txt)) == {"stddef.h", "stdint.h"}
    code = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    assert "hipStream_t" not in code and "torch" not in code.lower()


def test_null_arguments_return_invalid():
    assert R.lib.rt2_scene_load(None, 0, None) == -1
    assert b"null" in R.lib.rt2_last_error()
    assert R.lib.rt2_tracer_render(None, 1) == -1
    assert R.lib.rt2_write_image(None, 1, 1, b"/tmp/x.png", 1) == -1


def test_tracer_create_without_gpu_fails_cleanly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    s = R.Scene(scene_path("cornell_box_original"))
    with pytest.raises(R.Rt2Error) as e:
        R.RayTracer(s, 0)
    assert e.value.code == -4  # RT2_ERR_HIP


def test_version_string():
    assert b"gfx950" in R.lib.rt2_version()


def test_cpp_mirror_header_compiles():
    # include/rt2/RayTracer.hpp: the C++ drop-in mirror of cpu::RayTracer over the C ABI
    src = os.path.join(ROOT, "tests", "cpp", "mirror_compile.cpp")
    r = subprocess.run(["g++", "-std=c++17", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                        "-fsyntax-only", src], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


@pytest.mark.parametrize("scene,expect", [("book2_final_scene_10000_samples", 1), ("final_render_book_1", 1),
                                          ("cornell_box_original", 0)])
def test_paired_program_steps_are_well_formed(tmp_path, scene, expect):
    """compile.cpp's paired BVH / list-tree steps (host only): a paired step precedes its near child,
    carries that child's box and skip index, and no skip index lands on the child; sphere scenes
    pair, the Cornell box does not (its kernel has no second test)."""
    csrc = os.path.join(ROOT, "raytrace2_amd", "csrc")
    exe = str(tmp_path / "program_pairs")
    r = subprocess.run(["g++", "-O1", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", "-I", csrc,
                        "-o", exe, os.path.join(ROOT, "tests", "cpp", "program_pairs.cpp")]
                       + [os.path.join(csrc, f) for f in ("json.cpp", "scene.cpp", "compile.cpp")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    r = subprocess.run([exe, os.path.join(ROOT, "scenes", scene + ".json"), str(expect)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith("pairs=")


def test_box_level_test_decides_as_the_six_face_run(tmp_path):
    """boxaa.h (the kernel's box-level tests, host only): on random MakeBox boxes compiled by the product,
    for rays entering through faces, edges and corners, grazing, leaving a face from a rounded hit point,
    starting inside, passing near and with zero direction components, every lane BoxAATest certifies gets
    exactly the six-face run's answer (face and final interval key), and every lane BoxAAPair certifies
    gets exactly the two ConstantMedium boundary queries' answers (t1, t2); the certified fractions are
    printed (tests/cpp/box_cert.cpp)."""
    csrc = os.path.join(ROOT, "raytrace2_amd", "csrc")
    exe = str(tmp_path / "box_cert")
    r = subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                        "-I", csrc, "-o", exe, os.path.join(ROOT, "tests", "cpp", "box_cert.cpp")]
                       + [os.path.join(csrc, f) for f in ("json.cpp", "scene.cpp", "compile.cpp")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    for seed in (1, 2):
        r = subprocess.run([exe, "300", "12000", str(seed), str(tmp_path)], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr + r.stdout
        assert "boxes=" in r.stdout
        cert = {l.split(" rays")[0].strip(): float(l.split()[-1]) for l in r.stdout.splitlines()
                if "certified" in l and not l.startswith("boxes")}
        assert cert["enter face"] > 0.9 and cert["inside"] > 0.99, cert


def test_quadaa_bounds_decide_as_quad_hit(tmp_path):
    """compile.cpp CoordRange (host only): the kernel's QUADAA interior test, lo <= p <= hi on the hit
    point's two in-plane coordinates, decides as Quad::Hit's alpha/beta test (Quad.cpp:27-36) for
    random rectangles of every orientation and hit points on, beside and far from the bounds, +-0,
    +-inf and NaN (about 10 M decisions)."""
    csrc = os.path.join(ROOT, "raytrace2_amd", "csrc")
    exe = str(tmp_path / "quadaa_bounds")
    r = subprocess.run(["g++", "-O1", "-std=c++17", "-ffp-contract=off", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                        "-I", csrc, "-o", exe, os.path.join(ROOT, "tests", "cpp", "quadaa_bounds.cpp")]
                       + [os.path.join(csrc, f) for f in ("json.cpp", "scene.cpp", "compile.cpp")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    r = subprocess.run([exe, "20000", "7"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr + r.stdout
    assert r.stdout.startswith("rects=")
