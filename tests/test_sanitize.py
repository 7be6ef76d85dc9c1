"""ASan + UBSan build of the host code (SURVEY.md §5 "Race detection / sanitizers").

json.cpp, scene.cpp, compile.cpp, image.cpp (the product's loader, scene compiler and image writer) and
oracle/rt_oracle.cpp (the CPU restatement) are compiled with -fsanitize=address,undefined and
-fno-sanitize-recover=all, and tests/cpp/sanitize_host.cpp drives them over every committed scene (load,
compile in both list modes, camera at the BASELINE sizes, a small oracle render in both product orders),
every byte prefix and 400 single-byte corruptions of each scene document, the malformed documents of
tests/test_loader.py, the camera files' WriteCamera round trip and WriteImage in both formats. Any
sanitizer report aborts the run. CPU only; the GPU code is not built here (no device sanitizer on this
pool)."""
import glob
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "raytrace2_amd", "csrc")

BAD_DOCS = [
    '{"materials": [{"type": "plastic"}], "camera": {}}',
    '{"materials": [{"albedo": [1,1,1]}], "camera": {}}',
    '{"camera": {}, "materials": [{"type":"lambertian"}], "primitives": [{"type":"quad"}], "scene": [{"primitive": 3}]}',
    '{"camera": {}, "materials": [], "primitives": [], "scene": []}',
    '{"camera": {}, "materials": [{"type":"lambertian"}], "primitives": [{"type":"quad","material":5}], '
    '"scene": [{"primitive": 0}]}',
    '{"camera": {"fov": 40,',
    '{"camera": {"center": [0, 0, 1]}, "materials": [{"type": "lambertian"}], '
    '"primitives": {"triangles": [{"material_id": 0}]}}',
    '{"camera": {}, "materials": [{"type":"lambertian"}], "primitives": [{"type":"sphere","center":[0,0]}], '
    '"scene": [{"primitive": 0}]}',
    '{"camera": {}, "materials": [{"type":"lambertian"}], "primitives": [{"type":"quad"}], '
    '"scene": [{"children": [{"children": [{"primitive": -1}]}]}]}',
    '[1e999999, "\\ud800", "\\u00zz"]',
    '{"a": ' * 4000,
    '',
]


@pytest.fixture(scope="module")
def sanitized(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("asan") / "sanitize_host")
    flags = ["-O1", "-g", "-std=c++17", "-ffp-contract=off", "-fno-omit-frame-pointer",
             "-fsanitize=address,undefined,float-cast-overflow", "-fno-sanitize-recover=all", "-pthread"]
    srcs = [os.path.join(ROOT, "tests", "cpp", "sanitize_host.cpp"), os.path.join(ROOT, "oracle", "rt_oracle.cpp")]
    srcs += [os.path.join(CSRC, f) for f in ("json.cpp", "scene.cpp", "compile.cpp", "image.cpp")]
    r = subprocess.run(["g++", *flags, "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", "-I", CSRC, "-o", exe, *srcs],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    return exe


def test_host_code_is_clean_under_asan_and_ubsan(sanitized, tmp_path):
    scenes = sorted(p for p in glob.glob(os.path.join(ROOT, "scenes", "*.json")) if not p.endswith("cam.json")
                    and not p.endswith("cam1.json"))
    scenes += sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "scenes", "*.json")))
    bad = []
    for i, doc in enumerate(BAD_DOCS):
        p = tmp_path / f"bad{i}.json"
        p.write_text(doc)
        bad.append(str(p))
    cams = [os.path.join(ROOT, "scenes", "cam1.json"), os.path.join(ROOT, "scenes", "scene2_cam.json")]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([sanitized, "--out", str(tmp_path), "--good", *scenes, "--bad", *bad, "--camera", *cams],
                       capture_output=True, text=True, env=env, timeout=1200)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-6000:])
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-6000:]
    assert r.stdout.startswith("documents=")
    assert int(r.stdout.split()[0].split("=")[1]) > 5000  # (every scene, its prefixes and corruptions)
