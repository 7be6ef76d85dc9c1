"""Known-answer and distributional tests of the CPU restatement (oracle/), pinning it before it is
trusted as the parity reference. Hand-derived values cite the reference function they follow."""
import math

import numpy as np
import pytest

from conftest import scene_path
from oracle import oracle as O

F32_MAX = 3.4028234663852886e38


def test_philox_random123_kat():
    # Random123 kat_vectors, philox4x32 with 10 rounds
    assert O.philox([0, 0, 0, 0], [0, 0]) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    assert O.philox([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2) == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]
    assert O.philox([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0]) == \
        [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def test_uniform_stream_is_24bit_and_in_unit_interval():
    u = O.uniforms(1234, 7, 3, 4096)
    assert u.min() >= 0.0 and u.max() < 1.0
    assert np.all(u * 16777216.0 == np.round(u * 16777216.0))  # exact 24-bit grid
    assert abs(u.mean() - 0.5) < 0.02
    # the stream is a function of (seed, pixel, frame): distinct keys differ, same keys repeat
    assert np.array_equal(u, O.uniforms(1234, 7, 3, 4096))
    assert not np.array_equal(u, O.uniforms(1234, 8, 3, 4096))
    assert not np.array_equal(u, O.uniforms(1234, 7, 4, 4096))


def test_quad_hit_kat():
    # Quad.cpp:19-43: unit quad in the z=0 plane, ray straight down the -z axis
    out = O.quad_hit([0, 0, 0], [1, 0, 0], [0, 1, 0], [0.25, 0.5, 2.0], [0, 0, -1])
    assert out[0] == 1 and out[1] == pytest.approx(2.0)
    assert list(out[2:5]) == pytest.approx([0.25, 0.5, 0.0])
    # n = normalize(u x v) = +z; the ray travels -z so it hits the front face, normal stays +z
    assert list(out[5:8]) == [0, 0, 1] and out[8] == 1
    assert list(out[9:11]) == pytest.approx([0.25, 0.5])  # uv = (alpha, beta)
    # from below: back face, normal flipped (HitRecord::SetFaceNormal)
    out = O.quad_hit([0, 0, 0], [1, 0, 0], [0, 1, 0], [0.25, 0.5, -2.0], [0, 0, 1])
    assert out[0] == 1 and out[8] == 0 and list(out[5:8]) == [0, 0, -1]
    # outside the parallelogram, parallel ray, behind the interval
    assert O.quad_hit([0, 0, 0], [1, 0, 0], [0, 1, 0], [1.5, 0.5, 2.0], [0, 0, -1])[0] == 0
    assert O.quad_hit([0, 0, 0], [1, 0, 0], [0, 1, 0], [0.5, 0.5, 2.0], [1, 0, 0])[0] == 0
    assert O.quad_hit([0, 0, 0], [1, 0, 0], [0, 1, 0], [0.5, 0.5, 2.0], [0, 0, -1], tmin=0.001, tmax=1.5)[0] == 0
    # Interval::Contains is inclusive: t == tmax hits, the edge alpha == 1 is inside
    assert O.quad_hit([0, 0, 0], [1, 0, 0], [0, 1, 0], [0.5, 0.5, 2.0], [0, 0, -1], tmax=2.0)[0] == 1
    assert O.quad_hit([0, 0, 0], [1, 0, 0], [0, 1, 0], [1.0, 0.5, 2.0], [0, 0, -1])[0] == 1


def test_sphere_hit_kat():
    # Sphere.cpp:7-37: unit sphere at the origin, ray from z=5 toward -z: nearest root t = 4
    out = O.sphere_hit([0, 0, 0], [0, 0, 0], 1.0, [0, 0, 5], [0, 0, -1])
    assert out[0] == 1 and out[1] == pytest.approx(4.0)
    assert list(out[5:8]) == pytest.approx([0, 0, 1]) and out[8] == 1
    # from inside: the far root, back face (normal flipped toward the ray)
    out = O.sphere_hit([0, 0, 0], [0, 0, 0], 1.0, [0, 0, 0], [0, 0, -1])
    assert out[1] == pytest.approx(1.0) and out[8] == 0 and list(out[5:8]) == pytest.approx([0, 0, 1])
    # moving sphere: center(t) = c0 + disp * time
    out = O.sphere_hit([0, 0, 0], [0, 2, 0], 1.0, [0, 1, 5], [0, 0, -1], time=0.5)
    assert out[0] == 1 and out[1] == pytest.approx(4.0)
    # Interval::Surrounds is strict: t == tmax does not hit
    assert O.sphere_hit([0, 0, 0], [0, 0, 0], 1.0, [0, 0, 5], [0, 0, -1], tmax=4.0)[0] == 0
    # non-normalised direction: t is in units of |d|
    out = O.sphere_hit([0, 0, 0], [0, 0, 0], 1.0, [0, 0, 5], [0, 0, -2])
    assert out[1] == pytest.approx(2.0)


def test_aabb_slab_kat():
    # AABB.hpp:34-47
    assert O.aabb_hit([0, 0, 0], [1, 1, 1], [0.5, 0.5, 5], [0, 0, -1])
    assert not O.aabb_hit([0, 0, 0], [1, 1, 1], [1.5, 0.5, 5], [0, 0, -1])
    assert not O.aabb_hit([0, 0, 0], [1, 1, 1], [0.5, 0.5, 5], [0, 0, -1], tmax=3.9)
    assert O.aabb_hit([0, 0, 0], [1, 1, 1], [0.5, 0.5, 5], [0, 0, -1], tmax=4.1)
    # ray starting inside
    assert O.aabb_hit([0, 0, 0], [1, 1, 1], [0.5, 0.5, 0.5], [1, 1, 1])


def test_transform_kat():
    # ParseTransform (Serialize.cpp:106-132): T * R * S, rotation = angleAxis(radians(a), axis)
    m, inv = O.transform([265, 0, 295], [90, 0, 1, 0], [1, 1, 1])
    # rotation +90 deg about y maps x -> -z, z -> +x; translation in column 3 (glm column-major)
    assert m[0][:3] == pytest.approx([0, 0, -1], abs=1e-6)
    assert m[2][:3] == pytest.approx([1, 0, 0], abs=1e-6)
    assert m[3][:3] == pytest.approx([265, 0, 295])
    assert (np.asarray(m, np.float64).T @ np.asarray(inv, np.float64).T) == pytest.approx(np.eye(4), abs=1e-4)
    m, _ = O.transform([0, 0, 0], [0, 0, 1, 0], [2, 3, 4])
    assert np.diag(m)[:3] == pytest.approx([2, 3, 4])


def test_camera_basis_kat():
    # Camera.hpp:16-48 for the Cornell camera at 400x400, spp 64 (hand-derived):
    # w = (0,0,-1), u = (-1,0,0), v = (0,1,0); viewport = 2*tan(20 deg)*focus(1)
    s = O.OracleScene(scene_path("cornell_box_original"))
    p = s.camera_params(400, 400, 64)
    vh = 2 * math.tan(math.radians(20.0))
    du = vh / 400
    assert list(p[3:6]) == pytest.approx([-du, 0, 0], rel=1e-6)
    assert list(p[6:9]) == pytest.approx([0, du, 0], rel=1e-6)
    assert list(p[0:3]) == pytest.approx([278 + vh / 2 - du / 2, 278 - vh / 2 + du / 2, -799], abs=1e-4)
    assert p[19] == pytest.approx(1 / 8) and p[20] == 8  # sqrt(64) strata per axis
    # spp 1000 -> 31 strata per axis (int(sqrt(1000)))
    assert s.camera_params(1024, 1024, 1000)[20] == 31


def test_scene_hit_cornell_walls():
    s = O.OracleScene(scene_path("cornell_box_original"))
    # above the tall box, straight into the room: the back wall z = 555 (material 1, white); its
    # normal u x v points +z, so the ray sees its back face and the normal is flipped
    h = s.hit([450, 450, -800], [0, 0, 1])
    assert h[0] == 1 and h[1] == pytest.approx(1355.0) and h[9] == 1
    assert h[8] == 0 and list(h[5:8]) == pytest.approx([0, 0, -1])
    # down the middle: the tall box (translated (265,0,295), rotated 15 deg) is in front of the wall;
    # its t comes from inside a TransformedHittable (model-space t, equal here since |d| = 1)
    h = s.hit([278, 278, -800], [0, 0, 1])
    assert h[0] == 1 and 295 - 80 < h[4] < 295 + 20 and h[9] == 1
    # upward from the floor center: the ceiling light (material 3) at y=554 under the ceiling
    h = s.hit([278, 1, 278], [0, 1, 0])
    assert h[0] == 1 and h[1] == pytest.approx(553.0) and h[9] == 3


def test_rand_unit_vec3_distribution():
    # RandUnitVec3 (Math.hpp:26-43) is uniform on the unit sphere; the restatement draws it by the
    # inverse-CDF map (z = 1 - 2u, phi = 2 pi v): unit length, z uniform on [-1, 1] (Archimedes),
    # isotropic first and second moments, and the same z / azimuth law as normalize(rejection
    # sample in the unit ball) drawn from the same stream.
    v = O.unit_vectors(99, 1, 2, 40000).astype(np.float64)
    assert np.abs(np.linalg.norm(v, axis=1) - 1).max() < 1e-6
    assert np.abs(v.mean(0)).max() < 0.02
    assert (v * v).mean(0) == pytest.approx([1 / 3] * 3, abs=0.01)
    z = np.sort(v[:, 2])
    assert np.abs(z - np.linspace(-1, 1, z.size)).max() < 0.02  # uniform z
    u = O.uniforms(7, 3, 4, 3 * 40000).reshape(-1, 3).astype(np.float64) * 2 - 1
    ok = ((u * u).sum(1) <= 1) & ((u * u).sum(1) > 0)
    assert ok.mean() == pytest.approx(math.pi / 6, abs=0.01)  # the reference's acceptance rate
    r = u[ok] / np.linalg.norm(u[ok], axis=1, keepdims=True)
    for a in (v, r):
        assert np.histogram(a[:, 2], bins=8, range=(-1, 1))[0].min() > a.shape[0] / 8 * 0.9


def test_rand_in_unit_disk_distribution():
    p = O.unit_disk(5, 6, 7, 40000).astype(np.float64)
    r2 = (p[:, :2] ** 2).sum(1)
    assert (p[:, 2] == 0).all() and r2.max() <= 1.0
    assert np.abs(np.sort(r2) - np.linspace(0, 1, r2.size)).max() < 0.02  # r^2 uniform
    assert np.abs(p[:, :2].mean(0)).max() < 0.02


def test_cos_sin_2pi_polynomial():
    # the shared quarter-turn polynomial (oracle CosSin2Pi == kernel cos_sin_2pi): max error 3e-7
    v = (np.arange(1 << 20, dtype=np.float64) / (1 << 20)).astype(np.float32)
    cs = O.cos_sin_2pi(v).astype(np.float64)
    ang = 2 * np.pi * v.astype(np.float64)
    assert np.abs(cs[:, 0] - np.cos(ang)).max() < 3e-7
    assert np.abs(cs[:, 1] - np.sin(ang)).max() < 3e-7
    assert cs[0, 0] == 1.0 and cs[0, 1] == 0.0


def test_sin_f_restatement():
    # the marble texture's sin (Texture.cpp:16; oracle SinF == kernel sin_f): within 9e-8 of sin over
    # the marble's argument range and beyond, odd, exact at 0, 0 / NaN past 2^24
    rng = np.random.default_rng(5)
    v = np.concatenate([rng.uniform(-5000, 5000, 1 << 18), rng.uniform(-4, 4, 1 << 18),
                        np.arange(-20000, 20000, dtype=np.float64) * (np.pi / 4)]).astype(np.float32)
    s = O.sin_f(v).astype(np.float64)
    assert np.abs(s - np.sin(v.astype(np.float64))).max() < 1e-7
    assert np.array_equal(O.sin_f(-v), -O.sin_f(v))
    sp = O.sin_f(np.array([0.0, -0.0, 2.0 ** 24, -(2.0 ** 30), np.inf, np.nan], np.float32))
    assert sp[0] == 0 and sp[2] == 0 and sp[3] == 0 and np.isnan(sp[4]) and np.isnan(sp[5])


def test_medium_free_flight_fraction(tmp_path):
    # ConstantMedium.cpp:14-58: a ray crossing a slab of length L inside a medium of density rho
    # scatters with probability 1 - exp(-rho L).
    import json
    scene = {"camera": {"center": [0, 0, -10], "look_at": [0, 0, 0], "width": 8, "aspect_ratio": 1.0},
             "materials": [{"type": "lambertian", "albedo": [0.5, 0.5, 0.5]}],
             "primitives": [{"type": "box", "a": [-1, -1, -1], "b": [1, 1, 1], "material": 0,
                             "constant_medium": {"density": 0.5, "albedo": [1, 1, 1]}}],
             "scene": [{"primitive": 0}, {"primitive": 0}]}
    p = tmp_path / "medium.json"
    p.write_text(json.dumps(scene))
    s = O.OracleScene(str(p))
    n = 4000
    hits = sum(int(s.hit([0, 0, -10], [0, 0, 1], seed=k)[0]) for k in range(n))
    # the node appears twice at top level (a 2-leaf BVH): each test draws its own number, so the
    # ray scatters unless both draws fly through: 1 - exp(-2 rho L)
    expect = 1 - math.exp(-2 * 0.5 * 2.0)
    assert hits / n == pytest.approx(expect, abs=4 * math.sqrt(expect * (1 - expect) / n))


def test_log_u_within_one_ulp_for_every_uniform():
    """LogU (ConstantMedium's free-flight draw, ConstantMedium.cpp:38; the kernel's log_u computes the
    same bits) on every 24-bit uniform k / 2^24: within 1 ulp of ln in double, -inf at 0."""
    k = np.arange(1 << 24, dtype=np.float64)
    u = (k / 16777216.0).astype(np.float32)
    got = O.log_u(u).astype(np.float64)
    assert got[0] == -np.inf
    ref = np.log(u[1:].astype(np.float64))
    ulp = np.spacing(np.abs(ref).astype(np.float32)).astype(np.float64)
    err = np.abs(got[1:] - ref) / ulp
    assert err.max() < 0.9, err.max()  # measured 0.87 ulp
    # and equals the correctly rounded value for most (measured 93 %)
    assert np.mean(got[1:] == ref.astype(np.float32)) > 0.9
