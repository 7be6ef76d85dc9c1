"""ctypes front-end of the CPU restatement (oracle/rt_oracle.cpp). TEST INFRASTRUCTURE ONLY.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg may import this
module, and only as the checker or the timed CPU baseline — never as the product path.
Parity status: see the header of rt_oracle.cpp (partially pinned).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "librt2_oracle.so")
_lib = None


class Counters(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in
                ("rays", "bvh", "quad", "sphere", "xform", "medium", "list", "rng_draws")]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


class SceneInfo(ctypes.Structure):
    _fields_ = [("dims_x", ctypes.c_int), ("dims_y", ctypes.c_int),
                ("n_materials", ctypes.c_int), ("n_textures", ctypes.c_int),
                ("n_primitives", ctypes.c_int), ("n_top_nodes", ctypes.c_int),
                ("background", ctypes.c_float * 3), ("cam_center", ctypes.c_float * 3),
                ("cam_lookat", ctypes.c_float * 3), ("cam_vfov", ctypes.c_float),
                ("cam_defocus_angle", ctypes.c_float), ("cam_focus_dist", ctypes.c_float)]


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        vp, fp, u64, i32 = ctypes.c_void_p, ctypes.POINTER(ctypes.c_float), ctypes.c_uint64, ctypes.c_int
        L.oracle_scene_load.restype = vp
        L.oracle_scene_load.argtypes = [ctypes.c_char_p, u64]
        L.oracle_scene_free.argtypes = [vp]
        L.oracle_last_error.restype = ctypes.c_char_p
        L.oracle_scene_get_info.argtypes = [vp, ctypes.POINTER(SceneInfo)]
        L.oracle_scene_materials.argtypes = [vp, fp, i32]
        L.oracle_scene_textures.argtypes = [vp, fp, i32]
        L.oracle_scene_perlin.argtypes = [vp, i32, fp, ctypes.POINTER(ctypes.c_int)]
        L.oracle_camera_params.argtypes = [vp, i32, i32, i32, fp]
        L.oracle_scene_set_camera.argtypes = [vp, fp]
        L.oracle_scene_set_camera.restype = None
        L.oracle_scene_hit.argtypes = [vp, fp, fp, ctypes.c_float, ctypes.c_float, ctypes.c_float, u64, fp]
        L.oracle_philox.argtypes = [ctypes.POINTER(ctypes.c_uint32)] * 3
        L.oracle_uniforms.argtypes = [u64, ctypes.c_uint32, ctypes.c_uint32, i32, fp]
        L.oracle_samples.argtypes = [i32, u64, ctypes.c_uint32, ctypes.c_uint32, i32, fp, fp]
        L.oracle_quad_hit.argtypes = [fp, fp]
        L.oracle_sphere_hit.argtypes = [fp, fp]
        L.oracle_aabb_hit.argtypes = [fp]
        L.oracle_transform.argtypes = [fp, fp, fp]
        L.oracle_set_controls.argtypes = [i32]
        L.oracle_set_controls.restype = None
        L.oracle_get_controls.restype = i32
        L.oracle_render.argtypes = [vp, i32, i32, i32, i32, u64, i32, i32, i32, i32, i32, fp,
                                    ctypes.POINTER(ctypes.c_uint32), i32, i32, ctypes.POINTER(Counters)]
        _lib = L
    return _lib


def _f(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _u(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))


class OracleScene:
    """A scene loaded by the restated SceneLoader (Serialize.cpp:199-360) with the top-level BVH."""

    def __init__(self, path: str, seed: int = 0x5EED2024):
        self.path = path
        self.seed = seed
        self._h = lib().oracle_scene_load(path.encode(), seed)
        if not self._h:
            raise RuntimeError(lib().oracle_last_error().decode())

    def __del__(self):
        if getattr(self, "_h", None):
            lib().oracle_scene_free(self._h)
            self._h = None

    def info(self) -> SceneInfo:
        s = SceneInfo()
        lib().oracle_scene_get_info(self._h, ctypes.byref(s))
        return s

    def materials(self) -> np.ndarray:
        n = self.info().n_materials
        out = np.zeros((max(n, 1), 8), np.float32)
        lib().oracle_scene_materials(self._h, _f(out), n)
        return out[:n]

    def textures(self) -> np.ndarray:
        n = self.info().n_textures
        out = np.zeros((max(n, 1), 8), np.float32)
        lib().oracle_scene_textures(self._h, _f(out), n)
        return out[:n]

    def perlin(self, tex: int):
        vec = np.zeros((4096, 3), np.float32)
        perm = np.zeros(3 * 4096, np.int32)
        pc = lib().oracle_scene_perlin(self._h, tex, _f(vec), perm.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
        if pc < 0:
            raise ValueError("not a noise texture")
        return vec[:pc].copy(), perm[:3 * pc].reshape(3, pc).copy()

    def set_camera(self, center, look_at, view_up, vfov, defocus_angle, focus_distance) -> None:
        """Camera setters (Camera.hpp:69-101) for the renders that follow."""
        v = np.array(list(center) + list(look_at) + list(view_up) + [vfov, defocus_angle, focus_distance],
                     np.float32)
        lib().oracle_scene_set_camera(self._h, _f(v))

    def camera_params(self, w: int, h: int, spp: int) -> np.ndarray:
        out = np.zeros(21, np.float32)
        lib().oracle_camera_params(self._h, w, h, spp, _f(out))
        return out

    def hit(self, o, d, time=0.0, tmin=0.001, tmax=3.4028234663852886e38, seed=1):
        o = np.asarray(o, np.float32)
        d = np.asarray(d, np.float32)
        out = np.zeros(10, np.float32)
        lib().oracle_scene_hit(self._h, _f(o), _f(d), time, tmin, tmax, seed, _f(out))
        return out

    def render(self, w, h, spp_setting, frames, *, frame_begin=0, max_depth=50, seed=None, band_h=0,
               rank=0, world=1, accum=None, ray_counts=None, threads=0, forward=False):
        """Frames [frame_begin, frame_begin+frames) of RayTracer::Update (RayTracer.cpp:55-70)."""
        seed = self.seed if seed is None else seed
        bh = band_h or h
        rows = [y for y in range(h) if ((y // bh) % world + (y // bh) // world) % world == rank]
        if accum is None:
            accum = np.zeros((len(rows), w, 3), np.float32)
        if ray_counts is None:
            ray_counts = np.zeros((len(rows), w), np.uint32)
        cnt = Counters()
        lib().oracle_render(self._h, w, h, spp_setting, max_depth, seed, frame_begin, frames, band_h, rank, world,
                            _f(accum), _u(ray_counts), threads, 1 if forward else 0, ctypes.byref(cnt))
        return accum, ray_counts, cnt.as_dict()


# Controls that REMOVE one reference quirk each (rt_oracle.cpp g_controls): tests of the power of
# the screenshot pins only. 0 = the faithful restatement.
CTL_WORLD_T = 1      # transformed children report world-space t (Transform.cpp:13-20,75-88 quirk removed)
CTL_SINGLE_LEAF = 2  # span-1 BVH leaves tested once (BVH.cpp:18-20,50-55 quirk removed)
CTL_INF = 4          # kInfinity = +inf instead of FLT_MAX (Defs.hpp:17)
# ... and one that RESTORES the reference's sampling and libm calls where the restatement deviates
CTL_REF_MATH = 8     # rejection RandInUnitSphere/Disk, std::log, std::sin(float), std::pow(double, 5)


class controls:
    """Context manager: scenes loaded and rendered inside it use the given control mask."""

    def __init__(self, mask: int):
        self.mask = mask

    def __enter__(self):
        self.prev = lib().oracle_get_controls()
        lib().oracle_set_controls(self.mask)
        return self

    def __exit__(self, *exc):
        lib().oracle_set_controls(self.prev)
        return False


def philox(ctr, key):
    c = (ctypes.c_uint32 * 4)(*ctr)
    k = (ctypes.c_uint32 * 2)(*key)
    o = (ctypes.c_uint32 * 4)()
    lib().oracle_philox(c, k, o)
    return list(o)


def uniforms(seed, pixel, frame, n):
    out = np.zeros(n, np.float32)
    lib().oracle_uniforms(seed, pixel, frame, n, _f(out))
    return out


def unit_vectors(seed, pixel, frame, n):
    """n RandUnitVec3 draws (inverse-CDF map) from the path stream."""
    out = np.zeros((n, 3), np.float32)
    lib().oracle_samples(0, seed, pixel, frame, n, _f(np.zeros(1, np.float32)), _f(out))
    return out


def unit_disk(seed, pixel, frame, n):
    out = np.zeros((n, 3), np.float32)
    lib().oracle_samples(1, seed, pixel, frame, n, _f(np.zeros(1, np.float32)), _f(out))
    return out


def cos_sin_2pi(v):
    v = np.ascontiguousarray(v, np.float32)
    out = np.zeros((v.size, 2), np.float32)
    lib().oracle_samples(2, 0, 0, 0, v.size, _f(v), _f(out))
    return out


def log_u(v):
    """LogU (ConstantMedium's ln of a uniform; shared with the kernel's log_u)."""
    v = np.ascontiguousarray(v, np.float32)
    out = np.zeros(v.size, np.float32)
    lib().oracle_samples(3, 0, 0, 0, v.size, _f(v), _f(out))
    return out


def sin_f(v):
    """SinF (the marble texture's sin of a float; shared with the kernel's sin_f)."""
    v = np.ascontiguousarray(v, np.float32)
    out = np.zeros(v.size, np.float32)
    lib().oracle_samples(4, 0, 0, 0, v.size, _f(v), _f(out))
    return out


def quad_hit(q, u, v, o, d, tmin=0.001, tmax=3.4028234663852886e38):
    inp = np.array(list(q) + list(u) + list(v) + list(o) + list(d) + [tmin, tmax], np.float32)
    out = np.zeros(11, np.float32)
    lib().oracle_quad_hit(_f(inp), _f(out))
    return out


def sphere_hit(center, disp, radius, o, d, time=0.0, tmin=0.001, tmax=3.4028234663852886e38):
    inp = np.array(list(center) + list(disp) + [radius] + list(o) + list(d) + [time, tmin, tmax], np.float32)
    out = np.zeros(9, np.float32)
    lib().oracle_sphere_hit(_f(inp), _f(out))
    return out


def aabb_hit(mn, mx, o, d, tmin=0.001, tmax=3.4028234663852886e38):
    inp = np.array(list(mn) + list(mx) + list(o) + list(d) + [tmin, tmax], np.float32)
    return bool(lib().oracle_aabb_hit(_f(inp)))


def transform(translation, rotation, scale):
    inp = np.array(list(translation) + list(rotation) + list(scale), np.float32)
    m = np.zeros(16, np.float32)
    inv = np.zeros(16, np.float32)
    lib().oracle_transform(_f(inp), _f(m), _f(inv))
    return m.reshape(4, 4), inv.reshape(4, 4)  # [column][row]
