"""ctypes binding of include/rt2.h (lib/librt2.so). No fallback: if the library is missing or fails
to load, importing raytrace2_amd raises."""
from __future__ import annotations

import ctypes
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RT2_LIB") or os.path.join(_HERE, "lib", "librt2.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "rt2.h")

RT2_OK = 0
RT2_ERR_INVALID = -1
RT2_ERR_IO = -2
RT2_ERR_SCENE = -3
RT2_ERR_HIP = -4
UNIQUE_ID_BYTES = 128  # RT2_UNIQUE_ID_BYTES


class Rt2Error(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"rt2 error {code}: {msg}")
        self.code = code


class SceneInfo(ctypes.Structure):
    _fields_ = [("dims_x", ctypes.c_int), ("dims_y", ctypes.c_int),
                ("n_materials", ctypes.c_int), ("n_textures", ctypes.c_int),
                ("n_primitives", ctypes.c_int), ("n_top_nodes", ctypes.c_int),
                ("background", ctypes.c_float * 3), ("legacy_schema", ctypes.c_int),
                ("bvh_nodes", ctypes.c_int), ("quads", ctypes.c_int), ("spheres", ctypes.c_int),
                ("lists", ctypes.c_int), ("xforms", ctypes.c_int), ("media", ctypes.c_int),
                ("max_stack", ctypes.c_int), ("bvh_depth", ctypes.c_int), ("node_bytes", ctypes.c_uint64),
                ("acc_lists", ctypes.c_int), ("acc_nodes", ctypes.c_int), ("linear_steps", ctypes.c_int),
                ("origins_bounded", ctypes.c_int), ("box_steps", ctypes.c_int)]


class CameraDesc(ctypes.Structure):
    _fields_ = [("center", ctypes.c_float * 3), ("look_at", ctypes.c_float * 3),
                ("view_up", ctypes.c_float * 3), ("vfov", ctypes.c_float),
                ("defocus_angle", ctypes.c_float), ("focus_distance", ctypes.c_float)]


class AppSettings(ctypes.Structure):
    _fields_ = [("render_once", ctypes.c_int), ("save_after_render_once", ctypes.c_int),
                ("num_samples", ctypes.c_int64), ("max_depth", ctypes.c_int64),
                ("render_window", ctypes.c_int)]


class PartPlan(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("device", "rank", "world", "band_h", "local_rows", "rows_max")]


class Stats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in
                ("rays", "paths", "bvh_tests", "quad_tests", "sphere_tests", "xform_visits",
                 "medium_tests", "list_visits", "overflow", "launches")] + [("kernel_ms", ctypes.c_double),
                                                                           ("stamps", ctypes.c_uint64 * 4),
                                                                           ("diag", ctypes.c_uint64 * 8),
                                                                           ("gathers", ctypes.c_uint64),
                                                                           ("gather_ms", ctypes.c_double),
                                                                           ("enqueue_ms", ctypes.c_double),
                                                                           ("readbacks", ctypes.c_uint64),
                                                                           ("readback_ms", ctypes.c_double),
                                                                           ("host_waits", ctypes.c_uint64),
                                                                           ("launch_ms_sum", ctypes.c_double),
                                                                           ("sample_buffer_bytes", ctypes.c_uint64),
                                                                           ("device_bytes_peak", ctypes.c_uint64),
                                                                           ("box_tests", ctypes.c_uint64),
                                                                           ("box_certified", ctypes.c_uint64),
                                                                           ("box_wave_visits", ctypes.c_uint64),
                                                                           ("box_wave_runs", ctypes.c_uint64)]

    def as_dict(self):
        d = {n: (getattr(self, n) if n.endswith("_ms") else int(getattr(self, n))) for n, _ in self._fields_
             if n not in ("stamps", "diag")}
        d["stamps"] = [int(x) for x in self.stamps]
        d["diag"] = [int(x) for x in self.diag]
        return d


def declared_symbols(header: str = HEADER_PATH):
    """Every RT2_API function name declared in include/rt2.h."""
    txt = open(header).read()
    return re.findall(r"RT2_API\s+[\w\s\*]+?\b(rt2_\w+)\s*\(", txt)


def _load():
    # One HIP runtime per process: torch's libraries load torch/lib/libamdhip64.so by the name
    # "libamdhip64.so"; librt2 asks for the SONAME libamdhip64.so.7, which the dynamic linker then
    # resolves to that same already-loaded copy. Loading librt2 first would pull in
    # /opt/rocm/lib's runtime and torch would add its own beside it.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"raytrace2_amd: {LIB_PATH} is missing — run `python -c 'import __graft_entry__ as g; "
                          f"g.build()'` (or make -C raytrace2_amd/csrc); there is no CPU fallback")
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, i64, u64, f32 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_uint64, ctypes.c_float
    fp = ctypes.POINTER(ctypes.c_float)
    pp = ctypes.POINTER(ctypes.c_void_p)
    sig = {
        "rt2_last_error": (ctypes.c_char_p, []),
        "rt2_version": (ctypes.c_char_p, []),
        "rt2_scene_load": (i32, [ctypes.c_char_p, u64, pp]),
        "rt2_scene_free": (None, [vp]),
        "rt2_scene_get_info": (i32, [vp, ctypes.POINTER(SceneInfo)]),
        "rt2_scene_materials": (i32, [vp, fp, i32]),
        "rt2_scene_textures": (i32, [vp, fp, i32]),
        "rt2_scene_perlin": (i32, [vp, i32, fp, ctypes.POINTER(ctypes.c_int)]),
        "rt2_scene_get_camera": (i32, [vp, ctypes.POINTER(CameraDesc)]),
        "rt2_scene_set_camera": (i32, [vp, ctypes.POINTER(CameraDesc)]),
        "rt2_camera_params": (i32, [vp, i32, i32, i32, fp]),
        "rt2_camera_load": (i32, [ctypes.c_char_p, ctypes.POINTER(CameraDesc)]),
        "rt2_camera_write": (i32, [ctypes.POINTER(CameraDesc), ctypes.c_char_p]),
        "rt2_settings_load": (i32, [ctypes.c_char_p, ctypes.POINTER(AppSettings)]),
        "rt2_tracer_create": (i32, [vp, i32, pp]),
        "rt2_tracer_destroy": (None, [vp]),
        "rt2_tracer_set_stream": (i32, [vp, vp]),
        "rt2_tracer_set_max_depth": (i32, [vp, i32]),
        "rt2_tracer_set_samples_per_pixel": (i32, [vp, i32]),
        "rt2_tracer_set_seed": (i32, [vp, u64]),
        "rt2_tracer_set_partition": (i32, [vp, i32, i32, i32]),
        "rt2_tracer_set_launch_frames": (i32, [vp, i32]),
        "rt2_tracer_set_lazy_frames": (i32, [vp, i32]),
        "rt2_tracer_flush": (i32, [vp]),
        "rt2_tracer_set_work_split": (i32, [vp, i32]),
        "rt2_tracer_set_sample_budget": (i32, [vp, u64]),
        "rt2_tracer_set_batch_max": (i32, [vp, i32]),
        "rt2_tracer_pixels_async": (i32, [vp, ctypes.POINTER(ctypes.c_uint8)]),
        "rt2_tracer_query": (i32, [vp]),
        "rt2_host_alloc": (i32, [ctypes.c_size_t, ctypes.POINTER(vp)]),
        "rt2_host_free": (None, [vp]),
        "rt2_tracer_last_launch": (i32, [vp, ctypes.POINTER(i32), ctypes.POINTER(i32), ctypes.POINTER(i32)]),
        "rt2_tracer_on_resize": (i32, [vp, i32, i32]),
        "rt2_tracer_reset": (i32, [vp]),
        "rt2_tracer_update": (i32, [vp]),
        "rt2_tracer_render": (i32, [vp, i32]),
        "rt2_tracer_synchronize": (i32, [vp]),
        "rt2_tracer_frame_idx": (i64, [vp]),
        "rt2_tracer_dims": (i32, [vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
        "rt2_tracer_local_rows": (i32, [vp]),
        "rt2_tracer_non_converted_pixels": (i32, [vp, fp]),
        "rt2_tracer_accumulation": (i32, [vp, fp]),
        "rt2_tracer_pixels": (i32, [vp, ctypes.POINTER(ctypes.c_uint8)]),
        "rt2_tracer_copy_accum_device": (i32, [vp, vp, vp]),
        "rt2_tracer_enable_ray_counts": (i32, [vp, i32]),
        "rt2_tracer_ray_counts": (i32, [vp, ctypes.POINTER(ctypes.c_uint32)]),
        "rt2_tracer_enable_stats": (i32, [vp, i32]),
        "rt2_tracer_get_stats": (i32, [vp, ctypes.POINTER(Stats)]),
        "rt2_tracer_part_stats": (i32, [vp, i32, ctypes.POINTER(Stats)]),
        "rt2_multi_plan": (i32, [i32, ctypes.POINTER(ctypes.c_int), i32, i32, i32, ctypes.POINTER(PartPlan),
                                 ctypes.POINTER(ctypes.c_int)]),
        "rt2_tracer_image_non_converted_pixels_async": (i32, [vp, vp]),
        "rt2_tracer_reset_stats": (i32, [vp]),
        "rt2_write_image": (i32, [fp, i32, i32, ctypes.c_char_p, i32]),
        "rt2_tracer_set_camera": (i32, [vp, ctypes.POINTER(CameraDesc)]),
        "rt2_tracer_get_camera": (i32, [vp, ctypes.POINTER(CameraDesc)]),
        "rt2_tracer_create_multi": (i32, [vp, i32, ctypes.POINTER(ctypes.c_int), i32, pp]),
        "rt2_tracer_n_gpus": (i32, [vp]),
        "rt2_comm_unique_id": (i32, [ctypes.POINTER(ctypes.c_uint8), ctypes.c_size_t]),
        "rt2_tracer_join": (i32, [vp, ctypes.POINTER(ctypes.c_uint8), i32, i32, i32]),
        "rt2_tracer_gather": (i32, [vp]),
        "rt2_tracer_image_accumulation": (i32, [vp, fp]),
        "rt2_tracer_image_non_converted_pixels": (i32, [vp, fp]),
        "rt2_tracer_image_pixels": (i32, [vp, ctypes.POINTER(ctypes.c_uint8)]),
        "rt2_selftest": (i32, [i32, i32, u64, u64, ctypes.POINTER(u64), ctypes.POINTER(u64)]),
        "rt2_band_rows_max": (i32, [i32, i32, i32]),
        "rt2_deinterleave_host": (i32, [fp, fp, i32, i32, i32, i32, i32, i32]),
        "rt2_runtime_info": (i32, [ctypes.c_char_p, ctypes.c_size_t]),
    }
    # RT2_ALLOW_OLD_LIB=1 (tools/ A/B runs of earlier builds only): entry points the older library lacks
    # are left out; otherwise a library that does not export every entry point is a load error
    allow_old = os.environ.get("RT2_ALLOW_OLD_LIB") == "1"
    missing = [name for name in sig if not hasattr(L, name)]
    if missing and not allow_old:
        raise ImportError(f"raytrace2_amd: {LIB_PATH} does not export {missing} (a stale build? rebuild with "
                          f"make -C raytrace2_amd/csrc)")
    for name, (res, args) in sig.items():
        if name in missing:
            continue
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    del f32
    return L


lib = _load()


def check(rc: int):
    if rc < 0:
        raise Rt2Error(rc, lib.rt2_last_error().decode(errors="replace"))
    return rc


def selftest(which: int, n: int, seed: int = 1, device: int = 0):
    """Kernel arithmetic self-test (rt2_selftest): returns (mismatches, inputs checked)."""
    bad, checked = ctypes.c_uint64(0), ctypes.c_uint64(0)
    check(lib.rt2_selftest(device, which, n, seed, ctypes.byref(bad), ctypes.byref(checked)))
    return bad.value, checked.value


def multi_plan(n_gpus: int, devices=None, band_h: int = 0, width: int = 0, height: int = 0):
    """rt2_multi_plan: rt2_tracer_create_multi's argument checks and per-GPU partition, on the host
    (no GPU, no RCCL). Returns (list of part dicts, loopback)."""
    if devices is not None and len(devices) != n_gpus:
        raise ValueError(f"multi_plan: {len(devices)} device ids for n_gpus = {n_gpus}")
    plans = (PartPlan * max(1, n_gpus))()
    devs = (ctypes.c_int * len(devices))(*devices) if devices is not None else None
    lb = ctypes.c_int(0)
    check(lib.rt2_multi_plan(n_gpus, devs, band_h, width, height, plans, ctypes.byref(lb)))
    return [{f: getattr(plans[i], f) for f, _ in PartPlan._fields_} for i in range(n_gpus)], bool(lb.value)


def runtime_info() -> str:
    """rt2_runtime_info: the RCCL (version, path) and HIP runtime library this process runs."""
    buf = ctypes.create_string_buffer(1024)
    check(lib.rt2_runtime_info(buf, len(buf)))
    return buf.value.decode(errors="replace")
