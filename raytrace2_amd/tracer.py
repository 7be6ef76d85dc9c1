"""Python mirror of the reference's hot-path interface, over the C ABI (include/rt2.h).

Names follow the reference so callers read the same:
  serialize::SceneLoader::LoadScene   (src/Serialize.hpp:21-31)  -> SceneLoader().LoadScene(path)
  serialize::LoadCamera / WriteCamera (src/Serialize.hpp:34-35)  -> LoadCamera(path), WriteCamera(cam, path)
  serialize::LoadAppSettings          (src/Serialize.hpp:33)     -> LoadAppSettings(path)
  cpu::RayTracer                      (src/cpu_raytrace/RayTracer.hpp:15-42) -> RayTracer
  util::WriteImage                    (src/Util.hpp:11-12)       -> WriteImage(pixels, w, h, path)
Everything here is host plumbing; the per-pixel render loop runs in the gfx950 kernel.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np

from ._native import AppSettings as _AppSettings
from ._native import UNIQUE_ID_BYTES, CameraDesc, SceneInfo, Stats, check, lib

DEFAULT_SEED = 0x5EED2024


def _fp(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


@dataclass
class Camera:
    """Camera parameters that the scene files carry (Camera.hpp:113-123; Serialize.cpp:32-38)."""
    center: Tuple[float, float, float] = (0.0, 0.0, 1.0)
    look_at: Tuple[float, float, float] = (0.0, 0.0, 0.0)
    view_up: Tuple[float, float, float] = (0.0, 1.0, 0.0)
    vfov: float = 90.0
    defocus_angle: float = 0.0
    focus_distance: float = 1.0

    @classmethod
    def _from_desc(cls, d: CameraDesc) -> "Camera":
        return cls(tuple(d.center), tuple(d.look_at), tuple(d.view_up), d.vfov, d.defocus_angle, d.focus_distance)

    def _desc(self) -> CameraDesc:
        d = CameraDesc()
        d.center[:] = self.center
        d.look_at[:] = self.look_at
        d.view_up[:] = self.view_up
        d.vfov, d.defocus_angle, d.focus_distance = self.vfov, self.defocus_angle, self.focus_distance
        return d


@dataclass
class Settings:
    """AppSettings (src/Settings.hpp:5-11)."""
    render_once: bool = False
    save_after_render_once: bool = False
    num_samples: int = 1
    max_depth: int = 50
    render_window: bool = True


def LoadCamera(path: str) -> Camera:
    d = CameraDesc()
    check(lib.rt2_camera_load(path.encode(), ctypes.byref(d)))
    return Camera._from_desc(d)


def WriteCamera(cam: Camera, path: str) -> None:
    d = cam._desc()
    check(lib.rt2_camera_write(ctypes.byref(d), path.encode()))


def LoadAppSettings(path: str) -> Settings:
    s = _AppSettings()
    check(lib.rt2_settings_load(path.encode(), ctypes.byref(s)))
    return Settings(bool(s.render_once), bool(s.save_after_render_once), int(s.num_samples), int(s.max_depth),
                    bool(s.render_window))


def WriteImage(pixels: np.ndarray, width: int, height: int, path: str, png: bool = True) -> None:
    """util::WriteImage: `pixels` float32 (height, width, 3), row 0 = bottom row."""
    p = np.ascontiguousarray(pixels, dtype=np.float32)
    if p.size != width * height * 3:
        raise ValueError("pixels must hold width*height*3 floats")
    check(lib.rt2_write_image(_fp(p), width, height, path.encode(), 1 if png else 0))


class Scene:
    """A loaded + compiled scene (cpu::Scene after App.cpp:126 wraps the list in one BVHNode)."""

    def __init__(self, path: str, seed: int = DEFAULT_SEED):
        h = ctypes.c_void_p()
        check(lib.rt2_scene_load(path.encode(), seed, ctypes.byref(h)))
        self._h = h
        self.path = path
        self.seed = seed

    def __del__(self):
        if getattr(self, "_h", None) and self._h.value:
            lib.rt2_scene_free(self._h)
            self._h = None

    def info(self) -> SceneInfo:
        s = SceneInfo()
        check(lib.rt2_scene_get_info(self._h, ctypes.byref(s)))
        return s

    @property
    def dims(self) -> Tuple[int, int]:
        i = self.info()
        return i.dims_x, i.dims_y

    @property
    def background_color(self) -> Tuple[float, float, float]:
        return tuple(self.info().background)

    def materials(self) -> np.ndarray:
        n = check(lib.rt2_scene_materials(self._h, None, 0))
        out = np.zeros((max(n, 1), 8), np.float32)
        check(lib.rt2_scene_materials(self._h, _fp(out), n))
        return out[:n]

    def textures(self) -> np.ndarray:
        n = check(lib.rt2_scene_textures(self._h, None, 0))
        out = np.zeros((max(n, 1), 8), np.float32)
        check(lib.rt2_scene_textures(self._h, _fp(out), n))
        return out[:n]

    def perlin(self, tex: int):
        pc = check(lib.rt2_scene_perlin(self._h, tex, None, None))
        vec = np.zeros((pc, 3), np.float32)
        perm = np.zeros(3 * pc, np.int32)
        check(lib.rt2_scene_perlin(self._h, tex, _fp(vec), perm.ctypes.data_as(ctypes.POINTER(ctypes.c_int))))
        return vec, perm.reshape(3, pc)

    @property
    def cam(self) -> Camera:
        d = CameraDesc()
        check(lib.rt2_scene_get_camera(self._h, ctypes.byref(d)))
        return Camera._from_desc(d)

    @cam.setter
    def cam(self, c: Camera) -> None:
        d = c._desc()
        check(lib.rt2_scene_set_camera(self._h, ctypes.byref(d)))

    def camera_params(self, w: int, h: int, spp: int) -> np.ndarray:
        out = np.zeros(21, np.float32)
        check(lib.rt2_camera_params(self._h, w, h, spp, _fp(out)))
        return out


class SceneLoader:
    """serialize::SceneLoader: LoadScene returns a Scene, or None (std::nullopt) with `.error` set."""

    def __init__(self, seed: int = DEFAULT_SEED):
        self.seed = seed
        self.error: Optional[str] = None

    def LoadScene(self, filepath: str) -> Optional[Scene]:
        try:
            self.error = None
            return Scene(filepath, self.seed)
        except RuntimeError as e:
            self.error = str(e)
            return None


def band_rank(band: int, world: int) -> int:
    """Rank owning row band `band` (rt2_layout.h BandRank): period p = band // world, phase
    q = band % world, rank (q + p) % world — one band per period per rank, phases rotating."""
    return (band % world + band // world) % world


def local_rows(height: int, band_h: int, rank: int, world: int) -> List[int]:
    """Global rows owned by `rank` under the interleaved row-band partition, in increasing y."""
    bh = band_h if band_h > 0 else height
    return [y for y in range(height) if band_rank(y // bh, world) == rank]


def assemble_bands(parts: Sequence[np.ndarray], height: int, band_h: int) -> np.ndarray:
    """Inverse of the partition: parts[r] holds rank r's local rows (n_r, W, C) in increasing y."""
    world = len(parts)
    w = parts[0].shape[1]
    out = np.zeros((height, w) + parts[0].shape[2:], parts[0].dtype)
    for r, p in enumerate(parts):
        rows = local_rows(height, band_h, r, world)
        out[rows] = p[:len(rows)]
    return out


def comm_unique_id() -> bytes:
    """rt2_comm_unique_id: the RCCL id rank 0 makes and the caller broadcasts before join()."""
    buf = (ctypes.c_uint8 * UNIQUE_ID_BYTES)()
    check(lib.rt2_comm_unique_id(buf, UNIQUE_ID_BYTES))
    return bytes(buf)


class RayTracer:
    """cpu::RayTracer (RayTracer.hpp:15-42) on one or more MI355X GPUs.

    Update() renders one frame (one sample per pixel) exactly like RayTracer::Update; Render(n) is
    n Update() calls in one kernel launch. Image buffers hold this tracer's local rows (all rows
    unless set_partition()/join() was called). With `n_gpus` or `devices` the tracer renders on
    several GPUs of this process (rt2_tracer_create_multi: interleaved row bands, RCCL gather) and
    its readbacks return the full image.

    `camera`, like the reference's borrowed `Camera* camera` (RayTracer.hpp:31), is read at every
    Update()/Render() when set: a moved camera applies from the next frame (RayTracer.cpp:56).
    """

    def __init__(self, scene: Scene, device: int = 0, *, n_gpus: Optional[int] = None,
                 devices: Optional[Sequence[int]] = None, band_h: int = 0):
        h = ctypes.c_void_p()
        if n_gpus is None and devices is None:
            check(lib.rt2_tracer_create(scene._h, device, ctypes.byref(h)))
            self.devices = [device]
        else:
            devs = list(devices) if devices is not None else list(range(device, device + int(n_gpus)))
            arr = (ctypes.c_int * len(devs))(*devs)
            check(lib.rt2_tracer_create_multi(scene._h, len(devs), arr, int(band_h), ctypes.byref(h)))
            self.devices = devs
        self._h = h
        self.device = self.devices[0]
        self._max_depth = 50
        self.camera: Optional[Camera] = None

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            lib.rt2_tracer_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    # -- reference members ------------------------------------------------------------------
    @property
    def max_depth(self) -> int:
        return self._max_depth

    @max_depth.setter
    def max_depth(self, d: int) -> None:
        check(lib.rt2_tracer_set_max_depth(self._h, int(d)))
        self._max_depth = int(d)

    def SetSamplesPerPixel(self, spp: int) -> None:
        """scene.cam.SetSamplesPerPixel(settings.num_samples) (App.cpp:129): fixes the strata."""
        check(lib.rt2_tracer_set_samples_per_pixel(self._h, int(spp)))

    def OnResize(self, dims: Tuple[int, int]) -> None:
        check(lib.rt2_tracer_on_resize(self._h, int(dims[0]), int(dims[1])))

    def Reset(self) -> None:
        check(lib.rt2_tracer_reset(self._h))

    def _push_camera(self) -> None:
        if self.camera is not None:
            self.set_camera(self.camera)

    def Update(self, scene: Optional[Scene] = None) -> None:
        self._push_camera()  # camera->Update() (RayTracer.cpp:56)
        check(lib.rt2_tracer_update(self._h))

    def Render(self, n_frames: int) -> None:
        self._push_camera()
        check(lib.rt2_tracer_render(self._h, int(n_frames)))

    def FrameIdx(self) -> int:
        return int(lib.rt2_tracer_frame_idx(self._h))

    def Dims(self) -> Tuple[int, int]:
        w, h = ctypes.c_int(), ctypes.c_int()
        check(lib.rt2_tracer_dims(self._h, ctypes.byref(w), ctypes.byref(h)))
        return w.value, h.value

    def local_rows(self) -> int:
        return int(lib.rt2_tracer_local_rows(self._h))

    def NonConvertedPixels(self) -> np.ndarray:
        w, _ = self.Dims()
        out = np.zeros((self.local_rows(), w, 3), np.float32)
        check(lib.rt2_tracer_non_converted_pixels(self._h, _fp(out)))
        return out

    def Accumulation(self) -> np.ndarray:
        w, _ = self.Dims()
        out = np.zeros((self.local_rows(), w, 3), np.float32)
        check(lib.rt2_tracer_accumulation(self._h, _fp(out)))
        return out

    def Pixels(self) -> np.ndarray:
        w, _ = self.Dims()
        out = np.zeros((self.local_rows(), w, 4), np.uint8)
        check(lib.rt2_tracer_pixels(self._h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))))
        return out

    # -- MI355X extensions ------------------------------------------------------------------
    def set_camera(self, cam: Camera) -> None:
        """rt2_tracer_set_camera: the camera's setter fields for the next frames (queued frames
        keep the camera they were queued under; the accumulation is not reset)."""
        d = cam._desc()
        check(lib.rt2_tracer_set_camera(self._h, ctypes.byref(d)))

    def get_camera(self) -> Camera:
        d = CameraDesc()
        check(lib.rt2_tracer_get_camera(self._h, ctypes.byref(d)))
        return Camera._from_desc(d)

    def n_gpus(self) -> int:
        return int(check(lib.rt2_tracer_n_gpus(self._h)))

    def join(self, unique_id: bytes, world: int, rank: int, band_h: int = 0) -> None:
        """rt2_tracer_join: partition (band_h, rank, world) + this rank of an RCCL communicator."""
        buf = (ctypes.c_uint8 * UNIQUE_ID_BYTES).from_buffer_copy(unique_id[:UNIQUE_ID_BYTES])
        check(lib.rt2_tracer_join(self._h, buf, int(world), int(rank), int(band_h)))

    def gather(self) -> None:
        """rt2_tracer_gather: collective; the full image lands on rank 0 (enqueued, no wait)."""
        check(lib.rt2_tracer_gather(self._h))

    def image_accumulation(self) -> np.ndarray:
        w, h = self.Dims()
        out = np.zeros((h, w, 3), np.float32)
        check(lib.rt2_tracer_image_accumulation(self._h, _fp(out)))
        return out

    def image_non_converted_pixels(self) -> np.ndarray:
        w, h = self.Dims()
        out = np.zeros((h, w, 3), np.float32)
        check(lib.rt2_tracer_image_non_converted_pixels(self._h, _fp(out)))
        return out

    def image_pixels(self) -> np.ndarray:
        w, h = self.Dims()
        out = np.zeros((h, w, 4), np.uint8)
        check(lib.rt2_tracer_image_pixels(self._h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))))
        return out

    def set_seed(self, seed: int) -> None:
        check(lib.rt2_tracer_set_seed(self._h, int(seed)))

    def set_partition(self, band_h: int, rank: int, world: int) -> None:
        check(lib.rt2_tracer_set_partition(self._h, int(band_h), int(rank), int(world)))

    def set_launch_frames(self, n: int) -> None:
        check(lib.rt2_tracer_set_launch_frames(self._h, int(n)))

    def flush(self) -> None:
        """Launch the queued Update()/Render() frames now (does not wait for them)."""
        check(lib.rt2_tracer_flush(self._h))

    def query(self) -> int:
        """1 when every GPU has finished the work enqueued so far, 0 while some is still running
        (launches queued frames first, like flush(); never waits)."""
        r = lib.rt2_tracer_query(self._h)
        if r < 0:
            check(r)
        return r

    def set_lazy_frames(self, max_queued: int) -> None:
        check(lib.rt2_tracer_set_lazy_frames(self._h, int(max_queued)))

    def set_work_split(self, items_per_lane: int) -> None:
        check(lib.rt2_tracer_set_work_split(self._h, int(items_per_lane)))

    def set_sample_budget(self, nbytes: int) -> None:
        check(lib.rt2_tracer_set_sample_budget(self._h, int(nbytes)))

    def set_batch_max(self, items: int) -> None:
        check(lib.rt2_tracer_set_batch_max(self._h, int(items)))

    def last_launch(self) -> dict:
        g, c, v = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        check(lib.rt2_tracer_last_launch(self._h, ctypes.byref(g), ctypes.byref(c), ctypes.byref(v)))
        return {"grid": g.value, "chunk_frames": c.value, "variant": v.value}

    def set_stream(self, hip_stream_ptr: Optional[int]) -> None:
        check(lib.rt2_tracer_set_stream(self._h, ctypes.c_void_p(hip_stream_ptr or None)))

    def synchronize(self) -> None:
        check(lib.rt2_tracer_synchronize(self._h))

    def copy_accum_to(self, dst_ptr: int, stream_ptr: Optional[int] = None) -> None:
        check(lib.rt2_tracer_copy_accum_device(self._h, ctypes.c_void_p(dst_ptr), ctypes.c_void_p(stream_ptr or None)))

    def enable_ray_counts(self, on: bool = True) -> None:
        check(lib.rt2_tracer_enable_ray_counts(self._h, 1 if on else 0))

    def ray_counts(self) -> np.ndarray:
        w, _ = self.Dims()
        out = np.zeros((self.local_rows(), w), np.uint32)
        check(lib.rt2_tracer_ray_counts(self._h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))))
        return out

    def enable_stats(self, on: bool = True) -> None:
        check(lib.rt2_tracer_enable_stats(self._h, 1 if on else 0))

    def stats(self) -> dict:
        s = Stats()
        check(lib.rt2_tracer_get_stats(self._h, ctypes.byref(s)))
        return s.as_dict()

    def part_stats(self, part: int) -> dict:
        """Stats of GPU `part` of a multi-GPU tracer (rt2_tracer_part_stats)."""
        s = Stats()
        check(lib.rt2_tracer_part_stats(self._h, part, ctypes.byref(s)))
        return s.as_dict()

    def image_non_converted_pixels_async(self, out_ptr: int) -> None:
        """NonConvertedPixels of the gathered image into pinned host memory at out_ptr (rt2_host_alloc,
        height * width * 3 floats), enqueued; complete after synchronize() or query() == 1."""
        check(lib.rt2_tracer_image_non_converted_pixels_async(self._h, ctypes.c_void_p(out_ptr)))

    def reset_stats(self) -> None:
        check(lib.rt2_tracer_reset_stats(self._h))
