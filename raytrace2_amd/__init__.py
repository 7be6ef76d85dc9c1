"""raytrace2_amd — MI355X (gfx950) replacement for the per-pixel Monte-Carlo render loop of
tonadr1022/Raytrace2 (src/cpu_raytrace), behind the reference's RayTracer / SceneLoader surface.

The compute path is lib/librt2.so (hand-written HIP kernel + C ABI, include/rt2.h). Importing this
package fails loudly when that library is missing; there is no CPU fallback.
"""
from ._native import Rt2Error, declared_symbols, lib  # noqa: F401
from .tracer import (DEFAULT_SEED, Camera, LoadAppSettings, LoadCamera, RayTracer, Scene,  # noqa: F401
                     SceneLoader, Settings, WriteCamera, WriteImage, assemble_bands, comm_unique_id,
                     local_rows)

__all__ = ["Camera", "LoadAppSettings", "LoadCamera", "RayTracer", "Scene", "SceneLoader", "Settings",
           "WriteCamera", "WriteImage", "assemble_bands", "comm_unique_id", "local_rows", "Rt2Error", "DEFAULT_SEED"]
