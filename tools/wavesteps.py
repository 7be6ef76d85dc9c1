"""Per-wave linear-traversal step counts (build with HIPFLAGS_EXTRA=-DRT2_EXP_WAVESTEPS=1; RT2_LIB=...).
Prints, per ray cast, lane-level record tests and wave-level steps (a wave executes the union of the
steps its lanes need)."""
import json
import sys

import torch  # noqa: F401  (one HIP runtime)

sys.path.insert(0, ".")
import raytrace2_amd as R  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "scenes/cornell_box_original.json"
w, h = (int(v) for v in (sys.argv[3] if len(sys.argv) > 3 else "1024x1024").split("x"))
spp, frames = (int(sys.argv[4]) if len(sys.argv) > 4 else 1000), int(sys.argv[2]) if len(sys.argv) > 2 else 16
sc = R.Scene(scene)
tr = R.RayTracer(sc, 0)
tr.SetSamplesPerPixel(spp)
if len(sys.argv) > 5:
    tr.max_depth = int(sys.argv[5])
tr.enable_stats(True)
tr.OnResize((w, h))
tr.Render(frames)
st = tr.stats()
d = st["diag"]
rays = st["rays"]
wtrace = max(d[0], 1)
out = {
    "scene": scene, "max_depth": tr.max_depth, "rays": rays,
    "lane_per_ray": {k: st[k] / rays for k in ("bvh_tests", "quad_tests", "sphere_tests", "xform_visits",
                                                "medium_tests", "list_visits")},
    "wave_trace_calls": d[0], "active_lanes_per_trace": d[7] / wtrace,
    "wave_per_trace": {"steps": d[1] / wtrace, "bvh": d[2] / wtrace, "quad_runs": d[3] / wtrace,
                       "spheres": d[4] / wtrace, "media": d[5] / wtrace, "min_search_extra_trips": d[6] / wtrace},
}
print(json.dumps(out, indent=1))
