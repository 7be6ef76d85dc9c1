#!/usr/bin/env python3
"""Box-level test counters (rt2_stats box_*) of a short counting render (DESIGN.md §4 "Box-level test"):
lanes tested at flagged MakeBox runs, the certified fraction, and the fraction of wave visits in which the
wave still ran the six faces for an uncertified lane.
  python tools/box_stats.py [scene.json] [width height spp frames]   (GPU)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401  (one HIP runtime: torch first)
import raytrace2_amd as R  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "book2_final_scene_10000_samples.json"
w, h, spp, frames = (int(x) for x in (sys.argv[2:6] if len(sys.argv) > 5 else (800, 800, 10000, 16)))
sc = R.Scene(os.path.join(ROOT, "scenes", scene), R.DEFAULT_SEED)
tr = R.RayTracer(sc, 0)
tr.SetSamplesPerPixel(spp)
tr.OnResize((w, h))
tr.enable_stats(True)
tr.Render(frames)
st = tr.stats()
tr.close()
out = {"scene": scene, "size": [w, h], "spp": spp, "frames": frames, "box_steps": sc.info().box_steps,
       "rays": st["rays"], "quad_tests": st["quad_tests"], "box_tests": st["box_tests"],
       "box_certified": st["box_certified"], "box_wave_visits": st["box_wave_visits"],
       "box_wave_runs": st["box_wave_runs"]}
if st["box_tests"]:
    out["certified_frac"] = round(st["box_certified"] / st["box_tests"], 5)
    out["lanes_per_wave_visit"] = round(st["box_tests"] / max(1, st["box_wave_visits"]), 2)
    out["wave_visits_running_six_faces_frac"] = round(st["box_wave_runs"] / max(1, st["box_wave_visits"]), 4)
print(json.dumps(out))
