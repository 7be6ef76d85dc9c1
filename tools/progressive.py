#!/usr/bin/env python3
"""Progressive-display throughput on one GPU, Cornell 1024^2 by default.

Modes, each over the same F frames from Reset():
  reference_loop : Update() + Pixels() per frame (App.cpp:176-242 call pattern: one sample per
                   pixel and one readback per displayed frame)
  update_eager   : Update() per frame, each launched at once, no readback
  update_only    : Update() per frame, no readback (frames queued and launched together)
  progressive    : raytrace2_amd.progressive.ProgressiveLoop (frames per tick adapted to a
                   16 ms budget, one pinned Pixels() readback per tick)
  batch          : one Render(F)
Prints one JSON line per mode: Mray/s, frames/s, display ticks/s."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402,F401

import raytrace2_amd as R  # noqa: E402
from raytrace2_amd.progressive import ProgressiveLoop  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scene", default="cornell_box_original.json")
ap.add_argument("--size", type=int, default=1024)
ap.add_argument("--frames", type=int, default=1000)
ap.add_argument("--budget-ms", type=float, default=16.0)
a = ap.parse_args()

sc = R.Scene(os.path.join(ROOT, "scenes", a.scene), R.DEFAULT_SEED)
tr = R.RayTracer(sc, 0)
tr.SetSamplesPerPixel(a.frames)
tr.OnResize((a.size, a.size))


def timed(fn):
    tr.Reset()
    tr.synchronize()
    tr.reset_stats()
    t0 = time.perf_counter()
    ticks = fn()
    tr.synchronize()
    dt = time.perf_counter() - t0
    st = tr.stats()
    return dt, st["rays"], ticks, st["kernel_ms"], st["launches"]


def reference_loop():
    for _ in range(a.frames):
        tr.Update(sc)
        tr.Pixels()
    return a.frames


def update_only():  # App::Run headless pattern: Update() x F, then one readback (queued frames)
    for _ in range(a.frames):
        tr.Update(sc)
    return 0


def update_eager():  # the same with every Update() launched at once (rt2_tracer_set_lazy_frames(0))
    tr.set_lazy_frames(0)
    for _ in range(a.frames):
        tr.Update(sc)
    tr.set_lazy_frames(4096)
    return 0


def progressive():
    loop = ProgressiveLoop(tr, a.frames, budget_ms=a.budget_ms)
    loop.run()
    loop.close()
    return loop.ticks


def batch():
    tr.Render(a.frames)
    return 0


timed(batch)  # warm-up (sample buffer, code objects)
for name, fn in (("reference_loop", reference_loop), ("update_eager", update_eager), ("update_only", update_only),
                 ("progressive", progressive),
                 ("batch", batch)):
    dt, rays, ticks, kms, launches = timed(fn)
    print(json.dumps({"mode": name, "scene": a.scene, "size": a.size, "frames": a.frames, "seconds": round(dt, 4),
                      "render_kernel_ms": round(kms, 2), "launches": launches,
                      "mray_s": round(rays / dt / 1e6, 1), "frames_per_s": round(a.frames / dt, 1),
                      "display_ticks_per_s": round(ticks / dt, 1) if ticks else None}), flush=True)
tr.close()
