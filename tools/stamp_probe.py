#!/usr/bin/env python3
"""Per-section time split of the render loop (diagnostic build -DRT2_EXP_STAMPS=1, via RT2_LIB):
s_memtime sums over waves for work fetch, trace, shade and finish, as fractions, plus Mray/s.

  RT2_LIB=raytrace2_amd/lib/ablate/stamps.so python tools/stamp_probe.py <scene> <W>x<H> <spp> <frames>
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401
import raytrace2_amd as R  # noqa: E402

scene, dims, spp, frames = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
w, h = (int(v) for v in dims.split("x"))
sc = R.Scene(scene, R.DEFAULT_SEED)
tr = R.RayTracer(sc, 0)
tr.SetSamplesPerPixel(spp)
tr.OnResize((w, h))
tr.Render(frames)
tr.synchronize()
tr.Reset()
tr.reset_stats()
tr.Render(frames)
st = tr.stats()
s = st["stamps"]
tot = max(1, sum(s))
print(json.dumps({"scene": os.path.basename(scene), "mray_s": round(st["rays"] / st["kernel_ms"] / 1e3, 1),
                  "kernel_ms": round(st["kernel_ms"], 2),
                  "split": {k: round(v / tot, 4) for k, v in zip(("fetch", "trace", "shade", "finish"), s)}}))
tr.close()
