#!/usr/bin/env python3
"""Launch-tail probe (diagnostic build with -DRT2_EXP_ENDTIME=1): per-wave start / first-idle / end
times of one render launch, 100 MHz ticks. Prints, per configuration, the launch span, how long the
chip ran after the first wave ran out of work (the tail), and the mean wave time spent after its
first idle lane.

  RT2_LIB=raytrace2_amd/lib/ablate/endtime.so python tools/tail_probe.py [ranks]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401
import raytrace2_amd as R  # noqa: E402


def probe(scene, w, h, spp, band=0, rank=0, world=1, work_split=None, max_depth=50):
    sc = R.Scene(os.path.join("scenes", scene), R.DEFAULT_SEED)
    tr = R.RayTracer(sc, 0)
    tr.SetSamplesPerPixel(spp)
    tr.max_depth = max_depth
    tr.OnResize((w, h))
    if world > 1:
        tr.set_partition(band, rank, world)
    if work_split is not None:
        tr.set_work_split(work_split)
    tr.Render(spp)
    tr.synchronize()  # warm
    tr.Reset()
    tr.reset_stats()
    tr.Render(spp)
    st = tr.stats()
    d = st["diag"]
    m = (1 << 64) - 1
    t0, t0max, idle_min, t_end, idle_sum, wave_sum, waves, idle_max = (d[0] ^ m, d[1], d[2] ^ m, d[3], d[4], d[5],
                                                                         d[6], d[7])
    out = {"scene": scene, "w": w, "h": h, "spp": spp, "world": world, "work_split": work_split, "max_depth": max_depth,
           "kernel_ms": round(st["kernel_ms"], 3), "waves": waves, "launch_shape": tr.last_launch(),
           "span_ms": (t_end - t0) / 1e5, "start_spread_ms": (t0max - t0) / 1e5,
           "first_idle_ms": (idle_min - t0) / 1e5, "last_idle_ms": (idle_max - t0) / 1e5,
           "tail_ms": (t_end - idle_min) / 1e5, "mean_wave_after_idle_ms": idle_sum / max(1, waves) / 1e5,
           "mean_wave_ms": wave_sum / max(1, waves) / 1e5, "grays_s": st["rays"] / st["kernel_ms"] / 1e6}
    tr.close()
    print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in out.items()}), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "ranks":  # the headline and its 8-way rank
        probe("cornell_box_original.json", 1024, 1024, 1000)
        probe("cornell_box_original.json", 1024, 1024, 1000, band=2, rank=0, world=8)
        sys.exit(0)
    probe("cornell_box_original.json", 1024, 1024, 1000)
    probe("cornell_box_original.json", 1024, 1024, 125)
    probe("cornell_box_original.json", 1024, 1024, 1000, band=16, rank=0, world=8)
    probe("cornell_box_original.json", 1024, 1024, 125, work_split=16)
    probe("cornell_box_original.json", 1024, 1024, 125, work_split=256)
    probe("cornell_box_original.json", 1024, 1024, 125, max_depth=10)
    probe("cornell_box_original.json", 1024, 1024, 1000, max_depth=10)
