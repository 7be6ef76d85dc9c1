#!/usr/bin/env python3
"""The oracle's deliberate deviations (inverse-CDF sampling, LogU, double sin, explicit x^5) against
the reference's own sampling and libm calls (oracle control CTL_REF_MATH: rejection RandInUnitSphere /
RandInUnitDisk on the same Philox stream, std::log, std::sin(float), std::pow), at image level.

For each config: D1, D2 = default oracle at two seeds, C = reference-math oracle at a third seed.
  z_mean  = mean(C - D1) / (std(D1 - D2) / sqrt(N))     (difference of the image means in units of
            its sampling error; pixels are independent streams)
  r_mad   = median|C - D1| / median|D1 - D2|            (per-pixel noise distribution: a robust
            ratio, unmoved by the fireflies of book 2)
  r_var   = var(C - D1) / var(D1 - D2)                   (the same with the variance, heavy tailed)
  python3 tools/refmath_pin.py [--size 128 --spp 1024] > profiles/r04_refmath.json
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle.oracle import CTL_REF_MATH, OracleScene, controls  # noqa: E402

CONFIGS = [("C2", "cornell_box_original"), ("C4", "cornell_box_volume"), ("C5", "book2_final_scene_10000_samples")]
SEEDS = (0x11, 0x22, 0x33)


def render(name, size, spp, seed, mask, threads=0):
    with controls(mask):
        o = OracleScene(os.path.join(ROOT, "scenes", name + ".json"), 7)
        acc, _, cnt = o.render(size, size, spp, spp, seed=seed, threads=threads)
    return acc / np.float32(spp), cnt["rays"]


def compare(name, size, spp, threads=0):
    d1, r1 = render(name, size, spp, SEEDS[0], 0, threads)
    d2, r2 = render(name, size, spp, SEEDS[1], 0, threads)
    c, rc = render(name, size, spp, SEEDS[2], CTL_REF_MATH, threads)
    self_d, ref_d = (d1 - d2).astype(np.float64), (c - d1).astype(np.float64)
    n = self_d.size
    return {"z_mean": float(ref_d.mean() / (self_d.std() / np.sqrt(n))),
            "r_mad": float(np.median(np.abs(ref_d)) / np.median(np.abs(self_d))),
            "r_var": float(ref_d.var() / self_d.var()),
            "mean_default": float(d1.mean()), "mean_ref_math": float(c.mean()),
            "rays_per_sample": [r / (size * size * spp) for r in (r1, r2, rc)]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=128)
    ap.add_argument("--spp", type=int, default=1024)
    a = ap.parse_args()
    out = {"what": __doc__.strip().split("\n")[0], "size": a.size, "spp": a.spp, "seeds": SEEDS, "configs": {}}
    for tag, name in CONFIGS:
        out["configs"][tag] = {"scene": name, **compare(name, a.size, a.spp)}
        print(tag, out["configs"][tag], file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
