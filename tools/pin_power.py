#!/usr/bin/env python3
"""Power of the reference pins (tests/test_reference_pin.py): the same metrics computed for the
faithful restatement and for controls that each REMOVE one of the reference's quirks
(oracle.oracle.CTL_*: world-space t from transformed children, a single test of span-1 leaves,
+inf for kInfinity). A quirk is "pinned by the screenshot" when its control fails a check the
faithful oracle passes (the test's own tolerances, none tuned here), else "parity unpinned".

  python tools/pin_power.py [out.json]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import scene_path  # noqa: E402
from oracle.oracle import CTL_INF, CTL_SINGLE_LEAF, CTL_WORLD_T, OracleScene, controls  # noqa: E402
from test_reference_pin import encode_blocks  # noqa: E402

CONTROLS = {"faithful": 0, "world_space_t (Transform.cpp:82)": CTL_WORLD_T,
            "single_test_span1_leaf (BVH.cpp:18-20)": CTL_SINGLE_LEAF, "inf_not_flt_max (Defs.hpp:17)": CTL_INF}


def cornell_metrics(mask):
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "cornell_box_screenshot_blocks.json")))
    ref = np.array(g["blocks"])
    n, spp = ref.shape[0], 400
    with controls(mask):
        acc, _, cnt = OracleScene(scene_path("cornell_box_original")).render(5 * n, 5 * n, spp, spp)
    d = encode_blocks(acc, spp, n) - ref
    m = {"mean_abs": float(np.abs(d).mean()), "bias": float(d.mean()), "max_abs": float(np.abs(d).max()),
         "rays": cnt["rays"]}
    m["passes"] = m["mean_abs"] < 0.025 and abs(m["bias"]) < 0.02 and m["max_abs"] < 0.12
    return m


def book2_metrics(mask):
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "final_scene2_screenshot_blocks.json")))
    ref = np.array(g["blocks"])
    n, spp = ref.shape[0], 32
    with controls(mask):
        acc, _, cnt = OracleScene(scene_path("book2_final_scene_10000_samples")).render(5 * n, 5 * n, spp, spp,
                                                                                      forward=True)
    b = encode_blocks(acc, spp, n)
    m = {"corr": float(np.corrcoef(b.ravel(), ref.ravel())[0, 1]), "bias": float((b - ref).mean()),
         "mean_abs": float(np.abs(b - ref).mean()), "rays": cnt["rays"]}
    m["passes"] = m["corr"] > 0.9 and abs(m["bias"]) < 0.03 and m["mean_abs"] < 0.07
    return m


def main():
    out = {}
    for name, mask in CONTROLS.items():
        out[name] = {"cornell_box.png": cornell_metrics(mask), "final_scene2.png": book2_metrics(mask)}
        print(name, json.dumps(out[name]), flush=True)
    for name, r in out.items():
        if name == "faithful":
            continue
        caught = [k for k, v in r.items() if not v["passes"]]
        r["verdict"] = ("pinned by the screenshot (" + ", ".join(caught) + ")") if caught else "parity unpinned"
    path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "r03_pin_power.json")
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps({k: v.get("verdict") for k, v in out.items()}))


if __name__ == "__main__":
    main()
