#!/usr/bin/env python3
"""Re-derive the roofline fields of a configs.jsonl (tools/bench_configs.sh) whose lines were run before
the PMC profiles of the same kernel build were committed (their `roofline.profile_stale` is true):
for every such line, the committed profile with the line's workload, partition and kernel sha gives
the VALU instructions and HBM bytes per ray, applied to the line's own rays per launch and HIP-event
launch time exactly as bench.py roofline_for does. Lines without a matching profile are left alone.
  python tools/configs_reroof.py profiles/r03_configs.jsonl"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import HBM_PEAK_GBS, VALU_PEAK_TLANE_OPS, find_profile  # noqa: E402

path = sys.argv[1]
out = []
for line in open(path):
    d = json.loads(line)
    b = d.get("bench") or {}
    r = b.get("roofline") or {}
    if r.get("profile_stale"):
        key = {"workload": b["config"]["workload"], "partition": b["config"]["partition"],
               "kernel_sha": b["detail"]["kernel_sha"]}
        src, prof, stale = find_profile(key)
        if prof and not stale:
            pr = prof["per_ray"]
            launch_s = r["avg_launch_ms"] / 1e3
            # (frac is §8(d)'s useful-flop fraction, computed live by the bench; only the profile's
            # issue and traffic companions are filled in here)
            r["valu_issue_tlane_ops"] = round(pr["valu_insts"] * r["rays_per_launch"] * 64 / launch_s / 1e12, 3)
            r["valu_issue_frac"] = round(r["valu_issue_tlane_ops"] / VALU_PEAK_TLANE_OPS, 4)
            r["valu_insts_per_ray"] = round(pr["valu_insts"], 3)
            r["salu_insts_per_ray"] = round(pr.get("salu_insts", 0.0), 3)
            if pr.get("hbm_bytes") is not None:
                r["traffic"] = int(pr["hbm_bytes"] * r["rays_per_launch"])
                r["hbm_frac"] = round(r["traffic"] / launch_s / 1e9 / HBM_PEAK_GBS, 4)
            r["profile"], r["profile_stale"], r["profile_kernel_sha"] = src, False, key["kernel_sha"]
            r["recomputed"] = "after the run, from the committed profile of the same kernel build"
            print(f"{d['config']}: valu_issue_frac {r['valu_issue_frac']} from {src}")
    out.append(json.dumps(d))
open(path, "w").write("\n".join(out) + "\n")
