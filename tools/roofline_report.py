#!/usr/bin/env python3
"""Summarise a tools/profile.sh run (gpurun_out/prof) into profiles/<tag>_*: the rocprofv3
kernel-stats CSV of the bench command and a JSON with per-launch PMC figures of the render
kernel. HBM traffic per launch follows MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are KiB
from the TCC EA request counters; on gfx950 FETCH_SIZE reads half the bytes of wide streaming
reads, so the corrected figure doubles it (the raw sum is kept beside it)."""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "gpurun_out", "prof")


def per_dispatch(path, kernel_sub="render_kernel"):
    rows = list(csv.DictReader(open(path)))
    agg = defaultdict(lambda: defaultdict(float))
    names, dur = {}, {}
    for r in rows:
        if kernel_sub in r["Kernel_Name"]:
            agg[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"]
            dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    return agg, names, dur


def main(tag):
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    stats = os.path.join(PROF, "trace", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(ROOT, "profiles", f"{tag}_kernel_stats.csv"))
    kst = {r["Name"]: r for r in csv.DictReader(open(stats))}
    render = {k: v for k, v in kst.items() if "render_kernel" in k and ", false>" in k}
    bench_line = [l for l in open(os.path.join(PROF, "trace.log")) if l.startswith("{")]
    summary = {"tag": tag, "bench_under_rocprof": json.loads(bench_line[-1]) if bench_line else None,
               "render_kernel_stats": {k: {"calls": int(v["Calls"]), "avg_ns": float(v["AverageNs"]),
                                           "total_ns": float(v["TotalDurationNs"])} for k, v in render.items()},
               "pmc": {}}
    for d in sorted(glob.glob(os.path.join(PROF, "pmc_*"))):
        f = os.path.join(d, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        agg, names, dur = per_dispatch(f)
        # the timed render launch: the longest dispatch of the non-stats kernel
        timed = [d for d in agg if ", false>" in names[d]]
        if not timed:
            continue
        disp = max(timed, key=lambda d: dur[d])
        for k, v in agg[disp].items():
            summary["pmc"][k] = v
        summary["pmc"].setdefault("dispatch_ms", {})[os.path.basename(d)] = dur[disp]
    p = summary["pmc"]
    if "FETCH_SIZE" in p and "WRITE_SIZE" in p:
        fetch, write = p["FETCH_SIZE"] * 1024, p["WRITE_SIZE"] * 1024
        summary["hbm_bytes_per_launch"] = {"fetch_raw": fetch, "write": write, "raw_sum": fetch + write,
                                           "corrected": 2 * fetch + write}
    json.dump(summary, open(os.path.join(ROOT, "profiles", f"{tag}_summary.json"), "w"), indent=1)
    print(json.dumps({k: summary[k] for k in summary if k != "bench_under_rocprof"}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
