#!/usr/bin/env python3
"""Summarise a tools/profile.sh run (gpurun_out/prof_<name>) into profiles/<tag>_<name>_*:
the rocprofv3 kernel-stats CSV of the bench command and a JSON with the render kernel's PMC figures
per launch and per ray, keyed on the bench configuration (workload, partition) and the kernel build
(sha of its sources), which is what bench.py matches before it uses them.

HBM traffic follows MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are KiB from the TCC EA request
counters; on gfx950 FETCH_SIZE reads half the bytes of wide streaming reads, so the corrected figure
doubles it (the raw sum is kept beside it). The VALU issue fraction uses a wave64 VALU instruction =
2 SIMD cycles, 1024 SIMDs, and the clock from GRBM_GUI_ACTIVE / 8 XCDs / dispatch time.

  python tools/roofline_report.py <tag> <name>
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


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


def bench_line(log):
    lines = [l for l in open(log) if l.startswith("{")]
    return json.loads(lines[-1]) if lines else None


def main(tag, name):
    prof = os.path.join(ROOT, "gpurun_out", f"prof_{name}")
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    stats = os.path.join(prof, "trace", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(ROOT, "profiles", f"{tag}_{name}_kernel_stats.csv"))
    kst = {r["Name"]: r for r in csv.DictReader(open(stats))}
    render = {k: v for k, v in kst.items() if "render_kernel" in k and ", false>" in k}
    under = bench_line(os.path.join(prof, "trace.log"))
    summary = {"tag": tag, "name": name,
               "key": {"workload": under["config"]["workload"], "partition": under["config"]["partition"],
                       "kernel_sha": under["detail"]["kernel_sha"]},
               "bench_under_rocprof": under,
               "render_kernel_stats": {k: {"calls": int(v["Calls"]), "avg_ns": float(v["AverageNs"]),
                                           "total_ns": float(v["TotalDurationNs"])} for k, v in render.items()},
               "pmc": {}, "pmc_passes": {}}
    rays_per_launch = None
    for d in sorted(glob.glob(os.path.join(prof, "pmc_*"))):
        f = os.path.join(d, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        agg, names, dur = per_dispatch(f)
        # the product kernel's launches of the timed step (a step may be cut into several launches
        # by the sample-buffer budget: counters and durations are summed over all of them, and the
        # figures below are per average launch, like the bench's rays per launch)
        timed = [x for x in agg if ", false>" in names[x]]
        if not timed:
            continue
        line = bench_line(d + ".log")
        launches = max(1, line["detail"]["launches"])
        assert len(timed) == launches, (d, len(timed), launches)
        r = line["detail"]["rays"] / launches
        if rays_per_launch is None:
            rays_per_launch = r
        assert abs(r - rays_per_launch) < 1, "passes disagree on rays per launch"
        for k in agg[timed[0]]:
            summary["pmc"][k] = sum(agg[x][k] for x in timed) / launches
        summary["pmc_passes"][os.path.basename(d)] = {"dispatch_ms": sum(dur[x] for x in timed) / launches,
                                                      "dispatches": launches, "kernel": names[timed[0]]}
    p = summary["pmc"]
    summary["rays_per_launch"] = rays_per_launch
    per = {}
    if rays_per_launch:
        for k, n in (("SQ_INSTS_VALU", "valu_insts"), ("SQ_INSTS_SALU", "salu_insts"), ("SQ_INSTS_SMEM", "smem_insts"),
                     ("SQ_INSTS_VMEM_RD", "vmem_rd_insts"), ("SQ_INSTS_VMEM_WR", "vmem_wr_insts"),
                     ("SQ_INSTS_BRANCH", "branch_insts")):
            if k in p:
                per[n] = p[k] / rays_per_launch
    if "FETCH_SIZE" in p and "WRITE_SIZE" in p:
        fetch, write = p["FETCH_SIZE"] * 1024, p["WRITE_SIZE"] * 1024
        summary["hbm_bytes_per_launch"] = {"fetch_raw": fetch, "write": write, "raw_sum": fetch + write,
                                           "corrected": 2 * fetch + write}
        if rays_per_launch:
            per["hbm_bytes"] = (2 * fetch + write) / rays_per_launch
    summary["per_ray"] = per
    passes = summary["pmc_passes"]
    valu_pass = [v["dispatch_ms"] for k, v in passes.items() if "SQ_INSTS_VALU" in k]
    if "SQ_INSTS_VALU" in p and "GRBM_GUI_ACTIVE" in p and valu_pass:
        ms = valu_pass[0]
        clock = p["GRBM_GUI_ACTIVE"] / 8 / (ms / 1e3)
        summary["derived"] = {"clock_ghz": clock / 1e9,
                              "valu_issue_frac_at_clock": p["SQ_INSTS_VALU"] * 2 / (1024 * clock * ms / 1e3),
                              "valu_issue_frac_at_2p4ghz": p["SQ_INSTS_VALU"] * 2 / (1024 * 2.4e9 * ms / 1e3),
                              "salu_per_cu_cycle": p.get("SQ_INSTS_SALU", 0) / (256 * clock * ms / 1e3)}
        if "SQ_WAVE_CYCLES" in p and "SQ_WAIT_INST_ANY" in p:
            summary["derived"]["wait_inst_any_frac"] = p["SQ_WAIT_INST_ANY"] / p["SQ_WAVE_CYCLES"]
            summary["derived"]["active_inst_valu_frac"] = p.get("SQ_ACTIVE_INST_VALU", 0) / p["SQ_WAVE_CYCLES"]
    out = os.path.join(ROOT, "profiles", f"{tag}_{name}_summary.json")
    json.dump(summary, open(out, "w"), indent=1)
    print(json.dumps({k: summary[k] for k in ("key", "per_ray", "derived", "hbm_bytes_per_launch",
                                              "render_kernel_stats") if k in summary}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
