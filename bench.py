#!/usr/bin/env python3
"""Benchmark: Mray/s (samples x bounces) on the Cornell box at 1024^2 @ 1000 spp (BASELINE.json configs[1]).

One step = one full progressive render of the workload: Reset() + spp x Update() (launched as one
render, rt2.h lazy queue) + the gather of every GPU's row bands into the full image on the root GPU
+ the readback of that image's NonConvertedPixels() into host memory (App.cpp:163-174's headless
output; pinned, enqueued on the root's stream, complete at the step's closing synchronize).
Rays = closest-hit queries issued by RayColor (one per bounce level with depth > 0),
counted by the kernel. The scene program is resident in HBM before timing starts.

  python bench.py [--gpus N --steps K --warmup W]

Multi-GPU goes through the C ABI (include/rt2.h), not torch:
  * under torch.distributed.run (WORLD_SIZE = N): one process per GPU, rt2_tracer_join (partition +
    ncclCommInitRank; the id is broadcast over a gloo control-plane group) and rt2_tracer_gather
    (ncclGather of the row bands + de-interleave on rank 0) every step;
  * plain `python bench.py --gpus N`: one process driving N GPUs, rt2_tracer_create_multi
    (ncclCommInitAll); N = 1 is the same path with a communicator of size 1.
  * --emulate-world N [--emulate-rank r|all]: diagnostic, one GPU renders rank r's bands of an N-way
    split (all: every rank in turn); no gather.

Rank 0 prints one JSON line (contract in the task statement) with a `roofline` object for the render
kernel (frac: SURVEY §8(d)'s useful fp32 flops per ray x the live rays / the launches' own GPU time, over
the fp32 vector peak; the VALU and scalar issue fractions from a committed PMC profile of this kernel
build and config as named companions) and a `cpu_baseline` object (the oracle restatement on every
host core this process may use, bounded sample).
"""
import argparse
import glob
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402  (import before raytrace2_amd: one HIP runtime per process)
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP32_VALU_PEAK_TFLOPS = 157.3  # spec, FMA = 2 flops
MAX_CLOCK_HZ = 2.4e9           # MI355X_MICROARCH.md "Max clock"
SIMDS = 256 * 4
# VALU issue peak: a wave64 VALU instruction occupies a 32-lane SIMD for 2 cycles
VALU_PEAK_TLANE_OPS = SIMDS * 32 * MAX_CLOCK_HZ / 1e12  # 78.64 T lane-ops/s
# Scalar issue peak: one scalar unit per CU (MI355X_MICROARCH.md), one SALU instruction per cycle
SALU_PEAK_GINST = 256 * MAX_CLOCK_HZ / 1e9  # 614.4 G instructions/s
# Record sizes of the flattened scene program (rt2_layout.h) in bytes
REC_BYTES = {"bvh_tests": 32, "quad_tests": 80, "sphere_tests": 32, "xform_visits": 128, "medium_tests": 16,
             "list_visits": 16}
FLOPS = {"bvh_tests": 18, "quad_tests": 45, "sphere_tests": 30, "xform_visits": 45, "medium_tests": 20}
GATHER_REPS = 5  # isolated gathers timed after the steps (gather_ms_per_step)
KERNEL_SOURCES = ["raytrace2_amd/csrc/render.hip", "raytrace2_amd/csrc/rt2_layout.h", "raytrace2_amd/csrc/boxaa.h",
                  "raytrace2_amd/csrc/Makefile"]


def kernel_sha() -> str:
    """Identity of the render kernel sources in this tree: a profile only describes the build it was
    taken on."""
    h = hashlib.sha1()
    for f in KERNEL_SOURCES:
        h.update(open(os.path.join(ROOT, f), "rb").read())
    return h.hexdigest()[:12]


def library_kernel_sha(R) -> str:
    """The kernel sha the loaded librt2.so was built from (rt2_version's last field; the Makefile
    embeds it), which is what actually ran."""
    v = R.lib.rt2_version().decode(errors="replace").split()
    return v[-1] if len(v) >= 2 and v[-2] == "kernel" else "unknown"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scene", default="cornell_box_original.json")
    ap.add_argument("--width", type=int, default=1024)
    ap.add_argument("--height", type=int, default=1024)
    ap.add_argument("--spp", type=int, default=1000)
    ap.add_argument("--max-depth", type=int, default=50)
    ap.add_argument("--seed", type=int, default=0x5EED2024)
    ap.add_argument("--band-h", type=int, default=2, help="row-band height of the multi-GPU partition")
    ap.add_argument("--launch-frames", type=int, default=0, help="frames per kernel launch (0 = all)")
    ap.add_argument("--work-split", type=int, default=-1,
                    help="work items (pixel x frame chunk) per resident lane (-1: library default, 0: no split)")
    ap.add_argument("--batch-max", type=int, default=0, help="work items a wave reserves at once (0: default)")
    ap.add_argument("--sample-budget-gb", type=float, default=0.0, help="bound on both launch slots' per-frame sample buffers together, GiB (0: default 24)")
    ap.add_argument("--plain", action="store_true", help="one GPU, no gather (the one-GPU tracer alone)")
    ap.add_argument("--emulate-world", type=int, default=1,
                    help="diagnostic: render one rank's row bands of an N-GPU split on this one GPU (no gather)")
    ap.add_argument("--emulate-rank", default="0", help="rank to emulate, or 'all' (each rank timed in turn)")
    ap.add_argument("--cpu-frames", type=int, default=48, help="oracle sample: frames at full resolution")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--stats-frames", type=int, default=8)
    ap.add_argument("--out-image", default="")
    return ap.parse_args()


def host_cores():
    """Cores this process may run on, and the host's logical / physical counts (lscpu-equivalent)."""
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count() or 1
    logical, phys = 0, set()
    try:
        pid = cid = None
        for line in open("/proc/cpuinfo"):
            if line.startswith("processor"):
                logical += 1
            elif line.startswith("physical id"):
                pid = line.split(":")[1].strip()
            elif line.startswith("core id"):
                cid = line.split(":")[1].strip()
                phys.add((pid, cid))
    except OSError:
        pass
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = round(int(q) / int(period), 2)
    except (OSError, ValueError):
        pass
    return {"usable": usable, "logical": logical or usable, "physical": len(phys) or None, "cgroup_cpu_quota": quota}


def find_profile(key):
    """The newest committed profile summary taken on this exact config and kernel build."""
    best, stale = None, None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_summary.json")), reverse=True):
        try:
            prof = json.load(open(f))
        except (OSError, ValueError):
            continue
        k = prof.get("key") or {}
        if k.get("workload") != key["workload"] or k.get("partition") != key["partition"]:
            continue
        if "per_ray" not in prof:
            continue
        if k.get("kernel_sha") == key["kernel_sha"]:
            return os.path.relpath(f, ROOT), prof, False
        if stale is None:
            stale = (os.path.relpath(f, ROOT), prof, True)
    return stale if stale else (best, None, False)


def roofline_for(tr, rays_local, launches, kernel_ms, key, rank_stats_frames, spp_total, steps, ms_per_step):
    """Roofline of the render kernel on this GPU, as SURVEY.md §8(d) defines it.

    `frac` is §8(d)'s useful-flop fraction: rays/s x F_ray / the FP32 vector peak (157.3 TFLOP/s), with
    F_ray = the records each ray touched (counted by the kernel's counting pass at this run's seed) x the
    per-test flop constants (AABB 18, quad 45, sphere 30, transform 45, medium 20). The kernel is issue
    bound (DESIGN.md §4 Roofline), so the named companions say where the rest of the issue goes:
    `valu_issue_frac` (VALU wave instructions per ray of the matching PMC profile x 64 lanes x rays per
    launch / launch time / 78.6 T lane-op/s, masked lanes included) and `salu_frac` (the CU's one scalar
    unit, 614 G instructions/s). §8(d)'s HBM model (records x record bytes per ray) is reported as
    `record_rate_over_hbm_peak`: those records are scalar-cache hits on a few-KB scene program, so it is
    not a physical HBM fraction; `hbm_frac` is the PMC-measured one (profile traffic per ray, same scaling).
    Launch time = the render kernel's GPU time per launch (rt2_stats.kernel_ms: each launch timed by its
    own clock from its first wave to its last, overlapping launches counted once). A kernel time per step
    above the step's wall time would be a timing fault: then no fraction is reported."""
    tr.enable_stats(True)
    tr.Reset()
    tr.reset_stats()
    tr.Render(rank_stats_frames)
    s2 = tr.stats()
    tr.enable_stats(False)
    per_ray = {k: s2[k] / max(1, s2["rays"]) for k in REC_BYTES}
    b_ray = sum(REC_BYTES[k] * per_ray[k] for k in REC_BYTES)
    f_ray = sum(FLOPS.get(k, 0) * per_ray[k] for k in REC_BYTES)
    rays_per_launch = rays_local / max(1, launches)
    avg_launch_s = kernel_ms / 1e3 / max(1, launches)
    src, prof, stale = find_profile(key)
    out = {"bound": "valu", "model": "SURVEY §8(d) useful fp32 flops per ray x rays/s over the fp32 vector peak",
           "unit": "TFLOP/s", "peak": FP32_VALU_PEAK_TFLOPS,
           "achieved": None, "frac": None, "traffic": None, "traffic_unit": "HBM bytes per launch (PMC)",
           "kernel": "rt2::dev::render_kernel<..., false>", "avg_launch_ms": round(avg_launch_s * 1e3, 3),
           "rays_per_launch": int(rays_per_launch), "flops_per_ray": round(f_ray, 1), "profile": src,
           "profile_stale": stale, "kernel_ms_per_step": round(kernel_ms / max(1, steps), 2)}
    consistent = kernel_ms / max(1, steps) <= ms_per_step * 1.001
    if not consistent:
        out["invalid"] = (f"kernel time per step {kernel_ms / max(1, steps):.2f} ms exceeds the step's wall time "
                          f"{ms_per_step:.2f} ms: no fraction reported")
        return out
    useful = rays_per_launch * f_ray / avg_launch_s / 1e12
    out.update(achieved=round(useful, 3), frac=round(useful / FP32_VALU_PEAK_TFLOPS, 4))
    out["useful_flop_frac"] = out["frac"]
    if prof:
        pr = prof["per_ray"]
        valu = pr["valu_insts"] * rays_per_launch  # wave instructions per launch
        salu = pr.get("salu_insts", 0.0) * rays_per_launch
        valu_rate = valu * 64 / avg_launch_s / 1e12
        salu_rate = salu / avg_launch_s / 1e9
        out["valu_issue_frac"] = round(valu_rate / VALU_PEAK_TLANE_OPS, 4)
        out["valu_issue_tlane_ops"] = round(valu_rate, 3)
        out["valu_issue_peak"] = round(VALU_PEAK_TLANE_OPS, 2)
        out["salu_frac"] = round(salu_rate / SALU_PEAK_GINST, 4)
        out["valu_insts_per_ray"] = round(pr["valu_insts"], 3)
        out["salu_insts_per_ray"] = round(pr.get("salu_insts", 0.0), 3)
        # issued lane slots per useful flop (masked lanes, traversal bookkeeping, exact-division sequences)
        out["issued_lane_slots_per_useful_flop"] = round(pr["valu_insts"] * 64 / max(1e-9, f_ray), 3)
        if pr.get("hbm_bytes") is not None:
            out["traffic"] = int(pr["hbm_bytes"] * rays_per_launch)
            out["hbm_frac"] = round(out["traffic"] / avg_launch_s / 1e9 / HBM_PEAK_GBS, 4)
        out["profile_kernel_sha"] = (prof.get("key") or {}).get("kernel_sha")
    frame_bytes = 12 * spp_total  # the float3 sample store per (pixel, frame), per launch below
    out["record_rate_gbs"] = round((rays_per_launch * b_ray) / avg_launch_s / 1e9, 1)
    out["record_rate_over_hbm_peak"] = round(out["record_rate_gbs"] / HBM_PEAK_GBS, 3)
    out["record_rate_note"] = "§8(d) HBM model; the records are scalar-cache hits, not HBM traffic (see hbm_frac)"
    out["record_bytes_per_ray"] = round(b_ray, 1)
    out["records_per_ray"] = {k: round(v, 3) for k, v in per_ray.items()}
    out["sample_store_bytes_per_launch"] = frame_bytes
    return out


def cpu_baseline(a, scene_file):
    from oracle.oracle import OracleScene
    cores = host_cores()
    # every core this process may use: its affinity set, bounded by a cgroup CPU quota when one is
    # set (more threads than the quota only time-slice the same CPUs)
    threads = cores["usable"]
    if cores["cgroup_cpu_quota"]:
        threads = max(1, min(threads, int(-(-cores["cgroup_cpu_quota"] // 1))))
    o = OracleScene(scene_file, a.seed)
    tc = time.perf_counter()
    _, _, cnt = o.render(a.width, a.height, a.spp, a.cpu_frames, max_depth=a.max_depth, threads=threads,
                         forward=False)
    dt = time.perf_counter() - tc
    return {"value": round(cnt["rays"] / dt / 1e6, 3), "unit": "Mray/s", "cores": threads, "kind": "port",
            "host_cores": cores,
            "sample": f"{a.scene} {a.width}x{a.height}, frames 0..{a.cpu_frames - 1} of the spp={a.spp} "
                      f"stratification, oracle restatement (recursive RayColor), {threads} std::threads, "
                      f"{cnt['rays']} rays in {dt:.2f} s"}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    share = os.environ.get("RT2_BENCH_SHARE_GPU") == "1"  # rehearsal: every rank on GPU 0, gather via gloo
    # RT2_BENCH_RANKS=1: the one-process-per-GPU path even at WORLD_SIZE 1 (join + gather, comm of size 1)
    if world > 1 or os.environ.get("RT2_BENCH_RANKS") == "1":
        mode = "ranks"
        if a.gpus not in (1, world):
            raise SystemExit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}")
        n_gpus = world
        dist.init_process_group("gloo")  # control plane only: id broadcast, barriers, max-over-ranks
        if share:
            local_rank = 0
    elif a.emulate_world > 1:
        mode, n_gpus = "emulate", 1
    elif a.plain:
        mode, n_gpus = "plain", 1
    else:
        mode, n_gpus = "multi", a.gpus
        if torch.cuda.device_count() < n_gpus:
            raise SystemExit(f"bench.py: --gpus {n_gpus} but {torch.cuda.device_count()} GPU(s) visible")
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)

    import raytrace2_amd as R
    from raytrace2_amd._native import Rt2Error

    def fail(what, e):
        """A clear non-zero exit naming the C ABI's error text (rt2_last_error), e.g. an RCCL failure."""
        print(f"bench.py: {what} failed: {e}", file=sys.stderr, flush=True)
        sys.exit(3)

    scene_file = os.path.join(ROOT, "scenes", a.scene)
    if a.scene.startswith("gen:"):  # gen:<generator>:<n>:<seed> -> raytrace2_amd.authoring scene
        import random
        from raytrace2_amd import authoring
        _, gen, n, gseed = a.scene.split(":")
        scene_file = f"/tmp/rt2_{gen}_{n}_{gseed}.json"
        authoring.GENERATORS[gen](random.Random(int(gseed)), int(n)).dump(scene_file)
    t0 = time.perf_counter()
    sc = R.Scene(scene_file, a.seed)
    try:
        if mode == "multi":  # ncclCommInitAll for n_gpus > 1
            tr = R.RayTracer(sc, devices=list(range(n_gpus)), band_h=a.band_h)
        else:
            tr = R.RayTracer(sc, local_rank)
    except Rt2Error as e:
        fail("rt2_tracer_create" + ("_multi" if mode == "multi" else ""), e)
    tr.set_seed(a.seed)
    tr.max_depth = a.max_depth
    tr.SetSamplesPerPixel(a.spp)
    tr.OnResize((a.width, a.height))
    host_gather = None
    if mode == "ranks":
        if share:  # rehearsal only: RCCL cannot put two ranks on one GPU
            from raytrace2_amd.dist import BandGather
            tr.set_partition(a.band_h, rank, world)
            host_gather = BandGather(a.height, a.width, a.band_h, world, rank, torch.device("cpu"))
        else:
            uid = [R.comm_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            try:
                tr.join(uid[0], world, rank, a.band_h)  # ncclCommInitRank
            except Rt2Error as e:
                fail(f"rt2_tracer_join (rank {rank} of {world})", e)
    if a.launch_frames:
        tr.set_launch_frames(a.launch_frames)
    if a.work_split >= 0:
        tr.set_work_split(a.work_split)
    if a.batch_max > 0:
        tr.set_batch_max(a.batch_max)
    if a.sample_budget_gb > 0:
        tr.set_sample_budget(int(a.sample_budget_gb * (1 << 30)))
    tr.synchronize()
    # the root's host copy of the image (NonConvertedPixels, float3): pinned, read back every step
    readback = None
    # (an older library in a tools/ A/B run may lack the entry points used below)
    new_abi = hasattr(R._native.lib, "rt2_tracer_part_stats")
    if rank == 0 and mode in ("ranks", "multi") and host_gather is None and new_abi:
        from raytrace2_amd.progressive import PinnedBuffer
        readback = PinnedBuffer((a.height, a.width, 3), np.float32)
    setup_s = time.perf_counter() - t0

    def step():
        tr.Reset()
        tr.Render(a.spp)
        tr.flush()  # launch now: Render() only queues frames until a readback (rt2.h)
        if host_gather is not None:
            host_gather.local_view().copy_(torch.from_numpy(tr.Accumulation()))
            host_gather.gather()
        elif mode in ("ranks", "multi"):
            try:
                tr.gather()  # ncclGather of the row bands to rank 0 + de-interleave (rt2_tracer_gather)
            except Rt2Error as e:
                fail("rt2_tracer_gather (ncclGather)", e)
            if readback is not None:  # NonConvertedPixels() to the host (App.cpp:163-174)
                tr.image_non_converted_pixels_async(readback.array.ctypes.data)

    def sync_all():
        if mode == "multi":
            for d in range(n_gpus):
                torch.cuda.synchronize(d)
        else:
            torch.cuda.synchronize(dev)

    def timed(steps, warmup):
        for _ in range(warmup):
            step()
        sync_all()
        tr.reset_stats()
        if mode == "ranks":
            dist.barrier()
        sync_all()
        t_start = time.perf_counter()
        for _ in range(steps):
            step()
        sync_all()
        if mode == "ranks":
            dist.barrier()
        return time.perf_counter() - t_start, tr.stats()

    ranks_to_run = [0]
    if mode == "emulate":
        ranks_to_run = list(range(a.emulate_world)) if a.emulate_rank == "all" else [int(a.emulate_rank)]
    per_rank = []
    for er in ranks_to_run:
        if mode == "emulate":
            tr.set_partition(a.band_h, er, a.emulate_world)
        el, st = timed(a.steps, a.warmup)
        per_rank.append({"rank": er, "rows": tr.local_rows(), "elapsed_s": el, "rays": st["rays"],
                         "kernel_ms": st["kernel_ms"], "launch_ms_sum": st["launch_ms_sum"], "launches": st["launches"],
                         "gather_ms": st["gather_ms"],
                         "gathers": st["gathers"], "enqueue_ms": st.get("enqueue_ms", 0.0),
                         "readbacks": st.get("readbacks", 0), "readback_ms": st.get("readback_ms", 0.0),
                         "sample_buffer_bytes": st.get("sample_buffer_bytes", 0),
                         "device_bytes_peak": st.get("device_bytes_peak", 0),
                         "mray_s": st["rays"] / el / 1e6})
        if mode == "multi" and new_abi:  # each GPU of the one-process tracer
            per_rank[-1]["gpus"] = []
            for g in range(n_gpus):
                ps = tr.part_stats(g)
                per_rank[-1]["gpus"].append({"gpu": g, "rays": ps["rays"], "kernel_ms": ps["kernel_ms"],
                                             "enqueue_ms": ps["enqueue_ms"], "launches": ps["launches"]})
    # The exchange itself, timed on an otherwise idle GPU: in a run of back-to-back steps the gather's
    # small kernels (the RCCL gather, the de-interleave) wait for CUs behind the next step's render,
    # whose persistent waves hold them, so the event pair around a step's gather spans that queue time
    # (gather_span_ms_per_step). gather_ms_per_step is the mean over GATHER_REPS isolated gathers
    # (HIP events on the root stream around ncclGather + de-interleave); gather_readback_ms_isolated
    # is the host wall time of one gather + NonConvertedPixels() readback.
    gather_iso_ms = gather_ms_iso = None
    if mode in ("ranks", "multi") and host_gather is None:
        g0 = tr.stats()
        for _ in range(GATHER_REPS):
            sync_all()
            if mode == "ranks":
                dist.barrier()
            tr.gather()
            sync_all()
        g1 = tr.stats()
        if g1["gathers"] > g0["gathers"]:
            gather_ms_iso = (g1["gather_ms"] - g0["gather_ms"]) / (g1["gathers"] - g0["gathers"])
        sync_all()
        if mode == "ranks":
            dist.barrier()
        t_g = time.perf_counter()
        tr.gather()
        if readback is not None:
            tr.image_non_converted_pixels_async(readback.array.ctypes.data)
        sync_all()
        gather_iso_ms = round((time.perf_counter() - t_g) * 1e3, 3)
    launch_shape = tr.last_launch()  # the timed launches' shape (before the stats pass below)
    me = per_rank[-1] if mode != "emulate" else max(per_rank, key=lambda r: r["elapsed_s"])
    if mode == "ranks":
        gathered = [None] * world
        dist.all_gather_object(gathered, per_rank[0] | {"rank": rank})
        per_rank = gathered
    elapsed = max(r["elapsed_s"] for r in per_rank)
    rays_total = float(sum(r["rays"] for r in per_rank))

    if rank == 0 and a.out_image and mode != "emulate":
        img = (tr.image_accumulation() if mode != "plain" and host_gather is None else
               (host_gather.image.numpy() if host_gather is not None else tr.Accumulation()))
        R.WriteImage(img / np.float32(a.spp), a.width, a.height, a.out_image)

    workload = f"{a.scene} {a.width}x{a.height} @ {a.spp} spp, max_depth {a.max_depth}"
    if mode == "emulate":  # the same GPU work as that rank of a real N-GPU run: the same profile key
        partition = f"{a.emulate_world}-way h={a.band_h} rank {me['rank']}"
    elif n_gpus > 1:
        partition = f"{n_gpus}-way h={a.band_h} rank 0"
    else:
        partition = "1 GPU"
    lib_sha, src_sha = library_kernel_sha(R), kernel_sha()
    if lib_sha != src_sha:  # a library built from other sources than this tree's: key on what ran
        print(f"bench.py: librt2.so was built from kernel sources {lib_sha}, this tree has {src_sha}",
              file=sys.stderr)
    key = {"workload": workload, "partition": partition, "kernel_sha": lib_sha}
    roofline = None
    cpu = None
    if rank == 0:
        if mode == "emulate":  # the slowest rank's partition
            tr.set_partition(a.band_h, me["rank"], a.emulate_world)
        mine = me if mode != "ranks" else per_rank[0]
        gpu_rays, gpu_kernel_ms, launches = mine["rays"], mine["kernel_ms"], mine["launches"]
        if mode == "multi" and n_gpus > 1:  # per-GPU share (kernel_ms is the busiest GPU's)
            gpu_rays = mine["rays"] / n_gpus
        roofline = roofline_for(tr, gpu_rays, launches, gpu_kernel_ms, key, a.stats_frames,
                                tr.local_rows() * a.width * a.spp * a.steps // max(1, launches), a.steps,
                                mine["elapsed_s"] * 1e3 / a.steps)
        if not a.no_cpu:
            cpu = cpu_baseline(a, scene_file)

    if rank == 0:
        value = rays_total / elapsed / 1e6
        if mode == "ranks":
            par = (f"row-bands h={a.band_h} x {world} GPUs, one process per GPU, "
                   + ("host gather over gloo (rehearsal on one GPU)" if share else
                      "RCCL ncclGather to rank 0 through the C ABI (rt2_tracer_join/gather)"))
        elif mode == "multi":
            par = (f"row-bands h={a.band_h} x {n_gpus} GPU(s) in one process (rt2_tracer_create_multi), "
                   "RCCL ncclGather to GPU 0 + de-interleave")
        elif mode == "plain":
            par = "1 GPU, no gather (one-GPU tracer)"
        else:
            par = f"emulated rank(s) of a {a.emulate_world}-way row-band split on one GPU, no gather"
        default_workload = (a.scene == "cornell_box_original.json" and (a.width, a.height, a.spp, a.max_depth) ==
                            (1024, 1024, 1000, 50))
        metric = f"Mray/s (samples x bounces) {a.scene} {a.width}x{a.height} @ {a.spp} spp"
        if default_workload:  # BASELINE.json's headline metric, verbatim
            try:
                metric = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
            except (OSError, ValueError, KeyError):
                metric = "Mray/s (samples x bounces) Cornell Box 1024^2 @ 1000 spp; 1/2/4/8-GPU scaling"
        out = {
            "metric": metric,
            "value": round(value, 2),
            "unit": "Mray/s",
            "n_gpus": n_gpus,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed * 1e3 / a.steps, 2),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: committed scene JSON (scenes/), Philox4x32-10 sample streams seeded "
                    f"{a.seed:#x}",
            "config": {"workload": workload, "parallelism": par, "partition": partition,
                       "launch_frames": a.spp * a.steps // max(1, me["launches"]),
                       "work_split": launch_shape},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "detail": {"rays": int(rays_total), "launches": me["launches"], "setup_s": round(setup_s, 3),
                       "kernel_sha": key["kernel_sha"], "source_kernel_sha": src_sha,
                       "kernel_ms_per_step_max": round(max(r["kernel_ms"] for r in per_rank) / a.steps, 2),
                       "launch_ms_sum_per_step": round(per_rank[0]["launch_ms_sum"] / a.steps, 2),
                       "gather_ms_per_step": None if gather_ms_iso is None else round(gather_ms_iso, 3),
                       "gather_span_ms_per_step": round(per_rank[0]["gather_ms"] / a.steps, 3),
                       "gather_readback_ms_isolated": gather_iso_ms,
                       "readback_ms_per_step": round(per_rank[0]["readback_ms"] / a.steps, 3),
                       "readback_bytes_per_step": (a.width * a.height * 12 if per_rank[0]["readbacks"] else 0),
                       "enqueue_ms_per_step": round(per_rank[0]["enqueue_ms"] / a.steps, 3),
                       # device memory per GPU: both launch slots' sample buffers (bounded by the total
                       # sample budget, rt2.h) and the high-water mark of everything the tracer holds
                       "sample_buffer_bytes": max(r.get("sample_buffer_bytes", 0) for r in per_rank),
                       "device_bytes_peak_per_gpu": max(r.get("device_bytes_peak", 0) for r in per_rank),
                       "per_rank": [{"rank": r["rank"], "rows": r["rows"], "mray_s": round(r["mray_s"], 1),
                                     "ms_per_step": round(r["elapsed_s"] * 1e3 / a.steps, 2),
                                     "kernel_ms_per_step": round(r["kernel_ms"] / a.steps, 2)} for r in per_rank],
                       "runtime": R._native.runtime_info(),
                       "rays_per_sample": round(rays_total / (a.steps * a.spp * a.width *
                                                              sum(r["rows"] for r in per_rank)), 4)},
        }
        if cpu:
            out["detail"]["gpu_over_cpu"] = round(value / cpu["value"], 1)
        # per GPU (N > 1): kernel time and rays of each GPU, the host time of its launches' enqueue,
        # and the slowest / fastest GPU kernel-time ratio (the load balance of the row-band split)
        gpus = per_rank[0].get("gpus") if mode == "multi" else (
            [{"gpu": r["rank"], "rays": r["rays"], "kernel_ms": r["kernel_ms"], "enqueue_ms": r["enqueue_ms"],
              "launches": r["launches"]} for r in per_rank] if mode == "ranks" else None)
        if gpus:
            out["detail"]["per_gpu"] = [{"gpu": g["gpu"], "rays": int(g["rays"]),
                                         "kernel_ms_per_step": round(g["kernel_ms"] / a.steps, 3),
                                         "enqueue_ms_per_step": round(g["enqueue_ms"] / a.steps, 3),
                                         "launches": g["launches"]} for g in gpus]
            ks = [g["kernel_ms"] for g in gpus]
            out["detail"]["slowest_over_fastest_gpu"] = round(max(ks) / max(1e-9, min(ks)), 4)
        if mode == "emulate":
            out["config"]["emulated"] = (f"{len(per_rank)} rank(s) of {a.emulate_world} timed one after another on "
                                         "this GPU; value = their rays / the slowest rank's time (no gather)")
        print(json.dumps(out), flush=True)
    tr.close()
    if mode == "ranks":
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
