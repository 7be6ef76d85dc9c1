#!/usr/bin/env python3
"""Benchmark: Mray/s (samples x bounces) on the Cornell box at 1024^2 @ 1000 spp (BASELINE.json configs[1]).

One step = one full progressive render of the workload on the rank's share of the image:
Reset() + spp x Update() (executed as kernel launches of --launch-frames frames each) + the RCCL
gather of every rank's row bands to rank 0 and the de-interleave there. Rays = closest-hit
queries issued by RayColor (one per bounce level with depth > 0), counted by the
kernel. Inputs (scene program) are resident in HBM before timing starts.

  python bench.py [--gpus N --steps K --warmup W]      (N > 1: launched by torch.distributed.run)

Rank 0 prints one JSON line (contract in the task statement) with a `roofline` object for the
render kernel (algorithmic bytes per launch / HIP-event launch time vs 8 TB/s HBM) and a
`cpu_baseline` object (the oracle restatement timed on this host's cores on a bounded sample).
"""
import argparse
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402  (import before raytrace2_amd: one HIP runtime per process)
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP32_VALU_PEAK_TFLOPS = 157.3
# Record sizes of the flattened scene program (rt2_layout.h) in bytes
REC_BYTES = {"bvh_tests": 32, "quad_tests": 80, "sphere_tests": 32, "xform_visits": 128, "medium_tests": 16,
             "list_visits": 16}
FLOPS = {"bvh_tests": 18, "quad_tests": 45, "sphere_tests": 30, "xform_visits": 45, "medium_tests": 20}


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
    ap.add_argument("--band-h", type=int, default=16)
    ap.add_argument("--launch-frames", type=int, default=0, help="frames per kernel launch (0 = all)")
    ap.add_argument("--work-split", type=int, default=-1,
                    help="work items (pixel x frame chunk) per resident lane (-1: library default, 0: no split)")
    ap.add_argument("--batch-max", type=int, default=0, help="work items a wave reserves at once (0: default)")
    ap.add_argument("--sample-budget-gb", type=float, default=0.0, help="per-frame sample buffer bound (0: default)")
    ap.add_argument("--emulate-world", type=int, default=1,
                    help="diagnostic: render only rank 0's row bands of an N-GPU split on this one GPU (no gather)")
    ap.add_argument("--cpu-frames", type=int, default=48, help="oracle sample: frames at full resolution")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--stats-frames", type=int, default=8)
    ap.add_argument("--out-image", default="")
    return ap.parse_args()


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # RT2_BENCH_BACKEND=gloo + RT2_BENCH_SHARE_GPU=1: rehearsal of the N-rank flow with every rank
    # on GPU 0 and the gather over gloo through host memory (the real run is RCCL, one GPU per rank)
    backend = os.environ.get("RT2_BENCH_BACKEND", "nccl")
    if os.environ.get("RT2_BENCH_SHARE_GPU") == "1":
        local_rank = 0
    if world > 1:
        torch.cuda.set_device(local_rank)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)

    import raytrace2_amd as R

    scene_file = os.path.join(ROOT, "scenes", a.scene)
    if a.scene.startswith("gen:"):  # gen:<generator>:<n>:<seed> -> raytrace2_amd.authoring scene
        import random
        from raytrace2_amd import authoring
        _, gen, n, gseed = a.scene.split(":")
        scene_file = f"/tmp/rt2_{gen}_{n}_{gseed}.json"
        authoring.GENERATORS[gen](random.Random(int(gseed)), int(n)).dump(scene_file)
    t0 = time.perf_counter()
    sc = R.Scene(scene_file, a.seed)
    tr = R.RayTracer(sc, local_rank)
    # a dedicated (non-null) torch stream shared with the tracer, so torch events and RCCL calls
    # order against the render kernels
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    tr.set_stream(stream.cuda_stream)
    tr.set_seed(a.seed)
    tr.max_depth = a.max_depth
    tr.SetSamplesPerPixel(a.spp)
    tr.OnResize((a.width, a.height))
    emulate = a.emulate_world if world == 1 and a.emulate_world > 1 else 1
    tr.set_partition(a.band_h, rank, world * emulate)
    if a.launch_frames:
        tr.set_launch_frames(a.launch_frames)
    if a.work_split >= 0:
        tr.set_work_split(a.work_split)
    if a.batch_max > 0:
        tr.set_batch_max(a.batch_max)
    if a.sample_budget_gb > 0:
        tr.set_sample_budget(int(a.sample_budget_gb * (1 << 30)))
    tr.synchronize()
    setup_s = time.perf_counter() - t0
    rows = tr.local_rows()
    from raytrace2_amd.dist import BandGather
    host_gather = world > 1 and backend != "nccl"
    gath = (BandGather(a.height, a.width, a.band_h, world, rank, torch.device("cpu") if host_gather else dev)
            if emulate == 1 else None)
    assert gath is None or gath.local_view().shape[0] == rows

    def step():
        tr.Reset()
        tr.Render(a.spp)
        tr.flush()  # launch now: Render() only queues frames until a readback (rt2.h)
        if gath is not None:
            if host_gather:
                gath.local_view().copy_(torch.from_numpy(tr.Accumulation()))
            else:
                tr.copy_accum_to(gath.send.data_ptr(), stream.cuda_stream)
            gath.gather()  # RCCL gather of the row bands to rank 0 + de-interleave

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize(dev)
    tr.reset_stats()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t_start = time.perf_counter()
    ev0.record(stream)
    for _ in range(a.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    st = tr.stats()
    shape = tr.last_launch()
    stream_ms = ev0.elapsed_time(ev1)
    rays_local = st["rays"]
    kernel_ms = st["kernel_ms"]
    launches = max(1, st["launches"])
    if world > 1:
        t = torch.tensor([elapsed, float(rays_local)], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        tmax = t.clone()
        dist.all_reduce(tmax[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        elapsed = float(tmax[0])
        rays_total = float(t[1])
    else:
        rays_total = float(rays_local)

    if rank == 0 and a.out_image and gath is not None:
        img = gath.image.cpu().numpy() / np.float32(a.spp)
        R.WriteImage(img, a.width, a.height, a.out_image)

    workload = f"{a.scene} {a.width}x{a.height} @ {a.spp} spp, max_depth {a.max_depth}"
    # ---- algorithmic bytes per ray from a stats pass (same seed, same kernel family) ----
    roofline = None
    if rank == 0:
        tr.enable_stats(True)
        tr.Reset()
        tr.reset_stats()
        tr.Render(a.stats_frames)
        s2 = tr.stats()
        tr.enable_stats(False)
        per_ray = {k: s2[k] / max(1, s2["rays"]) for k in REC_BYTES}
        b_ray = sum(REC_BYTES[k] * per_ray[k] for k in REC_BYTES)
        f_ray = sum(FLOPS.get(k, 0) * per_ray[k] for k in REC_BYTES)
        rays_per_launch = rays_local / launches
        pixels_local = rows * a.width
        frame_bytes = pixels_local * 12 * (a.spp * a.steps / launches)  # float3 sample store per frame
        bytes_per_launch = rays_per_launch * b_ray + frame_bytes
        avg_launch_s = kernel_ms / 1e3 / launches
        achieved = bytes_per_launch / avg_launch_s / 1e9
        traffic, traffic_src, valu_issue = None, None, None
        for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_summary.json")), reverse=True):
            try:
                prof = json.load(open(f))
                under = prof.get("bench_under_rocprof") or {}
                if under.get("config", {}).get("workload") != workload or "hbm_bytes_per_launch" not in prof:
                    continue
                traffic = int(prof["hbm_bytes_per_launch"]["corrected"])
                traffic_src = os.path.relpath(f, ROOT)
                pmc = prof.get("pmc", {})
                if "SQ_INSTS_VALU" in pmc and "GRBM_GUI_ACTIVE" in pmc:
                    ms = pmc["dispatch_ms"]["pmc_SQ_WAVES_SQ_INSTS_VALU_SQ_INSTS_SALU_SQ_"]
                    clock = pmc["GRBM_GUI_ACTIVE"] / 8 / (ms / 1e3)  # MI355X_MICROARCH.md: sum over 8 XCDs
                    simds = 4 * 256
                    valu_issue = pmc["SQ_INSTS_VALU"] * 2 / (simds * clock * ms / 1e3)  # wave64 = 2 cycles/SIMD32
                break
            except (OSError, ValueError, KeyError):
                continue
        roofline = {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "traffic_unit": "bytes/launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, gfx950-corrected)",
            "traffic_source": traffic_src,
            "note": "algorithmic bytes = scene records touched per ray (SURVEY 8d) served from the scalar cache/L1; "
                    "frac > 1 means that record traffic exceeds what HBM alone could feed; measured HBM traffic is "
                    "`traffic`; the kernel is VALU-issue/latency bound (valu_issue_frac)",
            "valu_issue_frac": None if valu_issue is None else round(valu_issue, 3),
            "kernel": "rt2::dev::render_kernel<false>",
            "avg_launch_ms": round(kernel_ms / launches, 3),
            "bytes_per_ray": round(b_ray, 1),
            "records_per_ray": {k: round(v, 3) for k, v in per_ray.items()},
            "useful_flop_frac": round(rays_per_launch * f_ray / avg_launch_s / 1e12 / FP32_VALU_PEAK_TFLOPS, 4),
        }

    cpu = None
    if rank == 0 and not a.no_cpu and world == 1:
        from oracle.oracle import OracleScene
        try:
            cores = min(16, len(os.sched_getaffinity(0)))
        except AttributeError:
            cores = min(16, os.cpu_count() or 1)
        o = OracleScene(scene_file, a.seed)
        tc = time.perf_counter()
        _, _, cnt = o.render(a.width, a.height, a.spp, a.cpu_frames, max_depth=a.max_depth, threads=cores,
                             forward=False)
        dt = time.perf_counter() - tc
        cpu = {"value": round(cnt["rays"] / dt / 1e6, 3), "unit": "Mray/s", "cores": cores, "kind": "port",
               "sample": f"{a.scene} {a.width}x{a.height}, frames 0..{a.cpu_frames - 1} of the spp={a.spp} "
                         f"stratification, oracle restatement (recursive RayColor), {cnt['rays']} rays in "
                         f"{dt:.2f} s"}

    if rank == 0:
        value = rays_total / elapsed / 1e6
        out = {
            "metric": "Mray/s (samples x bounces) Cornell Box 1024^2 @ 1000 spp",
            "value": round(value, 2),
            "unit": "Mray/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed * 1e3 / a.steps, 2),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: committed scene JSON (scenes/), Philox4x32-10 sample streams seeded "
                    f"{a.seed:#x}",
            "config": {"workload": workload,
                       "parallelism": f"row-bands h={a.band_h} x {world} GPU(s), RCCL gather to rank 0",
                       "launch_frames": a.spp * a.steps // launches,
                       "work_split": shape},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "detail": {"rays": int(rays_total), "stream_ms": round(stream_ms, 2),
                       "kernel_ms_per_step": round(kernel_ms / a.steps, 2), "launches": launches,
                       "variant_features": hex(tr.last_variant_features()) if hasattr(tr, "last_variant_features") else None,
                       "setup_s": round(setup_s, 3), "stamps": st.get("stamps"),
                       "rays_per_sample": round(rays_total / (a.steps * a.spp * a.width * rows * world), 4)},
        }
        if cpu:
            out["detail"]["gpu_over_cpu"] = round(value / cpu["value"], 1)
        if emulate > 1:
            out["config"]["emulated"] = (f"rank 0 of {emulate}: {rows} of {a.height} rows on this GPU, no gather; "
                                         "value is this GPU's rate, not a job rate")
        print(json.dumps(out), flush=True)
    tr.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
