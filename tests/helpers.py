"""Shared helpers: product (GPU, through the C ABI) and oracle (CPU restatement) renders."""
import numpy as np

from conftest import scene_path

SEED = 0x5EED2024


def _gpu_render_once(name, w, h, spp, frames, *, seed, max_depth, band_h, rank, world, launch_frames, updates,
                     stats, work_split, sample_budget, batch_max, ray_counts, lazy):
    import torch  # noqa: F401
    import raytrace2_amd as R
    sc = R.Scene(scene_path(name), seed)
    tr = R.RayTracer(sc, 0)
    tr.set_seed(seed)
    tr.SetSamplesPerPixel(spp)
    tr.max_depth = max_depth
    if ray_counts:
        tr.enable_ray_counts(True)
    if stats:
        tr.enable_stats(True)
    tr.OnResize((w, h))
    if world > 1 or band_h:
        tr.set_partition(band_h, rank, world)
    if launch_frames:
        tr.set_launch_frames(launch_frames)
    if work_split is not None:
        tr.set_work_split(work_split)
    if sample_budget is not None:
        tr.set_sample_budget(sample_budget)
    if batch_max is not None:
        tr.set_batch_max(batch_max)
    if lazy is not None:
        tr.set_lazy_frames(lazy)
    if updates:
        for _ in range(frames):
            tr.Update(sc)
    else:
        tr.Render(frames)
    acc = tr.Accumulation()
    rc = tr.ray_counts() if ray_counts else None
    st = tr.stats()
    px = tr.Pixels()
    tr.close()
    return acc, rc, st, px


def gpu_render(name, w, h, spp, frames, *, seed=SEED, max_depth=50, band_h=0, rank=0, world=1,
               launch_frames=0, updates=False, stats=False, work_split=None, sample_budget=None, batch_max=None,
               counts=True, lazy=None):
    """Renders with the product kernel (no per-pixel counters) and, when `counts`, again with the
    counting kernel (per-pixel ray counts); the two must agree bit for bit. Returns the product
    render's (accumulation, ray counts of the counting render or None, stats, pixels)."""
    kw = dict(seed=seed, max_depth=max_depth, band_h=band_h, rank=rank, world=world, launch_frames=launch_frames,
              updates=updates, work_split=work_split, sample_budget=sample_budget, batch_max=batch_max, lazy=lazy)
    acc, _, st, px = _gpu_render_once(name, w, h, spp, frames, stats=stats, ray_counts=False, **kw)
    rc = None
    if counts:
        acc2, rc, st2, px2 = _gpu_render_once(name, w, h, spp, frames, stats=True, ray_counts=True, **kw)
        assert np.array_equal(acc.view(np.uint32), acc2.view(np.uint32)), "product and counting kernels differ"
        assert np.array_equal(px, px2)
        assert st["rays"] == st2["rays"] == int(rc.astype(np.uint64).sum()), (st["rays"], st2["rays"])
        assert st["paths"] == st2["paths"]
    return acc, rc, st, px


def oracle_render(name, w, h, spp, frames, *, seed=SEED, max_depth=50, band_h=0, rank=0, world=1,
                  forward=True, threads=0):
    from oracle.oracle import OracleScene
    o = OracleScene(scene_path(name), seed)
    acc, rc, cnt = o.render(w, h, spp, frames, max_depth=max_depth, band_h=band_h, rank=rank, world=world,
                            forward=forward, threads=threads)
    return acc, rc, cnt


def rmse(a, b):
    return float(np.sqrt(np.mean((np.asarray(a, np.float64) - np.asarray(b, np.float64)) ** 2)))
