"""N>1 path on the CPU: world_size-2/3 gloo process groups running the band partition + gather of the
C ABI's multi-GPU path: every rank sends its band stack padded to rt2_band_rows_max rows, the root
receives the rank-major stacks (the layout ncclGather delivers inside rt2_tracer_gather) and
de-interleaves them with rt2_deinterleave_host, the same index map (rt2_layout.h BandSource) as the
root's GPU kernel. Each rank renders its row bands with the CPU restatement (stand-in renderer, no GPU
here); the gathered image must equal the single-process render bit for bit, because sample streams
are keyed by global pixel and frame."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT, scene_path

W, H, BAND, SPP, FRAMES = 40, 45, 8, 16, 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_path):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from raytrace2_amd.dist import BandGather
    from oracle.oracle import OracleScene
    g = BandGather(H, W, BAND, world, rank, torch.device("cpu"))
    acc, _, _ = OracleScene(scene_path("cornell_box_original")).render(W, H, SPP, FRAMES, band_h=BAND, rank=rank,
                                                                       world=world, forward=True)
    assert acc.shape[0] == g.local_view().shape[0]
    g.local_view().copy_(torch.from_numpy(acc))
    img = g.gather()
    if rank == 0:
        np.save(out_path, img.numpy())
    else:
        assert img is None
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_band_gather_equals_single_render(tmp_path, world):
    out = str(tmp_path / "img.npy")
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    img = np.load(out)
    from oracle.oracle import OracleScene
    full, _, _ = OracleScene(scene_path("cornell_box_original")).render(W, H, SPP, FRAMES, forward=True)
    assert np.array_equal(img.view(np.uint32), full.view(np.uint32))


@pytest.mark.parametrize("h,band_h,world", [(45, 8, 3), (1024, 16, 8), (800, 16, 8), (1024, 8, 8), (10, 8, 4), (7, 1, 7)])
def test_band_partition_covers_every_row_once(h, band_h, world):
    """rt2_layout.h BandRank: the ranks' rows are disjoint, cover the image, and every rank owns one
    band of each full period, its phase rotating by one per period."""
    from raytrace2_amd.tracer import band_rank, local_rows
    parts = [local_rows(h, band_h, r, world) for r in range(world)]
    assert sorted(y for p in parts for y in p) == list(range(h))
    assert max(map(len, parts)) - min(map(len, parts)) <= band_h
    bands = -(-h // band_h)
    for p in range(bands // world):
        owners = [band_rank(p * world + q, world) for q in range(world)]
        assert sorted(owners) == list(range(world))
        assert owners[0] == p % world


@pytest.mark.parametrize("h,band_h,world", [(45, 8, 3), (47, 16, 1), (40, 16, 1), (10, 8, 4), (33, 2, 8), (9, 0, 1),
                                            (1024, 2, 8), (7, 1, 7)])
def test_c_abi_deinterleave_inverts_the_partition(h, band_h, world):
    """rt2_band_rows_max / rt2_deinterleave_host (the C ABI's gather layout) against the Python
    statement of the partition: random band stacks, padded rows poisoned, reassemble exactly."""
    from raytrace2_amd.dist import band_rows_max, deinterleave
    from raytrace2_amd.tracer import assemble_bands, local_rows
    w = 5
    rng = np.random.default_rng(h * 31 + band_h + world)
    mr = band_rows_max(h, band_h, world)
    rows = [local_rows(h, band_h, r, world) for r in range(world)]
    assert mr == max(len(r) for r in rows) or (band_h and mr - max(len(r) for r in rows) < band_h)
    parts = [rng.standard_normal((len(r), w, 3)).astype(np.float32) for r in rows]
    stacks = np.full((world, mr, w, 3), np.nan, np.float32)  # padding must never be read
    for r, p in enumerate(parts):
        stacks[r, :len(p)] = p
    img = deinterleave(stacks, h, band_h)
    assert np.array_equal(img.view(np.uint32), assemble_bands(parts, h, band_h).view(np.uint32))


@pytest.mark.parametrize("n,height,band_h", [(8, 1024, 0), (8, 1080, 2), (4, 45, 8), (2, 7, 3), (3, 1, 0), (1, 1024, 0)])
def test_multi_plan_partition_for_distinct_devices(n, height, band_h):
    """rt2_tracer_create_multi's argument checks and per-GPU partition (rt2_multi_plan), on the host:
    N distinct device ids without initialising RCCL or touching a GPU. Part i is rank i on device i,
    its rows are the Python statement of the band partition, and every part sends rows_max rows (whole
    bands for every period) in the gather."""
    from raytrace2_amd._native import multi_plan
    from raytrace2_amd.tracer import local_rows
    devices = list(range(n))[::-1]  # any distinct ids
    parts, loopback = multi_plan(n, devices, band_h, 1024, height)
    assert not loopback and len(parts) == n
    bh = band_h or 2
    rows = [len(local_rows(height, bh, r, n)) for r in range(n)]
    assert [p["device"] for p in parts] == devices and [p["rank"] for p in parts] == list(range(n))
    assert all(p["world"] == n and p["band_h"] == bh for p in parts)
    assert [p["local_rows"] for p in parts] == rows and sum(rows) == height
    bands = -(-height // bh)
    assert all(p["rows_max"] == -(-bands // n) * bh >= max(rows) for p in parts)  # whole bands per period


def test_multi_plan_rejects_bad_arguments():
    from raytrace2_amd._native import Rt2Error, multi_plan
    assert multi_plan(4, [2, 2, 2, 2])[1]  # one GPU listed n times: loopback (tests' configuration)
    assert not multi_plan(1, [5])[1]
    for args in [(0, None), (3, [0, 1, 1]), (2, [0, -1]), (2, [0, 1], -1)]:
        with pytest.raises(Rt2Error):
            multi_plan(*args)
    # a device list of another length than n_gpus is refused before the C call (the C
    # side reads n_gpus entries)
    for n, devs in [(3, [0, 1]), (1, [0, 1])]:
        with pytest.raises(ValueError):
            multi_plan(n, devs)
