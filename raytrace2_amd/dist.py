"""Multi-GPU plumbing for callers that move the band stacks themselves: the interleaved row-band
partition of the framebuffer and a torch.distributed gather of every rank's bands to rank 0 (RCCL
over xGMI with device tensors on MI355X, gloo with host tensors in the CPU tests). The product's own
gather is rt2_tracer_gather in librt2.so (ncclGather + the root's de-interleave kernel); this module
is the same layout in torch terms.

The render itself needs no communication: pixels are independent (RayTracer.cpp:62-69) and the
sample streams are keyed by (seed, global pixel, frame), so the gathered image is bit-identical to
a single-GPU render. The only exchange is this gather.
"""
from __future__ import annotations

from typing import List, Optional

import numpy as np
import torch
import torch.distributed as dist

from ._native import check, lib
from .tracer import _fp, local_rows


def band_rows_max(height: int, band_h: int, world: int) -> int:
    """Rows every rank sends (its band stack padded to the largest rank's; rt2_band_rows_max, the
    same function the C ABI's gather uses)."""
    return check(lib.rt2_band_rows_max(int(height), int(band_h), int(world)))


def deinterleave(stacks: np.ndarray, height: int, band_h: int) -> np.ndarray:
    """Rank-major padded band stacks (world, max_rows, W, C) -> the image (H, W, C), through the C
    ABI's host de-interleave (rt2_layout.h BandSource, the map of the root's GPU kernel)."""
    stacks = np.ascontiguousarray(stacks, np.float32)
    world, max_rows, w, c = stacks.shape
    out = np.empty((height, w, c), np.float32)
    check(lib.rt2_deinterleave_host(_fp(stacks), _fp(out), w, height, int(band_h), world, max_rows, c))
    return out


def source_rows(height: int, band_h: int, world: int) -> np.ndarray:
    """Image row y -> row of the rank-major padded stacks viewed as (world * max_rows) rows: the C
    ABI's host de-interleave applied to the stacks' own row numbers (one channel)."""
    max_rows = band_rows_max(height, band_h, world)
    ids = np.arange(world * max_rows, dtype=np.float32).reshape(world, max_rows, 1, 1)
    return deinterleave(ids, height, band_h)[:, 0, 0].astype(np.int64)


class BandGather:
    """Gathers (rows_r, W, C) float32 band stacks of every rank into one (H, W, C) image on rank 0:
    every rank sends its padded stack (band_rows_max rows) with one torch.distributed gather into a
    rank-major buffer (the layout ncclGather fills inside rt2_tracer_gather), which rank 0
    de-interleaves with one index_select on the buffer's device by the C ABI's row map
    (source_rows). The image stays where the stacks are: a device tensor for device buffers (no host
    copy), a host tensor for CPU ones."""

    def __init__(self, height: int, width: int, band_h: int, world: int, rank: int, device: torch.device,
                 channels: int = 3, group: Optional[dist.ProcessGroup] = None):
        self.height, self.width, self.band_h, self.world, self.rank = height, width, band_h, world, rank
        self.group = group
        self.rows = [local_rows(height, band_h, r, world) for r in range(world)]
        self.max_rows = band_rows_max(height, band_h, world)
        self.send = torch.zeros((self.max_rows, width, channels), dtype=torch.float32, device=device)
        self.stacks: Optional[torch.Tensor] = None
        self.image: Optional[torch.Tensor] = None
        if rank == 0:
            self.stacks = torch.zeros((world, self.max_rows, width, channels), dtype=torch.float32, device=device)
            self.image = torch.zeros((height, width, channels), dtype=torch.float32, device=device)
            self.src = torch.from_numpy(source_rows(height, band_h, world)).to(device)

    def local_view(self) -> torch.Tensor:
        """The part of the send buffer this rank fills (its local rows)."""
        return self.send[:len(self.rows[self.rank])]

    def gather(self) -> Optional[torch.Tensor]:
        """Collective: every rank calls it; rank 0 returns the assembled image (on the stacks' device),
        the others None."""
        if self.world == 1:
            self.stacks[0].copy_(self.send)
        else:
            recv: Optional[List[torch.Tensor]] = list(self.stacks.unbind(0)) if self.rank == 0 else None
            dist.gather(self.send, recv, dst=0, group=self.group)
            if self.rank != 0:
                return None
        flat = self.stacks.view(self.world * self.max_rows, self.width, -1)
        torch.index_select(flat, 0, self.src, out=self.image)
        return self.image
