"""Multi-GPU plumbing: interleaved row-band partition of the framebuffer and the gather of every
rank's bands to rank 0 (one process per GPU, torch.distributed; RCCL over xGMI on MI355X, gloo in
the CPU tests).

The render itself needs no communication: pixels are independent (RayTracer.cpp:62-69) and the
sample streams are keyed by (seed, global pixel, frame), so the gathered image is bit-identical to
a single-GPU render. The only exchange is this gather.
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist

from .tracer import local_rows


def band_rows_max(height: int, band_h: int, world: int) -> int:
    """Upper bound of the rows a rank owns (send-buffer height, equal on every rank)."""
    bands = -(-height // band_h)
    return -(-bands // world) * band_h


class BandGather:
    """Gathers (rows_r, W, C) float32 band stacks of every rank into one (H, W, C) image on rank 0."""

    def __init__(self, height: int, width: int, band_h: int, world: int, rank: int, device: torch.device,
                 channels: int = 3, group: Optional[dist.ProcessGroup] = None):
        self.height, self.width, self.band_h, self.world, self.rank = height, width, band_h, world, rank
        self.group = group
        self.rows = [local_rows(height, band_h, r, world) for r in range(world)]
        self.max_rows = band_rows_max(height, band_h, world)
        self.send = torch.zeros((self.max_rows, width, channels), dtype=torch.float32, device=device)
        self.recv: Optional[List[torch.Tensor]] = None
        self.image: Optional[torch.Tensor] = None
        self.index: Optional[List[torch.Tensor]] = None
        if rank == 0:
            self.recv = [torch.zeros_like(self.send) for _ in range(world)]
            self.image = torch.zeros((height, width, channels), dtype=torch.float32, device=device)
            self.index = [torch.tensor(r, dtype=torch.long, device=device) for r in self.rows]

    def local_view(self) -> torch.Tensor:
        """The part of the send buffer this rank fills (its local rows)."""
        return self.send[:len(self.rows[self.rank])]

    def gather(self) -> Optional[torch.Tensor]:
        """Collective: every rank calls it; rank 0 returns the assembled image, others None."""
        if self.world == 1:
            n = len(self.rows[0])
            self.image[:n].copy_(self.send[:n])  # rows == all rows, already in order
            return self.image
        dist.gather(self.send, self.recv if self.rank == 0 else None, dst=0, group=self.group)
        if self.rank != 0:
            return None
        for r in range(self.world):
            n = len(self.rows[r])
            if n:
                self.image.index_copy_(0, self.index[r], self.recv[r][:n])
        return self.image
