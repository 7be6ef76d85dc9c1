"""Progressive display loop: the reference's windowed loop without the window.

`App::Run` (src/App.cpp:176-242) calls `RayTracer::Update` once per displayed frame (one sample per
pixel) and uploads `Pixels()` to a GL texture, until `num_samples` frames are done. On a GPU one
1024^2 Cornell frame takes ~0.3 ms, so one sample per display refresh would leave it idle most of
the time, and a launch plus a readback per sample costs more than the sample itself. This loop
keeps the reference's frame semantics (frame f uses stratum (f % sq, f / sq % sq), samples are
summed in frame order, Pixels() = ToColor(clamp(accum / frame_idx))) but renders as many frames
per display tick as fit a time budget, adapting the count tick by tick, and reads Pixels() back
once per tick into pinned host memory. After F frames the accumulation is bit-identical to F
`Update()` calls.
"""
from __future__ import annotations

import ctypes
import time
from typing import Optional

import numpy as np

from ._native import check, lib


class PinnedBuffer:
    """Page-locked host memory (rt2_host_alloc) viewed as a numpy array."""

    def __init__(self, shape, dtype=np.uint8):
        self.nbytes = int(np.prod(shape)) * np.dtype(dtype).itemsize
        p = ctypes.c_void_p()
        check(lib.rt2_host_alloc(self.nbytes, ctypes.byref(p)))
        self._p = p
        buf = (ctypes.c_uint8 * self.nbytes).from_address(p.value)
        self.array = np.frombuffer(buf, dtype=dtype).reshape(shape)

    def close(self):
        if self._p is not None and self._p.value:
            lib.rt2_host_free(self._p)
        self._p = None

    def __del__(self):
        self.close()


class ProgressiveLoop:
    """Ticks of `frames_per_tick` frames, adapted so that a tick takes about `budget_ms`."""

    def __init__(self, tracer, total_frames: int, budget_ms: float = 16.0, first_frames: int = 1,
                 max_frames_per_tick: int = 4096):
        self.tr = tracer
        w, _ = tracer.Dims()
        self.pixels = PinnedBuffer((tracer.local_rows(), w, 4))
        self.total = int(total_frames)
        self.budget = float(budget_ms)
        self.n = max(1, int(first_frames))
        self.cap = int(max_frames_per_tick)
        self.ticks = 0
        self.frames_done = 0

    def done(self) -> bool:
        return self.frames_done >= self.total

    def tick(self) -> Optional[np.ndarray]:
        """Renders the next frames of the budget, returns Pixels() after them (None when done)."""
        if self.done():
            return None
        n = min(self.n, self.total - self.frames_done)
        t0 = time.perf_counter()
        self.tr.Render(n)
        check(lib.rt2_tracer_pixels_async(self.tr._h, self.pixels.array.ctypes.data_as(
            ctypes.POINTER(ctypes.c_uint8))))
        self.tr.synchronize()
        dt_ms = (time.perf_counter() - t0) * 1e3
        self.frames_done += n
        self.ticks += 1
        # next tick's frame count: proportional to the budget, at most doubling per tick
        scale = self.budget / max(dt_ms, 1e-3)
        self.n = int(max(1, min(self.cap, 2 * n, round(n * scale))))
        return self.pixels.array

    def run(self, on_tick=None) -> None:
        while not self.done():
            px = self.tick()
            if on_tick is not None:
                on_tick(self, px)

    def close(self):
        self.pixels.close()
