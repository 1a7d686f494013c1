"""Multi-GPU partition of the render (one process per GPU, torch.distributed).

The reference renders on one Taichi device only (renderer.py:16; no
collective anywhere). Pixels are independent (kernels.py:1184
writes only accum[py, px]) and every path's random stream is keyed by
(seed, pixel, sample) (include/ptmi_rng.h), so the render shards without any
exchange during rendering. Two partitions:

* ``tiles``: interleaved row bands (band_rows rows, round-robin over ranks)
  — every pixel is rendered entirely by one rank, so the gathered image is
  bit-identical to a 1-GPU render; one sum-reduce of the f32 accumulator
  (the other ranks' bands are zero) assembles it on the root.
* ``samples``: every rank renders the whole image for a disjoint set of
  sample indices (weak scaling: fixed work per GPU); the sum-reduce adds the
  partial accumulators (equal to the 1-GPU render up to f32 summation order).

The collective is a single ``reduce`` (RCCL over xGMI on MI355X; gloo in the
CPU tests): W*H*3*4 bytes = 7.7 MB at 800x800, once per render.
"""
from __future__ import annotations

from dataclasses import dataclass


@dataclass(frozen=True)
class Shard:
    rank: int
    world: int
    mode: str = 'samples'   # 'samples' | 'tiles'
    band_rows: int = 8

    @classmethod
    def balanced(cls, rank, world, mode, height, candidates=(8, 4, 2, 1), slack=0.01):
        """Shard whose band height gives every rank a near-equal row count
        (tiles): the tallest band among ``candidates`` whose largest rank
        share is within ``slack`` of the smallest achievable one. 800 rows
        over 8 ranks: 8-row bands give ranks 104 or 96 rows (100 bands, 4 %
        over the even share), 4-row bands 100 each; 2160 rows: 8-row bands
        (272 vs 270, kept). Taller bands keep more of a megakernel tile's 8
        rows adjacent in the image."""
        if mode != 'tiles' or world <= 1:
            return cls(rank, world, mode)

        def max_rows(b):
            return max(len(cls(r, world, mode, b).rows(height)) for r in range(world))
        best = min(max_rows(b) for b in candidates)
        band = next(b for b in candidates if max_rows(b) <= best * (1 + slack))
        return cls(rank, world, mode, band)

    def band(self):
        """(band_rows, band_stride, band_offset) for ptmi_frame."""
        if self.mode == 'tiles' and self.world > 1:
            return (self.band_rows, self.world, self.rank)
        return (1, 1, 0)

    def sample_range(self, step, spp_per_step):
        """First sample index and count this rank renders at `step`."""
        if self.mode == 'samples':
            return (step * self.world + self.rank) * spp_per_step, spp_per_step
        return step * spp_per_step, spp_per_step

    def rows(self, height):
        """Image rows this rank owns (tiles) or all rows (samples)."""
        b, s, o = self.band()
        return [r for r in range(height) if (r // b) % s == o]


def reduce_accum(accum, dst=0, group=None):
    """Sum-reduce the accumulator onto `dst` (in place); no-op for world 1."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        if accum.is_cuda and dist.get_backend(group) == 'gloo':  # rehearsal backend: reduce a host copy
            host = accum.cpu()
            dist.reduce(host, dst=dst, op=dist.ReduceOp.SUM, group=group)
            accum.copy_(host)
        else:
            dist.reduce(accum, dst=dst, op=dist.ReduceOp.SUM, group=group)
    return accum


def max_over_ranks(value, device=None, group=None):
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())
