"""Multi-GPU partition of the render (one process per GPU, torch.distributed).

The reference renders on one Taichi device only (renderer.py:16; no
collective anywhere). Pixels are independent (kernels.py:1184
writes only accum[py, px]) and every path's random stream is keyed by
(seed, pixel, sample) (include/ptmi_rng.h), so the render shards without any
exchange during rendering. Two partitions:

* ``tiles``: interleaved row bands (band_rows rows, round-robin over ranks)
  — every pixel is rendered entirely by one rank, so the assembled image is
  bit-identical to a 1-GPU render;
* ``samples``: every rank renders the whole image for a disjoint set of
  sample indices (weak scaling: fixed work per GPU); the sum-reduce adds the
  partial accumulators (equal to the 1-GPU render up to f32 summation order).

Image assembly is one collective per render (RCCL over xGMI on MI355X; gloo
in the CPU tests), ``assemble_image``:
* tiles: a ``gather`` of each rank's owned row bands onto the root (no
  arithmetic, so the image is bit-identical to one GPU; each rank sends only
  its own rows, W*rows*12 bytes: 7.7 MB / 8 at 800x800, 99.5 MB / 8 at
  3840x2160, instead of reducing a full-frame accumulator that is 7/8 zeros);
* samples: a sum-``reduce`` of the full accumulators (every rank holds every
  pixel).

Every collective here runs whenever a process group is initialised, at world
size 1 too (a gather / reduce / all-reduce / all-gather over one rank), so
``bench.py --gpus 1 --dist-backend nccl`` and tests/test_gpu_rccl.py execute
the exact RCCL calls of an N-GPU run on the one GPU of a test box. Without a
process group they are no-ops.
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


def _initialized():
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized()


def _host_staged(t, group=None):
    """gloo is only the multi-rank rehearsal backend: it reduces / gathers
    host tensors, so device tensors go through a host copy."""
    import torch.distributed as dist
    return t.is_cuda and dist.get_backend(group) == 'gloo'


def reduce_accum(accum, dst=0, group=None):
    """Sum-reduce the accumulator onto `dst` (in place); no-op without a
    process group."""
    import torch.distributed as dist
    if _initialized():
        if _host_staged(accum, group):
            host = accum.cpu()
            dist.reduce(host, dst=dst, op=dist.ReduceOp.SUM, group=group)
            accum.copy_(host)
        else:
            dist.reduce(accum, dst=dst, op=dist.ReduceOp.SUM, group=group)
    return accum


def max_over_ranks(value, device=None, group=None):
    import torch
    import torch.distributed as dist
    if not _initialized():
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def assemble_image(accum, shard, dst=0, group=None):
    """Assemble the image of a sharded render on `dst` (in place).

    tiles: every rank owns whole rows (shard.rows), so the root needs only the
    other ranks' rows, copied, not added: each rank packs its rows into a
    (max_rows, W, 3) buffer (max_rows = the largest rank share, so every
    gather buffer has one shape) and one ``gather`` brings them to the root,
    which writes them into its accumulator. samples: ``reduce_accum``.
    No-op without a process group; with one, the collective runs at every
    world size (at world 1 the root gathers its own rows)."""
    import torch
    import torch.distributed as dist
    if not _initialized():
        return accum
    if shard.mode != 'tiles':
        return reduce_accum(accum, dst, group)
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    H = accum.shape[0]
    rows_of = [Shard(r, world, 'tiles', shard.band_rows).rows(H) for r in range(world)]
    max_rows = max(len(r) for r in rows_of)
    dev = torch.device('cpu') if _host_staged(accum, group) else accum.device
    mine = torch.tensor(rows_of[rank], dtype=torch.long, device=accum.device)
    send = torch.zeros((max_rows,) + tuple(accum.shape[1:]), dtype=accum.dtype, device=accum.device)
    send[:len(rows_of[rank])] = accum.index_select(0, mine)
    send = send.to(dev)
    recv = [torch.empty_like(send) for _ in range(world)] if rank == dst else None
    dist.gather(send, gather_list=recv, dst=dst, group=group)
    if rank == dst:
        for r in range(world):
            if r != rank and rows_of[r]:
                idx = torch.tensor(rows_of[r], dtype=torch.long, device=accum.device)
                accum.index_copy_(0, idx, recv[r][:len(rows_of[r])].to(accum.device))
    return accum


def gather_ranks(vals, device=None, group=None):
    """Per-rank float rows (one ``all_gather`` of float64) -> list of lists,
    rank order; [vals] without a process group."""
    import torch
    import torch.distributed as dist
    if not _initialized():
        return [list(vals)]
    t = torch.tensor([float(v) for v in vals], dtype=torch.float64, device=device)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size(group))]
    dist.all_gather(out, t, group=group)
    return [o.cpu().tolist() for o in out]
