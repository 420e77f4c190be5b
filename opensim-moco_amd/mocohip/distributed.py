"""Mesh-interval sharding over ranks (one process per GPU).

The g rows and Jacobian nonzeros of mesh interval i are contiguous, and
every interval has the same row count and the same nonzero count
(CasOCTranscription.h:219-313). So rank r owns the
intervals [N*r/W, N*(r+1)/W) and evaluates only those (mh_options
interval_begin/interval_end). One all-gather of the fixed-size, padded
segments rebuilds the full g and Jacobian values on every rank, which is
what a single host IPOPT needs. The boundary grid point
between two shards is evaluated by both ranks: recomputing it is cheaper
than exchanging it.

The same code runs over RCCL (backend "nccl", device tensors, bench.py) and
over gloo on the CPU (tests/test_distributed.py).
"""
from __future__ import annotations

from typing import List, Tuple


def interval_shard(num_intervals: int, rank: int, world: int) -> Tuple[int, int]:
    """[begin, end) mesh intervals owned by ``rank``."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    return (num_intervals * rank) // world, (num_intervals * (rank + 1)) // world


def shard_counts(num_intervals: int, world: int) -> List[int]:
    return [e - b for b, e in (interval_shard(num_intervals, r, world) for r in range(world))]


class ShardGather:
    """Fixed-size segment buffers and their all-gather.

    Each rank writes its shard's g rows into ``gseg[:g_sizes[rank]]`` and its
    Jacobian values into ``vseg[:v_sizes[rank]]``.
    ``gather()`` all-gathers both. The results are padded per rank to the
    largest shard; ``full_g()`` / ``full_values()`` return the unpadded full
    vectors in the global row / nonzero order.
    """

    def __init__(self, num_intervals: int, rows_per_interval: int, nnz_per_interval: int,
                 world: int, device, group=None, tail_rows: int = 0, tail_nnz: int = 0):
        """``tail_rows`` / ``tail_nnz``: rows and nonzeros after the last
        interval (implicit dynamics: the final grid point's residuals), owned
        by the last rank (mh_nlp_info row_end / nnz_end)."""
        import torch
        self.N, self.rpi, self.nzi, self.world = num_intervals, rows_per_interval, nnz_per_interval, world
        self.group = group
        self.counts = shard_counts(num_intervals, world)
        self.tail = (tail_rows, tail_nnz)
        self.g_sizes = [c * rows_per_interval + (tail_rows if r == world - 1 else 0)
                        for r, c in enumerate(self.counts)]
        self.v_sizes = [c * nnz_per_interval + (tail_nnz if r == world - 1 else 0)
                        for r, c in enumerate(self.counts)]
        f64 = torch.float64
        self.gseg = torch.zeros(max(self.g_sizes), dtype=f64, device=device)
        self.vseg = torch.zeros(max(self.v_sizes), dtype=f64, device=device)
        self.gall = torch.zeros(world * self.gseg.numel(), dtype=f64, device=device)
        self.vall = torch.zeros(world * self.vseg.numel(), dtype=f64, device=device)
        self._g_index = self._unpad_index(self.g_sizes, self.gseg.numel(), device)
        self._v_index = self._unpad_index(self.v_sizes, self.vseg.numel(), device)

    def _unpad_index(self, sizes, seg: int, device):
        import torch
        parts = [torch.arange(r * seg, r * seg + n, device=device) for r, n in enumerate(sizes)]
        return torch.cat(parts)

    def gather(self):
        import torch.distributed as dist
        if self.world == 1:
            self.gall.copy_(self.gseg)
            self.vall.copy_(self.vseg)
            return
        dist.all_gather_into_tensor(self.gall, self.gseg, group=self.group)
        dist.all_gather_into_tensor(self.vall, self.vseg, group=self.group)

    def full_g(self):
        return self.gall[self._g_index]

    def full_values(self):
        return self.vall[self._v_index]
