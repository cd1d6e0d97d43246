"""Row-sharded exact top-k across GPUs.

The reference searches one faiss.IndexFlatIP (src/inference/vector_db.py:160,197).  Here the
catalog is split contiguously over the W ranks of a process group (rank r owns global rows
[r*N/W, (r+1)*N/W)), one process per GPU.  A search step for the buyers each rank encoded:

  1. all-gather the query batch                     [W*B, E]   (RCCL over xGMI)
  2. search the local shard for ALL queries          [W*B, k]   global row ids (row_base)
  3. all-to-all: the block of B rows for rank j goes back to rank j  -> [W, B, k]
  4. merge the W sorted lists (tt_topk_merge_f32)    [B, k]

A score does not depend on the shard, and the merge order is the scan's (score desc, lower
global row first), so the result is bit-identical to a single-GPU search of the whole
catalog.  ``TopkExchange`` is the collective part; the local search and the merge are passed
in, so the same code runs on GPUs (HIP kernels, nccl = RCCL) and in the gloo CPU tests.
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import torch
import torch.distributed as dist

Tensor = torch.Tensor


def shard_range(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous rows [lo, hi) of rank ``rank`` (sizes differ by at most one row)."""
    return rank * n // world, (rank + 1) * n // world


def _world(group) -> Tuple[int, int]:
    if not dist.is_available() or not dist.is_initialized():
        return 0, 1
    return dist.get_rank(group), dist.get_world_size(group)


class TopkExchange:
    """Collectives of one sharded search step for a fixed per-rank batch of B queries.

    Buffers are allocated once (no allocation inside a step)."""

    def __init__(self, b_local: int, width: int, k: int, device=None, group=None):
        self.group = group
        self.rank, self.world = _world(group)
        self.b, self.k = int(b_local), int(k)
        dev = device if device is not None else "cpu"
        self.qall = torch.empty((self.world * self.b, width), dtype=torch.float32, device=dev)
        self.s_recv = torch.empty((self.world, self.b, self.k), dtype=torch.float32, device=dev)
        self.i_recv = torch.empty((self.world, self.b, self.k), dtype=torch.int64, device=dev)

    def gather_queries(self, q: Tensor) -> Tensor:
        if q.shape[0] != self.b:
            raise ValueError(f"expected {self.b} local queries, got {q.shape[0]}")
        if self.world == 1:
            return q
        dist.all_gather_into_tensor(self.qall, q.contiguous(), group=self.group)
        return self.qall

    def return_results(self, s_shard: Tensor, i_shard: Tensor) -> Tuple[Tensor, Tensor]:
        """[W*B, k] per-shard results for every rank's queries -> [W, B, k] for my queries."""
        dist.all_to_all_single(self.s_recv.view(self.world * self.b, self.k),
                               s_shard.contiguous(), group=self.group)
        dist.all_to_all_single(self.i_recv.view(self.world * self.b, self.k),
                               i_shard.contiguous(), group=self.group)
        return self.s_recv, self.i_recv

    def search(self, q: Tensor, local_search: Callable[[Tensor], Tuple[Tensor, Tensor]],
               merge: Callable[[Tensor, Tensor, int], Tuple[Tensor, Tensor]]):
        """q: my B queries -> (scores [B, k], global ids [B, k]) over the whole catalog."""
        qall = self.gather_queries(q)
        s, i = local_search(qall)
        if self.world == 1:
            return s, i
        s_recv, i_recv = self.return_results(s, i)
        return merge(s_recv, i_recv, self.k)


def sharded_search(q: Tensor, k: int, local_search, merge, group=None):
    """Ragged variant: ranks may hold different numbers of queries.  Batches are padded to
    the group's maximum (one extra all-reduce) and the padding rows are dropped."""
    rank, world = _world(group)
    if world == 1:
        return local_search(q)
    b = torch.tensor([q.shape[0]], dtype=torch.int64, device=q.device)
    dist.all_reduce(b, op=dist.ReduceOp.MAX, group=group)
    bmax = int(b.item())
    qp = q
    if q.shape[0] < bmax:
        qp = torch.zeros((bmax, q.shape[1]), dtype=q.dtype, device=q.device)
        qp[: q.shape[0]] = q
    ex = TopkExchange(bmax, q.shape[1], k, device=q.device, group=group)
    s, i = ex.search(qp, local_search, merge)
    return s[: q.shape[0]], i[: q.shape[0]]


class ShardedFlatIP:
    """Rank-local shard of a row-sharded catalog, searched by the HIP kernels.

    ``add_shard`` takes this rank's rows (already normalised, like FlatIPIndex.add);
    ``search`` takes this rank's queries ([B, ep] device rows) and returns the global top-k.
    """

    def __init__(self, d: int, n_global: int, group=None, device=None):
        from .vector_db import FlatIPIndex

        self.group = group
        self.rank, self.world = _world(group)
        self.n_global = int(n_global)
        self.lo, self.hi = shard_range(self.n_global, self.rank, self.world)
        self.index = FlatIPIndex(d, device=device, row_base=self.lo)
        self._ex: Optional[TopkExchange] = None

    def add_shard(self, x) -> None:
        if x.shape[0] != self.hi - self.lo:
            raise ValueError(f"rank {self.rank} owns {self.hi - self.lo} rows, got {x.shape[0]}")
        self.index.add(x)

    def search(self, q: Tensor, k: int, method: str = "auto"):
        from . import kernels

        if self._ex is None or self._ex.b != q.shape[0] or self._ex.k != k:
            self._ex = TopkExchange(q.shape[0], q.shape[1], k, device=q.device, group=self.group)
        return self._ex.search(q, lambda qa: self._local(qa, k, method), kernels.merge_topk)

    def _local(self, qa: Tensor, k: int, method: str):
        """Local top-k with global ids; a shard smaller than k pads with (-inf, -1)."""
        kl = min(k, self.index.ntotal)
        if kl == k:
            return self.index.search_device(qa, k, method=method)
        s = torch.full((qa.shape[0], k), float("-inf"), dtype=torch.float32, device=qa.device)
        i = torch.full((qa.shape[0], k), -1, dtype=torch.int64, device=qa.device)
        if kl > 0:
            sl, il = self.index.search_device(qa, kl, method=method)
            s[:, :kl], i[:, :kl] = sl, il
        return s, i
