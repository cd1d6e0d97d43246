"""Row-sharded exact top-k across GPUs.

The reference searches one faiss.IndexFlatIP (src/inference/vector_db.py:160,197).  Here the
catalog is split contiguously over the W ranks of a process group (rank r owns global rows
[r*N/W, (r+1)*N/W)), one process per GPU.  A search step for the buyers each rank encoded:

  1. all-gather the query batch                     [W*B, E]   (RCCL over xGMI)
  2. search the local shard for ALL queries          [W*B, k]   global row ids (row_base)
  3. all-to-all: the block of B rows for rank j goes back to rank j  -> [W, B, k]
  4. merge the W sorted lists (tt_topk_merge_f32)    [B, k]

With the bf16 filter (k <= 128) step 2 is the staged protocol of include/twotower_hip.h
(tt_sharded_filter_*): each rank first derives its own queries' thresholds from a replicated
1/16 sample of the whole catalog (stats [B, 2], all-gathered with the queries), and one
all-reduce SUM of per-query probe counts [W*B, 16] int32 between the filter and the re-rank
lets every shard re-rank only rows that can reach the GLOBAL top-k.

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


def _dist_on() -> bool:
    """Collectives run whenever a process group exists -- at world size 1 too (trivially),
    so a one-GPU run exercises the RCCL calls of the W-GPU path."""
    return dist.is_available() and dist.is_initialized()


def _world(group) -> Tuple[int, int]:
    if not dist.is_available() or not dist.is_initialized():
        return 0, 1
    return dist.get_rank(group), dist.get_world_size(group)


class TopkExchange:
    """Collectives of one sharded search step for a fixed per-rank batch of B queries.

    Buffers are allocated once (no allocation inside a step)."""

    def __init__(self, b_local: int, width: int, k: int, device=None, group=None,
                 aux_width: int = 0):
        self.group = group
        self.rank, self.world = _world(group)
        self.active = _dist_on()
        self.b, self.k = int(b_local), int(k)
        dev = device if device is not None else "cpu"
        self.qall = torch.empty((self.world * self.b, width), dtype=torch.float32, device=dev)
        self.aux_all = (torch.empty((self.world * self.b, aux_width), dtype=torch.float32,
                                    device=dev) if aux_width else None)
        self.s_recv = torch.empty((self.world, self.b, self.k), dtype=torch.float32, device=dev)
        self.i_recv = torch.empty((self.world, self.b, self.k), dtype=torch.int64, device=dev)

    def gather_queries(self, q: Tensor, async_op: bool = False):
        """[B, w] my queries -> [W*B, w] every rank's (rank-major).  async_op: returns
        (qall, work); qall is valid on the current stream after work.wait()."""
        if q.shape[0] != self.b:
            raise ValueError(f"expected {self.b} local queries, got {q.shape[0]}")
        if not self.active:
            return (q, None) if async_op else q
        work = dist.all_gather_into_tensor(self.qall, q.contiguous(), group=self.group,
                                           async_op=async_op)
        return (self.qall, work) if async_op else self.qall

    def return_results(self, s_shard: Tensor, i_shard: Tensor) -> Tuple[Tensor, Tensor]:
        """[W*B, k] per-shard results for every rank's queries -> [W, B, k] for my queries."""
        dist.all_to_all_single(self.s_recv.view(self.world * self.b, self.k),
                               s_shard.contiguous(), group=self.group)
        dist.all_to_all_single(self.i_recv.view(self.world * self.b, self.k),
                               i_shard.contiguous(), group=self.group)
        return self.s_recv, self.i_recv

    def gather_aux(self, aux: Tensor) -> Tensor:
        """Per-query side data [B, aux_width] f32 (the sharded filter's stats), same order."""
        if not self.active:
            return aux
        dist.all_gather_into_tensor(self.aux_all, aux.contiguous(), group=self.group)
        return self.aux_all

    def search(self, q: Tensor, local_search: Callable[..., Tuple[Tensor, Tensor]],
               merge: Callable[[Tensor, Tensor, int], Tuple[Tensor, Tensor]],
               aux: Optional[Tensor] = None):
        """q: my B queries -> (scores [B, k], global ids [B, k]) over the whole catalog.
        With aux [B, a]: local_search(qall, aux_all) gets every rank's aux rows too.  aux may
        be a callable producing them (the sharded filter's begin stage): the query all-gather
        is then launched first, asynchronously, and overlaps that computation."""
        if callable(aux):
            qall, work = self.gather_queries(q, async_op=True)
            aux_all = self.gather_aux(aux())
            if work is not None:
                work.wait()
            s, i = local_search(qall, aux_all)
        elif aux is not None:
            s, i = local_search(self.gather_queries(q), self.gather_aux(aux))
        else:
            s, i = local_search(self.gather_queries(q))
        if not self.active:
            return s, i
        s_recv, i_recv = self.return_results(s, i)
        return merge(s_recv, i_recv, self.k)


class PipelinedStagedExchange:
    """The staged sharded search (tt_sharded_filter_begin / _full / _finish) with the ranks'
    queries in ``chunks`` chunks whose collectives overlap the next chunk's shard filter.

    Per step (every rank, C chunks of its B queries):
      1. per chunk: all-gather the queries (async on RCCL's stream), begin() on my chunk while
         it is in flight, all-gather its stats;
      2. chunk c: full(c) -> probe counts, all-reduce SUM launched async; chunk c-1's finish()
         and its result all-to-all (async) are issued after chunk c's filter was enqueued, so
         the all-reduce and all-to-all of one chunk run under the filter of the next;
      3. per chunk: wait for its all-to-all, merge the W sorted lists.
    ``begin(q_c) -> stats [b_c, 2]``; ``full(c, qall_c, sall_c) -> pcount [W*b_c, P] int32``;
    ``finish(c, qall_c, sall_c, pcount) -> (scores, ids) [W*b_c, k]`` (chunk-private
    workspaces: chunk c's band lists live until its finish).  Queries are independent, so the
    result is bit-identical to one unchunked search (and to one GPU searching the catalog)."""

    def __init__(self, b_local: int, width: int, k: int, chunks: int = 2, device=None,
                 group=None):
        self.group = group
        self.rank, self.world = _world(group)
        self.active = _dist_on()
        self.b, self.k = int(b_local), int(k)
        chunks = max(1, min(int(chunks), self.b))
        cut = [self.b * c // chunks for c in range(chunks + 1)]
        self.bounds = [(cut[c], cut[c + 1]) for c in range(chunks)]
        self.ex = [TopkExchange(hi - lo, width, k, device=device, group=group, aux_width=2)
                   for lo, hi in self.bounds]

    def _a2a(self, ex: TopkExchange, s: Tensor, i: Tensor):
        if not self.active:
            return None
        w1 = dist.all_to_all_single(ex.s_recv.view(self.world * ex.b, self.k), s.contiguous(),
                                    group=self.group, async_op=True)
        w2 = dist.all_to_all_single(ex.i_recv.view(self.world * ex.b, self.k), i.contiguous(),
                                    group=self.group, async_op=True)
        return (w1, w2)

    def search(self, q: Tensor, begin, full, finish, merge):
        if q.shape[0] != self.b:
            raise ValueError(f"expected {self.b} local queries, got {q.shape[0]}")
        C = len(self.ex)
        qc = [q[lo:hi] for lo, hi in self.bounds]
        gathered = [ex.gather_queries(x, async_op=True) for ex, x in zip(self.ex, qc)]
        sall = [ex.gather_aux(begin(x)) for ex, x in zip(self.ex, qc)]
        qall = []
        for qa, work in gathered:
            if work is not None:
                work.wait()
            qall.append(qa)
        outs = [None] * C
        pend = None
        for c in range(C + 1):
            nxt = None
            if c < C:
                pc = full(c, qall[c], sall[c])
                w = (dist.all_reduce(pc, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
                     if self.active else None)
                nxt = (c, pc, w)
            if pend is not None:
                cp, pcp, wp = pend
                if wp is not None:
                    wp.wait()
                s, i = finish(cp, qall[cp], sall[cp], pcp)
                outs[cp] = (s, i, self._a2a(self.ex[cp], s, i))
            pend = nxt
        res_s, res_i = [], []
        for c, (s, i, works) in enumerate(outs):
            if works is None:  # no process group: the local result is the global one
                res_s.append(s)
                res_i.append(i)
                continue
            for wk in works:
                wk.wait()
            ms, mi = merge(self.ex[c].s_recv, self.ex[c].i_recv, self.k)
            res_s.append(ms)
            res_i.append(mi)
        return torch.cat(res_s), torch.cat(res_i)


def sharded_search(q: Tensor, k: int, local_search, merge, group=None):
    """Ragged variant: ranks may hold different numbers of queries.  Batches are padded to
    the group's maximum (one extra all-reduce) and the padding rows are dropped."""
    if not _dist_on():
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

    ``add_shard`` takes this rank's rows (already normalised, like FlatIPIndex.add) and builds
    the replicated catalog sample + whole-catalog bf16 bounds (collectives, once);
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
        self._pipe: Optional[PipelinedStagedExchange] = None
        self._ws_chunks = []
        self.chunks = 2  # staged search: query chunks whose collectives overlap the next filter
        self.sample16: Optional[Tensor] = None
        self.bounds = (0.0, 0.0)
        self._ws_begin: Optional[Tensor] = None

    def add_shard(self, x) -> None:
        if x.shape[0] != self.hi - self.lo:
            raise ValueError(f"rank {self.rank} owns {self.hi - self.lo} rows, got {x.shape[0]}")
        self.index.add(x)
        if _dist_on():
            self._build_sample()

    def _build_sample(self) -> None:
        """Global rows 0, 16, 32, ... of the bf16 image on every rank (all-gather, padded to
        the largest rank's count) and the bounds MAX over ranks."""
        from . import _lib

        st = _lib.TT_SHARD_SAMPLE_STRIDE
        ix = self.index
        mine = ix.xb16[(-self.lo) % st: ix.ntotal: st]
        cnt = torch.tensor([mine.shape[0]], dtype=torch.int64, device=ix.device)
        cnts = [torch.zeros_like(cnt) for _ in range(self.world)]
        dist.all_gather(cnts, cnt, group=self.group)
        cnts = [int(c.item()) for c in cnts]
        cmax = max(cnts)
        pad = torch.zeros((cmax, ix.ep), dtype=torch.bfloat16, device=ix.device)
        pad[: mine.shape[0]] = mine
        allp = torch.empty((self.world * cmax, ix.ep), dtype=torch.bfloat16, device=ix.device)
        dist.all_gather_into_tensor(allp.view(torch.int32), pad.view(torch.int32),
                                    group=self.group)
        self.sample16 = torch.cat([allp[r * cmax: r * cmax + c] for r, c in enumerate(cnts)])
        b = torch.tensor(ix.bounds, dtype=torch.float32, device=ix.device)
        dist.all_reduce(b, op=dist.ReduceOp.MAX, group=self.group)
        self.bounds = tuple(b.tolist())

    def _staged(self, k: int, method: str) -> bool:
        """Every rank takes the same branch: decided from (n_global, world, k, method) only."""
        smallest = self.n_global // self.world
        return (_dist_on() and method in ("auto", "bf16") and 1 <= k <= 128
                and smallest >= k)

    def search(self, q: Tensor, k: int, method: str = "auto"):
        from . import kernels

        staged = self._staged(k, method)
        if staged:
            return self._search_staged(q, k)
        if self._ex is None or self._ex.b != q.shape[0] or self._ex.k != k:
            self._ex = TopkExchange(q.shape[0], q.shape[1], k, device=q.device, group=self.group)
        return self._ex.search(q, lambda qa: self._local(qa, k, method), kernels.merge_topk)

    def _search_staged(self, q: Tensor, k: int):
        """The staged bf16 protocol through PipelinedStagedExchange (self.chunks chunks)."""
        from . import kernels

        ix = self.index
        p = self._pipe
        if p is None or p.b != q.shape[0] or p.k != k or len(p.ex) != min(self.chunks, q.shape[0]):
            p = self._pipe = PipelinedStagedExchange(q.shape[0], q.shape[1], k, self.chunks,
                                                     device=q.device, group=self.group)
        bmax = max(ex.b for ex in p.ex)
        need = kernels.filter_workspace_bytes(self.sample16.shape[0], ix.d, bmax,
                                              min(k, self.sample16.shape[0]))
        if self._ws_begin is None or self._ws_begin.numel() < need:
            self._ws_begin = torch.empty(need, dtype=torch.uint8, device=ix.device)
        while len(self._ws_chunks) < len(p.ex):
            self._ws_chunks.append(None)
        for c, ex in enumerate(p.ex):  # chunk-private: chunk c's bands live until its finish
            need = kernels.sharded_workspace_bytes(ix.ntotal, ix.d, p.world * ex.b, k)
            if self._ws_chunks[c] is None or self._ws_chunks[c].numel() < need:
                self._ws_chunks[c] = torch.empty(need, dtype=torch.uint8, device=ix.device)
        ws = self._ws_chunks
        return p.search(
            q,
            lambda x: kernels.sharded_begin(self.sample16, ix.d, x, k, workspace=self._ws_begin),
            lambda c, qa, sa: kernels.sharded_full(ix.xb16, ix.ntotal, ix.d, qa, k, self.bounds,
                                                   sa, ws[c]),
            lambda c, qa, sa, pc: kernels.sharded_finish(ix.xb, ix.xb16, ix.ntotal, ix.d, qa, k,
                                                         ix.row_base, sa, pc, ws[c]),
            kernels.merge_topk)

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
