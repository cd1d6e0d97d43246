"""Row-sharded search (twotower.sharded) on CPU with gloo.

The collective layout (all-gather of queries, all-to-all of per-shard top-k, merge) is the
same code the GPU path runs over RCCL; here the local search is the CPU oracle and the merge
a numpy restatement of tt_topk_merge_f32's order (score desc, lower global row).  Result:
bit-identical to one search over the whole catalog, for even and ragged query batches.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "two-tower-model-v2_amd"))
sys.path.insert(0, ROOT)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def merge_np(s_recv, i_recv, k):
    """[W, B, k_in] sorted lists (global ids, -1 = empty) -> [B, k], tt_topk_merge_f32 order."""
    W, B, kin = s_recv.shape
    out_s = torch.full((B, k), float("-inf"))
    out_i = torch.full((B, k), -1, dtype=torch.int64)
    for b in range(B):
        cand = [(float(s_recv[w, b, j]), int(i_recv[w, b, j])) for w in range(W) for j in range(kin)
                if int(i_recv[w, b, j]) >= 0 and s_recv[w, b, j] == s_recv[w, b, j]]
        cand.sort(key=lambda t: (-t[0], t[1]))
        for j, (sc, ix) in enumerate(cand[:k]):
            out_s[b, j], out_i[b, j] = sc, ix
    return out_s, out_i


def data(n=3001, d=48, nq=37, seed=5):
    from oracle import oracle as O

    rng = np.random.default_rng(seed)
    x = O.l2norm_rows(rng.standard_normal((n, d)).astype(np.float32), 0)
    x[100:140] = x[0:40]  # exact duplicates straddling nothing / ties across ranks below
    x[n // 2: n // 2 + 30] = x[0:30]
    q = O.l2norm_rows(rng.standard_normal((nq, d)).astype(np.float32), 0)
    return x, q


def _worker(rank, world, port, k, ragged, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O
        from twotower.sharded import TopkExchange, shard_range, sharded_search

        x, q = data()
        lo, hi = shard_range(x.shape[0], rank, world)
        xs = x[lo:hi]
        # this rank's buyers
        if ragged:
            cuts = [0, 5, q.shape[0]] if world == 2 else np.linspace(0, q.shape[0], world + 1).astype(int)
        else:
            cuts = [r * (q.shape[0] // world) for r in range(world + 1)]
        qa, qb = int(cuts[rank]), int(cuts[rank + 1])
        ql = torch.from_numpy(q[qa:qb].copy())

        def local(qall):
            s, i = O.scan_topk(xs, qall.numpy(), k, row_base=lo)
            return torch.from_numpy(s), torch.from_numpy(i)

        if ragged:
            s, i = sharded_search(ql, k, local, merge_np)
        else:
            ex = TopkExchange(ql.shape[0], q.shape[1], k)
            s, i = ex.search(ql, local, merge_np)
        np.save(os.path.join(out_dir, f"s{rank}.npy"), s.numpy())
        np.save(os.path.join(out_dir, f"i{rank}.npy"), i.numpy())
        np.save(os.path.join(out_dir, f"r{rank}.npy"), np.array([qa, qb]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,k,ragged", [(2, 10, False), (2, 100, True), (3, 64, True)])
def test_sharded_search_bit_identical_to_single(tmp_path, world, k, ragged):
    from oracle import oracle as O

    port = _free_port()
    mp.start_processes(_worker, args=(world, port, k, ragged, str(tmp_path)), nprocs=world,
                       join=True, start_method="fork")
    x, q = data()
    rs, ri = O.scan_topk(x, q, k)
    for r in range(world):
        qa, qb = np.load(tmp_path / f"r{r}.npy")
        s, i = np.load(tmp_path / f"s{r}.npy"), np.load(tmp_path / f"i{r}.npy")
        assert np.array_equal(i, ri[qa:qb]) and np.array_equal(s, rs[qa:qb])


def test_shard_range_covers_catalog():
    from twotower.sharded import shard_range

    for n in (1, 7, 1000, 10_000_001):
        for w in (1, 2, 3, 8):
            rs = [shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[j][1] == rs[j + 1][0] for j in range(w - 1))
            assert max(b - a for a, b in rs) - min(b - a for a, b in rs) <= 1


def test_exchange_single_process_is_passthrough():
    from twotower.sharded import TopkExchange

    ex = TopkExchange(4, 8, 3)
    q = torch.randn(4, 8)
    s, i = ex.search(q, lambda qa: (qa[:, :3], torch.zeros(4, 3, dtype=torch.int64)), None)
    assert torch.equal(s, q[:, :3])


def _aux_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from twotower.sharded import TopkExchange

        B, k = 5, 3
        q = torch.arange(B * 4, dtype=torch.float32).view(B, 4) + 100 * rank
        aux = torch.stack([q[:, 0], -q[:, 0]], 1)  # per-query stats travel with the query
        seen = {}

        def local(qall, aux_all):
            seen["ok"] = bool(torch.equal(aux_all[:, 0], qall[:, 0])
                              and torch.equal(aux_all[:, 1], -qall[:, 0]))
            # the staged filter's probe-count exchange: SUM over ranks in place
            pc = torch.full((qall.shape[0], 16), rank + 1, dtype=torch.int32)
            dist.all_reduce(pc, op=dist.ReduceOp.SUM)
            seen["sum"] = int(pc[0, 0])
            s = qall[:, :k].clone()
            i = torch.arange(qall.shape[0] * k, dtype=torch.int64).view(-1, k)
            return s, i

        ex = TopkExchange(B, 4, k, aux_width=2)
        ex.search(q, local, lambda s, i, kk: (s[rank], i[rank]), aux=aux)
        ok0 = seen.pop("ok")
        # aux as a callable (the bench's overlapped form: async query gather under it)
        ex.search(q, local, lambda s, i, kk: (s[rank], i[rank]), aux=lambda: aux.clone())
        np.save(os.path.join(out_dir, f"aux{rank}.npy"),
                np.array([ok0 and seen["ok"], seen["sum"]], dtype=np.int64))
    finally:
        dist.destroy_process_group()


def test_exchange_gathers_aux_rows_with_queries(tmp_path):
    """The sharded filter's stats [B, 2] are all-gathered in query order next to the queries
    (TopkExchange aux), and the probe counts SUM over ranks."""
    world = 3
    mp.start_processes(_aux_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                       join=True, start_method="fork")
    for r in range(world):
        ok, tot = np.load(tmp_path / f"aux{r}.npy")
        assert ok == 1 and tot == sum(range(1, world + 1))


def _grad_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from twotower.train import allreduce_mean

        g = torch.Generator().manual_seed(rank)
        grads = {"proj0.w": torch.randn(256, 512, generator=g), "att2.b": torch.randn(1, generator=g),
                 "brand": torch.randn(51, 64, generator=g)}
        allreduce_mean(grads)
        # numpy by value: a torch tensor crosses the queue as a shared-memory handle that dies
        # with this process if it exits before the parent has received it
        q.put((rank, {k: v.numpy().copy() for k, v in grads.items()}))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_train_gradient_allreduce_mean(world):
    """configs[4] data-parallel step: every rank ends with the mean of all ranks' gradients
    (one flat-bucket all-reduce, same key order on every rank)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_grad_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    exp = {}
    for r in range(world):
        g = torch.Generator().manual_seed(r)
        for k, v in {"proj0.w": torch.randn(256, 512, generator=g),
                     "att2.b": torch.randn(1, generator=g),
                     "brand": torch.randn(51, 64, generator=g)}.items():
            exp[k] = exp.get(k, 0) + v / world
    for r in range(world):
        for k in exp:
            torch.testing.assert_close(torch.from_numpy(res[r][k]), exp[k], rtol=1e-6, atol=1e-6)


def _pipe_worker(rank, world, port, k, chunks, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O
        from twotower.sharded import PipelinedStagedExchange, shard_range

        x, q = data(nq=36)
        lo, hi = shard_range(x.shape[0], rank, world)
        xs = x[lo:hi]
        B = q.shape[0] // world
        ql = torch.from_numpy(q[rank * B:(rank + 1) * B].copy())
        checks = []

        def begin(xq):  # per-query stats: must reach full() in the gathered query order
            return torch.stack([xq[:, 0], -xq[:, 0]], 1).contiguous()

        def full(c, qall, sall):
            checks.append(bool(torch.equal(sall[:, 0], qall[:, 0])))
            return torch.full((qall.shape[0], 16), rank + 1, dtype=torch.int32)

        def finish(c, qall, sall, pc):
            checks.append(int(pc[0, 0]) == world * (world + 1) // 2)  # summed over ranks
            s, i = O.scan_topk(xs, qall.numpy(), k, row_base=lo)
            return torch.from_numpy(s), torch.from_numpy(i)

        ex = PipelinedStagedExchange(B, q.shape[1], k, chunks=chunks)
        s, i = ex.search(ql, begin, full, finish, merge_np)
        np.save(os.path.join(out_dir, f"s{rank}.npy"), s.numpy())
        np.save(os.path.join(out_dir, f"i{rank}.npy"), i.numpy())
        np.save(os.path.join(out_dir, f"c{rank}.npy"), np.array(checks))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,chunks,k", [(2, 2, 10), (3, 3, 64), (2, 1, 100)])
def test_pipelined_staged_exchange_bit_identical(tmp_path, world, chunks, k):
    """The chunked staged exchange (PipelinedStagedExchange: per-chunk query / stats
    all-gathers, async probe-count all-reduce and result all-to-all overlapping the next
    chunk's filter) returns the single-catalog top-k, bit for bit."""
    from oracle import oracle as O

    mp.start_processes(_pipe_worker, args=(world, _free_port(), k, chunks, str(tmp_path)),
                       nprocs=world, join=True, start_method="fork")
    x, q = data(nq=36)
    rs, ri = O.scan_topk(x, q, k)
    B = q.shape[0] // world
    for r in range(world):
        s, i = np.load(tmp_path / f"s{r}.npy"), np.load(tmp_path / f"i{r}.npy")
        assert np.array_equal(i, ri[r * B:(r + 1) * B]) and np.array_equal(s, rs[r * B:(r + 1) * B])
        assert np.load(tmp_path / f"c{r}.npy").all()
