"""ShardedFlatIP end to end on the GPU with W=2 ranks sharing cuda:0 (gloo moves the device
tensors; the 8-GPU RCCL run is the driver's): replicated sample + global bounds built by
add_shard, staged bf16 filter search, merge -> bit-identical to the single-catalog oracle."""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "two-tower-model-v2_amd"))
sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _data(n, nq, seed=11):
    from oracle import oracle as O

    rng = np.random.default_rng(seed)
    x = O.l2norm_rows(rng.standard_normal((n, 384)).astype(np.float32), 0)
    x[n // 2: n // 2 + 40] = x[:40]
    q = O.l2norm_rows(rng.standard_normal((nq, 384)).astype(np.float32), 0)
    return x, q


def _worker(rank, world, port, n, nq, k, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from twotower import _lib
        from twotower.sharded import ShardedFlatIP

        x, q = _data(n, nq)
        idx = ShardedFlatIP(384, n, device=torch.device("cuda", 0))
        idx.add_shard(x[idx.lo:idx.hi])
        b = nq // world
        ql = torch.zeros((b, _lib.padded_dim(384)), device="cuda")
        ql[:, :384] = torch.from_numpy(q[rank * b:(rank + 1) * b])
        assert idx._staged(k, "auto")
        s, i = idx.search(ql, k)
        np.save(os.path.join(out_dir, f"s{rank}.npy"), s.cpu().numpy())
        np.save(os.path.join(out_dir, f"i{rank}.npy"), i.cpu().numpy())
        np.save(os.path.join(out_dir, f"n{rank}.npy"), np.array([idx.sample16.shape[0]]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n,nq,k", [(200003, 24, 100), (40000, 10, 17)])
def test_sharded_index_two_ranks_bit_exact(tmp_path, oracle_mod, n, nq, k):
    import torch.multiprocessing as mp

    world = 2
    mp.start_processes(_worker, args=(world, _port(), n, nq, k, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    x, q = _data(n, nq)
    rs, ri = oracle_mod.scan_topk(x, q, k)
    b = nq // world
    for r in range(world):
        assert int(np.load(tmp_path / f"n{r}.npy")[0]) == (n + 15) // 16
        s, i = np.load(tmp_path / f"s{r}.npy"), np.load(tmp_path / f"i{r}.npy")
        assert np.array_equal(i, ri[r * b:(r + 1) * b]) and np.array_equal(s, rs[r * b:(r + 1) * b])


def _worker_nccl(rank, world, port, n, nq, k, out_dir):
    """The same path over the nccl backend (= RCCL) at world size 1: every collective the
    sharded index and the bench's TopkExchange issue (all_gather, all_gather_into_tensor,
    all_reduce SUM/MAX, all_to_all_single) runs through RCCL on device tensors."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    try:
        from twotower import _lib, kernels
        from twotower.sharded import ShardedFlatIP, TopkExchange

        assert dist.get_backend() == "nccl"
        x, q = _data(n, nq)
        ep = _lib.padded_dim(384)
        idx = ShardedFlatIP(384, n, device=dev)
        idx.add_shard(x[idx.lo:idx.hi])
        ql = torch.zeros((nq, ep), device=dev)
        ql[:, :384] = torch.from_numpy(q)
        assert idx._staged(k, "auto")
        s, i = idx.search(ql, k)
        # bench.py's exchange: all-gather queries + stats, all-to-all of the shard top-k
        ex = TopkExchange(nq, ep, k, device=dev, aux_width=2)
        stats = torch.randn((nq, 2), device=dev)
        seen = {}

        def local(qall, sall):
            seen["q"], seen["s"] = qall.clone(), sall.clone()
            return kernels.scan_topk(idx.index.xb, idx.index.ntotal, 384, qall, k)

        s2, i2 = ex.search(ql, local, kernels.merge_topk, aux=stats)
        torch.cuda.synchronize()
        assert torch.equal(seen["q"], ql) and torch.equal(seen["s"], stats)
        np.save(os.path.join(out_dir, "s.npy"), s.cpu().numpy())
        np.save(os.path.join(out_dir, "i.npy"), i.cpu().numpy())
        np.save(os.path.join(out_dir, "s2.npy"), s2.cpu().numpy())
        np.save(os.path.join(out_dir, "i2.npy"), i2.cpu().numpy())
    finally:
        dist.destroy_process_group()


def test_sharded_index_rccl_world1_bit_exact(tmp_path, oracle_mod):
    import torch.multiprocessing as mp

    n, nq, k = 120001, 16, 100
    mp.start_processes(_worker_nccl, args=(1, _port(), n, nq, k, str(tmp_path)), nprocs=1,
                       join=True, start_method="spawn")
    x, q = _data(n, nq)
    rs, ri = oracle_mod.scan_topk(x, q, k)
    for tag in ("", "2"):
        s, i = np.load(tmp_path / f"s{tag}.npy"), np.load(tmp_path / f"i{tag}.npy")
        assert np.array_equal(i, ri) and np.array_equal(s, rs)
