"""Diagnostic: one TwoTowerTrainStep forward+backward eagerly vs the same launches replayed
from a HIP graph, buffer by buffer (first divergence).  python tools/debug_graph_step.py"""
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "two-tower-model-v2_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from twotower.buyer_tower import BuyerTower
    from twotower.item_tower import ItemTower
    from twotower.train import TwoTowerTrainStep

    class Dim:
        def get_sentence_embedding_dimension(self):
            return 384

    for prec in ("f32", "bf16"):
        B, N, S, E = 128, 4, 20, 768
        torch.manual_seed(9)
        it0 = ItemTower(embedding_dim=E, text_encoder=Dim())
        it0.initialize_categorical_embeddings([f"b{i}" for i in range(5)], [f"c{i}" for i in range(5)])
        bt0 = BuyerTower(E, "attention")
        rng = np.random.default_rng(9)
        cu = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
        items = cu(rng.standard_normal((B, S, E)).astype(np.float32))
        w = cu(rng.integers(1, 11, (B, S)).astype(np.float32))
        pos = cu(rng.standard_normal((B, 384)).astype(np.float32))
        neg = cu(rng.standard_normal((B, N, 384)).astype(np.float32))
        ids = [cu(rng.integers(0, 6, s).astype(np.int32)) for s in ((B,), (B,), (B, N), (B, N))]
        batch = (items, w, pos, neg, *ids)
        it, bt = copy.deepcopy(it0).cuda().eval(), copy.deepcopy(bt0).cuda()
        st = TwoTowerTrainStep(it, bt, lr=1e-3, prec=prec, graph=False)
        loss, g = st.forward_backward(*batch)
        torch.cuda.synchronize()
        key = next(iter(st._bufs))
        bb = st._bufs[key]
        names = [n for n in vars(bb) if isinstance(getattr(bb, n), torch.Tensor)]
        eager = {n: getattr(bb, n).clone() for n in names}
        eager_g = {k: v.clone() for k, v in g.items()}
        eager_loss = float(loss)
        for n in names:  # poison the buffers, then replay from a graph
            t = getattr(bb, n)
            if t.dtype == torch.float32 and n not in ("items", "w", "text", "W3T", "W0cT"):
                t.fill_(float("nan"))
        st.flat_g.fill_(float("nan"))
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            st._launch(bb, key, grads=True)
        graph.replay()
        torch.cuda.synchronize()
        print(prec, "loss eager", eager_loss, "graph", float(bb.loss))
        for n in names:
            a, b = eager[n], getattr(bb, n)
            if a.dtype in (torch.float32, torch.bfloat16):
                d = (a.float() - b.float()).abs().max().item() if a.numel() else 0.0
                nan = torch.isnan(b.float()).sum().item()
                print(f"  {n:8s} {tuple(a.shape)} maxdiff {d:.3e} nan {nan}")
        for k in eager_g:
            d = (eager_g[k] - st.g[k]).abs().max().item()
            print(f"  grad {k:8s} maxdiff {d:.3e} (scale {eager_g[k].abs().max().item():.3e})")


if __name__ == "__main__":
    main()
