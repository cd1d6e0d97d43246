"""configs[4] training step timing (post-encode part): twotower.train.TwoTowerTrainStep at
B = 512, 4 negatives, S = 20, E = 768, attention aggregation, bf16 and f32, eager launches vs
the HIP-graph replay (graph=True), plus the graph step's agreement with the eager step.

    python tools/train_step_prof.py [--steps 50] [--json out.json]

Run under rocprofv3 --kernel-trace --stats for the per-kernel split.  Synthetic batch
(random-normal text / history embeddings, event-mix weights), random-init weights."""
import argparse
import copy
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "two-tower-model-v2_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    from twotower.buyer_tower import BuyerTower
    from twotower.item_tower import ItemTower
    from twotower.train import TwoTowerTrainStep

    class _Dim:
        def get_sentence_embedding_dimension(self):
            return 384

    dev = torch.device("cuda", 0)
    B, N, S, E = 512, 4, 20, 768
    torch.manual_seed(0)
    it0 = ItemTower(embedding_dim=E, text_encoder=_Dim())
    it0.initialize_categorical_embeddings([f"b{i}" for i in range(500)],
                                          [f"c{i}" for i in range(50)])
    bt0 = BuyerTower(E, "attention")
    g = torch.Generator(device=dev).manual_seed(17)
    items = torch.randn((B, S, E), generator=g, device=dev)
    u = torch.rand((B, S), generator=g, device=dev)
    w = torch.where(u > 0.92, 10.0, torch.where(u > 0.75, 5.0, 1.0))
    pos = torch.randn((B, 384), generator=g, device=dev)
    neg = torch.randn((B, N, 384), generator=g, device=dev)
    pb, pc = (torch.randint(0, m, (B,), generator=g, device=dev, dtype=torch.int32)
              for m in (501, 51))
    nb, nc = (torch.randint(0, m, (B, N), generator=g, device=dev, dtype=torch.int32)
              for m in (501, 51))
    batch = (items, w, pos, neg, pb, pc, nb, nc)
    out = {"shape": {"B": B, "N": N, "S": S, "E": E}}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for prec in ("bf16", "f32"):
        res = {}
        losses = {}
        for mode in ("eager", "graph"):
            it, bt = copy.deepcopy(it0).to(dev), copy.deepcopy(bt0).to(dev)
            st = TwoTowerTrainStep(it, bt, lr=1e-4, prec=prec, graph=mode == "graph")
            it.eval()  # deterministic comparison: no dropout
            tr = []
            for _ in range(5):
                tr.append(float(st.step(*batch)))
            losses[mode] = tr
            it.train()
            for _ in range(3):
                st.step(*batch)
            torch.cuda.synchronize()
            ev[0].record()
            for _ in range(a.steps):
                st.step(*batch)
            ev[1].record()
            torch.cuda.synchronize()
            res[mode + "_ms"] = ev[0].elapsed_time(ev[1]) / a.steps
            if mode == "graph":
                # the same steps with the inputs written in place (no copies)
                bi = st.input_buffers(B, S, N)
                bi[0].copy_(items)
                bi[1].copy_(w)
                bi[2][:B].copy_(pos)
                bi[2][B:].copy_(neg.reshape(B * N, -1))
                bi[3][:B].copy_(pb)
                bi[3][B:].copy_(nb.reshape(-1))
                bi[4][:B].copy_(pc)
                bi[4][B:].copy_(nc.reshape(-1))
                ni, nw, nt, nbi, nci = bi
                args = (ni, nw, nt[:B], nt[B:].view(B, N, -1), nbi[:B], nci[:B], nbi[B:].view(B, N),
                        nci[B:].view(B, N))
                st.step(*args)
                torch.cuda.synchronize()
                ev[0].record()
                for _ in range(a.steps):
                    st.step(*args)
                ev[1].record()
                torch.cuda.synchronize()
                res["graph_inplace_inputs_ms"] = ev[0].elapsed_time(ev[1]) / a.steps
            del st, it, bt
        res["loss_eager_first5"] = losses["eager"]
        res["loss_graph_first5"] = losses["graph"]
        res["max_loss_diff_graph_vs_eager"] = max(abs(x - y) for x, y in zip(losses["eager"],
                                                                              losses["graph"]))
        out[prec] = res
        print(prec, json.dumps(res), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
