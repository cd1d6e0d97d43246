"""Retrieval fixtures produced by the REFERENCE wrappers (run in the build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_retrieval_golden.py

Imported from /root/reference (read-only; never shipped, never on the GPU box):
  src.inference.vector_db.VectorDatabase   (vector_db.py:10-231)  -> vectordb.npz
      build_index / retrieve / retrieve_batch / save_index run as written: the reference's
      own normalisation (:44-45, :152-153, :189-190), float32 casts (:51, :156, :193),
      k clamp (:159, :196), `idx < len(product_ids)` filter (:165, :202) and id mapping;
      save_index's side files (product_ids.npy, product_id_to_index.json, :119-126) are
      stored byte for byte.
  src.api.server (FastAPI app, /retrieve :212-286)                -> server.json
      driven through fastapi.testclient with its module globals set to a stub encoder, the
      reference VectorDatabase above and a products DataFrame / photo dict (the startup hook
      that loads checkpoints from disk is not run).

faiss (requirements.txt:26, faiss-cpu>=1.7.4) is not installed.  A test-only stand-in module
supplies IndexFlatIP with faiss's documented flat inner-product semantics: exact inner
products (accumulated in float64 here, returned as float32), descending, ties to the lower
row.  faiss's own float32 summation order and tie order therefore stay PARITY UNPINNED; what
these fixtures pin is everything the reference wraps around the index.  write_index /
read_index of the stand-in are not used for any fixture (the .faiss bytes are faiss's).
"""
from __future__ import annotations

import json
import os
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import inputs as gi  # noqa: E402

REF = os.environ.get("REFERENCE_ROOT", "/root/reference")
sys.path.insert(0, REF)

CAPTURE = {}


class _IndexFlatIP:
    """Test-only stand-in for faiss.IndexFlatIP (exact search, see module docstring)."""

    def __init__(self, d):
        self.d = int(d)
        self.xb = np.zeros((0, self.d), np.float32)
        self.ntotal = 0
        self.is_trained = True

    def add(self, x):
        x = np.ascontiguousarray(x)
        assert x.dtype == np.float32 and x.shape[1] == self.d  # faiss requires float32
        self.xb = np.concatenate([self.xb, x])
        self.ntotal = self.xb.shape[0]
        CAPTURE["xb"] = self.xb.copy()

    def search(self, q, k):
        q = np.ascontiguousarray(q)
        assert q.dtype == np.float32 and q.shape[1] == self.d
        CAPTURE["q"] = q.copy()
        s = q.astype(np.float64) @ self.xb.astype(np.float64).T
        rows = np.broadcast_to(np.arange(self.ntotal), s.shape)
        order = np.lexsort((rows, -s), axis=1)[:, :k]
        return np.take_along_axis(s, order, 1).astype(np.float32), order.astype(np.int64)


def _install_stubs():
    import torch

    if "faiss" not in sys.modules or not hasattr(sys.modules["faiss"], "IndexFlatIP"):
        mod = types.ModuleType("faiss")
        mod.IndexFlatIP = _IndexFlatIP

        def _no_io(*a, **k):
            raise NotImplementedError("faiss file I/O is not restated by the stand-in")

        mod.write_index = lambda index, path: open(path, "wb").close()  # bytes not fixtured
        mod.read_index = _no_io
        sys.modules["faiss"] = mod
    if "sentence_transformers" not in sys.modules:
        class _StubST(torch.nn.Module):
            def __init__(self, name):
                super().__init__()

            def get_sentence_embedding_dimension(self):
                return 384

        st = types.ModuleType("sentence_transformers")
        st.SentenceTransformer = _StubST
        sys.modules["sentence_transformers"] = st


def _results_arrays(res, k, pid_to_row):
    """List[List[(pid, score)]] -> ([Q, k] int64 rows (-2 = no entry), [Q, k] f32 scores,
    [Q] lengths)."""
    rows = np.full((len(res), k), -2, np.int64)
    sc = np.zeros((len(res), k), np.float32)
    ln = np.zeros(len(res), np.int64)
    for a, r in enumerate(res):
        ln[a] = len(r)
        for b, (pid, s) in enumerate(r):
            rows[a, b] = pid_to_row[pid]
            sc[a, b] = s
    return rows, sc, ln


def vectordb_fixtures():
    _install_stubs()
    from src.inference.vector_db import VectorDatabase  # reference module

    out = {}
    for name, spec in gi.VDB_CASES.items():
        x, q, ids = gi.vdb_inputs(spec)
        E = x.shape[1]
        db = VectorDatabase(E)
        db.build_index(x, ids)
        pid_to_row = {p: j for j, p in enumerate(ids)}
        res = db.retrieve_batch(q, k=spec["k"])
        qn = CAPTURE["q"]
        rows, sc, ln = _results_arrays(res, spec["k"], pid_to_row)
        one = db.retrieve(q[0], k=spec["k"])  # the 1-D query path (:148-149)
        r1, s1, _ = _results_arrays([one], spec["k"], pid_to_row)
        out[name + "__xn_sha"] = np.frombuffer(gi.sha(CAPTURE["xb"]).encode(), np.uint8)
        out[name + "__qn"] = qn
        out[name + "__rows"], out[name + "__scores"], out[name + "__len"] = rows, sc, ln
        out[name + "__one_rows"], out[name + "__one_scores"] = r1[0], s1[0]
    # save_index side files, byte for byte (vector_db.py:119-126)
    x, q, ids = gi.vdb_inputs(gi.VDB_CASES["unicode_ids"])
    db = VectorDatabase(x.shape[1])
    db.build_index(x, ids)
    with tempfile.TemporaryDirectory() as d:
        db.save_index(os.path.join(d, "i.faiss"), os.path.join(d, "ids.npy"),
                      os.path.join(d, "map.json"))
        out["save__ids_npy"] = np.frombuffer(open(os.path.join(d, "ids.npy"), "rb").read(),
                                             np.uint8)
        out["save__map_json"] = np.frombuffer(open(os.path.join(d, "map.json"), "rb").read(),
                                              np.uint8)
    np.savez_compressed(os.path.join(HERE, "vectordb.npz"), **out)


def server_fixtures():
    """/retrieve responses of the reference FastAPI app (server.py:212-286)."""
    _install_stubs()
    import pandas as pd
    from fastapi.testclient import TestClient

    import src.api.server as S  # reference module
    from src.inference.vector_db import VectorDatabase

    x, _, ids = gi.vdb_inputs(gi.VDB_CASES["server"])
    db = VectorDatabase(x.shape[1])
    db.build_index(x, ids)

    class StubEncoder:
        def encode_buyer(self, interactions):
            return gi.stub_buyer_embedding(interactions, x.shape[1])

    df = pd.DataFrame(gi.server_products())
    S.encoder, S.vector_db, S.products_df = StubEncoder(), db, df
    S.product_photos = gi.server_photos()
    client = TestClient(S.app)  # no `with`: the disk-loading startup hook is not run
    cases = []
    for req in gi.server_requests():
        r = client.post("/retrieve", json=req)
        cases.append({"request": req, "status": r.status_code, "response": r.json()})
    with open(os.path.join(HERE, "server.json"), "w", encoding="utf-8") as f:
        json.dump(cases, f, ensure_ascii=False, indent=1)


if __name__ == "__main__":
    vectordb_fixtures()
    server_fixtures()
    for f in ("vectordb.npz", "server.json"):
        print(f, os.path.getsize(os.path.join(HERE, f)))
