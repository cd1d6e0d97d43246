"""VectorDatabase result assembly (reference vector_db.py:162-167 / 199-207) on host arrays:
(product_id, float(score)) per slot, ids past the catalog dropped, -1 passing through to the
last id exactly as the reference's `if idx < len(self.product_ids)` does."""
import numpy as np

from twotower.vector_db import VectorDatabase


def _reference_loop(product_ids, scores, indices):
    out = []
    for query_scores, query_indices in zip(scores, indices):
        res = []
        for idx, score in zip(query_indices, query_scores):
            if idx < len(product_ids):
                res.append((product_ids[idx], float(score)))
        out.append(res)
    return out


def test_to_results_matches_reference_loop():
    rng = np.random.default_rng(0)
    vdb = VectorDatabase(8)
    vdb.product_ids = [f"p{i}" for i in range(50)]
    scores = rng.standard_normal((3, 7)).astype(np.float32)
    indices = rng.integers(0, 50, (3, 7)).astype(np.int64)
    indices[0, 3] = -1   # faiss' "no result": passes the reference's check (last id)
    indices[1, 5] = 57   # past the catalog: dropped
    scores[2, 0] = np.float32(np.nextafter(np.float32(0.5), np.float32(1)))
    got = vdb._to_results(scores, indices)
    ref = _reference_loop(vdb.product_ids, scores, indices)
    assert got == ref
    assert all(type(s) is float for r in got for _, s in r)
    assert got[0][3][0] == "p49" and len(got[1]) == 6
