"""VectorDatabase and /retrieve against outputs of the REFERENCE wrappers themselves
(tests/golden/make_retrieval_golden.py imported src/inference/vector_db.py and
src/api/server.py with a test-only exact faiss.IndexFlatIP stand-in): normalisation,
float32 casts, k clamp, the idx < len(product_ids) filter, id mapping, save_index side
files and the /retrieve response records come from the reference; faiss's own f32 summation
and tie order stay parity unpinned (faiss absent), so scores are compared within 1e-5 and
ids wherever the reference's scores are separated by more than 1e-6."""
import json
import os
import struct

import numpy as np
import pandas as pd
import pytest

import inputs as gi

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _rows(res, ids):
    m = {p: j for j, p in enumerate(ids)}
    return [m[p] for p, _ in res], np.array([s for _, s in res], np.float64)


def _same_ranking(got_rows, got_s, ref_rows, ref_s, gap=1e-6):
    """ids equal at every rank whose reference score is > gap from its neighbours."""
    assert len(got_rows) == len(ref_rows)
    np.testing.assert_allclose(got_s, ref_s, rtol=0, atol=1e-5)
    for r in range(len(ref_rows)):
        lo = ref_s[r + 1] if r + 1 < len(ref_s) else -np.inf
        hi = ref_s[r - 1] if r > 0 else np.inf
        if hi - ref_s[r] > gap and ref_s[r] - lo > gap:
            assert got_rows[r] == ref_rows[r], r


@pytest.mark.parametrize("case", list(gi.VDB_CASES))
def test_vector_db_matches_reference_wrapper(golden, case):
    from twotower import VectorDatabase

    g = golden("vectordb.npz")
    spec = gi.VDB_CASES[case]
    x, q, ids = gi.vdb_inputs(spec)
    vdb = VectorDatabase(x.shape[1])
    vdb.build_index(x, ids)
    # build_index normalisation (vector_db.py:44-51) bit-identical to the reference's array
    xn = np.ascontiguousarray(vdb.index.xb[:, : x.shape[1]].cpu().numpy())
    assert gi.sha(xn) == bytes(g[case + "__xn_sha"]).decode()
    if q.dtype == np.float32:  # query normalisation (:189-193) on the device path
        import torch

        qd = torch.from_numpy(q).cuda()
        qn = vdb.normalize_queries(qd)[:, : x.shape[1]].cpu().numpy()
        assert np.array_equal(qn, g[case + "__qn"])
    res = vdb.retrieve_batch(q, k=spec["k"])
    rows, lens, scores = g[case + "__rows"], g[case + "__len"], g[case + "__scores"]
    assert [len(r) for r in res] == lens.tolist()  # clamp (:196) + id filter (:202)
    for a, r in enumerate(res):
        gr, gs = _rows(r, ids)
        _same_ranking(gr, gs, rows[a, : lens[a]].tolist(), scores[a, : lens[a]].astype(np.float64))
    one = vdb.retrieve(q[0], k=spec["k"])  # 1-D query (:148-149)
    n1 = int((g[case + "__one_rows"] >= 0).sum())
    gr, gs = _rows(one, ids)
    _same_ranking(gr, gs, g[case + "__one_rows"][:n1].tolist(),
                  g[case + "__one_scores"][:n1].astype(np.float64))


def test_save_index_side_files_match_reference(golden, tmp_path):
    """product_ids.npy and product_id_to_index.json byte-identical to the reference's
    save_index (vector_db.py:119-126) on Arabic product ids."""
    from twotower import VectorDatabase

    g = golden("vectordb.npz")
    x, _, ids = gi.vdb_inputs(gi.VDB_CASES["unicode_ids"])
    vdb = VectorDatabase(x.shape[1])
    vdb.build_index(x, ids)
    vdb.save_index(str(tmp_path / "i.faiss"), str(tmp_path / "ids.npy"), str(tmp_path / "m.json"))
    assert (tmp_path / "ids.npy").read_bytes() == bytes(g["save__ids_npy"])
    assert (tmp_path / "m.json").read_bytes() == bytes(g["save__map_json"])
    b = VectorDatabase(x.shape[1])
    b.load_index(str(tmp_path / "i.faiss"), str(tmp_path / "ids.npy"), str(tmp_path / "m.json"))
    assert b.product_ids == ids and b.index_to_id[3] == ids[3]


def test_faiss_flat_ip_header_layout(tmp_path):
    """.faiss bytes follow faiss's documented IndexFlatIP serialisation (faiss/impl/
    index_write.cpp, faiss-cpu >= 1.7.4 per requirements.txt:26): fourcc 'IxFI'; header
    d:int32, ntotal:int64, two int64 dummies = 1<<20, is_trained:uint8 = 1, metric_type:int32
    = 0 (METRIC_INNER_PRODUCT, no metric_arg since type <= 1); codes as a uint64 count of
    floats (ntotal*d) followed by the float32 rows.  faiss itself is absent: unpinned against
    faiss.read_index, so this checks the layout field by field, not a faiss-written file."""
    from twotower import VectorDatabase

    rng = np.random.default_rng(3)
    x = rng.standard_normal((37, 100)).astype(np.float32)
    vdb = VectorDatabase(100)
    vdb.build_index(x, [str(i) for i in range(37)])
    p = tmp_path / "i.faiss"
    vdb.save_index(str(p))
    raw = p.read_bytes()
    assert raw[:4] == b"IxFI"
    d, ntotal, d1, d2 = struct.unpack_from("<iqqq", raw, 4)
    trained, metric = struct.unpack_from("<Bi", raw, 32)
    (count,) = struct.unpack_from("<Q", raw, 37)
    assert (d, ntotal, d1, d2, trained, metric, count) == (100, 37, 1 << 20, 1 << 20, 1, 0, 3700)
    body = np.frombuffer(raw, "<f4", offset=45)
    assert len(raw) == 45 + 4 * 3700
    assert np.array_equal(body.reshape(37, 100), vdb.index.xb[:, :100].cpu().numpy())


def test_retrieve_endpoint_matches_reference_server(golden):
    """The /retrieve data path (retrieve_products: encode_buyer -> VectorDatabase.retrieve on
    HIP -> ProductCatalog) vs the reference FastAPI handler's JSON responses for the same
    catalog, products_df, photos and requests (k from 1 to 1000 > ntotal)."""
    from twotower import VectorDatabase
    from twotower.serving import ProductCatalog, retrieve_products

    cases = json.load(open(os.path.join(GOLD, "server.json"), encoding="utf-8"))
    x, _, ids = gi.vdb_inputs(gi.VDB_CASES["server"])
    vdb = VectorDatabase(x.shape[1])
    vdb.build_index(x, ids)

    class StubEncoder:
        def encode_buyer(self, interactions):
            return gi.stub_buyer_embedding(interactions, x.shape[1])

    cat = ProductCatalog(pd.DataFrame(gi.server_products()), gi.server_photos())
    for c in cases:
        req = c["request"]
        body = retrieve_products(StubEncoder(), vdb, cat, req["buyer_id"],
                                 req["recent_interactions"], k=req["k"])
        ref = c["response"]
        assert body["buyer_id"] == ref["buyer_id"]
        got_p, ref_p = body["products"], ref["products"]
        _same_ranking([ids.index(p["product_id"]) for p in got_p],
                      np.array([p["score"] for p in got_p]),
                      [ids.index(p["product_id"]) for p in ref_p],
                      np.array([p["score"] for p in ref_p]))
        for gp, rp in zip(got_p, ref_p):
            if gp["product_id"] == rp["product_id"]:
                assert {k: v for k, v in gp.items() if k != "score"} == \
                       {k: v for k, v in rp.items() if k != "score"}


def test_retrieve_serving_path_threads_and_device_path_agree():
    """VectorDatabase.retrieve / retrieve_batch run the serving path (FlatIPIndex.search_host:
    a serving slot's own stream, pinned staging, device normalisation).
    Results equal the device path (normalize_queries + search) bit for bit, and four threads
    calling retrieve concurrently on one index get the same answers as one thread."""
    import threading

    import torch

    from twotower import VectorDatabase

    rng = np.random.default_rng(11)
    n, d, k = 20000, 384, 100
    x = rng.standard_normal((n, d)).astype(np.float32)
    ids = [f"p{i}" for i in range(n)]
    vdb = VectorDatabase(d)
    vdb.build_index(x, ids)
    q = rng.standard_normal((64, d)).astype(np.float32)
    s_dev, i_dev = vdb.search(torch.from_numpy(q).cuda(), k)
    s_dev, i_dev = s_dev.cpu().numpy(), i_dev.cpu().numpy()
    want = [[(ids[j], float(s)) for j, s in zip(i_dev[b], s_dev[b])] for b in range(len(q))]
    assert vdb.retrieve_batch(q, k=k) == want
    assert [vdb.retrieve(q[b], k=k) for b in range(len(q))] == want
    got, errs = [None] * len(q), []

    def work(t):
        try:
            for b in range(t, len(q), 4):
                for _ in range(3):
                    got[b] = vdb.retrieve(q[b], k=k)
        except Exception as e:  # pragma: no cover - reported below
            errs.append(e)

    th = [threading.Thread(target=work, args=(t,)) for t in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs and got == want
    assert vdb.retrieve(q[0], k=n + 5)[:k] == want[0]  # k clamp (:159): all rows, same head


def test_retrieve_per_request_k_no_reallocation_and_threads():
    """/retrieve takes any k in 1..1000 per request (server.py:46).  Cycling k over 20 values x
    50 calls (k <= 128: the bf16 filter; k > 128: scores + radix select) reuses the serving
    slot's buffers: no allocation after the first pass, and every answer equals the device
    path's bit for bit.  Four threads cycling k concurrently (each call on its own slot's
    stream, the index lock not held across the kernels) get the same answers."""
    import threading

    import torch

    from twotower import VectorDatabase

    rng = np.random.default_rng(12)
    n, d = 30000, 384
    x = rng.standard_normal((n, d)).astype(np.float32)
    ids = [f"p{i}" for i in range(n)]
    vdb = VectorDatabase(d)
    vdb.build_index(x, ids)
    ks = [1, 2, 5, 10, 16, 20, 33, 50, 64, 99, 100, 127, 128, 129, 200, 256, 500, 512, 999, 1000]
    q = rng.standard_normal((8, d)).astype(np.float32)
    want = {}
    for k in ks:
        s_dev, i_dev = vdb.search(torch.from_numpy(q).cuda(), k)
        s_dev, i_dev = s_dev.cpu().numpy(), i_dev.cpu().numpy()
        want[k] = [[(ids[j], float(v)) for j, v in zip(i_dev[b], s_dev[b])] for b in range(len(q))]
    for k in ks:  # warm-up pass
        assert vdb.retrieve(q[0], k=k) == want[k][0]
    warm = vdb.index.allocations
    for c in range(50):
        for j, k in enumerate(ks):
            b = (c + j) % len(q)
            assert vdb.retrieve(q[b], k=k) == want[k][b], (c, k)
    assert vdb.index.allocations == warm, (warm, vdb.index.allocations)
    errs = []

    def work(t):
        try:
            for c in range(10):
                for j, k in enumerate(ks):
                    b = (t + c + j) % len(q)
                    if vdb.retrieve(q[b], k=k) != want[k][b]:
                        errs.append((t, c, k))
        except Exception as e:  # pragma: no cover - reported below
            errs.append(e)

    th = [threading.Thread(target=work, args=(t,)) for t in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs[:5]


def test_retrieve_coalesces_concurrent_requests_bit_identical():
    """Concurrent single-query retrieve calls are served as batched searches (FlatIPIndex
    request coalescing): 6 threads x 40 calls with per-request k (filter and select paths)
    get exactly the single-request answers; the coalescing counters account for every call."""
    import threading

    import torch

    from twotower import VectorDatabase

    rng = np.random.default_rng(13)
    n, d = 50000, 384
    x = rng.standard_normal((n, d)).astype(np.float32)
    ids = [f"p{i}" for i in range(n)]
    vdb = VectorDatabase(d)
    vdb.build_index(x, ids)
    q = rng.standard_normal((12, d)).astype(np.float32)
    ks = [1, 7, 50, 100, 128, 129, 300, 1000]
    want = {}
    for k in ks:
        s_dev, i_dev = vdb.search(torch.from_numpy(q).cuda(), k)
        s_dev, i_dev = s_dev.cpu().numpy(), i_dev.cpu().numpy()
        want[k] = [[(ids[j], float(v)) for j, v in zip(i_dev[b], s_dev[b])] for b in range(len(q))]
    errs = []
    st0 = list(vdb.index.coalesce_stats)

    def work(t):
        try:
            for c in range(40):
                k, b = ks[(t + c) % len(ks)], (3 * t + c) % len(q)
                if vdb.retrieve(q[b], k=k) != want[k][b]:
                    errs.append((t, c, k, b))
        except Exception as e:  # pragma: no cover - reported below
            errs.append(e)

    th = [threading.Thread(target=work, args=(t,)) for t in range(6)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs[:5]
    nb, nr = (vdb.index.coalesce_stats[0] - st0[0], vdb.index.coalesce_stats[1] - st0[1])
    assert nr == 240 and 1 <= nb <= 240
    print(f"coalesced 240 requests into {nb} searches")


class _Abort(BaseException):
    """Stands for KeyboardInterrupt / SystemExit raised inside a serving thread."""


def test_retrieve_survives_a_base_exception_in_the_coalescing_leader():
    """A BaseException (KeyboardInterrupt, SystemExit) raised inside the thread that leads the
    coalesced searches must not leave the lead held: that thread sees the exception, requests
    queued behind it still get their answers (the lead is handed over), and later retrieve
    calls return (FlatIPIndex._serve's finally)."""
    import threading

    from twotower import VectorDatabase

    rng = np.random.default_rng(17)
    n, d, k = 20000, 384, 10
    vdb = VectorDatabase(d)
    vdb.build_index(rng.standard_normal((n, d)).astype(np.float32), [f"p{i}" for i in range(n)])
    q = rng.standard_normal((4, d)).astype(np.float32)
    want = [vdb.retrieve(q[b], k=k) for b in range(4)]
    ix = vdb.index
    real = ix._run_batch
    entered, release = threading.Event(), threading.Event()
    calls = []

    def flaky(xs, kk, normalize, state=None):  # the first batch blocks, then aborts
        calls.append(xs.shape[0])
        if len(calls) == 1:
            entered.set()
            release.wait(30)
            raise _Abort()
        return real(xs, kk, normalize, state)

    ix._run_batch = flaky
    out = {}

    def lead():
        try:
            vdb.retrieve(q[0], k=k)
            out["lead"] = "returned"
        except _Abort:
            out["lead"] = "aborted"

    def follow(b):
        try:
            out[b] = vdb.retrieve(q[b], k=k)
        except Exception as e:  # pragma: no cover - reported by the asserts
            out[b] = e

    try:
        t0 = threading.Thread(target=lead)
        t0.start()
        assert entered.wait(30)
        followers = [threading.Thread(target=follow, args=(b,)) for b in (1, 2, 3)]
        for t in followers:
            t.start()
        while len(ix._queue) < 3 and all(t.is_alive() for t in followers):
            threading.Event().wait(0.01)
        release.set()
        for t in [t0] + followers:
            t.join(60)
            assert not t.is_alive(), "a retrieve call hung after the leader's BaseException"
    finally:
        release.set()
        ix._run_batch = real
    assert out["lead"] == "aborted"
    for b in (1, 2, 3):
        assert out[b] == want[b], (b, out[b])
    assert not ix._leading and not ix._queue
    res = {}
    th = threading.Thread(target=lambda: res.setdefault("r", vdb.retrieve(q[2], k=k)))
    th.start()
    th.join(60)
    assert not th.is_alive() and res["r"] == want[2]
