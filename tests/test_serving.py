"""ProductCatalog (twotower.serving) == the reference /retrieve response loop
(src/api/server.py:246-283, restated below with its O(N) DataFrame scan) on duplicates,
NaN / None cells, missing columns, unknown ids and photo links."""
import os
import sys

import numpy as np
import pandas as pd
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "two-tower-model-v2_amd"))


def reference_loop(products_df, product_photos, results):
    """server.py:248-279 as written (per result: boolean-mask scan, first row)."""
    out = []
    for product_id, score in results:
        product_row = products_df[products_df["product_id"] == product_id]
        photo_link = product_photos.get(product_id, None)
        if not product_row.empty:
            row = product_row.iloc[0]
            out.append(dict(
                product_id=product_id, title=str(row.get("title", "N/A")),
                description=str(row.get("description", "N/A")),
                brand=str(row.get("brand", None)) if pd.notna(row.get("brand")) else None,
                category=str(row.get("category", None)) if pd.notna(row.get("category")) else None,
                score=float(score), photo_link=photo_link))
        else:
            out.append(dict(product_id=product_id, title="N/A", description="N/A", brand=None,
                            category=None, score=float(score), photo_link=photo_link))
    return out


def _df(drop=()):
    df = pd.DataFrame({
        "product_id": ["a", "b", "c", "a", "d", "e"],
        "title": ["خاتم ذهب", "ring", np.nan, "dup-title", "t4", None],
        "description": ["desc a", "", "desc c", "dup", np.nan, "e"],
        "brand": ["Damas", np.nan, None, "Other", "Acme", 7],
        "category": ["rings", "necklaces", np.nan, "x", None, "oil"],
    })
    return df.drop(columns=list(drop))


@pytest.mark.parametrize("drop", [(), ("brand",), ("title", "category"), ("description",)])
def test_catalog_matches_reference_loop(drop):
    from twotower.serving import ProductCatalog

    df = _df(drop)
    photos = {"a": "http://x/a.jpg", "zz": "http://x/zz.jpg"}
    results = [("a", np.float32(0.93)), ("zz", 0.5), ("c", 0.25), ("e", np.float32(-0.1)),
               ("b", 1.0), ("d", 0.0)]
    got = ProductCatalog(df, photos).assemble(results)
    assert got == reference_loop(df, photos, results)


def test_retrieve_products_flow():
    from twotower.serving import ProductCatalog, retrieve_products

    class Enc:
        def encode_buyer(self, inter):
            assert inter[0]["product_id"] == "a"
            return np.ones(4, np.float32)

    class DB:
        def retrieve(self, emb, k=10):
            return [("b", 0.75), ("a", 0.5)][:k]

    body = retrieve_products(Enc(), DB(), ProductCatalog(_df()), "u1",
                             [{"product_id": "a", "event_type": "view"}], k=2)
    assert body["buyer_id"] == "u1" and [p["product_id"] for p in body["products"]] == ["b", "a"]
    assert body["products"][1]["title"] == "خاتم ذهب"


def test_catalog_matches_reference_server_fixture(golden):
    """Responses of the reference FastAPI /retrieve handler itself (server.py:212-286, run
    through fastapi.testclient by tests/golden/make_retrieval_golden.py): assembling the
    reference's own retrieved (id, score) lists gives the same records, field for field."""
    import json

    import inputs as gi
    from twotower.serving import ProductCatalog

    cases = json.load(open(os.path.join(ROOT, "tests", "golden", "server.json"),
                           encoding="utf-8"))
    cat = ProductCatalog(pd.DataFrame(gi.server_products()), gi.server_photos())
    assert len(cases) == len(gi.server_requests())
    for c in cases:
        assert c["status"] == 200
        ref = c["response"]["products"]
        got = cat.assemble([(p["product_id"], p["score"]) for p in ref])
        assert got == ref
