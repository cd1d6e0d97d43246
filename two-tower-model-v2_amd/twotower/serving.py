"""/retrieve response assembly with O(1) product lookups.

The reference handler (src/api/server.py:246-283) turns each of the k retrieved
``(product_id, score)`` pairs into a ``ProductInfo`` by scanning the whole products
DataFrame (``products_df[products_df['product_id'] == product_id]``, :250): O(k * N) per
request, which at N = 1M rows costs far more than the GPU encode + search it follows.
``ProductCatalog`` builds the id -> row mapping once and produces the same records:

  * the FIRST row of a duplicated product_id wins (``product_row.iloc[0]``, :256)
  * title / description: ``str(row.get(col, 'N/A'))`` -- a missing column gives 'N/A', a
    NaN cell gives 'nan' (:259-260)
  * brand / category: ``str(value)`` if ``pd.notna(value)`` else None (:261-262)
  * score: ``float(score)``; photo_link from the photo dict, None if absent (:253, :264)
  * unknown product_id: title / description 'N/A', brand / category None (:267-276)

``retrieve_products`` is the handler's data path (encode_buyer -> retrieve -> assemble,
:236-283) without the FastAPI layer, which stays out of scope.
"""
from __future__ import annotations

from typing import Any, Dict, Iterable, List, Optional, Tuple


def _is_na(v) -> bool:
    import pandas as pd

    try:
        return bool(pd.isna(v))
    except (TypeError, ValueError):  # list-like cells: pd.isna is element-wise
        return False


class ProductCatalog:
    """id -> ProductInfo fields, built once from the products DataFrame (reference schema:
    product_id, title, description, brand, category)."""

    def __init__(self, products_df, product_photos: Optional[Dict[str, str]] = None):
        self.product_photos = product_photos or {}
        cols = set(products_df.columns)
        self._rows: Dict[str, Tuple[str, str, Optional[str], Optional[str]]] = {}

        def col(name):
            return products_df[name].tolist() if name in cols else None

        ids = products_df["product_id"].tolist()
        title, desc, brand, cat = col("title"), col("description"), col("brand"), col("category")
        for i, pid in enumerate(ids):
            if pid in self._rows:  # first occurrence wins, as .iloc[0] of the mask
                continue
            b = brand[i] if brand is not None else None
            c = cat[i] if cat is not None else None
            self._rows[pid] = (
                str(title[i]) if title is not None else "N/A",
                str(desc[i]) if desc is not None else "N/A",
                None if b is None or _is_na(b) else str(b),
                None if c is None or _is_na(c) else str(c),
            )

    def __len__(self) -> int:
        return len(self._rows)

    def product_info(self, product_id: str, score) -> Dict[str, Any]:
        row = self._rows.get(product_id)
        title, desc, brand, cat = row if row is not None else ("N/A", "N/A", None, None)
        return {"product_id": product_id, "title": title, "description": desc, "brand": brand,
                "category": cat, "score": float(score),
                "photo_link": self.product_photos.get(product_id, None)}

    def assemble(self, results: Iterable[Tuple[str, float]]) -> List[Dict[str, Any]]:
        return [self.product_info(pid, score) for pid, score in results]


def retrieve_products(encoder, vector_db, catalog: ProductCatalog, buyer_id: str,
                      interactions: List[Dict[str, Any]], k: int = 10) -> Dict[str, Any]:
    """The /retrieve response body (server.py:225-283): {'buyer_id', 'products': [...]}."""
    buyer_embedding = encoder.encode_buyer(interactions)
    results = vector_db.retrieve(buyer_embedding, k=k)
    return {"buyer_id": buyer_id, "products": catalog.assemble(results)}
