"""Evaluator with batched buyer encode + retrieval.

Reference: src/evaluation/metrics.py.  The metric functions (:17-340) are restated with the
same definitions (they stay host Python: set arithmetic over k ids).  The reference
``Evaluator`` encodes and searches every test buyer one at a time (nq = 1) in each of
evaluate_retrieval, evaluate_diversity (x2) and evaluate_coverage (:419-429, 569-576,
619-626): four single-query passes per buyer.  Here one batched pass -- the encoder's
``encode_buyers`` and the index's ``retrieve_batch`` (the HIP top-k over the whole batch) --
is made once per (test set, k) and cached, and every evaluation reads the cache.  Aggregates,
keys and skip-on-error behaviour are the reference's (a batch that raises is redone buyer by
buyer so that only the failing buyers are skipped, as in the reference loop).
"""
from __future__ import annotations

import copy
import json
from pathlib import Path
from typing import Dict, List, Optional, Sequence, Set, Tuple

import numpy as np

from .config import DEFAULT_CONFIG, load_config


# ----------------------------------------------------------------- metric functions (:17-340)
def compute_recall_at_k(retrieved_items: List[str], relevant_items: Set[str], k: int) -> float:
    if not relevant_items:
        return 0.0
    return len(set(retrieved_items[:k]) & relevant_items) / len(relevant_items)


def compute_precision_at_k(retrieved_items: List[str], relevant_items: Set[str], k: int) -> float:
    if k == 0:
        return 0.0
    return len(set(retrieved_items[:k]) & relevant_items) / k


def _dcg_terms(n: int) -> List[float]:
    return [1.0 / np.log2(i + 1) for i in range(1, n + 1)]


def compute_ndcg_at_k(retrieved_items: List[str], relevant_items: Set[str], k: int) -> float:
    if not relevant_items:
        return 0.0
    dcg = 0.0
    for i, item in enumerate(retrieved_items[:k], 1):
        if item in relevant_items:
            dcg += 1.0 / np.log2(i + 1)
    idcg = 0.0
    for term in _dcg_terms(min(len(relevant_items), k)):
        idcg += term
    return 0.0 if idcg == 0.0 else dcg / idcg


def compute_mrr(retrieved_items: List[str], relevant_items: Set[str]) -> float:
    return next((1.0 / r for r, item in enumerate(retrieved_items, 1) if item in relevant_items),
                0.0)


def compute_hit_rate_at_k(retrieved_items: List[str], relevant_items: Set[str], k: int) -> float:
    return 1.0 if set(retrieved_items[:k]) & relevant_items else 0.0


def compute_diversity(retrieved_items: List[str], product_metadata: Dict,
                      attribute: str = "category") -> float:
    if not retrieved_items:
        return 0.0
    values = {product_metadata.get(p, {}).get(attribute) for p in retrieved_items}
    values.discard(None)
    values = {v for v in values if v}
    return len(values) / len(retrieved_items)


def compute_coverage(all_retrieved_items: Set[str], all_product_ids: Set[str]) -> float:
    if not all_product_ids:
        return 0.0
    return len(all_retrieved_items) / len(all_product_ids)


def _overlap(retrieved_items, buyer_history_items, product_metadata, attribute) -> float:
    if not retrieved_items or not buyer_history_items:
        return 0.0
    seen = {product_metadata.get(p, {}).get(attribute) for p in buyer_history_items}
    seen = {v for v in seen if v}
    if not seen:
        return 0.0
    hits = 0
    for p in retrieved_items:
        v = product_metadata.get(p, {}).get(attribute)
        if v and v in seen:
            hits += 1
    return hits / len(retrieved_items)


def compute_category_overlap(retrieved_items, buyer_history_items, product_metadata) -> float:
    return _overlap(retrieved_items, buyer_history_items, product_metadata, "category")


def compute_brand_overlap(retrieved_items, buyer_history_items, product_metadata) -> float:
    return _overlap(retrieved_items, buyer_history_items, product_metadata, "brand")


def compute_relevance_score(retrieved_items, buyer_history_items, product_metadata) -> float:
    cat = compute_category_overlap(retrieved_items, buyer_history_items, product_metadata)
    brand = compute_brand_overlap(retrieved_items, buyer_history_items, product_metadata)
    return 0.7 * cat + 0.3 * brand


def compute_embedding_stats(embeddings: np.ndarray) -> Dict[str, float]:
    norms = np.linalg.norm(embeddings, axis=1)
    n = min(1000, len(embeddings))
    sample = embeddings[np.random.choice(len(embeddings), n, replace=False)]
    unit = sample / (np.linalg.norm(sample, axis=1, keepdims=True) + 1e-8)
    sims = np.dot(unit, unit.T)[~np.eye(n, dtype=bool)]
    return {"mean_norm": float(np.mean(norms)), "std_norm": float(np.std(norms)),
            "min_norm": float(np.min(norms)), "max_norm": float(np.max(norms)),
            "mean_similarity": float(np.mean(sims)), "std_similarity": float(np.std(sims)),
            "min_similarity": float(np.min(sims)), "max_similarity": float(np.max(sims))}


def _aggregate(metrics: Dict[str, List[float]]) -> Dict[str, float]:
    out = {}
    for key, values in metrics.items():
        if values:
            out[f"{key}_mean"] = float(np.mean(values))
            out[f"{key}_std"] = float(np.std(values))
            out[f"{key}_median"] = float(np.median(values))
    return out


# ------------------------------------------------------------------------- Evaluator (:343)
class Evaluator:
    """Mirror of reference ``Evaluator`` (metrics.py:343-700) over batched retrieval."""

    def __init__(self, encoder, vector_db, config_path: Optional[str] = "configs/config.yaml",
                 batch_size: int = 1024, mode: str = "A"):
        self.encoder = encoder
        self.vector_db = vector_db
        self.config = (load_config(config_path) if config_path is not None
                       else copy.deepcopy(DEFAULT_CONFIG))
        self.product_metadata = None
        self.batch_size, self.mode = batch_size, mode
        self._cache: Dict[Tuple[int, int], List[Optional[List[str]]]] = {}

    def set_product_metadata(self, product_metadata: Dict):
        self.product_metadata = product_metadata

    # one batched pass per (test set, k); None marks a buyer whose encode / search raised
    def _retrieved(self, test_pairs: Sequence, k: int, verbose: bool = False):
        key = (id(test_pairs), k)
        if key in self._cache:
            return self._cache[key]
        out: List[Optional[List[str]]] = []
        for b0 in range(0, len(test_pairs), self.batch_size):
            chunk = test_pairs[b0: b0 + self.batch_size]
            try:
                out.extend(self._batch(chunk, k))
            except Exception:  # redo one by one: skip only the failing buyers
                for buyer_id, interactions, _ in chunk:
                    try:
                        out.extend(self._batch([(buyer_id, interactions, None)], k))
                    except Exception as e:  # reference :481-484
                        if verbose:
                            print(f"Error evaluating buyer {buyer_id}: {e}")
                        out.append(None)
        self._cache[key] = out
        return out

    def _batch(self, chunk, k) -> List[List[str]]:
        histories = [inter for _, inter, _ in chunk]
        if hasattr(self.encoder, "encode_buyers"):
            emb = self.encoder.encode_buyers(histories, mode=self.mode)
        else:
            emb = np.stack([self.encoder.encode_buyer(h) for h in histories])
        results = self.vector_db.retrieve_batch(np.asarray(emb, dtype=np.float32), k=k)
        return [[pid for pid, _ in r] for r in results]

    # reference :372-512
    def evaluate_retrieval(self, test_pairs, k_values: List[int] = [1, 5, 10, 20, 50],
                           verbose: bool = True) -> Dict[str, float]:
        if self.product_metadata is None:
            raise ValueError("Product metadata must be set before evaluation")
        meta = self.product_metadata
        metrics: Dict[str, List[float]] = {}
        for k in k_values:
            for name in ("recall", "precision", "ndcg", "hit_rate", "category_overlap",
                         "brand_overlap", "relevance_score"):
                metrics[f"{name}@{k}"] = []
        metrics["mrr"] = []
        diag = {"avg_history_size": [], "avg_relevant_items": [], "avg_retrieved_items": [],
                "buyers_with_category_info": 0, "buyers_with_brand_info": 0}
        retrieved_all = self._retrieved(test_pairs, max(k_values), verbose)
        for (buyer_id, interactions, relevant), retrieved in zip(test_pairs, retrieved_all):
            if retrieved is None:
                continue
            history = [i["product_id"] for i in interactions]
            for k in k_values:
                top = retrieved[:k]
                metrics[f"recall@{k}"].append(compute_recall_at_k(retrieved, relevant, k))
                metrics[f"precision@{k}"].append(compute_precision_at_k(retrieved, relevant, k))
                metrics[f"ndcg@{k}"].append(compute_ndcg_at_k(retrieved, relevant, k))
                metrics[f"hit_rate@{k}"].append(compute_hit_rate_at_k(retrieved, relevant, k))
                metrics[f"category_overlap@{k}"].append(compute_category_overlap(top, history, meta))
                metrics[f"brand_overlap@{k}"].append(compute_brand_overlap(top, history, meta))
                metrics[f"relevance_score@{k}"].append(compute_relevance_score(top, history, meta))
            metrics["mrr"].append(compute_mrr(retrieved, relevant))
            diag["avg_history_size"].append(len(history))
            diag["avg_relevant_items"].append(len(relevant))
            diag["avg_retrieved_items"].append(len(retrieved))
            if any(meta.get(p, {}).get("category") for p in history):
                diag["buyers_with_category_info"] += 1
            if any(meta.get(p, {}).get("brand") for p in history):
                diag["buyers_with_brand_info"] += 1
        out = _aggregate(metrics)
        if diag["avg_history_size"]:
            out["diagnostics"] = {
                "avg_history_size": float(np.mean(diag["avg_history_size"])),
                "avg_relevant_items": float(np.mean(diag["avg_relevant_items"])),
                "avg_retrieved_items": float(np.mean(diag["avg_retrieved_items"])),
                "buyers_with_category_info": diag["buyers_with_category_info"],
                "buyers_with_brand_info": diag["buyers_with_brand_info"],
                "total_buyers_evaluated": len(diag["avg_history_size"]),
            }
        return out

    # reference :514-546
    def evaluate_embedding_quality(self, product_ids: Optional[List[str]] = None,
                                   sample_size: int = 10000) -> Dict[str, float]:
        if self.product_metadata is None:
            raise ValueError("Product metadata must be set before evaluation")
        if product_ids is None:
            product_ids = list(self.product_metadata.keys())
        if len(product_ids) > sample_size:
            product_ids = np.random.choice(product_ids, sample_size, replace=False).tolist()
        print(f"Encoding {len(product_ids)} products...")
        return compute_embedding_stats(self.encoder.encode_items(product_ids, batch_size=32))

    # reference :548-593
    def evaluate_diversity(self, test_pairs, k: int = 10,
                           attribute: str = "category") -> Dict[str, float]:
        if self.product_metadata is None:
            raise ValueError("Product metadata must be set before evaluation")
        div = [compute_diversity(r, self.product_metadata, attribute)
               for r in self._retrieved(test_pairs, k, True) if r is not None]
        if not div:
            return {}
        return {f"diversity_{attribute}_mean": float(np.mean(div)),
                f"diversity_{attribute}_std": float(np.std(div)),
                f"diversity_{attribute}_median": float(np.median(div))}

    # reference :595-639
    def evaluate_coverage(self, test_pairs, k: int = 10,
                          all_product_ids: Optional[List[str]] = None) -> Dict[str, float]:
        if self.product_metadata is None:
            raise ValueError("Product metadata must be set before evaluation")
        if all_product_ids is None:
            all_product_ids = list(self.product_metadata.keys())
        seen: Set[str] = set()
        for r in self._retrieved(test_pairs, k, True):
            if r is not None:
                seen.update(r)
        return {"coverage": compute_coverage(seen, set(all_product_ids)),
                "unique_retrieved": len(seen), "total_products": len(all_product_ids)}

    # reference :641-700
    def evaluate_all(self, test_pairs, k_values: List[int] = [1, 5, 10, 20, 50],
                     all_product_ids: Optional[List[str]] = None,
                     output_path: Optional[str] = None) -> Dict:
        results = {"retrieval": self.evaluate_retrieval(test_pairs, k_values),
                   "embedding_quality": self.evaluate_embedding_quality()}
        kmax = max(k_values)
        results["diversity"] = {**self.evaluate_diversity(test_pairs, kmax, "category"),
                                **self.evaluate_diversity(test_pairs, kmax, "brand")}
        results["coverage"] = self.evaluate_coverage(test_pairs, kmax, all_product_ids)
        if output_path:
            output_path = Path(output_path)
            output_path.parent.mkdir(parents=True, exist_ok=True)
            with open(output_path, "w", encoding="utf-8") as f:
                json.dump(results, f, indent=2, ensure_ascii=False)
            print(f"\nResults saved to: {output_path}")
        return results
