"""Deterministic inputs for the golden fixtures (seeded numpy PCG64 streams).

Both tests/golden/make_golden.py (reference side) and the tests regenerate inputs here;
the fixtures store a sha256 of the inputs so a drifting generator is detected.
"""
from __future__ import annotations

import hashlib
import json

import numpy as np

EVENT_MIX = (np.array([1.0, 5.0, 10.0], np.float32), np.array([0.75, 0.17, 0.08]))


def sha(*arrays) -> str:
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def event_weights(rng, shape):
    vals, p = EVENT_MIX
    return vals[rng.choice(3, size=shape, p=p)].astype(np.float32)


# ----------------------------------------------------------------------------- buyer tower
BUYER_CASES = {
    "wavg_reftest": dict(method="weighted_avg", E=384, B=2, S=5, seed=11, w="reftest"),
    "wavg_b8_s20": dict(method="weighted_avg", E=384, B=8, S=20, seed=12),
    "wavg_s100": dict(method="weighted_avg", E=384, B=4, S=100, seed=13),
    "wavg_s1": dict(method="weighted_avg", E=384, B=3, S=1, seed=14),
    "wavg_pad": dict(method="weighted_avg", E=384, B=4, S=20, seed=15, pad=8),
    "wavg_zero_w": dict(method="weighted_avg", E=384, B=2, S=5, seed=16, w="zero"),
    "wavg_e768": dict(method="weighted_avg", E=768, B=4, S=20, seed=17),
    "wavg_scaled": dict(method="weighted_avg", E=384, B=4, S=20, seed=18, scale=1000.0),
    "wavg_e100": dict(method="weighted_avg", E=100, B=3, S=7, seed=19),
    "attn_reftest": dict(method="attention", E=384, B=2, S=5, seed=21, w="reftest"),
    "attn_b8_s20": dict(method="attention", E=384, B=8, S=20, seed=22),
    "attn_pad": dict(method="attention", E=384, B=4, S=20, seed=23, pad=8),
    "attn_e768": dict(method="attention", E=768, B=3, S=20, seed=24),
    "attn_s100": dict(method="attention", E=384, B=2, S=100, seed=25),
}


def buyer_inputs(spec):
    rng = np.random.default_rng(spec["seed"])
    B, S, E = spec["B"], spec["S"], spec["E"]
    items = rng.standard_normal((B, S, E), dtype=np.float32)
    if "scale" in spec:
        items *= np.float32(spec["scale"])
    if spec.get("w") == "reftest":  # reference tests/test_buyer_tower.py:25
        w = np.array([[1.0, 5.0, 10.0, 1.0, 1.0], [1.0, 1.0, 5.0, 5.0, 1.0]], np.float32)
    elif spec.get("w") == "zero":
        w = np.zeros((B, S), np.float32)
    else:
        w = event_weights(rng, (B, S))
    if spec.get("pad"):
        p = spec["pad"]
        items[:, S - p:, :] = 0.0
        w[:, S - p:] = 0.0
    return items, w


def attn_weights(spec):
    rng = np.random.default_rng(1000 + spec["seed"])
    E, H = spec["E"], spec.get("H", 128)
    a, b = 1.0 / np.sqrt(E), 1.0 / np.sqrt(H)
    W1 = rng.uniform(-a, a, (H, E)).astype(np.float32)
    b1 = rng.uniform(-a, a, (H,)).astype(np.float32)
    W2 = rng.uniform(-b, b, (1, H)).astype(np.float32)
    b2 = rng.uniform(-b, b, (1,)).astype(np.float32)
    return W1, b1, W2, b2


# ----------------------------------------------------------------------------- InfoNCE
INFONCE_CASES = {
    "b8_e384": dict(B=8, E=384, N=4, tau=0.07, seed=31),
    "b64_e768": dict(B=64, E=768, N=4, tau=0.07, seed=32),
    "b32_e384_t05": dict(B=32, E=384, N=4, tau=0.5, seed=33),
}


def _unit(x):
    return (x / np.linalg.norm(x, axis=-1, keepdims=True)).astype(np.float32)


def infonce_inputs(spec):
    rng = np.random.default_rng(spec["seed"])
    B, E, N = spec["B"], spec["E"], spec["N"]
    return (_unit(rng.standard_normal((B, E), dtype=np.float32)),
            _unit(rng.standard_normal((B, E), dtype=np.float32)),
            _unit(rng.standard_normal((B, N, E), dtype=np.float32)))


# ----------------------------------------------------------------------------- item head
BRANDS = ["Acme", "Dubai Gold", "Lazurde", "Damas", "Tiffany"]
CATEGORIES = ["rings", "necklaces", "bracelets", "engine-oil"]


def item_text_embeddings():
    rng = np.random.default_rng(41)
    return rng.standard_normal((16, 384), dtype=np.float32) * np.float32(0.3)


def item_head_weights(use_cat: bool):
    """Seeded ItemTower head parameters (names as in the reference module, item_tower.py:58-63,
    84-97).  Embedding row 0 (<UNK>, padding_idx) stays zero as nn.Embedding initialises it."""
    rng = np.random.default_rng(42 if use_cat else 43)
    din = 384 + (128 if use_cat else 0)
    w = {
        "projection.0.weight": rng.uniform(-1, 1, (256, din)) / np.sqrt(din),
        "projection.0.bias": rng.uniform(-1, 1, (256,)) / np.sqrt(din),
        "projection.3.weight": rng.uniform(-1, 1, (384, 256)) / 16.0,
        "projection.3.bias": rng.uniform(-1, 1, (384,)) / 16.0,
    }
    if use_cat:
        for name, n in (("brand_embedding.weight", len(BRANDS) + 1),
                        ("category_embedding.weight", len(CATEGORIES) + 1)):
            e = rng.standard_normal((n, 64))
            e[0] = 0.0
            w[name] = e
    return {k: v.astype(np.float32) for k, v in w.items()}


def item_batch():
    texts = [f"p#{i}" for i in range(12)]
    brands = ["Acme", "Damas", None, "Unknown", "Tiffany", "Lazurde", "", "Dubai Gold", "Acme",
              "Damas", None, "Tiffany"]
    cats = ["rings", None, "necklaces", "bracelets", "engine-oil", "nope", "rings", "",
            "bracelets", "rings", "necklaces", None]
    return texts, brands, cats


# ----------------------------------------------------------------------------- flat IP
FLATIP_CASES = {
    "n1_k10": dict(N=1, Q=4, k=10, seed=51),
    "n99_k100": dict(N=99, Q=16, k=100, seed=52),
    "n100_k100": dict(N=100, Q=16, k=100, seed=53),
    "n101_k100": dict(N=101, Q=16, k=100, seed=54),
    "n4096_k1": dict(N=4096, Q=16, k=1, seed=55),
    "n4096_k10": dict(N=4096, Q=16, k=10, seed=56),
    "n4096_k100": dict(N=4096, Q=16, k=100, seed=57),
    "n4096_k1000": dict(N=4096, Q=8, k=1000, seed=58),
    "dups_k100": dict(N=600, Q=8, k=100, seed=59, dups=True),
    "e768_k100": dict(N=2000, Q=8, k=100, seed=60, E=768),
}


def flatip_inputs(spec):
    rng = np.random.default_rng(spec["seed"])
    E = spec.get("E", 384)
    x = rng.standard_normal((spec["N"], E), dtype=np.float32)
    if spec.get("dups"):
        # every row appears 3 times (exact ties at every score) -> tie order by row index
        base = x[: spec["N"] // 3]
        x = np.concatenate([base, base, base])[: spec["N"]].copy()
    q = rng.standard_normal((spec["Q"], E), dtype=np.float32)
    return x, q


# --------------------------------------------------------------- evaluation metrics (f4)
EVAL_K = [1, 5, 10, 20]


def eval_cases(seed: int = 21, n_products: int = 60, n_buyers: int = 40):
    """Synthetic evaluation set: metadata (some categories / brands missing or empty),
    per buyer: interactions, relevant set (0..5 items, some outside the catalog) and the
    retrieved list (20 distinct ids) a stub index returns."""
    rng = np.random.default_rng(seed)
    pids = [f"p{i}" for i in range(n_products)]
    cats = ["rings", "necklaces", "oil", None, ""]
    brands = ["Acme", "Damas", None, "Lazurde"]
    meta = {p: {"text": f"item {p}", "category": cats[rng.integers(0, len(cats))],
                "brand": brands[rng.integers(0, len(brands))]} for p in pids}
    events = ["view", "add_to_cart", "purchase"]
    cases = []
    for b in range(n_buyers):
        hist = [{"product_id": pids[rng.integers(0, n_products)],
                 "event_type": events[rng.integers(0, 3)], "timestamp": None}
                for _ in range(rng.integers(0, 7))]
        rel = {pids[j] for j in rng.integers(0, n_products, rng.integers(0, 6))}
        if b % 7 == 3:
            rel.add("unknown-item")
        ret = [pids[j] for j in rng.permutation(n_products)[:20]]
        cases.append((f"u{b}", hist, rel, ret))
    return pids, meta, cases


# ------------------------------------------------ VectorDatabase / server fixtures (a10-a12, f1, f2)
# Generated by tests/golden/make_retrieval_golden.py through the reference's own VectorDatabase
# and FastAPI /retrieve handler.
VDB_CASES = dict(
    {name: dict(spec) for name, spec in FLATIP_CASES.items()},
    short_ids=dict(N=50, Q=6, k=45, seed=61, n_ids=40),       # idx < len(product_ids) filter
    f64_input=dict(N=300, Q=6, k=20, seed=62, dtype="f64"),   # normalised in f64, then cast
    unicode_ids=dict(N=30, Q=4, k=10, seed=63, unicode=True),
    scaled_zero_row=dict(N=500, Q=6, k=50, seed=64, scale=1e3, zero_row=7),
    server=dict(N=200, Q=1, k=10, seed=65, prefix="SKU-"),
)


def vdb_inputs(spec):
    """(embeddings, queries, product_ids) of one VectorDatabase case."""
    x, q = flatip_inputs(spec)
    if "scale" in spec:
        x = x * np.float32(spec["scale"])
    if "zero_row" in spec:
        x[spec["zero_row"]] = 0.0
    if spec.get("dtype") == "f64":
        rng = np.random.default_rng(spec["seed"] + 1000)
        x = x.astype(np.float64) + rng.standard_normal(x.shape) * 1e-9
        q = q.astype(np.float64)
    n_ids = spec.get("n_ids", x.shape[0])
    if spec.get("unicode"):
        ids = [f"منتج-{j}" for j in range(n_ids)]
    else:
        ids = [f"{spec.get('prefix', 'p')}{j}" for j in range(n_ids)]
    return x, q, ids


def stub_buyer_embedding(interactions, E):
    """Deterministic stand-in for EmbeddingEncoder.encode_buyer in the /retrieve fixtures:
    a seeded vector keyed by the interaction list."""
    import zlib

    key = "|".join(f"{i['product_id']}:{i['event_type']}" for i in interactions)
    rng = np.random.default_rng(zlib.crc32(key.encode("utf-8")))
    return rng.standard_normal(E).astype(np.float32)


def server_products():
    """products_df columns (reference schema): duplicates (first row wins), NaN / None
    cells, Arabic text; SKU-3, SKU-11 and SKU-150..199 are absent (-> 'N/A' records)."""
    rng = np.random.default_rng(66)
    ids = [f"SKU-{j}" for j in range(150) if j not in (3, 11)] + ["SKU-5", "SKU-8"]
    brands = ["Damas", "Lazurde", None, float("nan"), "Acme"]
    cats = ["خواتم", "rings", float("nan"), None, "oil"]
    return {
        "product_id": ids,
        "title": [f"خاتم ذهب {j}" if j % 3 else (float("nan") if j % 2 else f"title {j}")
                  for j in range(len(ids))],
        "description": [f"desc {j}" if j % 5 else "" for j in range(len(ids))],
        "brand": [brands[int(rng.integers(0, len(brands)))] for _ in ids],
        "category": [cats[int(rng.integers(0, len(cats)))] for _ in ids],
    }


def server_photos():
    return {f"SKU-{j}": f"https://img.example/{j}.jpg" for j in range(0, 200, 4)}


def server_requests():
    rng = np.random.default_rng(67)
    events = ["view", "add_to_cart", "purchase", "AddToCart", "buy", "wishlist"]
    reqs = []
    for b, k in enumerate([10, 1, 5, 50, 200, 250, 1000]):
        n = int(rng.integers(1, 8))
        inter = [{"product_id": f"SKU-{int(rng.integers(0, 200))}",
                  "event_type": events[int(rng.integers(0, len(events)))],
                  "timestamp": None if b % 2 else f"2024-01-0{1 + j}T10:00:00"}
                 for j in range(n)]
        reqs.append({"buyer_id": f"buyer-{b}", "recent_interactions": inter, "k": k})
    return reqs


# ------------------------------------------------ Trainer._encode_buyer_sequences_batched (f3)
def trainer_texts():
    return [f"نص المنتج {j}" for j in range(40)] + ["positive fallback A", "positive fallback B"]


def trainer_batch():
    """(product_metadata, buyer_sequences, positive_texts) in the collate_fn format: tuples of
    (pid, weight) / (pid, weight, timestamp), malformed entries, unknown ids, an empty and an
    all-unknown history (-> positive-text fallback), a 130-item history (-> last 100)."""
    rng = np.random.default_rng(71)
    texts = trainer_texts()
    meta = {f"p{j}": {"text": texts[j], "brand": None, "category": None} for j in range(40)}
    seqs = []
    for b in range(5):
        seq = []
        for _ in range(int(rng.integers(1, 25))):
            pid = f"p{int(rng.integers(0, 45))}"  # p40..p44: not in the metadata
            w = float(rng.choice([1.0, 5.0, 10.0]))
            seq.append((pid, w, "2024-01-01") if rng.random() < 0.5 else (pid, w))
        if b == 2:
            seq.append(("p1",))  # malformed: skipped
        seqs.append(seq)
    seqs.append([])                                     # empty -> fallback
    seqs.append([("p41", 5.0), ("p44", 1.0)])           # all unknown -> fallback
    seqs.append([(f"p{j % 40}", float(1 + j % 3)) for j in range(130)])  # truncation
    pos = [texts[j] for j in range(5)] + [texts[40], texts[41], texts[7]]
    return meta, seqs, pos


# ----------------------------------------------------------------------------- configs[0] pipeline
# BASELINE.json configs[0]: 1k products in the reference CSV schema (processor.py:71-112: id,
# title, description, metadata JSON {brand, catalog_id}), 100 buyers x 20 events (event mix
# 0.75 / 0.17 / 0.08, DATA_PREPROCESSING.md:97-99), seed 0, k = 10 (scripts/evaluate.py).
PIPE_WORDS = ["خاتم", "ذهب", "عيار", "21", "18", "سلسال", "اسورة", "فضة", "زيت", "محرك",
              "5W-30", "gold", "ring", "necklace", "bracelet", "silver", "engine", "oil",
              "Damas", "classic", "new", "مميز", "هدية", "لامع"]
PIPE_BRANDS = ["Damas", "Lazurde", "Acme", "Tiffany", "Dubai Gold", "Mobil", "Shell", "Tanagra"]
PIPE_CATS = [f"cat_{i:02d}" for i in range(12)]


def pipeline_products(n: int = 1000, seed: int = 0):
    """Product rows (dicts; None = empty CSV cell).  ~3% are content duplicates of an earlier
    row under another id (processor.py:243-284 keeps one per dedup key), ~2% lack a title or
    a description, 3 have neither (dropped: empty text, :104), ~10% have no metadata."""
    rng = np.random.default_rng(seed)
    rows = []
    for i in range(n):
        pid = f"P{int(rng.integers(0, 10**6)):06d}-{i}"
        title = " ".join(rng.choice(PIPE_WORDS, int(rng.integers(1, 6))))
        desc = " ".join(rng.choice(PIPE_WORDS, int(rng.integers(0, 12))))
        brand = PIPE_BRANDS[int(rng.integers(0, len(PIPE_BRANDS)))]
        cat = PIPE_CATS[int(rng.integers(0, len(PIPE_CATS)))]
        r = rng.random()
        if r < 0.03 and rows:  # duplicate content (case / spacing changed) of an earlier row
            src = rows[int(rng.integers(0, len(rows)))]
            title = (src["title"] or "").upper() + "  "
            desc, meta = src["description"], src["metadata"]
        else:
            meta = json.dumps({"brand": brand, "catalog_id": cat}, ensure_ascii=False) \
                if rng.random() > 0.1 else None
        if 0.03 <= r < 0.04:
            title = None
        elif 0.04 <= r < 0.05:
            desc = None
        if i in (17, 401, 902):
            title, desc = None, "   "
        rows.append({"id": pid, "title": title, "description": desc or None, "metadata": meta})
    return rows


def pipeline_events(product_ids, n_buyers: int = 100, per_buyer: int = 20, seed: int = 0):
    """Event rows (distinct_id, product_id, event_name, created_at) in the reference events
    schema (processor.py:24-69 renames them).  Product ids are drawn from the whole CSV, so
    some point at deduplicated / dropped products (metadata {} -> text ' ', encoder.py:280);
    event names vary in case and spacing; two events have no timestamp."""
    rng = np.random.default_rng(seed + 1)
    names = [["view", "View", "page view"], ["add_to_cart", "Add To Cart", "AddToCart"],
             ["purchase", "Purchase", "buy"]]
    rows = []
    for b in range(n_buyers):
        for e in range(per_buyer):
            kind = int(rng.choice(3, p=EVENT_MIX[1]))
            name = names[kind][int(rng.integers(0, 3))]
            t = int(rng.integers(0, 365 * 24 * 3600))
            ts = f"2024-{1 + t // (31 * 24 * 3600) % 12:02d}-{1 + t // 86400 % 28:02d} " \
                 f"{t // 3600 % 24:02d}:{t // 60 % 60:02d}:{t % 60:02d}"
            rows.append({"distinct_id": f"B{b:03d}",
                         "product_id": product_ids[int(rng.integers(0, len(product_ids)))],
                         "event_name": name, "created_at": ts})
    rows[5]["created_at"] = None
    rows[333]["created_at"] = None
    return rows


def stub_text_embedding(texts, dim: int = 384) -> np.ndarray:
    """Deterministic stand-in for SentenceTransformer.encode (item_tower.py:116-122; the real
    MiniLM is absent offline): per text, a PCG64 normal vector seeded by blake2b(text)."""
    out = np.empty((len(texts), dim), np.float32)
    for j, t in enumerate(texts):
        s = int.from_bytes(hashlib.blake2b(t.encode("utf-8"), digest_size=8).digest(), "little")
        out[j] = np.random.default_rng(s).standard_normal(dim).astype(np.float32) * np.float32(0.5)
    return out


def pipeline_weights(n_brand: int, n_cat: int, E: int = 384, seed: int = 7):
    """Seeded checkpoint weights (reference state-dict names, trainer.py:327-340) for the
    configs[0] pipeline: ItemTower head + categorical tables (row 0 = padding, zero) and the
    BuyerTower attention MLP."""
    rng = np.random.default_rng(seed)
    din = 384 + 128
    w = {
        "item_tower.projection.0.weight": rng.uniform(-1, 1, (256, din)) / np.sqrt(din),
        "item_tower.projection.0.bias": rng.uniform(-1, 1, (256,)) / np.sqrt(din),
        "item_tower.projection.3.weight": rng.uniform(-1, 1, (E, 256)) / 16.0,
        "item_tower.projection.3.bias": rng.uniform(-1, 1, (E,)) / 16.0,
        "item_tower.brand_embedding.weight": rng.standard_normal((n_brand, 64)),
        "item_tower.category_embedding.weight": rng.standard_normal((n_cat, 64)),
        "buyer_tower.attention.0.weight": rng.uniform(-1, 1, (128, E)) / np.sqrt(E),
        "buyer_tower.attention.0.bias": rng.uniform(-1, 1, (128,)) / np.sqrt(E),
        "buyer_tower.attention.2.weight": rng.uniform(-1, 1, (1, 128)) / np.sqrt(128),
        "buyer_tower.attention.2.bias": rng.uniform(-1, 1, (1,)) / np.sqrt(128),
    }
    w["item_tower.brand_embedding.weight"][0] = 0.0
    w["item_tower.category_embedding.weight"][0] = 0.0
    return {k: v.astype(np.float32) for k, v in w.items()}


def encoder_buyer_cases(product_ids):
    """Adversarial interaction lists for EmbeddingEncoder.encode_buyer (encoder.py:244-305):
    timestamp sort iff every one is present (ISO strings, :263-264), > 100 events (last
    max_interaction_history kept, :267-268), unknown ids and event names (weight 1), aliases
    (AddToCart / buy), one event, products with empty text."""
    rng = np.random.default_rng(77)
    P = list(product_ids)

    def ev(pid, name, ts):
        d = {"product_id": pid, "event_type": name}
        if ts is not None:
            d["timestamp"] = ts
        return d

    cases = []
    # 1. all timestamps present, shuffled -> sorted
    cases.append([ev(P[int(rng.integers(0, len(P)))], n, f"2024-03-{d:02d}T10:00:00")
                  for n, d in zip(["view", "purchase", "AddToCart", "buy", "share"],
                                  [9, 2, 17, 5, 11])])
    # 2. one timestamp missing -> input order kept
    c = [ev(P[int(rng.integers(0, len(P)))], "view", f"2024-05-{d:02d}") for d in (30, 3, 12)]
    c[1]["timestamp"] = None
    cases.append(c)
    # 3. 130 events, every one timestamped -> sort, keep the last 100
    cases.append([ev(P[int(rng.integers(0, len(P)))], ["view", "add_to_cart", "purchase"][i % 3],
                     f"2023-{1 + i % 12:02d}-{1 + (i * 7) % 28:02d}T{i % 24:02d}:00:00")
                  for i in range(130)])
    # 4. 120 events, no timestamps -> input order, last 100
    cases.append([ev(P[(37 * i) % len(P)], "view" if i % 4 else "Purchase", None)
                  for i in range(120)])
    # 5. unknown product ids (metadata {} -> text '' -> ' ') mixed with known ones
    cases.append([ev("not-a-product", "view", None), ev(P[3], "purchase", None),
                  ev("ghost-2", "AddToCart", None)])
    # 6. a single event
    cases.append([ev(P[11], "add_to_cart", "2024-01-01")])
    return cases
