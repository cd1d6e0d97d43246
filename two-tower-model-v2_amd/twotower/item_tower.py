"""ItemTower on MI355X: drop-in for the reference's sentence-transformers-backed module.

Reference: src/models/item_tower.py (class ItemTower :10).  Same constructor arguments,
``initialize_categorical_embeddings`` / ``encode_text`` / ``encode_categorical`` /
``forward`` / ``encode_batch``, state-dict keys ``projection.{0,3}.{weight,bias}``,
``brand_embedding.weight``, ``category_embedding.weight``; outputs L2-normalised float32.

The text encoder is ``BertEncoder``: the MiniLM-class BertModel (12 layers, hidden 384,
12 heads, FFN 1536, GELU, LayerNorm eps 1e-12) + masked mean pooling that
SentenceTransformer("paraphrase-multilingual-MiniLM-L12-v2").encode runs (item_tower.py:116),
executed by the HIP kernels of csrc/tt_encoder.hip over packed (unpadded) token sequences.
Its weights come from a Hugging Face BertModel state dict; offline there is no checkpoint,
so ``random_bert_state_dict`` provides seeded weights of the same architecture.

Tokenisation: the reference's XLM-R SentencePiece tokenizer ships with the model files, which
are absent offline.  ``ItemTower`` accepts any ``tokenizer(texts) -> list of id lists``; the
default ``HashTokenizer`` is a deterministic stand-in (``<s>`` text-pieces ``</s>``, ids hashed
into the vocabulary, truncation to 128 tokens) -- parity of token ids with the real tokenizer
is unpinned; everything from token ids on is the reference's arithmetic.
"""
from __future__ import annotations

import ctypes
import hashlib
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.nn as nn

from . import _lib, kernels
from ._lib import check, lib, stream_ptr

MINILM_L12 = dict(vocab=250037, hidden=384, layers=12, heads=12, intermediate=1536,
                  max_positions=512, type_vocab=2, ln_eps=1e-12)
MAX_SEQ_LENGTH = 128  # sentence-transformers max_seq_length of the MiniLM model


def random_bert_state_dict(cfg: Dict, seed: int = 0, std: float = 0.02) -> Dict[str, torch.Tensor]:
    """Seeded float32 weights of a BertModel (Hugging Face key names, no pooler).

    numpy's PCG64 stream, drawn in a fixed key order: reproducible on any host."""
    rng = np.random.default_rng(seed)
    H, I, V = cfg["hidden"], cfg["intermediate"], cfg["vocab"]

    def n(*shape, s=std):
        return torch.from_numpy((rng.standard_normal(shape) * s).astype(np.float32))

    sd = {
        "embeddings.word_embeddings.weight": n(V, H),
        "embeddings.position_embeddings.weight": n(cfg["max_positions"], H),
        "embeddings.token_type_embeddings.weight": n(cfg["type_vocab"], H),
        "embeddings.LayerNorm.weight": 1.0 + n(H, s=0.1),
        "embeddings.LayerNorm.bias": n(H),
    }
    for l in range(cfg["layers"]):
        p = f"encoder.layer.{l}."
        for name in ("query", "key", "value"):
            sd[p + f"attention.self.{name}.weight"] = n(H, H)
            sd[p + f"attention.self.{name}.bias"] = n(H)
        sd[p + "attention.output.dense.weight"] = n(H, H)
        sd[p + "attention.output.dense.bias"] = n(H)
        sd[p + "attention.output.LayerNorm.weight"] = 1.0 + n(H, s=0.1)
        sd[p + "attention.output.LayerNorm.bias"] = n(H)
        sd[p + "intermediate.dense.weight"] = n(I, H)
        sd[p + "intermediate.dense.bias"] = n(I)
        sd[p + "output.dense.weight"] = n(H, I)
        sd[p + "output.dense.bias"] = n(H)
        sd[p + "output.LayerNorm.weight"] = 1.0 + n(H, s=0.1)
        sd[p + "output.LayerNorm.bias"] = n(H)
    return sd


def pack_sequences(seqs: Sequence[Sequence[int]], device=None):
    """List of token-id lists -> (ids int32 [T], cu_seqlens int32 [n+1], max_len) on device."""
    lens = [len(s) for s in seqs]
    if any(L < 1 for L in lens):
        raise ValueError("every sequence needs at least one token")
    cu = np.zeros(len(seqs) + 1, np.int32)
    cu[1:] = np.cumsum(lens)
    flat = np.fromiter((t for s in seqs for t in s), dtype=np.int32, count=int(cu[-1]))
    dev = device or _lib.device()
    # pinned + non-blocking: a pageable copy waits for the stream, so the host could not pack
    # the next batch while this one is encoded
    up = (lambda a: torch.from_numpy(a).pin_memory().to(dev, non_blocking=True)) \
        if torch.device(dev).type == "cuda" else (lambda a: torch.from_numpy(a).to(dev))
    return up(flat), up(cu), max(lens) if lens else 0


def x3_split_weights(w: torch.Tensor) -> torch.Tensor:
    """[N, K] f32 (device) -> the x3 GEMM's pre-split image [N, 2K] bf16 (tt_x3_split_weights)."""
    N, K = w.shape
    out = torch.empty((N, 2 * K), dtype=torch.bfloat16, device=w.device)
    check(lib().tt_x3_split_weights(w.data_ptr(), w.stride(0), N, K, out.data_ptr(), out.stride(0),
                                    stream_ptr()), "tt_x3_split_weights")
    return out


def x3i_weights(w: torch.Tensor) -> torch.Tensor:
    """[N, K] f32 (device) -> the x3 encoder's x3i image [N, 2K] bf16: per 32 k, 32 hi =
    bf16(W) then 32 lo = bf16(W - hi) (tt_x3i_weights)."""
    N, K = w.shape
    out = torch.empty((N, 2 * K), dtype=torch.bfloat16, device=w.device)
    check(lib().tt_x3i_weights(w.data_ptr(), w.stride(0), N, K, out.data_ptr(), out.stride(0),
                               stream_ptr()), "tt_x3i_weights")
    return out


class BertEncoder:
    """Device-resident BertModel weights + the fused HIP forward (tt_bert_encode).

    ``prec`` "f32": every GEMM on f32 MFMA (parity path); "x3": the f32 path with each GEMM's
    f32 operands split on the fly into bf16 hi + lo, products as three bf16 MFMAs (the parity
    precision class at bf16 MFMA rates); "bf16": GEMMs on bf16 MFMA with f32 accumulation and
    f32 residual stream / LayerNorm / softmax / pooling (throughput path)."""

    _PREC = {"f32": _lib.TT_PREC_F32, "bf16": _lib.TT_PREC_BF16, "x3": _lib.TT_PREC_X3}

    def __init__(self, state_dict: Dict[str, torch.Tensor], cfg: Dict = MINILM_L12,
                 device=None, prec: str = "x3"):
        if prec not in self._PREC:
            raise ValueError("prec must be 'f32', 'x3' or 'bf16'")
        self.cfg = dict(cfg)
        self.prec = prec
        self.device = device or _lib.device()
        H, nl = cfg["hidden"], cfg["layers"]
        dev = self.device

        def t(key):
            return state_dict[key].detach().to(device=dev, dtype=torch.float32).contiguous()

        self._keep = []  # tensors referenced by raw pointers in the ctypes structs

        def ptr(x):
            self._keep.append(x)
            return x.data_ptr()

        m = _lib.BertModel()
        m.vocab, m.hidden, m.heads = cfg["vocab"], H, cfg["heads"]
        m.intermediate, m.layers, m.max_positions = cfg["intermediate"], nl, cfg["max_positions"]
        m.ln_eps = cfg["ln_eps"]
        m.word_emb = ptr(t("embeddings.word_embeddings.weight"))
        m.pos_emb = ptr(t("embeddings.position_embeddings.weight"))
        m.type_emb = ptr(t("embeddings.token_type_embeddings.weight"))
        m.emb_ln_g = ptr(t("embeddings.LayerNorm.weight"))
        m.emb_ln_b = ptr(t("embeddings.LayerNorm.bias"))
        layers = (_lib.BertLayer * max(nl, 1))()
        for l in range(nl):
            p = f"encoder.layer.{l}."
            wqkv = torch.cat([t(p + f"attention.self.{n}.weight") for n in ("query", "key", "value")])
            bqkv = torch.cat([t(p + f"attention.self.{n}.bias") for n in ("query", "key", "value")])
            L = layers[l]
            L.wqkv, L.bqkv = ptr(wqkv), ptr(bqkv)
            wo, w1, w2 = (t(p + "attention.output.dense.weight"), t(p + "intermediate.dense.weight"),
                          t(p + "output.dense.weight"))
            L.wo, L.bo = ptr(wo), ptr(t(p + "attention.output.dense.bias"))
            L.ln1_g = ptr(t(p + "attention.output.LayerNorm.weight"))
            L.ln1_b = ptr(t(p + "attention.output.LayerNorm.bias"))
            L.w1, L.b1 = ptr(w1), ptr(t(p + "intermediate.dense.bias"))
            L.w2, L.b2 = ptr(w2), ptr(t(p + "output.dense.bias"))
            L.ln2_g = ptr(t(p + "output.LayerNorm.weight"))
            L.ln2_b = ptr(t(p + "output.LayerNorm.bias"))
            if prec == "x3":  # the weights' hi / lo split once (tt_x3_split_weights), and
                # their x3i interleaved form for the bf16 GEMM kernels (H = 384: tt_bert_encode's
                # x3i path)
                L.wqkv_x3, L.wo_x3, L.w1_x3, L.w2_x3 = (ptr(x3_split_weights(x))
                                                        for x in (wqkv, wo, w1, w2))
                L.wqkv_x3i, L.wo_x3i, L.w1_x3i, L.w2_x3i = (ptr(x3i_weights(x))
                                                            for x in (wqkv, wo, w1, w2))
            if prec == "bf16":
                L.wqkv_bf16 = ptr(wqkv.to(torch.bfloat16))
                L.wo_bf16 = ptr(wo.to(torch.bfloat16))
                L.w1_bf16 = ptr(w1.to(torch.bfloat16))
                L.w2_bf16 = ptr(w2.to(torch.bfloat16))
        m.layer = ctypes.cast(layers, ctypes.POINTER(_lib.BertLayer))
        self._layers = layers
        self._model = m
        # per HIP stream (encodes may run concurrently on several streams), bounded LRU
        self._ws = _lib.StreamWorkspaces(4)

    @property
    def hidden(self) -> int:
        return self.cfg["hidden"]

    def workspace_bytes(self, T: int) -> int:
        b = ctypes.c_int64(0)
        check(lib().tt_bert_workspace_bytes(T, self.hidden, self.cfg["intermediate"],
                                            self._PREC[self.prec], ctypes.byref(b)),
              "tt_bert_workspace_bytes")
        return b.value

    def encode_packed(self, ids: torch.Tensor, cu_seqlens: torch.Tensor, max_len: int,
                      out: torch.Tensor = None) -> torch.Tensor:
        """ids int32 [T], cu_seqlens int32 [n+1] (device) -> mean-pooled [n, H] float32."""
        if ids.dtype != torch.int32 or cu_seqlens.dtype != torch.int32:
            raise TypeError("ids and cu_seqlens must be int32")
        n, T = cu_seqlens.numel() - 1, ids.numel()
        if out is None:
            out = torch.empty((n, self.hidden), dtype=torch.float32, device=ids.device)
        if n == 0:
            return out
        if max_len > self.cfg["max_positions"]:
            raise ValueError(f"sequence longer than max_position_embeddings ({max_len})")
        need = self.workspace_bytes(T)
        st = stream_ptr()
        ws = self._ws.get(need, ids.device)
        check(lib().tt_bert_encode(ctypes.byref(self._model), ids.data_ptr(),
                                   cu_seqlens.data_ptr(), n, T, int(max_len),
                                   self._PREC[self.prec], out.data_ptr(), out.stride(0), ws.data_ptr(), ws.numel(), st),
              "tt_bert_encode")
        return out

    def encode_ids(self, seqs: Sequence[Sequence[int]]) -> torch.Tensor:
        ids, cu, mx = pack_sequences(seqs, self.device)
        return self.encode_packed(ids, cu, mx)


class HashTokenizer:
    """Deterministic stand-in for the XLM-R SentencePiece tokenizer (absent offline):
    ``<s>`` (0), one id per whitespace-separated piece (blake2b hash into [3, vocab)), ``</s>``
    (2), truncated to ``max_length``.  Token-id parity with the real tokenizer is unpinned."""

    def __init__(self, vocab: int = MINILM_L12["vocab"], max_length: int = MAX_SEQ_LENGTH):
        self.vocab, self.max_length = vocab, max_length

    def __call__(self, texts: Sequence[str]) -> List[List[int]]:
        out = []
        for t in texts:
            ids = [0]
            for piece in t.split():
                h = int.from_bytes(hashlib.blake2b(piece.encode(), digest_size=8).digest(), "little")
                ids.append(3 + h % (self.vocab - 3))
            ids = ids[: self.max_length - 1] + [2]
            out.append(ids)
        return out


class _HipTextEncoder:
    """The ``text_encoder`` of ItemTower: tokenizer + BertEncoder (the SentenceTransformer
    surface the reference uses: ``encode``, ``get_sentence_embedding_dimension``)."""

    def __init__(self, encoder: BertEncoder, tokenizer):
        self.encoder, self.tokenizer = encoder, tokenizer

    def get_sentence_embedding_dimension(self) -> int:
        return self.encoder.hidden

    def encode(self, texts, **kw) -> torch.Tensor:
        return self.encoder.encode_ids(self.tokenizer(texts))


def _device_ids(v, dev):
    """Categorical ids -> int32 on ``dev`` without stalling the host: a device tensor is used
    as is, a host list goes through pinned memory with a non-blocking copy (torch.tensor(...,
    device=dev) is a synchronous copy that waits for the stream, so the host could not queue
    the next batch's launches while this one runs)."""
    if v is None:
        return None
    if isinstance(v, torch.Tensor):
        return v.to(dev, torch.int32, non_blocking=True).contiguous()
    return torch.tensor(v, dtype=torch.int32).pin_memory().to(dev, non_blocking=True)


class ItemTower(nn.Module):
    """Mirror of reference ``ItemTower`` (src/models/item_tower.py:10-243)."""

    def __init__(self, text_encoder_name: str = "paraphrase-multilingual-MiniLM-L12-v2",
                 embedding_dim: int = 384, use_categorical_features: bool = True,
                 categorical_embedding_dim: int = 64, projection_hidden_dim: int = 256,
                 freeze_text_encoder: bool = True, text_encoder=None, tokenizer=None,
                 encoder_state_dict: Optional[Dict[str, torch.Tensor]] = None,
                 encoder_cfg: Dict = MINILM_L12, prec: str = "x3", seed: int = 0):
        super().__init__()
        self.embedding_dim = embedding_dim
        self.use_categorical_features = use_categorical_features
        if text_encoder is None:  # the HIP MiniLM encoder (seeded weights unless given)
            sd = encoder_state_dict or random_bert_state_dict(encoder_cfg, seed)
            text_encoder = _HipTextEncoder(BertEncoder(sd, encoder_cfg, prec=prec),
                                           tokenizer or HashTokenizer(encoder_cfg["vocab"]))
        self.text_encoder = text_encoder  # not an nn.Module: frozen, never trained here
        text_dim = self.text_encoder.get_sentence_embedding_dimension()
        if use_categorical_features:
            self.brand_embedding = None
            self.category_embedding = None
            self.categorical_embedding_dim = categorical_embedding_dim
            input_dim = text_dim + 2 * categorical_embedding_dim
        else:
            input_dim = text_dim
        self.projection = nn.Sequential(nn.Linear(input_dim, projection_hidden_dim), nn.ReLU(),
                                        nn.Dropout(0.1),
                                        nn.Linear(projection_hidden_dim, embedding_dim))
        self._categorical_vocabs = {"brand": set(), "category": set()}
        # precision of the projection head's two GEMMs at inference: "x3" (split-bf16 products,
        # k_gemm<float, 1>: the f32 precision class at 16x the f32 MFMA rate -- a batch of 256
        # is 4 tiles, 47 + 27 us on f32 MFMA) with the x3 encoder, else "f32"
        enc = getattr(self.text_encoder, "encoder", None)
        self.head_prec = "x3" if getattr(enc, "prec", None) == "x3" else "f32"

    # reference :68-98
    def initialize_categorical_embeddings(self, brand_vocab: Optional[List[str]] = None,
                                          category_vocab: Optional[List[str]] = None):
        if not self.use_categorical_features:
            return
        if brand_vocab is not None:
            brand_vocab = ["<UNK>"] + sorted(set(brand_vocab))
            self.brand_embedding = nn.Embedding(len(brand_vocab), self.categorical_embedding_dim,
                                                padding_idx=0)
            self.brand_vocab = {b: i for i, b in enumerate(brand_vocab)}
        if category_vocab is not None:
            category_vocab = ["<UNK>"] + sorted(set(category_vocab))
            self.category_embedding = nn.Embedding(len(category_vocab),
                                                   self.categorical_embedding_dim, padding_idx=0)
            self.category_vocab = {c: i for i, c in enumerate(category_vocab)}

    def _device(self):
        return _lib.device()

    # reference :100-124
    def encode_text(self, texts: List[str]) -> torch.Tensor:
        texts = [t if t and len(t.strip()) > 0 else " " for t in texts]
        with torch.no_grad():
            emb = self.text_encoder.encode(texts, convert_to_tensor=True, show_progress_bar=False,
                                           normalize_embeddings=False)
        return emb.to(self._device(), torch.float32)

    # reference :126-172 (ids only; the rows are gathered on the device by tt_item_concat)
    def _categorical_ids(self, brands, categories):
        if not self.use_categorical_features:
            return None
        if self.brand_embedding is None or self.category_embedding is None:
            return None
        bid = [self.brand_vocab.get(b, 0) if b else 0 for b in brands] if brands else None
        cid = [self.category_vocab.get(c, 0) if c else 0 for c in categories] if categories else None
        return bid, cid

    def encode_categorical(self, brands=None, categories=None) -> Optional[torch.Tensor]:
        ids = self._categorical_ids(brands, categories)
        if ids is None:
            return None
        n = len(brands) if brands else len(categories) if categories else 1
        C = self.categorical_embedding_dim
        dev = self._device()
        out = torch.zeros((n, 2 * C), dtype=torch.float32, device=dev)
        if ids[0] is not None:
            out[:, :C] = self.brand_embedding.weight.detach().to(dev)[torch.tensor(ids[0], device=dev)]
        if ids[1] is not None:
            out[:, C:] = self.category_embedding.weight.detach().to(dev)[torch.tensor(ids[1], device=dev)]
        return out

    def head(self, text_emb: torch.Tensor, brand_ids=None, cat_ids=None,
             use_cat: bool = False) -> torch.Tensor:
        """Device path of forward() after the text encoder: concat -> Linear -> ReLU ->
        Linear -> F.normalize, all HIP kernels.  text_emb [B, Ht] f32 device."""
        dev = text_emb.device
        B, Ht = text_emb.shape
        C = self.categorical_embedding_dim if use_cat else 0
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            from .autograd_ops import ItemHeadFn  # training: HIP forward + backward
            from .train import dropout_keep

            l0, l3 = self.projection[0], self.projection[3]
            ids = lambda v: (torch.tensor(v, dtype=torch.int32, device=dev)  # noqa: E731
                             if v is not None else None)
            bt = self.brand_embedding.weight.to(dev) if use_cat else None
            ct = self.category_embedding.weight.to(dev) if use_cat else None
            pdrop = self.projection[2].p if self.training else 0.0
            keep = dropout_keep((text_emb.shape[0], l0.weight.shape[0]), pdrop, dev) \
                if pdrop > 0 else None
            return ItemHeadFn.apply(text_emb, ids(brand_ids) if use_cat else None,
                                    ids(cat_ids) if use_cat else None, bt, ct,
                                    l0.weight.to(dev), l0.bias.to(dev), l3.weight.to(dev),
                                    l3.bias.to(dev), keep, pdrop)
        width = Ht + 2 * C
        l0, l3 = self.projection[0], self.projection[3]
        x = torch.empty((B, width), dtype=torch.float32, device=dev)
        te = text_emb.contiguous()
        if use_cat:
            bt = self.brand_embedding.weight.detach().to(dev, torch.float32).contiguous()
            ct = self.category_embedding.weight.detach().to(dev, torch.float32).contiguous()
            bi, ci = _device_ids(brand_ids, dev), _device_ids(cat_ids, dev)
            check(lib().tt_item_concat(te.data_ptr(), te.stride(0), Ht,
                                       bi.data_ptr() if bi is not None else None,
                                       bt.data_ptr() if bi is not None else None,
                                       ci.data_ptr() if ci is not None else None,
                                       ct.data_ptr() if ci is not None else None, C, B,
                                       x.data_ptr(), x.stride(0), None, stream_ptr()),
                  "tt_item_concat")
        else:
            x.copy_(te)
        w0 = l0.weight.detach().to(dev, torch.float32).contiguous()
        b0 = l0.bias.detach().to(dev, torch.float32).contiguous()
        w3 = l3.weight.detach().to(dev, torch.float32).contiguous()
        b3 = l3.bias.detach().to(dev, torch.float32).contiguous()
        hdim, E = w0.shape[0], w3.shape[0]
        if w0.shape[1] != width:  # what nn.Linear raises (reference H1: no cat init)
            raise RuntimeError(f"mat1 and mat2 shapes cannot be multiplied ({B}x{width} and "
                               f"{w0.shape[1]}x{hdim})")
        h = torch.empty((B, hdim), dtype=torch.float32, device=dev)
        gemm = lib().tt_gemm_x3 if self.head_prec == "x3" else lib().tt_gemm_f32
        check(gemm(x.data_ptr(), x.stride(0), w0.data_ptr(), w0.stride(0), b0.data_ptr(), None, 0,
                   h.data_ptr(), h.stride(0), None, 0, B, hdim, width, _lib.TT_ACT_RELU,
                   stream_ptr()), "projection.0")
        if self.training and self.projection[2].p > 0:  # nn.Dropout (:61) in train mode
            from .train import apply_dropout, dropout_keep

            p = self.projection[2].p
            apply_dropout(h, dropout_keep(h.shape, p, dev), p)
        y = torch.empty((B, E), dtype=torch.float32, device=dev)
        check(gemm(h.data_ptr(), h.stride(0), w3.data_ptr(), w3.stride(0), b3.data_ptr(), None, 0,
                   y.data_ptr(), y.stride(0), None, 0, B, E, hdim, _lib.TT_ACT_NONE,
                   stream_ptr()), "projection.3")
        return kernels.l2norm_rows(y, E, _lib.TT_NORM_MAX_EPS, out=y)

    # reference :174-211
    def forward(self, texts: List[str], brands: Optional[List[str]] = None,
                categories: Optional[List[str]] = None) -> torch.Tensor:
        text_emb = self.encode_text(texts)
        ids = self._categorical_ids(brands, categories) if self.use_categorical_features else None
        if ids is None:
            return self.head(text_emb)  # text only (reference :201-204)
        return self.head(text_emb, ids[0], ids[1], use_cat=True)

    # reference :213-243
    # texts per device call in encode_batch: every output row depends only on its own text
    # (packed varlen encoder, row-wise GEMMs / LayerNorm / pooling), so chunking changes no
    # result -- only how full the GPU is (64 texts ~ 4.6k tokens leave most CUs idle; 4096
    # texts run the encoder's persistent GEMMs at full occupancy).
    device_batch = 4096

    def encode_batch(self, texts: List[str], brands: Optional[List[str]] = None,
                     categories: Optional[List[str]] = None, batch_size: int = 32) -> np.ndarray:
        """item_tower.py:213-243.  ``batch_size`` is honoured as the minimum chunk; chunks of
        ``device_batch`` texts (same results) keep the MI355X busy."""
        self.eval()
        step = max(int(batch_size), int(self.device_batch))
        outs = []
        with torch.no_grad():
            for i in range(0, len(texts), step):
                outs.append(self.forward(texts[i:i + step],
                                         brands[i:i + step] if brands else None,
                                         categories[i:i + step] if categories else None))
        return torch.cat(outs).cpu().numpy()
