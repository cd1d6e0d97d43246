"""twotower -- MI355X-native two-tower retrieval hot path.

Mirrors the reference's hot-path classes (HeikalPro/two-tower-model-v2):
  VectorDatabase  <- src/inference/vector_db.py   (FAISS IndexFlatIP -> HIP scan + top-k)
  BuyerTower      <- src/models/buyer_tower.py    (weighted-avg / attention -> HIP kernels)
  load_config, get_event_weight <- src/utils/config.py
The numeric work runs in libtwotower_hip.so (C ABI: include/twotower_hip.h).
"""
from ._lib import HipUnavailable, build  # noqa: F401
from .buyer_tower import BuyerTower  # noqa: F401
from .config import DEFAULT_CONFIG, get_event_weight, load_config  # noqa: F401
from .vector_db import FlatIPIndex, VectorDatabase  # noqa: F401

__version__ = "0.1.0"
