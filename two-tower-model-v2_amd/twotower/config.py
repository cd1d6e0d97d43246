"""Config helpers, same behaviour as reference src/utils/config.py.

``get_event_weight`` produces the buyer-tower weights on the hot path
(src/inference/encoder.py:273 -> src/utils/config.py:27-50).
"""
from __future__ import annotations

from pathlib import Path
from typing import Any, Dict

import yaml


def load_config(config_path: str = "configs/config.yaml") -> Dict[str, Any]:
    """reference src/utils/config.py:8-24"""
    config_path = Path(config_path)
    if not config_path.exists():
        raise FileNotFoundError(f"Configuration file not found: {config_path}")
    with open(config_path, "r", encoding="utf-8") as f:
        return yaml.safe_load(f)


_EVENT_ALIASES = {
    "view": "view",
    "addtocart": "add_to_cart",
    "add_to_cart": "add_to_cart",
    "purchase": "purchase",
    "buy": "purchase",
}


def get_event_weight(event_name: str, config: Dict[str, Any]) -> int:
    """reference src/utils/config.py:27-50: lower-case, alias, default weight 1."""
    event_weights = config.get("event_weights", {})
    name = event_name.lower()
    return event_weights.get(_EVENT_ALIASES.get(name, name), 1)


# The reference's shipped configuration (configs/config.yaml), used when no file is given.
DEFAULT_CONFIG: Dict[str, Any] = {
    "model": {
        "embedding_dim": 384,
        "item_tower": {
            "text_encoder": "paraphrase-multilingual-MiniLM-L12-v2",
            "use_categorical_features": True,
            "categorical_embedding_dim": 64,
            "projection_hidden_dim": 256,
        },
        "buyer_tower": {
            "aggregation_method": "attention",
            "attention_hidden_dim": 128,
            "max_interaction_history": 100,
        },
    },
    "training": {
        "batch_size": 512, "learning_rate": 0.001, "num_epochs": 3, "temperature": 0.07,
        "num_negatives": 4, "validation_split": 0.1, "checkpoint_dir": "checkpoints",
        "save_every_n_epochs": 2, "freeze_text_encoder": True,
    },
    "event_weights": {"view": 1, "add_to_cart": 5, "purchase": 10},
    "inference": {
        "embeddings_dir": "outputs/embeddings", "index_dir": "outputs/index",
        "model_checkpoint": "checkpoints/best_model.pt", "device": "cuda",
    },
}
