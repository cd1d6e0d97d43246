"""EmbeddingEncoder host rules (no GPU) against captures of the REFERENCE encode_buyer
(src/inference/encoder.py:244-305, tests/golden/pipeline.json made by make_pipeline_golden.py):
timestamp sort iff every interaction has one (:263-264), the last max_interaction_history = 100
kept (:267-268), get_event_weight incl. aliases and the default 1 (:273 -> config.py:27-50),
metadata lookups with '' / None for unknown ids (:280-284), categorical lists passed because
use_categorical_features is set (:288-292).  The arithmetic after these rules is the GPU test
tests/test_gpu_pipeline_configs0.py."""
import json
import os

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_encode_buyer_host_rules_match_reference_captures():
    from twotower.encoder import EmbeddingEncoder

    with open(os.path.join(GOLD, "pipeline.json"), encoding="utf-8") as f:
        doc = json.load(f)
    enc = EmbeddingEncoder.__new__(EmbeddingEncoder)  # host state only: no device needed
    enc.config = doc["config"]
    enc.product_metadata = {pid: m for pid, m in doc["metadata"]}
    cases = doc["encode_buyer_cases"]
    assert [len(c["interactions"]) for c in cases] == [5, 3, 130, 120, 3, 1]
    for c in cases:
        pids, weights = enc._history(c["interactions"])
        texts, brands, cats = enc._item_inputs(pids)
        assert weights == c["weights"]
        assert texts == c["texts"]
        assert brands == c["brands"] and cats == c["categories"]
    assert len(cases[2]["weights"]) == 100 and len(cases[3]["weights"]) == 100
    assert cases[4]["texts"][0] == "" and cases[4]["brands"][0] is None
