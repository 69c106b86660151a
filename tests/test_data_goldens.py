"""Data-side parity, pinned by fixtures generated from the reference's own modules
(tests/golden/make_data_goldens.py runs src/preprocessing.py + src/data_processing.py +
src/config.py): vocab order, StringLookup ids, labels, class weights, config defaults, and the
evaluation's validation sample."""
import json
import os

import numpy as np
import pandas as pd
import pytest

from conftest import oracle, pkg

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def g():
    return dict(np.load(os.path.join(GOLD, "data_goldens.npz"), allow_pickle=False))


def frames(g):
    train = pd.DataFrame({"user_id": g["train_user_id"], "movie_id": g["train_movie_id"],
                          "rating": g["train_rating"], "y_implicit": g["train_y_implicit"]})
    val = pd.DataFrame({"user_id": g["val_user_id"], "movie_id": g["val_movie_id"],
                        "rating": g["val_rating"], "y_implicit": g["val_y_implicit"]})
    return train, val


def test_vocab_is_lexicographic_string_order(g):
    lookup = pkg("lookup")
    train, _ = frames(g)
    tr = pkg("trainer").normalize_columns(train)
    assert lookup.build_vocab(tr["user_id"].unique()) == g["user_vocab"].tolist()
    assert lookup.build_vocab(tr["movie_id"].unique()) == g["item_vocab"].tolist()
    assert g["user_vocab"].tolist()[:3] == sorted(g["user_vocab"].tolist())[:3]


def test_string_lookup_ids_match_reference(g):
    lookup = pkg("lookup")
    train, val = frames(g)
    ul = lookup.StringLookup(g["user_vocab"].tolist())
    il = lookup.StringLookup(g["item_vocab"].tolist())
    assert np.array_equal(ul(train["user_id"].astype(str).values), g["train_uid"])
    assert np.array_equal(il(train["movie_id"].astype(str).values), g["train_iid"])
    # validation contains cold-start ids -> OOV bucket 0
    assert np.array_equal(ul(val["user_id"].astype(str).values), g["val_uid"])
    assert np.array_equal(il(val["movie_id"].astype(str).values), g["val_iid"])
    assert (g["val_uid"] == 0).any() or (g["val_iid"] == 0).any()
    # the oracle's restatement agrees too
    O = oracle()
    assert np.array_equal(O.string_lookup(g["user_vocab"].tolist(), train["user_id"].values), g["train_uid"])


def test_labels_and_class_weights(g):
    tr = pkg("trainer")
    data = pkg("data")
    train, _ = frames(g)
    rating, yi = data.split_labels(train)
    assert np.array_equal(rating, g["train_rating"])
    assert np.array_equal(yi, g["train_y_implicit"])
    cw = tr.balanced_class_weights(yi)
    assert np.allclose([cw[0], cw[1]], g["class_weights"], rtol=0, atol=1e-12)
    O = oracle()
    ocw = O.balanced_class_weights(yi)
    assert np.allclose([ocw[0], ocw[1]], g["class_weights"], rtol=0, atol=1e-12)


def test_y_implicit_fallback_is_rating_ge_3():
    data = pkg("data")
    df = pd.DataFrame({"user_id": [1, 2, 3], "movie_id": [4, 5, 6], "rating": [2.0, 3.0, 5.0]})
    _, yi = data.split_labels(df)
    assert yi.tolist() == [0.0, 1.0, 1.0]          # src/trainer.py:105-106 (>= 3.0, not 4)


def test_validation_sample_matches_reference(g):
    _, val = frames(g)
    idx = val.sample(n=min(1000, len(val)), random_state=42).index.values
    assert np.array_equal(idx, g["val_sample_index"])


def test_model_config_defaults_match_reference():
    cfg = pkg("config").ModelConfig()
    ref = json.load(open(os.path.join(GOLD, "config_defaults.json")))
    mine = cfg.to_dict()
    for k, v in ref.items():
        assert mine[k] == v, k
    # build-only extensions are appended after the reference fields
    assert set(mine) - set(ref) == {"ctr_loss_mode", "clipnorm", "contraction_precision", "early_stopping_restore"}
    # round trip through to_dict like config.json
    assert pkg("config").ModelConfig(**ref).to_dict()["cross_layers"] == 3


def test_normalize_columns_aliases_and_errors():
    tr = pkg("trainer")
    df = pd.DataFrame({"UserID": [1, 2], "MovieID": [3, 4], "rating": [5, 4]})
    out = tr.normalize_columns(df)
    assert out["user_id"].tolist() == ["1", "2"] and out["movie_id"].tolist() == ["3", "4"]
    with pytest.raises(ValueError):
        tr.normalize_columns(pd.DataFrame({"u": [1], "movie_id": [2]}))
