"""Generate the data-side golden fixtures by RUNNING the reference's importable modules.

Run once in the build container (it reads /root/reference; the GPU box never does):
    python tests/golden/make_data_goldens.py

What it pins: vocabulary order, StringLookup indices,
rating / y_implicit labels, balanced class weights, and ModelConfig defaults, exactly as the
reference's own src/preprocessing.py + src/data_processing.py + src/config.py produce them.
src/models.py / src/trainer.py cannot be imported here (TensorFlow is absent), so the
trainer-side steps are restated with the reference expressions quoted in comments:
  vocab = sorted(train_df[col].unique().tolist())                       (src/trainer.py:81-82)
  StringLookup(vocabulary=vocab, mask_token=None): index = 1 + position (src/models.py:70,73)
  labels rating / y_implicit as float32                                 (src/trainer.py:99-106)
  compute_class_weight('balanced', classes=[0, 1], y=y_implicit)        (src/trainer.py:139-145)

Inputs: the reference's real data/raw/movies.dat and users.dat plus a seeded synthetic
ratings table (ratings.dat is not shipped: SURVEY §0 item 10). Only data (inputs and outputs)
is written to data_goldens.npz / config_defaults.json — no reference source.
"""
import importlib
import json
import os
import sys
import types

import numpy as np
import pandas as pd

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def import_reference():
    # package shim so src/__init__.py (which imports TF via trainer) is not executed
    pkg = types.ModuleType("refsrc")
    pkg.__path__ = [os.path.join(REF, "src")]
    sys.modules["refsrc"] = pkg
    return (importlib.import_module("refsrc.config"), importlib.import_module("refsrc.preprocessing"),
            importlib.import_module("refsrc.data_processing"))


def synthetic_ratings(movies, users, n=20000, seed=0):
    rng = np.random.default_rng(seed)
    uids = users["user_id"].values
    mids = movies["movie_id"].values
    # skewed popularity, ML-1M-like rating marginal, timestamps over 2000-04-25 .. 2003-02-28
    u = uids[np.minimum(rng.zipf(1.3, n) - 1, len(uids) - 1)]
    u[: len(uids)] = rng.permutation(uids)   # every user rates at least once (users.to_dict needs it)
    m = mids[np.minimum(rng.zipf(1.2, n) - 1, len(mids) - 1)]
    r = rng.choice([1, 2, 3, 4, 5], size=n, p=[0.056, 0.108, 0.261, 0.349, 0.226])
    t = rng.integers(956703932, 1046454590, size=n)
    return pd.DataFrame({"user_id": u, "movie_id": m, "rating": r, "timestamp": t})


def main():
    cfgmod, prep, dp = import_reference()
    raw = os.path.join(REF, "data", "raw")
    movies = pd.read_csv(os.path.join(raw, "movies.dat"), sep="::", header=None,
                         names=["movie_id", "title", "genres"], engine="python", encoding="latin-1")
    users = pd.read_csv(os.path.join(raw, "users.dat"), sep="::", header=None,
                        names=["user_id", "gender", "age", "occupation", "zip-code"], engine="python")
    ratings = synthetic_ratings(movies, users)
    inputs = ratings.copy()

    processed = prep.preprocessing_pipeline(ratings, movies.copy(), users.copy())
    config = cfgmod.ModelConfig()
    proc = dp.DataProcessor(config)
    data = {"train_ratings": processed["train_ratings"], "val_ratings": processed["val_ratings"],
            "test_ratings": processed["test_ratings"], "user_features": processed["user_features"],
            "movie_features": processed["movie_features"]}
    # load_and_validate_data's dict branch (features dicts become empty frames)
    user_features = data["user_features"] if isinstance(data["user_features"], pd.DataFrame) else pd.DataFrame()
    item_features = data["movie_features"] if isinstance(data["movie_features"], pd.DataFrame) else pd.DataFrame()
    train_df = proc.engineer_features(data["train_ratings"], user_features, item_features, "train")
    val_df = proc.engineer_features(data["val_ratings"], user_features, item_features, "val")

    user_vocab = sorted(train_df["user_id"].unique().tolist())     # src/trainer.py:81
    item_vocab = sorted(train_df["movie_id"].unique().tolist())     # src/trainer.py:82
    uindex = {s: i + 1 for i, s in enumerate(user_vocab)}
    iindex = {s: i + 1 for i, s in enumerate(item_vocab)}

    def lookup(df):
        return (np.array([uindex.get(s, 0) for s in df["user_id"].astype(str).values], np.int64),
                np.array([iindex.get(s, 0) for s in df["movie_id"].astype(str).values], np.int64))

    tr_u, tr_i = lookup(train_df)
    va_u, va_i = lookup(val_df)
    from sklearn.utils.class_weight import compute_class_weight
    cw = compute_class_weight("balanced", classes=np.array([0, 1]), y=train_df["y_implicit"].values)

    np.savez_compressed(
        os.path.join(HERE, "data_goldens.npz"),
        in_user_id=inputs["user_id"].values.astype(np.int64),
        in_movie_id=inputs["movie_id"].values.astype(np.int64),
        in_rating=inputs["rating"].values.astype(np.int64),
        in_timestamp=inputs["timestamp"].values.astype(np.int64),
        # preprocessing_pipeline outputs (remapped ids, temporal split)
        train_user_id=data["train_ratings"]["user_id"].values.astype(np.int64),
        train_movie_id=data["train_ratings"]["movie_id"].values.astype(np.int64),
        val_user_id=data["val_ratings"]["user_id"].values.astype(np.int64),
        val_movie_id=data["val_ratings"]["movie_id"].values.astype(np.int64),
        # what reaches the model
        user_vocab=np.array(user_vocab), item_vocab=np.array(item_vocab),
        train_uid=tr_u, train_iid=tr_i, val_uid=va_u, val_iid=va_i,
        train_rating=train_df["rating"].astype(np.float32).values,
        train_y_implicit=train_df["y_implicit"].astype(np.float32).values,
        val_rating=val_df["rating"].astype(np.float32).values,
        val_y_implicit=val_df["y_implicit"].astype(np.float32).values,
        class_weights=np.asarray(cw, np.float64),
        val_sample_index=val_df.sample(n=min(1000, len(val_df)), random_state=42).index.values.astype(np.int64),
    )
    with open(os.path.join(HERE, "config_defaults.json"), "w") as f:
        json.dump(config.to_dict(), f, indent=2, sort_keys=True)
    print("wrote", os.path.join(HERE, "data_goldens.npz"), len(train_df), "train rows,",
          len(user_vocab), "users,", len(item_vocab), "items")


if __name__ == "__main__":
    main()
