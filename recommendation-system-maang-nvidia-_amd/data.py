"""Input pipeline of the trainer (§8f row 2).

Reference (src/trainer.py:95-117, make_ds): features = {'user_id', 'movie_id'} as strings,
labels = {'rating' (fp32), 'y_implicit' (fp32; column if present, else rating >= 3.0)},
shuffle(50000) for training, batch(B) keeping the partial last batch, prefetch.

Here the StringLookup runs ONCE over the whole split (vectorised, lookup.StringLookup) and the
int64 ids + fp32 labels live in HBM for the whole run; an epoch is a device-side permutation
(seeded, identical on every data-parallel rank) sliced into batches. Under data parallelism
each rank takes its contiguous 1/N of every global batch, as MirroredStrategy splits a batch
across replicas. The epoch order is tf.data's shuffle-buffer process with the reference's
buffer of 50,000 (``rs_shuffle_buffer_order_i64``: output i comes from inputs < i + 50000, a
fresh order every epoch); the reference leaves that shuffle unseeded, so the window, not a
particular order, is what is kept (seeded here by (seed, epoch) so every rank agrees).
``shuffle_buffer=None`` gives a full permutation instead.
"""
from __future__ import annotations

import ctypes
from typing import Dict, Iterator, Optional, Tuple

import numpy as np
import torch

from . import _native
from .lookup import StringLookup


SHUFFLE_BUFFER = 50000  # ds.shuffle(50000), src/trainer.py:116


def shuffle_buffer_order(n: int, buffer_size: int, seed: int = 0, epoch: int = 0) -> torch.Tensor:
    """One epoch's element order under tf.data's shuffle buffer (include/recsys_hip.h
    rs_shuffle_buffer_order_i64; host int64 tensor of n indices)."""
    out = torch.empty(int(n), dtype=torch.int64)
    _native.call("rs_shuffle_buffer_order_i64", int(n), int(buffer_size), int(seed) & (2 ** 64 - 1),
                 int(epoch) & (2 ** 64 - 1), ctypes.c_void_p(out.data_ptr() if n else 0))
    return out


class InMemoryDataset:
    """Device-resident (ids, labels) of one split; iterates ({'user_id','movie_id'}, labels)."""

    def __init__(self, user_ids: np.ndarray, item_ids: np.ndarray, rating: Optional[np.ndarray],
                 y_implicit: Optional[np.ndarray], batch_size: int, device, shuffle: bool = False,
                 seed: int = 0, rank: int = 0, world: int = 1,
                 shuffle_buffer: Optional[int] = SHUFFLE_BUFFER):
        self.n = int(len(user_ids))
        self.shuffle_buffer = shuffle_buffer
        self.batch_size = int(batch_size)
        self.device = device
        self.shuffle = shuffle
        self.seed = seed
        self.rank, self.world = rank, world
        self.epoch = 0
        self.uid = torch.as_tensor(np.asarray(user_ids, np.int64)).to(device)
        self.iid = torch.as_tensor(np.asarray(item_ids, np.int64)).to(device)
        self.labels: Dict[str, torch.Tensor] = {}
        if rating is not None:
            self.labels["rating"] = torch.as_tensor(np.asarray(rating, np.float32)).to(device)
        if y_implicit is not None:
            self.labels["y_implicit"] = torch.as_tensor(np.asarray(y_implicit, np.float32)).to(device)

    def __len__(self) -> int:
        return (self.n + self.batch_size - 1) // self.batch_size

    def _order(self):
        if not self.shuffle:
            return None
        if self.shuffle_buffer is None:
            g = torch.Generator(device="cpu")
            g.manual_seed(self.seed * 1_000_003 + self.epoch)
            return torch.randperm(self.n, generator=g).to(self.device)
        return shuffle_buffer_order(self.n, self.shuffle_buffer, self.seed, self.epoch).to(self.device)

    def __iter__(self) -> Iterator[Tuple[dict, dict]]:
        order = self._order()
        self.epoch += 1
        for b0 in range(0, self.n, self.batch_size):
            b1 = min(self.n, b0 + self.batch_size)
            # this rank's contiguous share of the global batch (MirroredStrategy split)
            per = (b1 - b0 + self.world - 1) // self.world
            s0 = min(b1, b0 + self.rank * per)
            s1 = min(b1, s0 + per)
            if s1 <= s0:
                continue
            if order is None:
                sl = slice(s0, s1)
                feats = {"user_id": self.uid[sl], "movie_id": self.iid[sl]}
                labs = {k: v[sl] for k, v in self.labels.items()}
            else:
                idx = order[s0:s1]
                feats = {"user_id": self.uid[idx], "movie_id": self.iid[idx]}
                labs = {k: v[idx] for k, v in self.labels.items()}
            yield feats, labs


def split_labels(df):
    """src/trainer.py:99-106: rating fp32; y_implicit from its column, else rating >= 3.0."""
    rating = df["rating"].astype(np.float32).values if "rating" in df.columns else None
    if "y_implicit" in df.columns:
        yi = df["y_implicit"].astype(np.float32).values
    elif rating is not None:
        yi = (df["rating"] >= 3.0).astype(np.float32).values
    else:
        yi = None
    return rating, yi


def make_dataset(df, user_lookup: StringLookup, item_lookup: StringLookup, batch_size: int, device,
                 training: bool = False, seed: int = 0, rank: int = 0, world: int = 1):
    """src/trainer.py:95-117 (make_ds) on device-resident tensors."""
    if df is None or len(df) == 0:
        return None
    uid = user_lookup(df["user_id"].astype(str).values)
    iid = item_lookup(df["movie_id"].astype(str).values)
    rating, yi = split_labels(df)
    return InMemoryDataset(uid, iid, rating, yi, batch_size, device, shuffle=training, seed=seed,
                           rank=rank, world=world)
