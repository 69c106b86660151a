"""Host-side string-id vocabulary and StringLookup.

Reference: vocab = sorted(train_df[col].unique().tolist()) on string ids (src/trainer.py:81-82;
ids are cast with .astype(str) at src/data_processing.py:77-78 and src/trainer.py:109-110) and
keras.layers.StringLookup(vocabulary=vocab, mask_token=None) (src/models.py:70,73): index =
1 + position in the vocabulary, out-of-vocabulary -> 0 (one OOV bucket, Keras default).

TF runs StringLookup per batch on the host inside the fit loop; here the mapping is a
vectorised numpy searchsorted over the sorted vocabulary, done ONCE per dataset, and the
device only ever sees int64 row ids.
"""
from __future__ import annotations

from typing import Iterable, List, Sequence

import numpy as np


def build_vocab(values: Iterable) -> List[str]:
    """sorted(unique(str(v))) — Python string order, e.g. ['0', '1', '10', '100', ...]."""
    arr = np.asarray(list(values) if not isinstance(values, np.ndarray) else values)
    return sorted(set(np.asarray(arr).astype(str).tolist()))


def _as_str_array(values) -> np.ndarray:
    if isinstance(values, np.ndarray) and values.dtype.kind == "U":
        return values
    return np.asarray(values).astype(str)


class StringLookup:
    """keras.layers.StringLookup(vocabulary=vocab, mask_token=None) on the host."""

    def __init__(self, vocabulary: Sequence[str]):
        self.vocabulary = list(vocabulary)
        voc = _as_str_array(self.vocabulary) if len(self.vocabulary) else np.asarray([], dtype="<U1")
        if len(set(voc.tolist())) != len(voc):
            raise ValueError("StringLookup vocabulary contains duplicate entries")
        self._order = np.argsort(voc, kind="stable")
        self._sorted = voc[self._order]

    def vocabulary_size(self) -> int:
        return len(self.vocabulary) + 1  # + the OOV bucket at index 0

    def __call__(self, values) -> np.ndarray:
        x = _as_str_array(values)
        if self._sorted.size == 0:
            return np.zeros(x.shape, dtype=np.int64)
        pos = np.searchsorted(self._sorted, x)
        pos_c = np.minimum(pos, self._sorted.size - 1)
        found = (pos < self._sorted.size) & (self._sorted[pos_c] == x)
        return np.where(found, self._order[pos_c] + 1, 0).astype(np.int64)
