"""Ranking-metric suite on the GPU.

`AdvancedMetrics` keeps the reference's static API (src/evaluation.py:22-104: recall_at_k,
precision_at_k, ndcg_at_k, map_at_k, mrr, coverage, diversity over Python lists of item ids,
strings or ints) and adds `evaluate`, the device fast path over an int64 [U, K] top-K tensor
(what `BruteForceIndex.search` returns). Every metric is computed by one rs_rank_metrics_i64
call (metrics.hip): host work is only the string -> int mapping of list inputs, as the
StringLookup layer does for the model.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import torch

from . import functional as F

_PAD = -3      # list padding (never read: per-list lengths are passed)
_UNKNOWN = -2  # a true item absent from every list


def _encode(predictions: Sequence[Sequence], truths: Optional[Sequence] = None, device=None):
    ids: Dict = {}
    rows = []
    for lst in predictions:
        rows.append([ids.setdefault(v, len(ids)) for v in lst])
    U = len(rows)
    K = max([len(r) for r in rows] + [1])
    pred = torch.full((U, K), _PAD, dtype=torch.int64)
    for u, r in enumerate(rows):
        if r:
            pred[u, :len(r)] = torch.tensor(r, dtype=torch.int64)
    lens = torch.tensor([len(r) for r in rows], dtype=torch.int32)
    truth = torch.tensor([ids.get(t, _UNKNOWN) for t in truths] if truths is not None else [_UNKNOWN] * U,
                         dtype=torch.int64)
    dev = device or torch.device("cuda")
    return pred.to(dev), lens.to(dev), truth.to(dev), len(ids)


class AdvancedMetrics:
    """Drop-in for src/evaluation.py:AdvancedMetrics; all arithmetic runs in metrics.hip."""

    @staticmethod
    def evaluate(pred_rows: torch.Tensor, true_rows: torch.Tensor, ks: Sequence[int], n_items: int,
                 lens: Optional[torch.Tensor] = None) -> Dict[str, float]:
        """Device fast path: pred_rows int64 [U, K] item rows, true_rows int64 [U] (negative =
        unknown), n_items = catalogue size for coverage."""
        ks = list(ks)
        m = F.rank_metrics(pred_rows.contiguous(), true_rows.contiguous(), ks, n_items, lens).cpu().tolist()
        out = {}
        for j, k in enumerate(ks):
            out[f"recall@{k}"], out[f"precision@{k}"], out[f"ndcg@{k}"], out[f"map@{k}"] = m[4 * j:4 * j + 4]
        out["mrr"], out["diversity"], out["coverage"] = m[4 * len(ks):]
        return out

    @staticmethod
    def _suite(predictions, ground_truth, ks):
        if len(predictions) == 0:
            return [0.0] * (4 * len(ks) + 3)
        pred, lens, truth, n = _encode(predictions, ground_truth)
        return F.rank_metrics(pred, truth, list(ks), n, lens).cpu().tolist()

    @staticmethod
    def recall_at_k(predictions: List[List], ground_truth: List, k: int) -> float:
        return AdvancedMetrics._suite(predictions, ground_truth, [k])[0]

    @staticmethod
    def precision_at_k(predictions: List[List], ground_truth: List, k: int) -> float:
        return AdvancedMetrics._suite(predictions, ground_truth, [k])[1]

    @staticmethod
    def ndcg_at_k(predictions: List[List], ground_truth: List, k: int) -> float:
        return AdvancedMetrics._suite(predictions, ground_truth, [k])[2]

    @staticmethod
    def map_at_k(predictions: List[List], ground_truth: List, k: int) -> float:
        return AdvancedMetrics._suite(predictions, ground_truth, [k])[3]

    @staticmethod
    def mrr(predictions: List[List], ground_truth: List) -> float:
        return AdvancedMetrics._suite(predictions, ground_truth, [1])[4]

    @staticmethod
    def diversity(recommendations: List[List]) -> float:
        return AdvancedMetrics._suite(recommendations, None, [1])[5]

    @staticmethod
    def coverage(recommendations: List[List], all_items: List) -> float:
        """|union of the lists| / len(all_items) (the union may hold items outside all_items, as
        in the reference)."""
        if not all_items:
            return 0.0
        if len(recommendations) == 0:
            return 0.0
        pred, lens, truth, n = _encode(recommendations)
        frac = F.rank_metrics(pred, truth, [1], n, lens).cpu().tolist()[6]
        return round(frac * n) / len(all_items)
