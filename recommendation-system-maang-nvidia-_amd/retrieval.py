"""Exact brute-force retrieval on the GPU top-K kernel.

Replaces, with one kernel family (rs_topk_ip_f32 / rs_topk_merge_f32):
  * ProductionTrainer._evaluate's np.dot(user_embs, item_embs.T) + np.argpartition
    (src/trainer.py:204-212) — raw inner product;
  * faiss.normalize_L2 + IndexFlatIP.add/search of _build_faiss and the serving
    RecommendationService (src/trainer.py:240-243, app/recommendation_service.py:71-72) —
    cosine = inner product of L2-normalised rows.
Results are ordered by (-score, index) (the build's deterministic contract).

ShardedBruteForceIndex row-shards the item table over the ranks of a process group (BASELINE
config 4: 100M items over 8 GPUs): each rank scans its rows with its global row offset, the
per-rank top-k lists are all-gathered (Q x k x (fp32 + int64) per rank) and merged on device.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.distributed as dist

from . import functional as F


def l2_normalize(x: torch.Tensor) -> torch.Tensor:
    """faiss.normalize_L2 (rows scaled to unit norm; zero rows stay zero) on the GPU kernel."""
    return F.l2_normalize_rows(x.contiguous())


class BruteForceIndex:
    """IndexFlatIP-equivalent on one GPU (metric 'ip' or 'cosine'). `precision` = the scan's
    contraction precision (functional.PREC_*; the split kernels serve > 64 queries at D = 128)."""

    def __init__(self, dim: int, metric: str = "ip", device=None, precision: int = 6):
        if metric not in ("ip", "cosine"):
            raise ValueError("metric must be 'ip' or 'cosine'")
        self.dim = dim
        self.metric = metric
        self.precision = precision
        self.device = device or torch.device("cuda")
        self.items = torch.empty((0, dim), dtype=torch.float32, device=self.device)

    @property
    def ntotal(self) -> int:
        return self.items.shape[0]

    def add(self, embs) -> None:
        x = torch.as_tensor(embs, dtype=torch.float32).to(self.device).contiguous()
        if self.metric == "cosine":
            x = l2_normalize(x)
        self.items = torch.cat([self.items, x]).contiguous()
        Dp = F._kernel_dim(self.dim)
        self._padded = F._pad_cols(self.items, Dp) if Dp != self.dim else None   # kernel width, once

    def set_items(self, items: torch.Tensor) -> None:
        """Install an already-prepared item matrix (e.g. the saved, normalised faiss.idx matrix)."""
        self.items = items.to(self.device, dtype=torch.float32).contiguous()
        Dp = F._kernel_dim(self.dim)
        self._padded = F._pad_cols(self.items, Dp) if Dp != self.dim else None

    def search(self, queries, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
        q = torch.as_tensor(queries, dtype=torch.float32).to(self.device).contiguous()
        if self.metric == "cosine":
            q = l2_normalize(q)
        k = min(int(k), self.ntotal)
        items = self.items if getattr(self, "_padded", None) is None else self._padded
        return F.topk_ip(q, items, k, precision=self.precision)


def shard_rows(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Rows [r0, r1) of an n-row table held by `rank` of `world` (contiguous, near-equal)."""
    per = -(-n // world) if world > 0 else n
    r0 = min(rank * per, n)
    return r0, min(r0 + per, n)


class ShardedBruteForceIndex:
    """Row-sharded exact top-k: this rank holds rows [row_offset, row_offset + n_local).
    ntotal: the rows of all shards (summed over the group when not given). A shard with fewer
    than k rows (or none) contributes its rows padded with (-inf, -1) entries, which the merge
    orders last."""

    def __init__(self, local_items: torch.Tensor, row_offset: int, metric: str = "ip", group=None,
                 precision: int = 6, ntotal: Optional[int] = None):
        self.local = BruteForceIndex(local_items.shape[1], metric, local_items.device, precision)
        if local_items.shape[0]:
            self.local.add(local_items)
        self.row_offset = int(row_offset)
        self.group = group
        if ntotal is None:
            ntotal = self.local.ntotal
            if dist.is_initialized() and dist.get_world_size(self.group) > 1:
                dev = self.local.device if dist.get_backend(self.group) == "nccl" else "cpu"
                t = torch.tensor([ntotal], dtype=torch.int64, device=dev)
                dist.all_reduce(t, group=self.group)
                ntotal = int(t.item())
        self.ntotal = int(ntotal)

    def search(self, queries, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
        q = torch.as_tensor(queries, dtype=torch.float32).to(self.local.device).contiguous()
        if self.local.metric == "cosine":
            q = l2_normalize(q)
        k = min(int(k), self.ntotal)
        n_local = self.local.ntotal
        kl = min(k, n_local)
        if kl > 0:
            items = self.local.items if getattr(self.local, "_padded", None) is None else self.local._padded
            s, i = F.topk_ip(q, items, kl, index_base=self.row_offset, precision=self.local.precision)
        else:
            s = torch.empty((q.shape[0], 0), dtype=torch.float32, device=q.device)
            i = torch.empty((q.shape[0], 0), dtype=torch.int64, device=q.device)
        if kl < k:   # (-inf, -1) pads: every shard's list has k entries for the all-gather
            s = torch.cat([s, torch.full((q.shape[0], k - kl), float("-inf"), device=q.device)], 1).contiguous()
            i = torch.cat([i, torch.full((q.shape[0], k - kl), -1, dtype=torch.int64, device=q.device)], 1).contiguous()
        if not dist.is_initialized() or dist.get_world_size(self.group) == 1:
            return s, i
        world = dist.get_world_size(self.group)
        gs = [torch.empty_like(s) for _ in range(world)]
        gi = [torch.empty_like(i) for _ in range(world)]
        dist.all_gather(gs, s, group=self.group)
        dist.all_gather(gi, i, group=self.group)
        return F.topk_merge(torch.stack(gs, 1).contiguous(), torch.stack(gi, 1).contiguous(), k)


def recall_at_k(index_or_items, user_embs: torch.Tensor, true_rows, ks) -> dict:
    """recall@k of ProductionTrainer._evaluate (src/trainer.py:206-213): 1 if the true item's row
    is among the top-k rows of the raw inner-product scores."""
    kmax = max(ks)
    if isinstance(index_or_items, torch.Tensor):
        _, idx = F.topk_ip(user_embs.contiguous(), index_or_items.contiguous(), min(kmax, index_or_items.shape[0]))
    else:
        _, idx = index_or_items.search(user_embs, kmax)
    true = torch.as_tensor(true_rows, dtype=torch.int64, device=idx.device).view(-1).contiguous()
    true = torch.where(true < 0, torch.full_like(true, -2), true)  # unknown items never match a -1 pad
    n_items = index_or_items.shape[0] if isinstance(index_or_items, torch.Tensor) else index_or_items.ntotal
    m = F.rank_metrics(idx.contiguous(), true, list(ks), n_items).cpu()
    return {f"recall@{k}": float(m[4 * j]) for j, k in enumerate(ks)}
