"""Serving path on the GPU index: the reference's RecommendationService
(app/recommendation_service.py:18-109) over this build's training artefacts.

`ProductionTrainer` writes `vocabs.json`, `config.json`, `item_map.json` (reference formats),
`encoder.pt` (Keras-layout state dict) and `faiss.idx` (the L2-normalised item matrix in faiss's
IndexFlatIP file format, faiss_io). `RecommendationService.load` rebuilds the two-tower encoder and a cosine
`BruteForceIndex`; `recommend` runs the user tower (GEMM kernels), normalises (metrics.hip) and
searches (topk.hip); `score` runs both towers and one GEMV (gemm.hip). Result dictionaries keep
the reference's keys (`item_id`, `score`, `rank`), its cold-start list and its errors.
"""
from __future__ import annotations

import json
import logging
from pathlib import Path
from typing import Dict, List, Optional, Sequence

import torch

from . import functional as F
from .config import load_config
from .faiss_io import read_index_flat
from .models import MultiTowerModel
from .retrieval import BruteForceIndex, l2_normalize

logger = logging.getLogger(__name__)


class RecommendationService:
    def __init__(self, model_dir: str = "outputs/models/experiment_001", device=None):
        self.model_dir = Path(model_dir)
        self.version = "1.2.0"
        self.device = device or torch.device("cuda")
        self.user_vocab: List[str] = []
        self.item_map: Dict[str, str] = {}
        self.encoder_model: Optional[MultiTowerModel] = None
        self.faiss_index: Optional[BruteForceIndex] = None
        self._user_set = set()

    def load(self):
        """app/recommendation_service.py:33-61: vocabularies, index + item map, encoder."""
        logger.info(f"Loading model artifacts from {self.model_dir}...")
        if not self.model_dir.exists():
            raise FileNotFoundError(f"Model directory not found: {self.model_dir}")
        with open(self.model_dir / "vocabs.json") as f:
            vocabs = json.load(f)
        self.user_vocab = vocabs["users"]
        self._user_set = set(self.user_vocab)
        with open(self.model_dir / "item_map.json") as f:
            self.item_map = json.load(f)
        item_vocab = vocabs.get("items") or [self.item_map[str(i)] for i in range(len(self.item_map))]
        cfg = load_config(self.model_dir)          # config.json (+ config_ext.json)
        enc = MultiTowerModel(cfg, self.user_vocab, item_vocab, {}, device=self.device)
        state = torch.load(self.model_dir / "encoder.pt", map_location="cpu", weights_only=True)
        enc.load_state_dict(state)
        self.encoder_model = enc
        if (self.model_dir / "faiss.idx").exists():      # app/recommendation_service.py:47
            _, xb = read_index_flat(self.model_dir / "faiss.idx")
            items = torch.from_numpy(xb)
        else:                                              # directories written by round-1 builds
            items = torch.load(self.model_dir / "item_index.pt", map_location="cpu", weights_only=True)
        index = BruteForceIndex(items.shape[1], "cosine", self.device)
        index.set_items(items)   # stored already normalised
        self.faiss_index = index
        logger.info(f"Loaded index with {index.ntotal} items; encoder ready.")

    def is_ready(self) -> bool:
        return all([self.encoder_model is not None, self.faiss_index is not None, self.user_vocab,
                    self.item_map])

    @torch.no_grad()
    def recommend(self, user_id: str, k: int = 10) -> List[Dict]:
        """app/recommendation_service.py:63-81 (unknown users get the cold-start list)."""
        if user_id not in self._user_set:
            logger.warning(f"User '{user_id}' not in vocabulary. Applying cold-start strategy.")
            return self._get_popular_items(k)
        return self.recommend_batch([user_id], k)[0]

    @torch.no_grad()
    def recommend_batch(self, user_ids: Sequence[str], k: int = 10) -> List[List[Dict]]:
        """Batched recommend: one user-tower pass and one top-k search for all known users."""
        known = [u for u in user_ids if u in self._user_set]
        res = {}
        if known:
            emb = self.encoder_model({"user_id": list(known)})["user_embedding"].contiguous()
            scores, idx = self.faiss_index.search(emb, k)
            scores, idx = scores.cpu().tolist(), idx.cpu().tolist()
            for j, u in enumerate(known):
                res[u] = [{"item_id": self.item_map[str(i)], "score": float(s), "rank": r + 1}
                          for r, (s, i) in enumerate(zip(scores[j], idx[j])) if i != -1]
        return [res[u] if u in res else self._get_popular_items(k) for u in user_ids]

    @torch.no_grad()
    def score(self, user_id: str, item_ids: List[str]) -> Dict[str, float]:
        """app/recommendation_service.py:83-93: item_embeddings . user_embedding (raw inner product)."""
        if user_id not in self._user_set:
            raise ValueError(f"User '{user_id}' not found in vocabulary.")
        out = self.encoder_model({"user_id": [user_id], "movie_id": list(item_ids)})
        u = out["user_embedding"].contiguous()
        c = out["item_embedding"].contiguous()
        s = F.gemm(c, u, trans_b=True)   # [n, D] x [1, D]^T -> [n, 1]
        return {item: float(v) for item, v in zip(item_ids, s[:, 0].cpu().tolist())}

    def _get_popular_items(self, k: int) -> List[Dict]:
        """app/recommendation_service.py:95-103 (the first k catalogue items, descending scores)."""
        return [{"item_id": self.item_map[str(i)], "score": 1.0 - (i * 0.05), "rank": i + 1}
                for i in range(min(k, len(self.item_map)))]

    def get_model_info(self) -> Dict:
        return {
            "version": self.version,
            "model_path": str(self.model_dir),
            "num_users": len(self.user_vocab),
            "faiss_index_items": self.faiss_index.ntotal if self.faiss_index else 0,
        }


__all__ = ["RecommendationService", "l2_normalize"]
