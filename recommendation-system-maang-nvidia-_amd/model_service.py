"""Second serving variant of the reference on the GPU index: the
RecommendationService of app/model_service.py:20-249 — raw inner product against precomputed
item-tower embeddings, no normalisation, no FAISS.

Differences from serving.py (app/recommendation_service.py), kept as the reference has them:
  * the full trained model is loaded (best_model.keras there, the trainer's best_model.pt
    here) and the item tower is run over the whole item vocabulary once, in chunks of 512
    (_precompute_item_embeddings, :71-91);
  * recommend scores `item_embeddings . user_embedding` (:137) and orders by descending score
    (argpartition + argsort, :140-141; this build breaks ties by ascending item row);
  * recommend_batch returns {"user_id", "recommendations", "status"[, "error"]} per user
    (:200-227); the cold-start list scores 1/rank (:229-239);
  * score drops item ids outside the vocabulary and raises if none is left (:172-175).
Every score is one GEMM/top-k kernel launch (gemm.hip, topk.hip); the host only maps strings.
"""
from __future__ import annotations

import json
import logging
from pathlib import Path
from typing import Dict, List, Optional

import torch

from . import functional as F
from .config import load_config
from .models import MultiTowerModel

logger = logging.getLogger(__name__)

_CHUNK = 512   # app/model_service.py:75


class RecommendationService:
    def __init__(self, model_dir: str = "outputs/models/experiment_001", device=None):
        self.model_dir = Path(model_dir)
        self.device = device or torch.device("cuda")
        self.model: Optional[MultiTowerModel] = None
        self.user_vocab: Optional[List[str]] = None
        self.item_vocab: Optional[List[str]] = None
        self.item_embeddings: Optional[torch.Tensor] = None
        self.config: Optional[Dict] = None
        self.version = "1.0.0"
        self._user_set = set()
        self._item_row: Dict[str, int] = {}

    def load_model(self):
        """app/model_service.py:32-69 (model, vocabs.json, config.json, item embeddings)."""
        logger.info(f"Loading model from {self.model_dir}")
        model_path = self.model_dir / "best_model.pt"
        if not model_path.exists():
            raise FileNotFoundError(f"Model not found at {model_path}")
        vocab_path = self.model_dir / "vocabs.json"
        if not vocab_path.exists():
            raise FileNotFoundError(f"Vocabularies not found at {vocab_path}")
        with open(vocab_path) as f:
            vocabs = json.load(f)
        self.user_vocab, self.item_vocab = vocabs["users"], vocabs["items"]
        self._user_set = set(self.user_vocab)
        self._item_row = {s: i for i, s in enumerate(self.item_vocab)}
        cfg = load_config(self.model_dir)          # config.json (+ config_ext.json)
        if (self.model_dir / "config.json").exists():
            with open(self.model_dir / "config.json") as f:
                self.config = json.load(f)
        state = torch.load(model_path, map_location="cpu", weights_only=True)
        enc_state = {k[len("encoder."):]: v for k, v in state.items() if k.startswith("encoder.")}
        if not enc_state:
            raise ValueError(f"{model_path} holds no encoder weights")
        enc = MultiTowerModel(cfg, self.user_vocab, self.item_vocab, {}, device=self.device)
        enc.load_state_dict(enc_state)
        self.model = enc
        self._precompute_item_embeddings()
        logger.info(" Model service ready")

    @torch.no_grad()
    def _precompute_item_embeddings(self):
        """app/model_service.py:71-91: the item tower over the vocabulary, 512 ids per call."""
        parts = [self.model({"movie_id": self.item_vocab[i:i + _CHUNK]})["item_embedding"]
                 for i in range(0, len(self.item_vocab), _CHUNK)]
        self.item_embeddings = torch.cat(parts).contiguous()
        Dp = F._kernel_dim(self.item_embeddings.shape[1])
        self._items_k = (F._pad_cols(self.item_embeddings, Dp) if Dp != self.item_embeddings.shape[1]
                         else self.item_embeddings)
        logger.info(f" Item embeddings computed: {tuple(self.item_embeddings.shape)}")

    def is_ready(self) -> bool:
        return (self.model is not None and self.user_vocab is not None and self.item_vocab is not None
                and self.item_embeddings is not None)

    def get_version(self) -> str:
        return self.version

    @torch.no_grad()
    def _user_embeddings(self, user_ids: List[str]) -> torch.Tensor:
        return self.model({"user_id": list(user_ids)})["user_embedding"].contiguous()

    @torch.no_grad()
    def recommend(self, user_id: str, k: int = 10, exclude_seen: bool = True) -> List[Dict]:
        """app/model_service.py:104-150 (exclude_seen is accepted and unused, as there)."""
        if user_id not in self._user_set:
            logger.warning(f"User {user_id} not in vocabulary, using cold-start strategy")
            return self._get_popular_items(k)
        return self._recommend_known([user_id], k)[0]

    def _recommend_known(self, users: List[str], k: int) -> List[List[Dict]]:
        k = min(int(k), len(self.item_vocab))
        if k <= 0:
            return [[] for _ in users]
        q = self._user_embeddings(users)
        Dp = self._items_k.shape[1]
        if Dp != q.shape[1]:
            q = F._pad_cols(q, Dp)
        scores, idx = F.topk_ip(q, self._items_k, k)
        scores, idx = scores.cpu().tolist(), idx.cpu().tolist()
        return [[{"item_id": self.item_vocab[i], "score": float(s), "rank": r + 1}
                 for r, (s, i) in enumerate(zip(scores[j], idx[j])) if 0 <= i < len(self.item_vocab)]
                for j in range(len(users))]

    @torch.no_grad()
    def score(self, user_id: str, item_ids: List[str]) -> Dict[str, float]:
        """app/model_service.py:152-198: dot(user_emb, item_emb) for the known items."""
        if user_id not in self._user_set:
            raise ValueError(f"User {user_id} not found")
        valid = [i for i in item_ids if i in self._item_row]
        if not valid:
            raise ValueError("No valid items found")
        u = self._user_embeddings([user_id])
        c = self.model({"movie_id": valid})["item_embedding"].contiguous()
        s = F.gemm(c, u, trans_b=True)[:, 0].cpu().tolist()
        return {item: float(v) for item, v in zip(valid, s)}

    def recommend_batch(self, user_ids: List[str], k: int = 10) -> List[Dict]:
        """app/model_service.py:200-227; known users share one tower pass and one top-k launch."""
        known = [u for u in dict.fromkeys(user_ids) if u in self._user_set]
        recs = {}
        err = None
        if known:
            try:
                recs = dict(zip(known, self._recommend_known(known, k)))
            except Exception as e:   # the reference reports per-user errors instead of raising
                err = str(e)
        out = []
        for u in user_ids:
            if u not in self._user_set:
                out.append({"user_id": u, "recommendations": self._get_popular_items(k), "status": "success"})
            elif err is None:
                out.append({"user_id": u, "recommendations": recs[u], "status": "success"})
            else:
                out.append({"user_id": u, "recommendations": [], "status": "error", "error": err})
        return out

    def _get_popular_items(self, k: int) -> List[Dict]:
        """app/model_service.py:229-239: the first k vocabulary items, score 1/rank."""
        return [{"item_id": item, "score": 1.0 / rank, "rank": rank}
                for rank, item in enumerate(self.item_vocab[:k], 1)]

    def get_model_info(self) -> Dict:
        return {
            "version": self.version,
            "num_users": len(self.user_vocab) if self.user_vocab else 0,
            "num_items": len(self.item_vocab) if self.item_vocab else 0,
            "embedding_dim": int(self.item_embeddings.shape[1]) if self.item_embeddings is not None else 0,
            "config": self.config,
            "model_path": str(self.model_dir),
        }


__all__ = ["RecommendationService"]
