"""ProductionTrainer — drop-in for src/trainer.py on the MI355X HIP path.

Same constructor and methods as the reference (src/trainer.py:37-248):
    trainer = ProductionTrainer(config, output_dir)
    model, history = trainer.train(pickle_path)          # history.history['loss'/'val_loss']
    trainer.prepare_datasets(data) -> {'train_ds','val_ds','train_df','val_df','user_vocab',
                                       'item_vocab','feature_specs'}
and the same artefacts in output_dir: best_model (state dict), training_log.csv, metrics.json,
encoder weights, vocabs.json, config.json, faiss.idx (the L2-normalised item matrix in faiss's
IndexFlatIP file format, searched by the GPU brute-force index) + item_map.json.

Semantics kept (file:line of the reference): lexicographic string vocabularies (:81-82);
labels (:99-106); balanced class weights on y_implicit (:139-145); MultiTaskModel with
Adagrad(ExponentialDecay(lr, 1000, 0.96, staircase), clipnorm=1.0) (:148-163); fit for
epochs_retrieval with EarlyStopping(val_loss, patience=20, restore_best_weights) — Keras 2
semantics: the best weights come back only when the stop triggers — and
ModelCheckpoint(save_best_only) (:165-183); recall@k on 1,000 sampled validation rows with
random_state=42 (:195-219); MirroredStrategy data parallelism when
distributed_strategy == 'mirrored' and more than one GPU process (:45-48), here one process per
GPU under torch.distributed (RCCL). Out of scope: the pandas feature engineering
of DataProcessor.engineer_features (its outputs never reach the model — only ids and labels
do), negative sampling (dead code in the reference), W&B / TensorBoard.
"""
from __future__ import annotations

import csv
import json
import logging
import math
import os
import time
from pathlib import Path
from typing import Any, Dict

import numpy as np
import torch
import torch.distributed as dist

from . import distributed as D
from . import functional as F
from .config import ModelConfig, save_config
from .data import make_dataset
from .faiss_io import write_index_flat
from .lookup import build_vocab
from .models import MultiTaskModel
from .optim import Adagrad, ExponentialDecay
from .retrieval import BruteForceIndex, ShardedBruteForceIndex, recall_at_k, shard_rows

logger = logging.getLogger(__name__)


class History:
    """keras.callbacks.History-compatible record (history.history[metric] -> per-epoch list)."""

    def __init__(self):
        self.history: Dict[str, list] = {}
        self.epoch: list = []

    def append(self, epoch: int, logs: Dict[str, float]):
        self.epoch.append(epoch)
        for k, v in logs.items():
            self.history.setdefault(k, []).append(v)


def load_and_validate_data(pickle_path: str) -> Dict[str, Any]:
    """src/data_processing.py:27-54: a pickled dict with train/val/test frames (or one frame)."""
    import pandas as pd
    data = pd.read_pickle(pickle_path)
    if isinstance(data, dict):
        train_df = data.get("train_ratings", data.get("train", pd.DataFrame()))
        val_df = data.get("val_ratings", data.get("val", pd.DataFrame()))
        test_df = data.get("test_ratings", data.get("test", pd.DataFrame()))
        uf = data.get("user_features", pd.DataFrame())
        itf = data.get("movie_features", data.get("item_features", pd.DataFrame()))
    else:
        train_df, val_df, test_df = data, pd.DataFrame(), pd.DataFrame()
        uf, itf = pd.DataFrame(), pd.DataFrame()
    as_df = lambda x: x if isinstance(x, pd.DataFrame) else pd.DataFrame(x)  # noqa: E731
    return {"train_df": as_df(train_df), "val_df": as_df(val_df), "test_df": as_df(test_df),
            "user_features": uf if isinstance(uf, pd.DataFrame) else pd.DataFrame(),
            "item_features": itf if isinstance(itf, pd.DataFrame) else pd.DataFrame()}


def normalize_columns(df):
    """The id-column part of engineer_features (src/data_processing.py:66-78): accept the
    reference's alternative column names, cast ids to str, fillna(0) (:279)."""
    if df is None or len(df) == 0:
        return df
    df = df.copy()
    for col, alts in (("user_id", ["user", "userid", "UserID"]),
                      ("movie_id", ["movie", "movieid", "item_id", "MovieID"])):
        if col not in df.columns:
            for a in alts:
                if a in df.columns:
                    df.rename(columns={a: col}, inplace=True)
                    break
            else:
                raise ValueError(f"Column {col} not found. Available: {df.columns.tolist()}")
    df["user_id"] = df["user_id"].astype(str)
    df["movie_id"] = df["movie_id"].astype(str)
    return df.fillna(0)


def balanced_class_weights(y) -> Dict[int, float]:
    """sklearn compute_class_weight('balanced', classes=[0, 1], y) (src/trainer.py:139-145)."""
    y = np.asarray(y).astype(np.int64)
    n = len(y)
    out = {}
    for c in (0, 1):
        cnt = int(np.count_nonzero(y == c))
        if cnt == 0:
            raise ValueError(f"classes should include all valid labels; class {c} absent from y")
        out[c] = n / (2.0 * cnt)
    return out


class EarlyStopping:
    """keras.callbacks.EarlyStopping(monitor, patience, restore_best_weights=True) (src/trainer.py:166)
    together with ModelCheckpoint(save_best_only=True) (:167): ``on_epoch_end`` returns
    (improved, stop) and the caller saves a checkpoint when improved; ``restore_at_end(stopped)``
    says whether the caller restores ``best_state`` after the last epoch. mode "keras3" (Keras 3,
    tf.keras from TF 2.16): restore whenever a best epoch exists, stopped or not; "keras2": only
    when the stop triggered; keras3 also records the first epoch with a monitor value as the best
    state when it does not improve (Keras 3 EarlyStopping.on_epoch_end). As in Keras, an epoch
    without a monitor value changes nothing."""

    def __init__(self, patience: int = 20, mode: str = "keras3"):
        if mode not in ("keras3", "keras2"):
            raise ValueError(f"EarlyStopping mode must be 'keras3' or 'keras2', got {mode!r}")
        self.patience = patience
        self.mode = mode
        self.best = math.inf
        self.wait = 0
        self.best_epoch = -1
        self.stopped_epoch = 0
        self.best_state = None

    def on_epoch_end(self, epoch: int, monitor, state_fn):
        if monitor is None:              # Keras returns before touching `wait`
            return False, False
        improved = monitor < self.best   # (False for a NaN monitor, as Keras' np.less)
        if self.mode == "keras3" and self.best_state is None and not improved:
            # Keras 3: "if best weights were never set, then the current weights are the best" —
            # the first epoch with a monitor value is recorded (and restored at train end) even
            # when it does not improve (a NaN val_loss)
            self.best_state = state_fn()
            self.best_epoch = epoch
        self.wait += 1
        if improved:
            self.best, self.best_epoch, self.wait = monitor, epoch, 0
            self.best_state = state_fn()
            return True, False
        if self.wait >= self.patience and epoch > 0:
            self.stopped_epoch = epoch
            return False, True
        return False, False

    def restore_at_end(self, stopped: bool) -> bool:
        if self.best_state is None:
            return False
        return stopped or self.mode == "keras3"


class ProductionTrainer:
    """Production-grade trainer (src/trainer.py:37)."""

    def __init__(self, config: ModelConfig, output_dir: str, device=None, seed: int = 0):
        self.config = config
        self.output_dir = Path(output_dir)
        self.output_dir.mkdir(parents=True, exist_ok=True)
        self.seed = seed
        # src/trainer.py:45-48: MirroredStrategy only when asked for and > 1 GPU
        self.distributed = False
        if config.distributed_strategy == "mirrored" and int(os.environ.get("WORLD_SIZE", "1")) > 1:
            self.distributed = D.init_process_group()
        self.rank = dist.get_rank() if self.distributed else 0
        self.world = dist.get_world_size() if self.distributed else 1
        if device is None:
            local = int(os.environ.get("LOCAL_RANK", "0"))
            device = torch.device("cuda", local) if torch.cuda.is_available() else torch.device("cpu")
        self.device = device

    # ------------------------------------------------------------------------------------------
    def prepare_datasets(self, data: Dict[str, Any]) -> Dict[str, Any]:
        """src/trainer.py:68-130."""
        import pandas as pd
        train_df = normalize_columns(data["train_df"])
        val_df = normalize_columns(data["val_df"])
        user_vocab = build_vocab(train_df["user_id"].unique())       # :81
        item_vocab = build_vocab(train_df["movie_id"].unique())      # :82
        feature_specs = {}
        for col in train_df.columns:                                 # :84-93
            if col in ["user_id", "movie_id", "rating", "y_implicit", "timestamp"]:
                continue
            if pd.api.types.is_numeric_dtype(train_df[col]):
                feature_specs[col] = {"type": "numerical"}
            else:
                nunique = train_df[col].nunique()
                if nunique < 10000:
                    feature_specs[col] = {"type": "categorical", "vocab_size": int(nunique)}
        from .lookup import StringLookup
        ul, il = StringLookup(user_vocab), StringLookup(item_vocab)
        B = self.config.batch_size
        train_ds = make_dataset(train_df, ul, il, B, self.device, training=True, seed=self.seed,
                                rank=self.rank, world=self.world)
        val_ds = make_dataset(val_df, ul, il, B, self.device, training=False, rank=self.rank, world=self.world)
        return {"train_ds": train_ds, "val_ds": val_ds, "train_df": train_df, "val_df": val_df,
                "user_vocab": user_vocab, "item_vocab": item_vocab, "feature_specs": feature_specs}

    # ------------------------------------------------------------------------------------------
    def build(self, datasets, class_weights):
        model = MultiTaskModel(self.config, datasets["user_vocab"], datasets["item_vocab"],
                               datasets["feature_specs"], class_weights=class_weights, seed=self.seed,
                               device=self.device)
        if self.distributed:  # identical initial replicas (MirroredStrategy mirrors variables)
            for p in model.parameters():
                dist.broadcast(p.data, 0)
        lr = ExponentialDecay(self.config.learning_rate_retrieval, decay_steps=1000, decay_rate=0.96,
                              staircase=True)
        opt = Adagrad(model.dense_parameters(), model.embedding_modules(), lr, clipnorm=self.config.clipnorm,
                      defer_reductions=not self.distributed)
        if self.distributed:   # bucketed dense all-reduce during the backward + deduplicated sparse exchange
            per_rank = -(-self.config.batch_size // self.world)
            opt.pre_apply_hooks.append(D.MirroredGradientExchange(max_rows=per_rank, dense_params=opt.dense,
                                                                  embeddings=opt.embeddings))
        return model, opt

    @staticmethod
    def train_step(model: MultiTaskModel, opt: Adagrad, batch) -> Dict[str, torch.Tensor]:
        """tfrs.models.Model.train_step [TF-ext]: loss + sum(model.losses), gradients, apply."""
        opt.zero_grad()
        # loss + sum(model.losses) formed in the loss node itself (no separate add launch)
        loss, total, reg = model.compute_loss(batch, training=True, with_regularization=True)
        total.backward(F.backward_seed(total))
        opt.step()
        return {"loss": loss.detach(), "regularization_loss": reg.detach(), "total_loss": total.detach()}

    @staticmethod
    @torch.no_grad()
    def test_step(model: MultiTaskModel, batch) -> Dict[str, torch.Tensor]:
        loss = model.compute_loss(batch, training=False)
        reg = sum(model.losses)
        return {"loss": loss, "regularization_loss": reg, "total_loss": loss + reg}

    def train(self, pickle_path: str):
        """src/trainer.py:132-193."""
        logger.info("=" * 80 + "\nSTARTING TRAINING\n" + "=" * 80)
        data = load_and_validate_data(pickle_path)
        return self.fit_data(data)

    def fit_data(self, data: Dict[str, Any]):
        datasets = self.prepare_datasets(data)
        cw = balanced_class_weights(datasets["train_df"]["y_implicit"].values
                                    if "y_implicit" in datasets["train_df"].columns
                                    else (datasets["train_df"]["rating"] >= 3.0).values)
        logger.info(f"Class weights computed: {cw}")
        model, opt = self.build(datasets, cw)
        self.model, self.optimizer = model, opt
        history = History()
        es = self.early_stopping = EarlyStopping(patience=20, mode=self.config.early_stopping_restore)  # :166
        log_path = self.output_dir / "training_log.csv"
        epoch_times = []
        for epoch in range(self.config.epochs_retrieval):
            t0 = time.time()
            last = None
            sums = {"loss": 0.0}
            nb = 0
            for batch in datasets["train_ds"]:
                last = self.train_step(model, opt, batch)
                sums["loss"] += float(last["loss"])
                nb += 1
            logs = {k: float(v) for k, v in (last or {}).items()}
            logs["epoch_mean_loss"] = sums["loss"] / max(nb, 1)
            if datasets["val_ds"] is not None:
                vlast = None
                for batch in datasets["val_ds"]:
                    vlast = self.test_step(model, batch)
                if vlast is not None:
                    for k, v in vlast.items():
                        logs[f"val_{k}"] = float(v)
            epoch_times.append(time.time() - t0)
            history.append(epoch, logs)
            if self.rank == 0:
                self._csv_log(log_path, epoch, logs)
            monitor = logs.get("val_loss", logs.get("loss"))
            improved, stop = es.on_epoch_end(
                epoch, monitor, lambda: {k: v.detach().clone() for k, v in model.state_dict().items()})
            if improved and self.rank == 0:                               # ModelCheckpoint (:167)
                torch.save(es.best_state, self.output_dir / "best_model.pt")
            if stop:
                logger.info(f"Early stopping at epoch {epoch}")
                break
        # restore_best_weights=True: Keras 3 restores at the end of training whenever a best epoch
        # exists, Keras 2 only when the stop triggered (config.early_stopping_restore); the restored
        # weights feed _evaluate / _save_artifacts / _build_faiss (src/trainer.py:185-189)
        if es.restore_at_end(es.stopped_epoch > 0):
            model.load_state_dict(es.best_state)
        for hook in opt.pre_apply_hooks:        # drop the data-parallel gradient hooks
            close = getattr(hook, "close", None)
            if close is not None:
                close()
        self.metrics = self._evaluate(model, datasets)   # every rank: the item rows are sharded (§8e)
        if self.rank == 0:
            with open(self.output_dir / "detailed_metrics.json", "w") as f:
                json.dump({"epoch_times": epoch_times, "total_time": float(sum(epoch_times))}, f, indent=2)
            self._save_artifacts(model, datasets)
            self._build_faiss(model, datasets["item_vocab"])
        logger.info("=" * 80 + "\nTRAINING COMPLETE\n" + "=" * 80)
        return model, history

    @staticmethod
    def _csv_log(path, epoch, logs):
        new = not path.exists()
        with open(path, "a", newline="") as f:
            w = csv.writer(f)
            keys = sorted(logs)
            if new:
                w.writerow(["epoch"] + keys)
            w.writerow([epoch] + [logs[k] for k in keys])

    # ------------------------------------------------------------------------------------------
    @torch.no_grad()
    def _get_item_embeddings(self, model, item_vocab, rows=None) -> torch.Tensor:
        """src/trainer.py:221-226 (chunks of 512 through the item tower), on the device; rows =
        (r0, r1) limits it to vocab rows [r0, r1) (a shard)."""
        r0, r1 = rows if rows is not None else (0, len(item_vocab))
        ids = torch.arange(r0 + 1, r1 + 1, dtype=torch.int64, device=self.device)
        out = [model.encoder({"movie_id": ids[i:i + 512]})["item_embedding"] for i in range(0, len(ids), 512)]
        if not out:
            return torch.empty((0, self.config.embedding_dim), dtype=torch.float32, device=self.device)
        return torch.cat(out).contiguous()

    @torch.no_grad()
    def _evaluate(self, model, datasets):
        """src/trainer.py:195-219: recall@k over 1,000 sampled validation rows. Under data
        parallelism (MirroredStrategy runs it on the mirrored model, :185) every rank takes part:
        each scores the sampled users against its shard of the item rows (its item-tower rows only)
        and the per-shard top-k lists meet in one all-gather + merge (ShardedBruteForceIndex, SURVEY
        §8e), so every rank returns the metrics; rank 0 writes metrics.json. The scan runs at the
        same contraction precision sharded or not (fp32 scores: the same lists)."""
        val_df = datasets["val_df"]
        if datasets["val_ds"] is None or val_df is None or len(val_df) == 0:
            logger.warning("No validation data available for evaluation.")
            return {}
        item_vocab = datasets["item_vocab"]
        if self.distributed and self.world > 1:
            rows = shard_rows(len(item_vocab), self.rank, self.world)
            index = ShardedBruteForceIndex(self._get_item_embeddings(model, item_vocab, rows), rows[0], "ip",
                                           precision=F.PREC_F32, ntotal=len(item_vocab))
        else:
            index = self._get_item_embeddings(model, item_vocab)
        sample = val_df.sample(n=min(1000, len(val_df)), random_state=42)
        user_embs = model.encoder({"user_id": sample["user_id"].values})["user_embedding"].contiguous()
        true_rows = model.encoder.item_lookup(sample["movie_id"].values) - 1   # -1: not in vocab
        metrics = recall_at_k(index, user_embs, true_rows, self.config.eval_topk)
        logger.info(f"Evaluation Results: {metrics}")
        if self.rank == 0:
            with open(self.output_dir / "metrics.json", "w") as f:
                json.dump(metrics, f, indent=2)
        return metrics

    def _save_artifacts(self, model, datasets):
        """src/trainer.py:228-234: encoder weights, vocabs.json, config.json (reference fields
        only; the build-only fields go to config_ext.json)."""
        torch.save({k: v.cpu() for k, v in model.encoder.state_dict().items()}, self.output_dir / "encoder.pt")
        with open(self.output_dir / "vocabs.json", "w") as f:
            json.dump({"users": datasets["user_vocab"], "items": datasets["item_vocab"]}, f)
        save_config(self.config, self.output_dir)   # config.json keeps the reference schema

    def _build_faiss(self, model, item_vocab):
        """src/trainer.py:236-248: the L2-normalised item matrix as faiss.idx in faiss's IndexFlatIP
        file format (faiss_io; the serving path searches it on the GPU brute-force index) and
        item_map.json."""
        idx = BruteForceIndex(self.config.embedding_dim, "cosine", self.device)
        idx.add(self._get_item_embeddings(model, item_vocab))
        write_index_flat(self.output_dir / "faiss.idx", idx.items.cpu().numpy(), "ip")
        with open(self.output_dir / "item_map.json", "w") as f:
            json.dump({str(i): item for i, item in enumerate(item_vocab)}, f)
        logger.info(f"Brute-force cosine index built with {len(item_vocab)} items.")
        return idx
