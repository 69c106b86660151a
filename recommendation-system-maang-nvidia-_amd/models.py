"""Model classes with the reference's construction API (src/models.py), on HIP kernels.

  DeepCrossNetwork(cross_layers=3, deep_layers=None, dropout_rate=0.2, l2_reg=1e-5)
      src/models.py:13-55
  MultiTowerModel(config, user_vocab, item_vocab, feature_specs)      src/models.py:58-102
  MultiTaskModel(config, user_vocab, item_vocab, feature_specs, class_weights=None)
      src/models.py:105-159 (+ the tfrs.models.Model train_step contract)

They are torch.nn.Modules whose every hot op is a librecsys_hip.so kernel (functional.py).
Parameter layout is Keras' (Dense kernel [in, out], Embedding [V+1, D] with row 0 = OOV;
DCN cross weights packed [L, d] = the L [d, 1] cross_w_i stacked) so reference weights load
without transposes. Embedding gradients never materialise as dense [V, D] tensors: they are
collected as (ids, rows) slices — the Keras IndexedSlices — and applied by the sparse Adagrad
kernel (optim.py).
"""
from __future__ import annotations

import math
from typing import Any, Dict, List, Optional

import numpy as np
import torch
from torch import nn

from .config import ModelConfig
from .functional import (PREC_F32_SPLIT6, HeadsLossTotalFn, DCN2TrunkFn, DCNCrossFn, DCNCrossMatFn, DenseFn, EmbeddingFn,
                         EmbeddingTablesFn, HeadsFn, MLPFn, MLPGroupFn, HeadsRankingLossFn, InBatchSoftmaxFn,
                         L2PenaltyFn, LossCombineFn, MultiEmbeddingFn, RetrievalCrossFn, SparseGradSink)
from . import functional as _F
from . import optim as _optim
from .lookup import StringLookup

DCN2_TRUNK = True  # DCNv2Ranker: cross stack + deep tower as one plane-pair-GEMM node at precision 6


def _default_device():
    return torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")


def _glorot(shape, gen, device):
    fan_in, fan_out = shape[0], shape[1]
    lim = math.sqrt(6.0 / (fan_in + fan_out))
    return (torch.rand(shape, generator=gen, dtype=torch.float32) * 2 - 1).mul_(lim).to(device)


def set_contraction_precision(module: nn.Module, precision: int) -> None:
    """Contraction precision (ModelConfig.contraction_precision; include/recsys_hip.h RS_PREC_*)
    of every GEMM-shaped kernel under `module`: Dense layers, the DCN-v2 cross stack and (through
    the config) the in-batch softmax."""
    if precision not in (0, 6, 9):
        raise ValueError(f"contraction precision must be 0, 6 or 9, got {precision!r}")
    for m in module.modules():
        if isinstance(m, (Dense, DCNv2Ranker)):
            m.precision = precision
        cfg = getattr(m, "config", None)
        if isinstance(cfg, ModelConfig):
            cfg.contraction_precision = precision


def _gen(seed):
    g = torch.Generator()
    g.manual_seed(int(seed))
    return g


# --------------------------------------------------------------------------------------------
# layers
# --------------------------------------------------------------------------------------------
class Dense(nn.Module):
    """keras.layers.Dense(units, activation in {None, 'relu', 'sigmoid'}) — kernel [in, units]."""

    def __init__(self, in_dim: int, units: int, activation: Optional[str] = None, seed: int = 0,
                 device=None, kernel_regularizer_l2: float = 0.0):
        super().__init__()
        device = device or _default_device()
        self.activation = activation
        self.l2 = kernel_regularizer_l2
        self.kernel = nn.Parameter(_glorot((in_dim, units), _gen(seed), device))
        self.bias = nn.Parameter(torch.zeros(units, dtype=torch.float32, device=device))
        self.precision = 0   # contraction precision of its GEMMs (set_contraction_precision)

    def forward(self, x):
        if self.activation == "sigmoid":
            raise NotImplementedError("sigmoid Dense is only used by the fused CTR head")
        return DenseFn.apply(x, self.kernel, self.bias, self.activation == "relu", self.precision)


class Embedding(nn.Module):
    """keras.layers.Embedding(input_dim, output_dim), uniform(-0.05, 0.05) init.
    The gradient is collected as IndexedSlices (ids, rows) in ``self.sink``."""

    def __init__(self, input_dim: int, output_dim: int, seed: int = 0, device=None):
        super().__init__()
        device = device or _default_device()
        w = torch.empty((input_dim, output_dim), dtype=torch.float32, device=device)
        g = torch.Generator(device=device)
        g.manual_seed(int(seed))
        w.uniform_(-0.05, 0.05, generator=g)
        self.weight = nn.Parameter(w)
        self.sink = SparseGradSink()

    def forward(self, ids: torch.Tensor):
        return EmbeddingFn.apply(ids, self.weight, self.sink)


class Tower(nn.Module):
    """keras.Sequential([Dense(u, 'relu') for u in dims] + [Dense(D)]) (src/models.py:76-77)."""

    def __init__(self, in_dim: int, dims: List[int], out_dim: int, seed: int = 0, device=None):
        super().__init__()
        layers = []
        prev = in_dim
        for j, u in enumerate(list(dims)):
            layers.append(Dense(prev, u, "relu", seed=seed + j, device=device))
            prev = u
        layers.append(Dense(prev, out_dim, None, seed=seed + len(dims), device=device))
        self.layers = nn.ModuleList(layers)

    def forward(self, x):
        return dense_stack(self.layers, x)


def dense_stack(layers, x, l2: float = 0.0):
    """x through a list of ReLU / linear Dense layers as one MLPFn node (fused backward); with
    l2 > 0 returns (y, l2 * sum ||W_k||^2) from the same node."""
    if len(layers) == 0:
        return (x, None) if l2 > 0 else x
    params = []
    for layer in layers:
        params += [layer.kernel, layer.bias]
    return MLPFn.apply(x, tuple(layer.activation == "relu" for layer in layers), layers[0].precision, float(l2),
                       *params)


def dense_stack_group(stacks, xs):
    """Several Dense stacks of one architecture on inputs of one shape (the user and item towers,
    src/models.py:86,90) through one MLPGroupFn node: every GEMM launch serves all stacks (same
    results, bitwise, as one dense_stack per stack); falls back to dense_stack per stack otherwise."""
    ref = stacks[0]
    same = (len(stacks) <= 4 and all(x.shape == xs[0].shape for x in xs)
            and all(len(st) == len(ref) for st in stacks)
            and all(a.kernel.shape == b.kernel.shape and a.activation == b.activation and a.precision == b.precision
                    for st in stacks for a, b in zip(st, ref)))
    if len(stacks) == 1 or not same or len(ref) == 0:
        return [dense_stack(st, x) for st, x in zip(stacks, xs)]
    params = []
    for st in stacks:
        for layer in st:
            params += [layer.kernel, layer.bias]
    return list(MLPGroupFn.apply(tuple(layer.activation == "relu" for layer in ref), ref[0].precision, len(stacks),
                                 *xs, *params))


# --------------------------------------------------------------------------------------------
# DeepCrossNetwork (src/models.py:13-55)
# --------------------------------------------------------------------------------------------
class DeepCrossNetwork(nn.Module):
    """Deep & Cross Network (v1, vector cross weight) — src/models.py:13-55.

    ``forward(inputs [B, d]) -> [B, d + deep_layers[-1]]`` like the Keras layer. Keras builds the
    cross weights lazily from the input width (build, :31-35); pass ``input_dim`` to build
    eagerly (MultiTaskModel does), otherwise the first forward builds them. ``dropout_rate`` is
    stored but — exactly like the reference — never applied.
    """

    def __init__(self, cross_layers: int = 3, deep_layers: List[int] = None, dropout_rate: float = 0.2,
                 l2_reg: float = 1e-5, input_dim: Optional[int] = None, seed: int = 100, device=None):
        super().__init__()
        self.cross_layers = cross_layers
        self.deep_layers = list(deep_layers or [256, 128, 64])   # src/models.py:21
        self.dropout_rate = dropout_rate
        self.l2_reg = l2_reg
        self._seed = seed
        self._device = device or _default_device()
        self.cross_w = None
        self.cross_b = None
        self.deep_nets = None
        if input_dim is not None:
            self.build(input_dim)

    def build(self, input_dim: int):
        g = _gen(self._seed)
        lim = math.sqrt(6.0 / (input_dim + 1))           # glorot_uniform on [d, 1]
        w = (torch.rand((self.cross_layers, input_dim), generator=g) * 2 - 1) * lim
        self.cross_w = nn.Parameter(w.to(self._device))
        self.cross_b = nn.Parameter(torch.zeros((self.cross_layers, input_dim), device=self._device))
        nets, prev = [], input_dim
        for j, u in enumerate(self.deep_layers):             # src/models.py:26-29
            nets.append(Dense(prev, u, "relu", seed=self._seed + 1 + j, device=self._device,
                              kernel_regularizer_l2=self.l2_reg))
            prev = u
        self.deep_nets = nn.ModuleList(nets)
        self.input_dim = input_dim

    @property
    def output_dim(self) -> int:
        return self.input_dim + self.deep_layers[-1]

    def cross_weight(self, i: int) -> torch.Tensor:
        """The reference's cross_w_i as a [d, 1] view."""
        return self.cross_w[i].view(-1, 1)

    def forward_pair(self, u: torch.Tensor, v: torch.Tensor):
        """Fused path: x0 = [u || v] is produced by the cross kernel itself.
        Returns (x0, x_L, deep_out)."""
        if self.cross_w is None:
            self.build(u.shape[1] + v.shape[1])
        x0, xl = DCNCrossFn.apply(u, v, self.cross_w, self.cross_b)
        h = self._deep(x0)                                    # deep net on x0 (:46-48)
        return x0, xl, h

    def _deep(self, x0):
        """The deep net on x0; under autograd with l2 > 0 the same node also computes the kernels'
        l2 regularizer, kept for the next regularization_loss() (Keras model.losses)."""
        if self.l2_reg > 0 and torch.is_grad_enabled() and len(self.deep_nets) > 0:
            h, self._reg_pending = dense_stack(self.deep_nets, x0, self.l2_reg)
            return h
        self._reg_pending = None
        return dense_stack(self.deep_nets, x0)

    def forward(self, inputs: torch.Tensor, training=None):
        d = inputs.shape[1]
        if self.cross_w is None:
            self.build(d)
        if d % 2 == 0:
            _, xl, h = self.forward_pair(inputs[:, : d // 2].contiguous(), inputs[:, d // 2:].contiguous())
            return torch.cat([xl, h], dim=1)                  # src/models.py:50
        # any width, like the Keras layer (:31-35): the fused kernel takes x0 as two equal halves,
        # so an odd width runs with one zero column appended (with zero cross weight and bias it
        # stays zero through every layer and changes no dot product); the deep net reads the
        # unpadded x0 and the padded gradient entries are dropped by autograd
        xp = torch.nn.functional.pad(inputs, (0, 1))
        hp = (d + 1) // 2
        wp = torch.nn.functional.pad(self.cross_w, (0, 1))
        bp = torch.nn.functional.pad(self.cross_b, (0, 1))
        x0p, xlp = DCNCrossFn.apply(xp[:, :hp].contiguous(), xp[:, hp:].contiguous(), wp, bp)
        h = self._deep(x0p[:, :d].contiguous())                    # deep net on x0 (:46-48)
        return torch.cat([xlp[:, :d], h], dim=1)

    def regularization_loss(self) -> torch.Tensor:
        """sum of kernel_regularizer=l2(l2_reg) terms (src/models.py:27)."""
        # the value the last training forward computed with the deep net (same weights: the
        # optimizer steps after model.losses is read), taken once; otherwise a penalty node
        reg, self._reg_pending = getattr(self, "_reg_pending", None), None
        if reg is not None:
            return reg
        return L2PenaltyFn.apply(float(self.l2_reg), *[n.kernel for n in self.deep_nets])

    def get_config(self):
        return {"cross_layers": self.cross_layers, "deep_layers": self.deep_layers,
                "dropout_rate": self.dropout_rate, "l2_reg": self.l2_reg}


# --------------------------------------------------------------------------------------------
# MultiTowerModel (src/models.py:58-102)
# --------------------------------------------------------------------------------------------
class MultiTowerModel(nn.Module):
    """Two-tower encoder. ``forward(features)`` accepts the reference's feature dict
    {'user_id': str ids, 'movie_id': str ids} (either key optional, :83-89) or, as a fast
    path, int64 device tensors that are already StringLookup outputs.

    Build extension: ``user_vocab`` / ``item_vocab`` may also be an int vocabulary SIZE (tables of
    size+1 rows, integer-id inputs only) for synthetic 10M-row tables where a Python list of
    10M strings would dominate start-up."""

    def __init__(self, config: ModelConfig, user_vocab, item_vocab,
                 feature_specs: Dict[str, Any], seed: int = 0, device=None):
        super().__init__()
        device = device or _default_device()
        self.config = config
        self.user_vocab = user_vocab if isinstance(user_vocab, int) else list(user_vocab)
        self.item_vocab = item_vocab if isinstance(item_vocab, int) else list(item_vocab)
        self.feature_specs = feature_specs
        D = config.embedding_dim
        nu = self.user_vocab if isinstance(self.user_vocab, int) else len(self.user_vocab)
        ni = self.item_vocab if isinstance(self.item_vocab, int) else len(self.item_vocab)
        self.user_lookup = None if isinstance(self.user_vocab, int) else StringLookup(self.user_vocab)  # :70
        self.user_embedding = Embedding(nu + 1, D, seed=seed + 1, device=device)                      # :71
        self.item_lookup = None if isinstance(self.item_vocab, int) else StringLookup(self.item_vocab)  # :73
        self.item_embedding = Embedding(ni + 1, D, seed=seed + 2, device=device)                      # :74
        self.user_tower = Tower(D, config.user_tower_dims, D, seed=seed + 10, device=device)       # :76
        self.item_tower = Tower(D, config.item_tower_dims, D, seed=seed + 30, device=device)       # :77
        set_contraction_precision(self, config.contraction_precision)

    @property
    def device(self):
        return self.user_embedding.weight.device

    def ids(self, values, lookup: Optional[StringLookup]) -> torch.Tensor:
        if isinstance(values, torch.Tensor) and values.dtype == torch.int64:
            return values.to(self.device, non_blocking=True).contiguous()
        if lookup is None:
            raise TypeError("this model was built from vocabulary sizes: pass int64 row-id tensors")
        return torch.from_numpy(lookup(values)).to(self.device, non_blocking=True)

    def user_ids(self, values):
        return self.ids(values, self.user_lookup)

    def item_ids(self, values):
        return self.ids(values, self.item_lookup)

    def forward(self, features: Dict[str, Any], training=None, orders=None):
        """orders (optional): each side's batch rows in ascending-id order (the in-batch id plan's,
        functional.inbatch_unique_ids_pair(order=True)): the gather reads the tables in that order
        (nearby rows per wave: few TLB pages), the same result."""
        user_emb = item_emb = None
        if "user_id" in features and "movie_id" in features:
            # both lookups (:85, :89) in one gather launch, then the towers (:86, :90)
            ue, ie = EmbeddingTablesFn.apply(
                [self.user_embedding.sink, self.item_embedding.sink], 2, orders, self.user_ids(features["user_id"]),
                self.item_ids(features["movie_id"]), self.user_embedding.weight, self.item_embedding.weight)
            u, i = dense_stack_group([self.user_tower.layers, self.item_tower.layers], [ue, ie])
            return {"user_embedding": u, "item_embedding": i}
        if "user_id" in features:                             # :84-85
            user_emb = self.user_tower(self.user_embedding(self.user_ids(features["user_id"])))
        if "movie_id" in features:                            # :88-89
            item_emb = self.item_tower(self.item_embedding(self.item_ids(features["movie_id"])))
        return {"user_embedding": user_emb, "item_embedding": item_emb}

    def get_config(self):
        return {"config": self.config.to_dict(), "user_vocab": self.user_vocab,
                "item_vocab": self.item_vocab, "feature_specs": self.feature_specs}

    @classmethod
    def from_config(cls, config, **kw):
        config = dict(config)
        config["config"] = ModelConfig(**config.pop("config"))
        return cls(**config, **kw)


# --------------------------------------------------------------------------------------------
# MultiTaskModel (src/models.py:105-159)
# --------------------------------------------------------------------------------------------
class MultiTaskModel(nn.Module):
    """Two towers -> in-batch retrieval loss and [u || i] -> DCN -> rating / CTR heads."""

    def __init__(self, config: ModelConfig, user_vocab: List[str], item_vocab: List[str],
                 feature_specs: Dict[str, Any], class_weights: Dict[int, float] = None,
                 seed: int = 0, device=None):
        super().__init__()
        device = device or _default_device()
        self.config = config
        self.encoder = MultiTowerModel(config, user_vocab, item_vocab, feature_specs, seed=seed, device=device)
        self.class_weights = dict(class_weights) if class_weights else None
        d = 2 * config.embedding_dim
        self.dcn = DeepCrossNetwork(config.cross_layers, config.dnn_dims, config.dropout_rate, config.l2_reg,
                                    input_dim=d, seed=seed + 100, device=device)      # :118
        dz = d + config.dnn_dims[-1]
        self.rating_head = Dense(dz, 1, None, seed=seed + 200, device=device)         # :119
        self.ctr_head = Dense(dz, 1, "sigmoid", seed=seed + 201, device=device)       # :120
        set_contraction_precision(self, config.contraction_precision)

    # ---- inputs ------------------------------------------------------------------------------
    @staticmethod
    def _split(data):
        if isinstance(data, tuple):
            return data[0], data[1]
        return data, data

    def _labels(self, labels, key):
        v = labels[key]
        if isinstance(v, torch.Tensor):
            return v.to(self.encoder.device, dtype=torch.float32, non_blocking=True).reshape(-1).contiguous()
        return torch.as_tensor(np.asarray(v, dtype=np.float32), device=self.encoder.device).reshape(-1)

    def _towers(self, features, orders=None):
        emb = self.encoder(features, orders=orders)
        return emb["user_embedding"], emb["item_embedding"]

    # ---- keras call / compute_loss -----------------------------------------------------------
    def forward(self, data, training=None):
        """MultiTaskModel.call (src/models.py:125-131)."""
        features, _ = self._split(data)
        u, i = self._towers(features)
        _, xl, h = self.dcn.forward_pair(u, i)
        r, p = HeadsFn.apply(xl, h, self.rating_head.kernel, self.rating_head.bias,
                             self.ctr_head.kernel, self.ctr_head.bias)
        return {"user_embedding": u, "item_embedding": i, "rating_prediction": r, "ctr_prediction": p}

    def compute_loss(self, data, training=False, return_parts: bool = False, with_regularization: bool = False):
        """MultiTaskModel.compute_loss (src/models.py:133-148): retrieval_weight * Retrieval(u, i)
        + rating_weight * Ranking(MSE) + ctr_weight * Ranking(BCE, class-weighted).
        with_regularization: also add the train step's sum(self.losses) (tfrs train_step) in the same
        node and return (loss, loss + regularization, regularization) — one launch sequence instead
        of a separate add (the trainer's path)."""
        self._prepare_stack_images(data)
        try:
            return self._compute_loss(data, training, return_parts, with_regularization)
        finally:
            _F.clear_prepared_images()   # images are valid for this forward only

    def _prepare_stack_images(self, data):
        """At batches the one-launch Dense stacks serve, the towers' and the deep net's weight
        images in one launch (functional.prepare_mlp_images) instead of one per stack node."""
        if not _F.MLP_PREPARE:
            return
        feats = data[0] if isinstance(data, (tuple, list)) else data
        uid = feats.get("user_id") if isinstance(feats, dict) else None
        if uid is None or not torch.is_tensor(uid) or uid.shape[0] > _F.MLP_FUSED_MAX_M or not uid.is_cuda:
            return
        enc = self.encoder
        if not hasattr(enc, "user_tower"):
            return
        nodes = [[[l.kernel for l in enc.user_tower.layers], [l.kernel for l in enc.item_tower.layers]]]
        if self.dcn.deep_nets is not None and len(self.dcn.deep_nets):
            nodes.append([[l.kernel for l in self.dcn.deep_nets]])
        for node in nodes:
            dims = [node[0][0].shape[0]] + [W.shape[1] for W in node[0]]
            if not (all(d % 32 == 0 for d in dims) and _F.mlp_fused_ok(uid.shape[0], dims[0], node[0],
                                                                         self.config.contraction_precision)):
                return
        _F.prepare_mlp_images(nodes)

    def _compute_loss(self, data, training, return_parts, with_regularization):
        features, labels = self._split(data)
        ids = None
        if "user_id" in features and "movie_id" in features:
            # the towers see only the ids (:85-90), so equal ids give equal embeddings: the
            # retrieval loss's deduplicated pair groups rows by id (functional.inbatch_dedup_plan)
            enc = self.encoder
            uid, iid = enc.user_ids(features["user_id"]), enc.item_ids(features["movie_id"])
            features = dict(features, user_id=uid, movie_id=iid)
            ids = (uid, iid, enc.user_embedding.weight.shape[0], enc.item_embedding.weight.shape[0])
        orders = None
        if ids is not None and _F.inbatch_plan_eligible(uid.shape[0], self.config):
            # the id plan (distinct rows, counts; with RS_GATHER_ORDERED each side's rows in ascending-id
            # order, for the gather) before the towers; the retrieval loss reuses the plan
            # each side's order is also the stable sort the tables' sparse update would run: the
            # sinks carry it to the optimizer (optim.SPARSE_USE_PLAN_ORDER), which then skips its sort
            want_order = _F.GATHER_ORDERED or _optim.SPARSE_USE_PLAN_ORDER
            # (module attribute: patchable, timed); the distinct ids for the distinct-row towers' gather
            plan = _F.inbatch_unique_ids_pair(*ids, order=want_order, dids=want_order and _F.PLAN_DIDS)
            ids = ids + (plan,)
            orders = (plan[0][5], plan[1][5]) if _F.GATHER_ORDERED else None
            if want_order and torch.is_grad_enabled():
                enc.user_embedding.sink.order = (uid, plan[0][5])
                enc.item_embedding.sink.order = (iid, plan[1][5])
                if len(plan[0]) > 7:   # the run heads: the update's apply pass, one slice per distinct id
                    enc.user_embedding.sink.heads = (plan[0][7], plan[0][6], plan[0][3][0:1])
                    enc.item_embedding.sink.heads = (plan[1][7], plan[1][6], plan[1][3][0:1])
                    # each side's deduplicated count, known from the forward on (the data-parallel
                    # exchange all-gathers these long before the backward ends: no drain at its host read)
                    ev = torch.cuda.Event() if uid.is_cuda else None
                    if ev is not None:
                        ev.record()
                    enc.user_embedding.sink.plan_counts = (plan[0][4][4:5], ev)
                    enc.item_embedding.sink.plan_counts = (plan[1][4][5:6], ev)
        enc = self.encoder
        if (ids is not None and len(ids) > 4 and hasattr(enc, "user_tower")
                and _F.distinct_towers_ok(uid.shape[0], [enc.user_tower.layers, enc.item_tower.layers],
                                          self.config.contraction_precision)):
            # the towers over the plan's distinct ids (the lookups and forward once per distinct id,
            # expanded to the batch rows; gradients per batch row: bitwise the per-row towers)
            ut, it = enc.user_tower.layers, enc.item_tower.layers
            params = [t for l in ut for t in (l.kernel, l.bias)] + [t for l in it for t in (l.kernel, l.bias)]
            u, i = _F.DistinctTowersFn.apply(
                [enc.user_embedding.sink, enc.item_embedding.sink], tuple(l.activation == "relu" for l in ut),
                self.config.contraction_precision, ids[4], uid, iid, enc.user_embedding.weight,
                enc.item_embedding.weight, *params)
        else:
            u, i = self._towers(features, orders)
        # the retrieval task (:137) and the concat + cross stack (:128, 38-44) read the same tower
        # outputs: one node, whose backward adds the retrieval gradient inside the cross kernel
        ret, _, x0, xl = RetrievalCrossFn.apply(u, i, self.dcn.cross_w, self.dcn.cross_b,
                                                self.config.contraction_precision, ids)
        h = self.dcn._deep(x0)                                                          # :46-48
        reg = None
        if with_regularization:
            losses = self.losses
            reg = losses[0] if len(losses) == 1 else sum(losses)
        rating = self._labels(labels, "rating")
        has_ctr = "y_implicit" in labels                                               # :141
        yi = self._labels(labels, "y_implicit") if has_ctr else torch.zeros_like(rating)
        c = self.config
        # heads (:119-120,131), both Ranking tasks (:138-145) and w_ret ret + w_rat l_rat + w_ctr
        # l_ctr (:147; no ctr term without CTR labels, :140) (+ the regularizer): one node
        total, total_reg, l_rat, l_ctr = HeadsLossTotalFn.apply(
            xl, h, self.rating_head.kernel, self.rating_head.bias, self.ctr_head.kernel, self.ctr_head.bias,
            ret.reshape(()), reg.reshape(()) if reg is not None else None, rating, yi,
            self.class_weights if has_ctr else None, self.config.ctr_mode_code if has_ctr else 0,
            c.retrieval_weight, c.rating_weight, c.ctr_weight, has_ctr,
            bool(self.dcn.deep_nets) and self.dcn.deep_nets[-1].activation == "relu")
        out = (total, total_reg, reg) if with_regularization else total
        if return_parts:
            return out, {"retrieval": ret, "rating": l_rat,
                         "ctr": l_ctr if has_ctr else torch.zeros((), device=rating.device)}
        return out

    @property
    def losses(self) -> List[torch.Tensor]:
        """Keras model.losses: the DCN deep-kernel l2 regularization terms."""
        return [self.dcn.regularization_loss()]

    def embedding_modules(self) -> List[Embedding]:
        return [self.encoder.user_embedding, self.encoder.item_embedding]

    def dense_parameters(self) -> List[nn.Parameter]:
        emb = {id(e.weight) for e in self.embedding_modules()}
        return [p for p in self.parameters() if id(p) not in emb]

    def get_config(self):
        return {"config": self.config.to_dict(), "user_vocab": self.encoder.user_vocab,
                "item_vocab": self.encoder.item_vocab, "feature_specs": self.encoder.feature_specs,
                "class_weights": self.class_weights}

    @classmethod
    def from_config(cls, config, **kw):
        config = dict(config)
        config["config"] = ModelConfig(**config.pop("config"))
        cw = config.get("class_weights")
        if cw:
            config["class_weights"] = {int(k): float(v) for k, v in cw.items()}
        return cls(**config, **kw)


# --------------------------------------------------------------------------------------------
# DCN-v2 ranker (BASELINE config 5 — an extension: the reference has no such model)
# --------------------------------------------------------------------------------------------
class DCNv2Ranker(nn.Module):
    """Criteo-shaped DCN-v2 CTR ranker: ``num_sparse`` embedding tables + ``num_dense`` dense
    features -> x0 (zero-padded to a multiple of 16 columns) -> ``cross_layers`` matrix cross
    layers x_{l+1} = x0 * (x_l W_l + b_l) + x_l  and a ReLU deep tower on x0 -> [x_L || h] ->
    Dense(1, sigmoid) -> BCE (the reference's ctr_task, src/models.py:120,123).
    Inputs: ``sparse_ids`` int64 [num_sparse, B] (feature-major), ``dense`` fp32 [B, num_dense].
    The zero padding is inert: padded x0 columns stay 0 through every layer and receive no
    gradient, so the model equals the unpadded one."""

    def __init__(self, vocab_sizes: List[int], embedding_dim: int = 128, num_dense: int = 13,
                 cross_layers: int = 4, deep_layers: List[int] = None, seed: int = 0, device=None,
                 pad_to: int = 16, precision: int = 6):
        super().__init__()
        device = device or _default_device()
        self.vocab_sizes = list(vocab_sizes)
        self.embedding_dim = E = embedding_dim
        self.num_dense = num_dense
        self.deep_layers = list(deep_layers or [1024, 1024, 1024])
        F_ = len(self.vocab_sizes)
        self.d_raw = F_ * E + num_dense
        self.d = d = (self.d_raw + pad_to - 1) // pad_to * pad_to
        self.tables = nn.ModuleList([Embedding(v + 1, E, seed=seed + 1 + f, device=device)
                                     for f, v in enumerate(self.vocab_sizes)])
        g = _gen(seed + 500)
        lim = math.sqrt(6.0 / (d + d))
        W = (torch.rand((cross_layers, d, d), generator=g) * 2 - 1) * lim
        W[:, self.d_raw:, :] = 0.0
        W[:, :, self.d_raw:] = 0.0
        self.cross_W = nn.Parameter(W.to(device))
        self.cross_b = nn.Parameter(torch.zeros((cross_layers, d), device=device))
        nets, prev = [], d
        for j, u in enumerate(self.deep_layers):
            nets.append(Dense(prev, u, "relu", seed=seed + 600 + j, device=device))
            prev = u
        self.deep_nets = nn.ModuleList(nets)
        dz = d + self.deep_layers[-1]
        self.rating_head = Dense(dz, 1, None, seed=seed + 700, device=device)   # unused (kept zero-weighted)
        self.ctr_head = Dense(dz, 1, "sigmoid", seed=seed + 701, device=device)
        self._ptrs = None
        set_contraction_precision(self, precision)

    def _table_arrays(self, device):
        ptrs = [t.weight.data_ptr() for t in self.tables]
        if self._ptrs is None or self._ptrs[0] != ptrs:
            self._ptrs = (ptrs, torch.tensor(ptrs, dtype=torch.int64, device=device),
                          torch.tensor([t.weight.shape[0] for t in self.tables], dtype=torch.int64, device=device))
        return self._ptrs[1], self._ptrs[2]

    def x0(self, sparse_ids: torch.Tensor, dense: torch.Tensor) -> torch.Tensor:
        tp, nr = self._table_arrays(sparse_ids.device)
        return MultiEmbeddingFn.apply(sparse_ids.contiguous(), dense.contiguous() if dense is not None else None,
                                      tp, nr, self.embedding_dim, self.d, [t.sink for t in self.tables],
                                      *[t.weight for t in self.tables])

    def _trunk(self, sparse_ids, dense):
        x0 = self.x0(sparse_ids, dense)
        if DCN2_TRUNK and self.precision == PREC_F32_SPLIT6 and self.cross_W.shape[0] > 0 and len(self.deep_nets):
            # cross stack + deep tower as one node, every GEMM on the plane-pair kernel
            params = []
            for layer in self.deep_nets:
                params += [layer.kernel, layer.bias]
            return DCN2TrunkFn.apply(x0, self.cross_W, self.cross_b,
                                     tuple(layer.activation == "relu" for layer in self.deep_nets), *params)
        xl = DCNCrossMatFn.apply(x0, self.cross_W, self.cross_b, self.precision)
        return xl, dense_stack(self.deep_nets, x0)

    def forward(self, sparse_ids, dense):
        xl, h = self._trunk(sparse_ids, dense)
        _, p = HeadsFn.apply(xl, h, self.rating_head.kernel, self.rating_head.bias,
                             self.ctr_head.kernel, self.ctr_head.bias)
        return p

    def compute_loss(self, sparse_ids, dense, labels, class_weights=None):
        """Binary cross-entropy of the CTR head (Keras BCE, mean over the batch)."""
        xl, h = self._trunk(sparse_ids, dense)
        y = labels.to(torch.float32).reshape(-1).contiguous()
        _, _, _, l_ctr = HeadsRankingLossFn.apply(xl, h, self.rating_head.kernel, self.rating_head.bias,
                                                  self.ctr_head.kernel, self.ctr_head.bias, torch.zeros_like(y),
                                                  y, class_weights, 0)
        return l_ctr

    def embedding_modules(self) -> List[Embedding]:
        return list(self.tables)

    def dense_parameters(self) -> List[nn.Parameter]:
        emb = {id(t.weight) for t in self.tables}
        return [p for p in self.parameters() if id(p) not in emb]
