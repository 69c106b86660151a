"""Adagrad + ExponentialDecay + clipnorm, as the reference trainer compiles it.

Reference: src/trainer.py:157-163
    lr = ExponentialDecay(learning_rate_retrieval, decay_steps=1000, decay_rate=0.96, staircase=True)
    model.compile(optimizer=keras.optimizers.Adagrad(lr, clipnorm=1.0))
with Keras >= 2.11 optimizer semantics [TF-ext, SURVEY Appendix A.7]: each gradient clipped by
its own norm (IndexedSlices: over the un-deduplicated values), sparse rows deduplicated (summed)
then `acc += g^2; var -= lr_t * g / sqrt(acc + 1e-7)`, accumulators start at 0.1, and
`lr_t` is the schedule evaluated at optimizer.iterations (incremented after every apply).

Dense variables: one multi-tensor kernel sequence (rs_adagrad_dense_f32) over a device slot
table. Embedding tables: the deterministic sort + segment-sum sparse kernel
(rs_sparse_adagrad_f32) — a [V, D] dense gradient is never formed. The iteration counter lives
on the device, so a captured step (hipGraph) replays with the right learning rate.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence

import torch

from . import functional as F
from ._native import call, query


SPARSE_MULTI_MIN_TABLES = 2  # tables of one width updated by one launch sequence from this many on
# the sparse update takes the step's id-plan order instead of sorting (RS_SPARSE_PLAN_ORDER=0: sort)
SPARSE_USE_PLAN_ORDER = True
# with the plan's order, its run heads too: the apply pass runs one slice per distinct id
SPARSE_USE_PLAN_HEADS = True


@dataclass
class ExponentialDecay:
    """tf.keras.optimizers.schedules.ExponentialDecay (staircase only is used by the reference)."""

    initial_learning_rate: float
    decay_steps: int = 1000
    decay_rate: float = 0.96
    staircase: bool = True

    def __call__(self, step: int) -> float:
        p = step / self.decay_steps
        if self.staircase:
            p = float(int(p))
        return self.initial_learning_rate * self.decay_rate ** p


class Adagrad:
    """keras.optimizers.Adagrad(learning_rate, initial_accumulator_value=0.1, epsilon=1e-7,
    clipnorm=...) over a MultiTaskModel (dense params + sparse embedding tables)."""

    def __init__(self, dense_params: Sequence[torch.nn.Parameter], embeddings: Sequence,
                 learning_rate=0.001, clipnorm: Optional[float] = 1.0,
                 initial_accumulator_value: float = 0.1, epsilon: float = 1e-7,
                 defer_reductions: bool = False):
        if isinstance(learning_rate, ExponentialDecay):
            if not learning_rate.staircase:
                raise NotImplementedError("only staircase=True ExponentialDecay is on the device path")
            self.schedule = learning_rate
        else:
            self.schedule = ExponentialDecay(float(learning_rate), 1, 1.0, True)  # constant
        self.clipnorm = float(clipnorm) if clipnorm else 0.0
        self.epsilon = float(epsilon)
        self.dense = [p for p in dense_params]
        self.embeddings = list(embeddings)
        dev = self.dense[0].device if self.dense else self.embeddings[0].weight.device
        self.device = dev
        self.accum = [torch.full_like(p, initial_accumulator_value) for p in self.dense]
        self.emb_accum = [torch.full_like(e.weight, initial_accumulator_value) for e in self.embeddings]
        self.iterations = torch.zeros((), dtype=torch.int64, device=dev)
        n = len(self.dense)
        self._slots_dev = torch.zeros((max(n, 1), 4), dtype=torch.int64, device=dev)
        self._slots_key = None
        self._pinned_slots = torch.zeros((max(n, 1), 4), dtype=torch.int64,
                                         pin_memory=dev.type == "cuda")
        self._pinned_used = False
        self._max_numel = max((p.numel() for p in self.dense), default=0)
        self._ws = torch.empty(max(query("rs_adagrad_dense_workspace_bytes", max(n, 1), self._max_numel), 256),
                               dtype=torch.uint8, device=dev)
        self.pre_apply_hooks: List[Callable] = []   # e.g. data-parallel gradient exchange
        # zero_grad() .. step(): the gradient reductions of the backward of THIS optimizer's
        # parameters are queued in its own ReductionQueue and run as one launch at the top of step();
        # the gradients are not readable in between, so this is for training loops with one
        # backward per step and no gradient hooks (never with a data-parallel exchange, whose hooks
        # read the gradients). The queue is attached (weakly) to the parameters, whose autograd nodes
        # record it: another model (another optimizer) in the process never queues into it. The most
        # recently created optimizer of a parameter owns it: a new one (deferring or not) flushes and
        # detaches the queue of the one it replaces (functional.attach_reduction_queue).
        self.defer_reductions = bool(defer_reductions)
        self._rq: Optional[F.ReductionQueue] = None
        if self.defer_reductions and dev.type == "cuda":
            self._rq = F.ReductionQueue()
        F.attach_reduction_queue(self.dense, self._rq)

    # Keras-compatible read-out of the current learning rate
    def learning_rate(self, step: Optional[int] = None) -> float:
        return self.schedule(int(self.iterations.item()) if step is None else step)

    def zero_grad(self):
        for p in self.dense:
            p.grad = None
        for e in self.embeddings:
            e.sink.clear()
        for hook in self.pre_apply_hooks:   # a new step: e.g. reset the data-parallel bucketer
            begin = getattr(hook, "begin_step", None)
            if begin is not None:
                begin()
        if self._rq is not None:
            if not self.pre_apply_hooks:
                self._rq.open()    # (launches the jobs an aborted step left queued first)
            else:
                self._rq.flush()
        else:   # a queue some other optimizer left open on these parameters is closed, not fed
            F.attach_reduction_queue(self.dense, None)

    def _refresh_slots(self, live):
        """Upload the (param, grad, accum, numel) table only when a gradient moved. The copy is
        from pageable host memory, so the host buffer is consumed before copy_ returns (no race
        with a step still queued on the device); the caching allocator normally hands autograd
        the same gradient addresses every step, so this is a no-op in steady state."""
        rows = [(p.data_ptr(), g.data_ptr(), a.data_ptr(), p.numel()) for p, g, a in live]
        key = tuple(rows)
        if key == self._slots_key:
            return
        host = torch.tensor(rows, dtype=torch.int64)
        if self.device.type == "cuda" and torch.cuda.is_current_stream_capturing():
            # inside a hipGraph capture the copy becomes a memcpy node that re-reads this pinned
            # buffer (allocated up front: no host allocation is legal during capture) on every
            # replay, so it is written once and never modified afterwards
            if self._pinned_used:
                raise RuntimeError("this optimizer already belongs to a captured graph; "
                                   "create a new Adagrad for a second capture")
            self._pinned_slots[: len(rows)].copy_(host)
            self._pinned_used = True
            self._slots_dev[: len(rows)].copy_(self._pinned_slots[: len(rows)], non_blocking=True)
        else:
            self._slots_dev[: len(rows)].copy_(host)
        self._slots_key = key

    @torch.no_grad()
    def step(self):
        if self._rq is not None:
            self._rq.flush()   # the queued gradient reductions (no-op when none)
        for hook in self.pre_apply_hooks:
            hook(self)
        s = self.schedule
        live = [(p, p.grad, a) for p, a in zip(self.dense, self.accum) if p.grad is not None]
        for p, g, _ in live:
            if not g.is_contiguous() or g.dtype != torch.float32:
                raise ValueError("dense gradients must be contiguous fp32")
        if live:
            self._refresh_slots(live)
            call("rs_adagrad_dense_f32", ctypes.c_void_p(self._slots_dev.data_ptr()), len(live),
                 self._max_numel, ctypes.c_void_p(self.iterations.data_ptr()),
                 float(s.initial_learning_rate), float(s.decay_rate), int(s.decay_steps), self.clipnorm,
                 self.epsilon, ctypes.c_void_p(self._ws.data_ptr()), self._ws.numel(), F._stream())
        # the tables' sparse updates: from SPARSE_MULTI_MIN_TABLES tables of one width on, one
        # launch sequence for all of them (rs_sparse_adagrad_multi_f32: one sort, clip-norm,
        # fragment and apply pass; C5's 26 tables: ~234 launches -> 9, bitwise the per-table
        # result when the tables' slice counts are equal), else one sequence per table
        todo = []
        for e, acc in zip(self.embeddings, self.emb_accum):
            sl = e.sink.gathered()
            if sl is not None:
                todo.append((e, acc, sl[0].contiguous(), sl[1], e.sink.sumsq))
        widths = {e.weight.shape[1] for e, *_ in todo}
        with_ssq = [t[4] is not None for t in todo]
        if len(todo) >= SPARSE_MULTI_MIN_TABLES and len(widths) == 1 and (all(with_ssq) or not any(with_ssq)):
            # the multi-table sequence also advances the step counter (its apply pass's last
            # workgroup: no iteration_increment launch); with every table's ids already ordered by
            # the step's id plan it skips its own sort
            orders = [e.sink.sorted_order() for e, *_ in todo] if SPARSE_USE_PLAN_ORDER else [None]
            heads = [e.sink.sorted_heads() for e, *_ in todo] if SPARSE_USE_PLAN_HEADS else [None]
            ordered = all(o is not None for o in orders)
            F.sparse_adagrad_multi([t[0].weight.data for t in todo], [t[1] for t in todo], [t[2] for t in todo],
                                   [t[3] for t in todo], self.iterations, s.initial_learning_rate, s.decay_rate,
                                   s.decay_steps, self.clipnorm, self.epsilon,
                                   sumsq=[t[4] for t in todo] if all(with_ssq) else None, increment=True,
                                   orders=orders if ordered else None,
                                   heads=heads if ordered and all(h is not None for h in heads) else None)
        else:
            for e, acc, ids, rows, ssq in todo:
                F.sparse_adagrad(e.weight.data, acc, ids, rows, self.iterations, s.initial_learning_rate,
                                 s.decay_rate, s.decay_steps, self.clipnorm, self.epsilon, sumsq=ssq)
            F.iteration_increment(self.iterations)

    def state_dict(self):
        return {"iterations": self.iterations.clone(), "accum": [a.clone() for a in self.accum],
                "emb_accum": [a.clone() for a in self.emb_accum]}

    def load_state_dict(self, st):
        self.iterations.copy_(st["iterations"])
        for a, b in zip(self.accum, st["accum"]):
            a.copy_(b)
        for a, b in zip(self.emb_accum, st["emb_accum"]):
            a.copy_(b)
