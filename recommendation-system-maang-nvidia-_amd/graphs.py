"""Whole-training-step hipGraph capture (the MI355X replacement for tf.function tracing).

A training step of the reference model is ~70 small kernel launches (towers, cross, heads,
losses, two in-batch passes, ~30 optimizer launches); at the ML-1M batch (4096) the host issue
cost of eager launches is comparable to the GPU work. ``GraphedTrainStep`` captures forward,
backward and the Adagrad update of one step into a single hipGraph and replays it with new
inputs copied into static buffers. Semantics are unchanged: the first call runs eagerly (a real
step, also loading every kernel's code object), the capture records without executing, and
every replay is exactly one more step (the iteration counter and learning rate live on the
device). Single-process only (the data-parallel exchange is not captured).
"""
from __future__ import annotations

from typing import Callable, Dict, Tuple

import torch


def _clone_batch(batch):
    feats, labels = batch
    return ({k: v.clone() for k, v in feats.items()}, {k: v.clone() for k, v in labels.items()})


def _detach(out):
    """Drop autograd history from a step's outputs: a live autograd graph from the eager step
    keeps AccumulateGrad nodes bound to the previous stream and invalidates the capture."""
    if isinstance(out, torch.Tensor):
        return out.detach()
    if isinstance(out, dict):
        return {k: _detach(v) for k, v in out.items()}
    if isinstance(out, (tuple, list)):
        return type(out)(_detach(v) for v in out)
    return out


def _copy_into(dst, src):
    for k, v in src[0].items():
        dst[0][k].copy_(v, non_blocking=True)
    for k, v in src[1].items():
        dst[1][k].copy_(v, non_blocking=True)


class GraphedTrainStep:
    def __init__(self, step_fn: Callable, example_batch: Tuple[Dict, Dict]):
        self.step_fn = step_fn
        self.static = _clone_batch(example_batch)
        self.graph = None
        self.out = None

    def _capture(self):
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        torch.cuda.current_stream().wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, stream=side):
            self.out = _detach(self.step_fn(self.static))
        torch.cuda.current_stream().wait_stream(side)

    def __call__(self, batch):
        if self.graph is None:
            # eager first step: a real training step that also warms every code object
            _copy_into(self.static, batch)
            out = _detach(self.step_fn(self.static))
            torch.cuda.synchronize()
            self._capture()
            return out
        if batch[0]["user_id"].shape != self.static[0]["user_id"].shape:
            return _detach(self.step_fn(batch))  # ragged last batch: run it eagerly
        _copy_into(self.static, batch)
        self.graph.replay()
        return self.out
