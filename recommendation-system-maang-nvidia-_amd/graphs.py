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


def _fields(batch):
    return [v for part in batch for v in part.values()]


class PackedBatch(tuple):
    """A (features, labels) batch made by ``pack_batch``: every field a view of one storage that
    holds nothing else (its byte size is the padded sum of the field sizes)."""

    packed_nbytes = 0


def _packed_layout(fs):
    offs, total = [], 0
    for f in fs:
        offs.append(total)
        total += (f.numel() * f.element_size() + 15) // 16 * 16
    return offs, total


def _packed_storage(batch):
    """The storage a ``pack_batch`` batch owns, else None. Only batches tagged by pack_batch
    qualify: fields that merely share a storage (e.g. slices of one preloaded dataset tensor)
    would make a static copy — and every replay's memcpy — the size of the whole storage."""
    if not isinstance(batch, PackedBatch):
        return None
    fs = _fields(batch)
    if not fs or not all(f.is_contiguous() for f in fs):
        return None
    st = fs[0].untyped_storage()
    if any(f.untyped_storage().data_ptr() != st.data_ptr() for f in fs):
        return None
    if st.nbytes() != batch.packed_nbytes or _packed_layout(fs)[1] != batch.packed_nbytes:
        return None
    return st


def _tag(parts, nbytes):
    out = PackedBatch(parts)
    out.packed_nbytes = nbytes
    return out


def _clone_batch(batch):
    """Static input buffers. A packed example batch (every field a view of one storage, as
    ``pack_batch`` makes) gets a packed static copy with the same layout, so a replay's input
    copy is one memcpy instead of one per field."""
    st = _packed_storage(batch)
    if st is not None:
        buf = torch.empty(st.nbytes(), dtype=torch.uint8, device=_fields(batch)[0].device)
        out = []
        for part in batch:
            d = {}
            for k, v in part.items():
                d[k] = torch.empty(0, dtype=v.dtype, device=v.device).set_(
                    buf.untyped_storage(), v.storage_offset(), v.shape, v.stride())
            out.append(d)
        return _tag(out, batch.packed_nbytes)
    feats, labels = batch
    return ({k: v.clone() for k, v in feats.items()}, {k: v.clone() for k, v in labels.items()})


def pack_batch(batch):
    """Copy a (features, labels) batch of device tensors into one storage (fields become views,
    16-B aligned), so graph replays copy it with a single memcpy."""
    fs = _fields(batch)
    offs, total = _packed_layout(fs)
    buf = torch.empty(total, dtype=torch.uint8, device=fs[0].device)
    out, i = [], 0
    for part in batch:
        d = {}
        for k, v in part.items():
            t = torch.empty(0, dtype=v.dtype, device=v.device).set_(
                buf.untyped_storage(), offs[i] // v.element_size(), v.shape, v.contiguous().stride())
            t.copy_(v)
            d[k] = t
            i += 1
        out.append(d)
    return _tag(out, total)


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


def _same_fields(dst, src):
    for pd, ps in zip(dst, src):
        if list(pd) != list(ps):
            return False
        for k in pd:
            a, b = pd[k], ps[k]
            if a.dtype != b.dtype or a.shape != b.shape or a.storage_offset() != b.storage_offset():
                return False
    return True


def _copy_into(dst, src):
    sd, ss = _packed_storage(dst), _packed_storage(src)
    if sd is not None and ss is not None and sd.nbytes() == ss.nbytes() and _same_fields(dst, src):
        torch.empty(0, dtype=torch.uint8, device=_fields(dst)[0].device).set_(sd).copy_(
            torch.empty(0, dtype=torch.uint8, device=_fields(src)[0].device).set_(ss), non_blocking=True)
        return
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
