"""Tensor-level wrappers over the C-ABI and the autograd Functions of the hot path.

Every op here launches hand-written gfx950 kernels from librecsys_hip.so on the current
PyTorch (HIP) stream; PyTorch only supplies device memory, streams and autograd plumbing.
Inputs must be contiguous float32 (int64 for ids) tensors on a ROCm device; anything else
raises — there is no CPU or eager fallback.
"""
from __future__ import annotations

import contextlib
import ctypes
import weakref
from typing import List, Optional, Sequence, Tuple

import torch

from . import _native
from ._native import call, query

_VP = ctypes.c_void_p


# --------------------------------------------------------------------------------------------
# plumbing
# --------------------------------------------------------------------------------------------
def _p(t: Optional[torch.Tensor]):
    return _VP(t.data_ptr()) if t is not None else _VP(0)


def _stream():
    return _VP(torch.cuda.current_stream().cuda_stream)


def _dev(t: torch.Tensor, name: str, dtype=torch.float32) -> torch.Tensor:
    if not t.is_cuda:
        raise RuntimeError(f"{name}: expected a ROCm device tensor, got {t.device} "
                           "(the hot path has no CPU implementation)")
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: expected a contiguous tensor")
    return t


def _ws(nbytes: int, device) -> torch.Tensor:
    return torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=device)


class ReductionQueue:
    """A caller-owned deferred-reduction queue (include/recsys_hip.h rs_reduction_queue_*): while
    open, the ops that end in an ordered parameter-gradient reduction (gemm_wgrad_bias[_group],
    relu_bwd_colsum, dcn_cross_bwd, heads_bwd) append their second stage to it instead of launching
    it, and flush() runs them all in one launch (bitwise the same sums). The queue is host memory
    owned here, so two training loops (two optimizers) never share jobs. It also keeps the storages
    of every workspace, addend and output of a queued job until the flush (storages, not tensors: an
    extra reference to a returned gradient would make AccumulateGrad copy it before it is written)."""

    def __init__(self):
        n = query("rs_reduction_queue_bytes")
        self._buf = (ctypes.c_uint64 * ((n + 7) // 8))()   # 8-byte aligned host memory
        call("rs_reduction_queue_init", ctypes.addressof(self._buf), ctypes.sizeof(self._buf))
        self._keep: list = []
        self.active = False

    @property
    def handle(self):
        return _VP(ctypes.addressof(self._buf))

    def pending(self) -> int:
        return query("rs_reduction_queue_pending", self.handle)

    def open(self):
        """Start queueing (jobs left from an aborted step are launched first)."""
        self.flush()
        self.active = True

    def keep(self, *ts):
        self._keep.extend(t.untyped_storage() for t in ts if t is not None)

    def flush(self):
        """Launch every queued reduction (one kernel on the current stream) and stop queueing; the
        kept storages go back to the caching allocator behind that launch."""
        if self.pending():
            call("rs_reduction_queue_flush", self.handle, _stream())
        self._keep = []
        self.active = False


def _queue_of(param) -> Optional[ReductionQueue]:
    """The queue an optimizer attached to a parameter it owns (optim.Adagrad(defer_reductions=True)),
    or None: the forward of a node records it, its backward queues into it while it is open. The
    parameter holds only a weak reference: a dropped optimizer's queue is never used again."""
    ref = getattr(param, "_rs_reduction_queue", None)
    return ref() if ref is not None else None


def attach_reduction_queue(params, queue: Optional[ReductionQueue]) -> None:
    """Make `queue` (or no queue) the one the backward of `params` defers into. A queue another
    optimizer attached before is flushed and closed first (its pending jobs launched), so a
    replaced or abandoned deferring optimizer can never hold back this one's gradients."""
    ref = weakref.ref(queue) if queue is not None else None
    for p in params:
        old = _queue_of(p)
        if old is not None and old is not queue:
            old.flush()
        if ref is not None:
            p._rs_reduction_queue = ref
        elif hasattr(p, "_rs_reduction_queue"):
            del p._rs_reduction_queue


def _q(queue: Optional[ReductionQueue]):
    """(queue to append to or None, its C handle or NULL)."""
    if queue is not None and queue.active:
        return queue, queue.handle
    return None, _VP(0)


_SEEDS = {}


def backward_seed(t: torch.Tensor) -> torch.Tensor:
    """A cached 1.0 of t's shape / dtype / device for t.backward(seed): the implicit seed is a fresh
    ones_like (one fill launch per step); this one is made once (before any graph capture)."""
    key = (t.device, t.dtype, tuple(t.shape))
    seed = _SEEDS.get(key)
    if seed is None:
        seed = _SEEDS[key] = torch.ones_like(t)
    return seed


# --------------------------------------------------------------------------------------------
# raw ops (no autograd)
# --------------------------------------------------------------------------------------------
def embedding_gather(table: torch.Tensor, ids: torch.Tensor, bad_ids: Optional[torch.Tensor] = None):
    """Embedding row gather (src/models.py:71,74) -> [n, D]."""
    _dev(table, "table")
    _dev(ids, "ids", torch.int64)
    n, D = ids.numel(), table.shape[1]
    out = torch.empty((n, D), dtype=torch.float32, device=table.device)
    call("rs_embedding_gather_f32", _p(table), table.shape[0], D, _p(ids), n, _p(out), _p(bad_ids), _stream())
    return out


def embedding_gather_tables(tables: Sequence[torch.Tensor], ids: Sequence[torch.Tensor], orders=None):
    """The lookups of several same-width tables in one launch (rs_embedding_gather_tables_f32)
    -> list of [n_j, D]. orders (int32 [n_j] per table, e.g. the id plan's ascending-id row
    orders): the rows are copied in that order (rs_embedding_gather_tables_ordered_f32), the same
    result."""
    k = len(tables)
    if k != len(ids) or k > 8:
        raise ValueError("embedding_gather_tables: 1..8 (table, ids) pairs")
    D = tables[0].shape[1]
    outs = []
    for t, i in zip(tables, ids):
        _dev(t, "table")
        _dev(i, "ids", torch.int64)
        if t.shape[1] != D:
            raise ValueError("embedding_gather_tables: tables must share one width")
        outs.append(torch.empty((i.numel(), D), dtype=torch.float32, device=t.device))
    arr_p = (_VP * k)(*[t.data_ptr() for t in tables])
    arr_r = (ctypes.c_int64 * k)(*[t.shape[0] for t in tables])
    arr_i = (_VP * k)(*[i.data_ptr() for i in ids])
    arr_n = (ctypes.c_int64 * k)(*[i.numel() for i in ids])
    arr_o = (_VP * k)(*[o.data_ptr() for o in outs])
    if orders is not None:
        for o, i in zip(orders, ids):
            if o is not None and (_dev(o, "order", torch.int32).numel() != i.numel()):
                raise ValueError("embedding_gather_tables: an order must list every row")
        arr_q = (_VP * k)(*[o.data_ptr() if o is not None else 0 for o in orders])
        call("rs_embedding_gather_tables_ordered_f32", k, ctypes.cast(arr_p, _VP), ctypes.cast(arr_r, _VP),
             ctypes.cast(arr_i, _VP), ctypes.cast(arr_q, _VP), ctypes.cast(arr_n, _VP), ctypes.cast(arr_o, _VP), D,
             _VP(0), _stream())
        return outs
    call("rs_embedding_gather_tables_f32", k, ctypes.cast(arr_p, _VP), ctypes.cast(arr_r, _VP),
         ctypes.cast(arr_i, _VP), ctypes.cast(arr_n, _VP), ctypes.cast(arr_o, _VP), D, _VP(0), _stream())
    return outs


GATHER_ROWS_DIMS = (32, 64, 128)   # the widths rs_embedding_gather_tables_rows_f32 is compiled for


def embedding_gather_tables_rows(tables: Sequence[torch.Tensor], ids: Sequence[torch.Tensor],
                                 reps: Sequence[torch.Tensor], counts: Sequence[torch.Tensor]):
    """The lookups over each table's distinct ids (rs_embedding_gather_tables_rows_f32): out_j[p] =
    table_j[ids_j[reps_j[p]]] for p below the device count counts_j (int64 [1]); rows past it unset."""
    k = len(tables)
    D = tables[0].shape[1]
    outs = []
    for t, i, r, c in zip(tables, ids, reps, counts):
        _dev(t, "table"), _dev(i, "ids", torch.int64), _dev(r, "reps", torch.int32), _dev(c, "counts", torch.int64)
        if t.shape[1] != D:
            raise ValueError("embedding_gather_tables_rows: tables must share one width")
        outs.append(torch.empty((i.numel(), D), dtype=torch.float32, device=t.device))
    arr = [(_VP * k)(*[t.data_ptr() for t in ts]) for ts in (tables, ids, reps, counts, outs)]
    arr_r = (ctypes.c_int64 * k)(*[t.shape[0] for t in tables])
    arr_n = (ctypes.c_int64 * k)(*[i.numel() for i in ids])
    call("rs_embedding_gather_tables_rows_f32", k, ctypes.cast(arr[0], _VP), ctypes.cast(arr_r, _VP),
         ctypes.cast(arr[1], _VP), ctypes.cast(arr[2], _VP), ctypes.cast(arr[3], _VP), ctypes.cast(arr_n, _VP),
         ctypes.cast(arr[4], _VP), D, _VP(0), _stream())
    return outs


def merge_runs_order(ids: torch.Tensor, run_offsets: Sequence[int]) -> torch.Tensor:
    """The stable ascending order (int32) of runs of ids concatenated, each run ascending without
    repeats (rs_merge_runs_order_i64): the permutation a stable sort gives, from binary searches."""
    _dev(ids, "ids", torch.int64)
    offs = [int(o) for o in run_offsets]
    if offs[0] != 0 or offs[-1] != ids.numel():
        raise ValueError("merge_runs_order: run offsets must span the ids")
    order = torch.empty((ids.numel(),), dtype=torch.int32, device=ids.device)
    arr = (ctypes.c_int64 * len(offs))(*offs)
    call("rs_merge_runs_order_i64", _p(ids), ctypes.cast(arr, _VP), len(offs) - 1, _p(order), _stream())
    return order


def embedding_gather_tables_ids(tables: Sequence[torch.Tensor], dids: Sequence[torch.Tensor], out=None):
    """The lookups straight from an id plan's distinct ids (rs_embedding_gather_tables_ids_f32):
    out_j[p] = table_j[dids_j[p]] where dids_j[p] >= 0 (a slot of the plan), rows past the plan's
    count (dids -1) unset; ids >= the table's rows give zero rows. out: preallocated [n_j, D] outputs."""
    k = len(tables)
    D = tables[0].shape[1]
    outs = []
    for j, (t, d) in enumerate(zip(tables, dids)):
        _dev(t, "table"), _dev(d, "dids", torch.int64)
        if t.shape[1] != D:
            raise ValueError("embedding_gather_tables_ids: tables must share one width")
        if out is not None:
            o = _dev(out[j], "out")
            if tuple(o.shape) != (d.numel(), D) or not o.is_contiguous():
                raise ValueError("embedding_gather_tables_ids: out must be contiguous [n, D]")
            outs.append(o)
        else:
            outs.append(torch.empty((d.numel(), D), dtype=torch.float32, device=t.device))
    arr = [(_VP * k)(*[t.data_ptr() for t in ts]) for ts in (tables, dids, outs)]
    arr_r = (ctypes.c_int64 * k)(*[t.shape[0] for t in tables])
    arr_n = (ctypes.c_int64 * k)(*[d.numel() for d in dids])
    call("rs_embedding_gather_tables_ids_f32", k, ctypes.cast(arr[0], _VP), ctypes.cast(arr_r, _VP),
         ctypes.cast(arr[1], _VP), ctypes.cast(arr_n, _VP), ctypes.cast(arr[2], _VP), D, _VP(0), _stream())
    return outs


def sparse_adagrad(table, accum, ids, rows, iteration, lr0, decay_rate=0.96, decay_steps=1000,
                   clipnorm=1.0, epsilon=1e-7, sumsq: Optional[torch.Tensor] = None):
    """Clip (over the raw rows) + dedupe + Adagrad row update, in place (src/trainer.py:157-163).
    ``rows`` may be a row-strided view (unit column stride), e.g. a column slice of dLoss/dx0.
    ``sumsq`` (device fp32 scalar): the clip norm^2 when the rows are not the raw ones (the
    data-parallel exchange's deduplicated rows, rs_sparse_adagrad_sumsq_f32)."""
    _dev(table, "table"), _dev(accum, "accum"), _dev(ids, "ids", torch.int64)
    _dev(iteration, "iteration", torch.int64)
    n, D = ids.numel(), table.shape[1]
    if n == 0:
        return
    if not rows.is_cuda or rows.dtype != torch.float32 or rows.dim() != 2 or rows.stride(1) != 1:
        raise ValueError("rows: expected a [n, D] fp32 device tensor with unit column stride")
    wsb = query("rs_sparse_adagrad_workspace_bytes", n, D, table.shape[0])
    ws = _ws(wsb, table.device)
    if sumsq is not None:
        call("rs_sparse_adagrad_sumsq_f32", _p(table), _p(accum), table.shape[0], D, _p(ids), _p(rows),
             rows.stride(0), n, _p(_dev(sumsq, "sumsq")), _p(iteration), float(lr0), float(decay_rate),
             int(decay_steps), float(clipnorm or 0.0), float(epsilon), _p(ws), ws.numel(), _stream())
        return
    call("rs_sparse_adagrad_ld_f32", _p(table), _p(accum), table.shape[0], D, _p(ids), _p(rows), rows.stride(0),
         n, _p(iteration), float(lr0), float(decay_rate), int(decay_steps), float(clipnorm or 0.0),
         float(epsilon), _p(ws), ws.numel(), _stream())


SPARSE_MULTI_MAX = 32  # tables per rs_sparse_adagrad_multi_f32 call


def sparse_adagrad_multi(tables, accums, ids, rows, iteration, lr0, decay_rate=0.96, decay_steps=1000,
                         clipnorm=1.0, epsilon=1e-7, sumsq: Optional[Sequence[torch.Tensor]] = None,
                         increment: bool = False, orders: Optional[Sequence[torch.Tensor]] = None,
                         heads: Optional[Sequence[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]]] = None):
    """sparse_adagrad over several tables of one width in one launch sequence per 32 tables (one
    sort, clip-norm, fragment and apply pass for all of them; rs_sparse_adagrad_multi_f32). Each
    table's update is bitwise its sparse_adagrad when all tables have the same row count.
    increment: also advance the step counter `iteration` once every table is updated (the last
    sequence's apply pass does it: rs_sparse_adagrad_multi_step_f32, no iteration_increment launch).
    orders (with increment, one sequence): each table's positions in stable ascending-id order (the
    in-batch id plan's order entries): the update skips its own sort
    (rs_sparse_adagrad_multi_step_ordered_f32; bitwise the same result). heads (with orders): per
    table the plan's (starts int32, distinct ids int64, distinct count int64 [1]) — the apply pass runs
    one slice per distinct id (rs_sparse_adagrad_multi_step_planned_f32; bitwise the same result)."""
    nt = len(tables)
    if not (len(accums) == len(ids) == len(rows) == nt) or (sumsq is not None and len(sumsq) != nt):
        raise ValueError("sparse_adagrad_multi: one accum, ids, rows (and sumsq) per table")
    if nt == 0:
        return
    _dev(iteration, "iteration", torch.int64)
    D = tables[0].shape[1]
    for k in range(nt):
        _dev(tables[k], f"tables[{k}]"), _dev(accums[k], f"accums[{k}]"), _dev(ids[k], f"ids[{k}]", torch.int64)
        r = rows[k]
        if (not r.is_cuda or r.dtype != torch.float32 or r.dim() != 2 or r.shape[1] != D
                or (r.stride(1) != 1 and r.numel() > 0)):
            raise ValueError(f"rows[{k}]: expected a [n, {D}] fp32 device tensor with unit column stride")
        if tables[k].shape[1] != D:
            raise ValueError("sparse_adagrad_multi: all tables must have the same width")
        if sumsq is not None:
            _dev(sumsq[k], f"sumsq[{k}]")
    for c0 in range(0, nt, SPARSE_MULTI_MAX):
        ks = range(c0, min(nt, c0 + SPARSE_MULTI_MAX))
        m = len(ks)
        P = ctypes.c_void_p * m
        I = ctypes.c_int64 * m
        n = I(*[ids[k].numel() for k in ks])
        ws = _ws(query("rs_sparse_adagrad_multi_workspace_bytes", m, ctypes.addressof(n), D), tables[0].device)
        arrs = (P(*[tables[k].data_ptr() for k in ks]), P(*[accums[k].data_ptr() for k in ks]),
                I(*[tables[k].shape[0] for k in ks]), P(*[ids[k].data_ptr() for k in ks]),
                P(*[rows[k].data_ptr() for k in ks]), I(*[max(rows[k].stride(0), D) for k in ks]))
        ssq = P(*[sumsq[k].data_ptr() for k in ks]) if sumsq is not None else None
        last = c0 + SPARSE_MULTI_MAX >= nt
        if orders is not None and increment and nt <= SPARSE_MULTI_MAX:
            for k in ks:
                _dev(orders[k], f"orders[{k}]", torch.int32)
                if orders[k].numel() != ids[k].numel():
                    raise ValueError(f"orders[{k}]: one entry per id")
            op = P(*[orders[k].data_ptr() for k in ks])
            common = (m, ctypes.addressof(arrs[0]), ctypes.addressof(arrs[1]), ctypes.addressof(arrs[2]), D,
                      ctypes.addressof(arrs[3]), ctypes.addressof(arrs[4]), ctypes.addressof(arrs[5]),
                      ctypes.addressof(n), ctypes.addressof(ssq) if ssq is not None else None, _p(iteration),
                      float(lr0), float(decay_rate), int(decay_steps), float(clipnorm or 0.0), float(epsilon),
                      ctypes.addressof(op))
            if heads is not None and all(h is not None for h in heads):
                for k in ks:
                    st, dd, cnt = heads[k]
                    _dev(st, f"heads[{k}] starts", torch.int32), _dev(dd, f"heads[{k}] ids", torch.int64)
                    _dev(cnt, f"heads[{k}] count", torch.int64)
                    if st.numel() < ids[k].numel() or dd.numel() < ids[k].numel():
                        raise ValueError(f"heads[{k}]: one start and id slot per id")
                hs = (P(*[heads[k][0].data_ptr() for k in ks]), P(*[heads[k][1].data_ptr() for k in ks]),
                      P(*[heads[k][2].data_ptr() for k in ks]))
                call("rs_sparse_adagrad_multi_step_planned_f32", *common, *[ctypes.addressof(h) for h in hs],
                     _p(ws), ws.numel(), _stream())
            else:
                call("rs_sparse_adagrad_multi_step_ordered_f32", *common, _p(ws), ws.numel(), _stream())
            continue
        call("rs_sparse_adagrad_multi_step_f32" if increment and last else "rs_sparse_adagrad_multi_f32", m, ctypes.addressof(arrs[0]), ctypes.addressof(arrs[1]),
             ctypes.addressof(arrs[2]), D, ctypes.addressof(arrs[3]), ctypes.addressof(arrs[4]),
             ctypes.addressof(arrs[5]), ctypes.addressof(n), ctypes.addressof(ssq) if ssq is not None else None,
             _p(iteration), float(lr0), float(decay_rate), int(decay_steps), float(clipnorm or 0.0),
             float(epsilon), _p(ws), ws.numel(), _stream())


def sparse_dedupe(ids: torch.Tensor, rows: torch.Tensor, num_rows: int, want_sumsq: bool = True, plan=None):
    """Locally deduplicated IndexedSlices -> (unique ids [n] (valid prefix), summed rows [n, D],
    count int64 0-dim, raw sum of squares fp32 0-dim or None), all on the device. plan = (order,
    starts, distinct ids, distinct count [1]) of an id plan of these ids: no sort
    (rs_sparse_dedupe_planned_f32, bitwise the same outputs)."""
    _dev(ids, "ids", torch.int64)
    if not rows.is_cuda or rows.dtype != torch.float32 or rows.dim() != 2 or rows.stride(1) != 1:
        raise ValueError("rows: expected a [n, D] fp32 device tensor with unit column stride")
    n, D = ids.numel(), rows.shape[1]
    out_ids = torch.empty((max(n, 1),), dtype=torch.int64, device=ids.device)
    out_rows = torch.empty((max(n, 1), D), dtype=torch.float32, device=ids.device)
    count = torch.empty((), dtype=torch.int64, device=ids.device)
    sumsq = torch.empty((), dtype=torch.float32, device=ids.device) if want_sumsq else None
    ws = _ws(query("rs_sparse_dedupe_workspace_bytes", max(n, 1), D, int(num_rows)), ids.device)
    if plan is not None and D in (32, 64, 128, 256):
        order, starts, dids, nslots = plan
        _dev(order, "order", torch.int32), _dev(starts, "starts", torch.int32), _dev(dids, "dids", torch.int64)
        _dev(nslots, "nslots", torch.int64)
        if order.numel() != n or starts.numel() < n or dids.numel() < n:
            raise ValueError("sparse_dedupe: the plan must cover these ids")
        call("rs_sparse_dedupe_planned_f32", _p(ids), _p(rows), rows.stride(0), n, int(num_rows), D, _p(order),
             _p(starts), _p(dids), _p(nslots), _p(out_ids), _p(out_rows), _p(count), _p(sumsq), _p(ws), ws.numel(),
             _stream())
    else:
        call("rs_sparse_dedupe_f32", _p(ids), _p(rows), rows.stride(0), n, int(num_rows), D, _p(out_ids),
             _p(out_rows), _p(count), _p(sumsq), _p(ws), ws.numel(), _stream())
    return out_ids, out_rows, count, sumsq


def multi_embedding_gather(table_ptrs, num_rows, E, ids, dense, ld, bad_ids=None):
    """Config-5 feature assembly: x0 [B, ld] = [emb_0 || ... || emb_{F-1} || dense || 0]."""
    _dev(ids, "ids", torch.int64)
    F_, B = ids.shape
    nd = dense.shape[1] if dense is not None else 0
    if dense is not None:
        _dev(dense, "dense")
    x0 = torch.empty((B, ld), dtype=torch.float32, device=ids.device)
    call("rs_multi_embedding_gather_f32", _p(table_ptrs), _p(num_rows), F_, int(E), _p(ids), B, _p(dense), nd,
         _p(x0), int(ld), _p(bad_ids), _stream())
    return x0


def dcn_cross_mat_fwd(x0, W, b, precision: int = 0):
    _dev(x0, "x0"), _dev(W, "W"), _dev(b, "b")
    B, d = x0.shape
    L = W.shape[0]
    xs = torch.empty((max(L, 1), B, d), dtype=torch.float32, device=x0.device)
    us = torch.empty_like(xs)
    call("rs_dcn_cross_mat_fwd_prec_f32", _p(x0), B, d, L, _p(W), _p(b), _p(xs), _p(us), int(precision), _stream())
    return xs, us


def dcn_cross_mat_fwd_planes(x0, W, b, precision: int = 6, want_x0_img: bool = False):
    """Plane-image path (precision 6): returns (xs, us, ximg); ximg (the images of x_0^T ..
    x_{L-1}^T) goes to dcn_cross_mat_bwd_planes. want_x0_img: also x0's xgemm image (4th item)."""
    _dev(x0, "x0"), _dev(W, "W"), _dev(b, "b")
    B, d = x0.shape
    L = W.shape[0]
    xs = torch.empty((max(L, 1), B, d), dtype=torch.float32, device=x0.device)
    us = torch.empty_like(xs)
    ximg = _ws(query("rs_dcn_cross_mat_planes_bytes", B, d, L), x0.device)
    ws = _ws(query("rs_dcn_cross_mat_fwd_planes_workspace_bytes", B, d), x0.device)
    x0_img = (torch.empty((query("rs_xgemm_image_bytes", B, d),), dtype=torch.uint8, device=x0.device)
              if want_x0_img else None)
    call("rs_dcn_cross_mat_fwd_planes_x0img_f32", _p(x0), B, d, L, _p(W), _p(b), _p(xs), _p(us), _p(ximg),
         _p(x0_img), int(precision), _p(ws), ws.numel(), _stream())
    return (xs, us, ximg, x0_img) if want_x0_img else (xs, us, ximg)


def dcn_cross_mat_bwd_planes(x0, xs, us, W, ximg, g_xl, g_x0_extra=None, precision: int = 6):
    B, d = x0.shape
    L = W.shape[0]
    g_x0 = torch.empty_like(x0)
    gW = torch.empty_like(W)
    gb = torch.empty((L, d), dtype=torch.float32, device=x0.device)
    ws = _ws(max(query("rs_dcn_cross_mat_bwd_planes_workspace_bytes", B, d, L),
                 query("rs_dcn_cross_mat_bwd_workspace_bytes", B, d, L)), x0.device)
    call("rs_dcn_cross_mat_bwd_planes_f32", _p(x0), _p(xs), _p(us), _p(W), _p(ximg), B, d, L,
         _p(_dev(g_xl, "g_xl")), _p(g_x0_extra), _p(g_x0), _p(gW), _p(gb), int(precision), _p(ws), ws.numel(),
         _stream())
    return g_x0, gW, gb


def dcn_cross_mat_bwd(x0, xs, us, W, g_xl, g_x0_extra=None, precision: int = 0):
    B, d = x0.shape
    L = W.shape[0]
    g_x0 = torch.empty_like(x0)
    gW = torch.empty_like(W)
    gb = torch.empty((L, d), dtype=torch.float32, device=x0.device)
    ws = _ws(query("rs_dcn_cross_mat_bwd_workspace_bytes", B, d, L), x0.device)
    call("rs_dcn_cross_mat_bwd_prec_f32", _p(x0), _p(xs), _p(us), _p(W), B, d, L, _p(_dev(g_xl, "g_xl")),
         _p(g_x0_extra), _p(g_x0), _p(gW), _p(gb), int(precision), _p(ws), ws.numel(), _stream())
    return g_x0, gW, gb


def gemm(a, b, trans_a=False, trans_b=False, bias=None, relu=False, mask=None, out=None, beta=0.0,
         precision: int = 0):
    """out = epilogue(op(a) @ op(b)) (row-major, contiguous); `precision` = contraction precision
    (PREC_F32: f32 MFMA; PREC_F32_SPLIT6 / 9: exact bf16 splits on the bf16 MFMA)."""
    _dev(a, "a"), _dev(b, "b")
    M = a.shape[1] if trans_a else a.shape[0]
    K = a.shape[0] if trans_a else a.shape[1]
    N = b.shape[0] if trans_b else b.shape[1]
    Kb = b.shape[1] if trans_b else b.shape[0]
    if K != Kb:
        raise ValueError(f"gemm: inner dims differ ({K} vs {Kb})")
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=a.device)
    if bias is not None:
        _dev(bias, "bias")
    if mask is not None:
        _dev(mask, "mask")
    call("rs_gemm_prec_f32", int(trans_a), int(trans_b), M, N, K, _p(a), a.shape[1], _p(b), b.shape[1],
         _p(out), N, _p(bias), 1 if relu else 0, _p(mask), N if mask is not None else 0, float(beta),
         int(precision), _stream())
    return out


def gemm_splitk(a, b, trans_a=True, trans_b=False, addend=None, addend_scale=0.0, precision: int = 0):
    """C = op(a) @ op(b) (+ addend_scale*addend) with a batch-sized reduction (weight grads)."""
    _dev(a, "a"), _dev(b, "b")
    M = a.shape[1] if trans_a else a.shape[0]
    K = a.shape[0] if trans_a else a.shape[1]
    N = b.shape[0] if trans_b else b.shape[1]
    out = torch.empty((M, N), dtype=torch.float32, device=a.device)
    ws = _ws(query("rs_gemm_splitk_workspace_bytes", M, N, K), a.device)
    call("rs_gemm_splitk_prec_f32", int(trans_a), int(trans_b), M, N, K, _p(a), a.shape[1], _p(b), b.shape[1],
         _p(out), N, _p(addend), float(addend_scale), int(precision), _p(ws), ws.numel(), _stream())
    return out


PLANE_KC, PLANE_KM = 0, 1   # plane-image layouts (rs_plane_image_f32): k = columns / k = rows


def plane_image(x: torch.Tensor, layout: int) -> torch.Tensor:
    """Pre-split bf16 plane image of an fp32 matrix for rs_gemm_planes_* (uint8 device tensor)."""
    _dev(x, "x")
    R, Cc = x.shape
    k_ext, ext = (Cc, R) if layout == PLANE_KC else (R, Cc)
    img = torch.empty((query("rs_plane_image_bytes", k_ext, ext),), dtype=torch.uint8, device=x.device)
    call("rs_plane_image_f32", _p(x), Cc, R, Cc, int(layout), _p(img), _stream())
    return img


def gemm_planes(a_img, b_img, M, N, K, trans_a=False, trans_b=False, bias=None, relu=False, out=None, beta=0.0,
                precision: int = 6):
    """out = act(op(A) op(B) + bias) + beta out from plane images (A: KC image of A, or KM image of
    A^T when trans_a; B: KM image of B, or KC image of B^T when trans_b)."""
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=a_img.device)
    call("rs_gemm_planes_prec_f32", int(trans_a), int(trans_b), M, N, K, _p(a_img), _p(b_img), _p(out), N,
         _p(bias), 1 if relu else 0, float(beta), int(precision), _stream())
    return out


def gemm_planes_splitk(a_img, b_img, M, N, K, trans_a=True, trans_b=False, addend=None, addend_scale=0.0,
                       precision: int = 6):
    out = torch.empty((M, N), dtype=torch.float32, device=a_img.device)
    ws = _ws(query("rs_gemm_planes_splitk_workspace_bytes", M, N, K), a_img.device)
    call("rs_gemm_planes_splitk_prec_f32", int(trans_a), int(trans_b), M, N, K, _p(a_img), _p(b_img), _p(out),
         _p(addend), float(addend_scale), int(precision), _p(ws), ws.numel(), _stream())
    return out


def xgemm_image(x: torch.Tensor, trans: bool = False) -> torch.Tensor:
    """xgemm image (three bf16 planes, 8 KB blocks) of x viewed as [rows][k]: x itself when not
    trans, x^T (x stored [k][rows]) when trans (rs_xgemm_image_f32)."""
    _dev(x, "x")
    if x.dim() != 2 or x.stride(1) != 1:
        raise ValueError("xgemm_image: a row-major 2-D tensor is required")
    rows, k = (x.shape[1], x.shape[0]) if trans else (x.shape[0], x.shape[1])
    img = torch.empty((query("rs_xgemm_image_bytes", rows, k),), dtype=torch.uint8, device=x.device)
    call("rs_xgemm_image_f32", _p(x), x.stride(0), rows, k, int(trans), _p(img), _stream())
    return img


def xgemm_image_dual(x: torch.Tensor, relu_y: Optional[torch.Tensor] = None, colsum: bool = False):
    """(image of x, image of x^T[, column sums]) from one read of x [rows][k] (rs_xgemm_image_dual_f32);
    with relu_y: of x * (relu_y > 0)."""
    _dev(x, "x")
    rows, k = x.shape
    img = torch.empty((query("rs_xgemm_image_bytes", rows, k),), dtype=torch.uint8, device=x.device)
    img_t = torch.empty((query("rs_xgemm_image_bytes", k, rows),), dtype=torch.uint8, device=x.device)
    cs = torch.empty((k,), dtype=torch.float32, device=x.device) if colsum else None
    ws = _ws(query("rs_xgemm_image_dual_workspace_bytes", rows, k), x.device)
    call("rs_xgemm_image_dual_f32", _p(x), _p(_dev(relu_y, "relu_y") if relu_y is not None else None), rows, k,
         _p(img), _p(img_t), _p(cs), _p(ws), ws.numel(), _stream())
    return img, img_t, cs


def xgemm(a_img, b_img, M, N, K, bias=None, relu=False, out=None, beta=0.0, precision: int = 6):
    """out = act(A B^T + bias) + beta out from xgemm images of A [M][K] and B [N][K]."""
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=a_img.device)
    call("rs_xgemm_prec_f32", M, N, K, _p(a_img), _p(b_img), _p(out), out.stride(0), _p(bias),
         1 if relu else 0, float(beta), int(precision), _stream())
    return out


def xgemm_splitk(a_img, b_img, M, N, K, addend=None, addend_scale=0.0, precision: int = 6):
    """A B^T (+ addend_scale addend) with the contraction split over workgroups (ordered slabs)."""
    out = torch.empty((M, N), dtype=torch.float32, device=a_img.device)
    ws = _ws(query("rs_xgemm_splitk_workspace_bytes", M, N, K), a_img.device)
    call("rs_xgemm_splitk_prec_f32", M, N, K, _p(a_img), _p(b_img), _p(out), _p(addend), float(addend_scale),
         int(precision), _p(ws), ws.numel(), _stream())
    return out


def gemm_wgrad_bias(x, g, precision: int = 0, W=None, w_scale: float = 0.0, w_dscale=None, queue=None):
    """(dW, db) = (x^T g [+ w_scale * w_dscale * W], column sums of g) in one split-K GEMM
    (rs_gemm_wgrad_bias_prec_f32: the bias gradient is the all-ones row appended to x^T; W adds
    the l2 regularizer gradient, w_dscale a device scalar). Views of one [in + 1, out] buffer.
    queue: a ReductionQueue that receives the reduction while open (else it launches now)."""
    _dev(x, "x")
    _dev(g, "g")
    K, M = x.shape
    N = g.shape[1]
    buf = torch.empty((M + 1, N), dtype=torch.float32, device=x.device)
    ws = _ws(query("rs_gemm_wgrad_bias_workspace_bytes", M, N, K), x.device)
    q, qh = _q(queue)
    call("rs_gemm_wgrad_bias_prec_f32", M, N, K, _p(x), x.stride(0), _p(g), g.stride(0), _p(buf), _p(W),
         float(w_scale), _p(w_dscale), int(precision), _p(ws), ws.numel(), _stream(), qh)
    if q is not None:
        q.keep(ws, W, w_dscale, buf)   # read / written by the queued reduction
    return buf[:M], buf[M]


def _ptrs(ts):
    arr = (_VP * len(ts))(*[t.data_ptr() if t is not None else 0 for t in ts])
    return arr, ctypes.cast(arr, _VP)


def gemm_group(a_list, b_list, trans_b=False, bias=None, relu=False, mask=None, precision: int = 0,
               b_img=None, mask_rows=None, m_dev=None, a_rows=None, m_rows=None):
    """[epilogue(a_g @ op(b_g)) for g] for 1..4 problems of one shape in one launch
    (rs_gemm_group_prec_f32; each result bitwise its gemm()). Views of one [G, M, N] buffer.
    b_img: per problem the device address of op(b_g)'s fragment image (mlp_layer_images), used by
    the large-batch skinny kernel (rs_gemm_group_img_prec_f32; bitwise the same results).
    mask_rows (int32 [M] per problem: the mask row of each output row), m_dev (a device int64
    per problem: the live row count, <= M; rows past it are left unwritten) and a_rows (int32 [M]
    per problem: the A row each output row reads; M = m_rows then): the distinct-row form
    (rs_gemm_group_rows_prec_f32, the weight-stationary kernel; same per-row arithmetic)."""
    G = len(a_list)
    for t in list(a_list) + list(b_list):
        _dev(t, "operand")
    M, K = a_list[0].shape
    if a_rows is not None:
        M = int(m_rows if m_rows is not None else a_rows[0].numel())
    N = b_list[0].shape[0] if trans_b else b_list[0].shape[1]
    for a, b in zip(a_list, b_list):
        if a.shape != a_list[0].shape or b.shape != b_list[0].shape:
            raise ValueError("gemm_group: all problems must have one shape")
    out = torch.empty((G, M, N), dtype=torch.float32, device=a_list[0].device)
    keep = [_ptrs(a_list), _ptrs(b_list), _ptrs([out[g] for g in range(G)])]
    if bias is not None:
        keep.append(_ptrs([_dev(t, "bias") for t in bias]))
    if mask is not None:
        keep.append(_ptrs([_dev(t, "mask") for t in mask]))
    args = (G, 0, int(trans_b), M, N, K, keep[0][1], a_list[0].shape[1], keep[1][1], b_list[0].shape[1],
            keep[2][1], N, keep[3][1] if bias is not None else None, 1 if relu else 0,
            keep[-1][1] if mask is not None else None, N if mask is not None else 0, 0.0, int(precision))
    if mask_rows is not None or m_dev is not None or a_rows is not None:
        rows = _ptrs([_dev(t, "mask_rows", torch.int32) for t in mask_rows]) if mask_rows is not None else None
        mdev = _ptrs([_dev(t, "m_dev", torch.int64) for t in m_dev]) if m_dev is not None else None
        arow = _ptrs([_dev(t, "a_rows", torch.int32) for t in a_rows]) if a_rows is not None else None
        call("rs_gemm_group_rows_prec_f32", G, int(trans_b), M, N, K, keep[0][1], a_list[0].shape[1],
             arow[1] if arow is not None else None, keep[1][1],
             b_list[0].shape[1], keep[2][1], N, keep[3][1] if bias is not None else None, 1 if relu else 0,
             keep[-1][1] if mask is not None else None, N if mask is not None else 0,
             rows[1] if rows is not None else None, mdev[1] if mdev is not None else None, int(precision),
             _stream())
    elif b_img is not None:
        arr = (_VP * G)(*b_img)
        call("rs_gemm_group_img_prec_f32", *args, ctypes.cast(arr, _VP), _stream())
    else:
        call("rs_gemm_group_prec_f32", *args, _stream())
    return [out[g] for g in range(G)]


# the large-batch Dense GEMMs read their weights from fragment images (one image launch per stack
# node per step; the skinny kernel then stages pre-split fragments). Module constants here are the
# product's kernel selection: only tests patch them (no environment reads)
SKINNY_IMG = True


def mlp_layer_images(imgs, dims):
    """Per layer l the (forward, chain) image addresses inside each stack's mlp_weight_image:
    returns fwd[l][s], chain[l][s] (ints)."""
    L = len(dims) - 1
    fwd, chain = [], []
    off = 0
    for l in range(L):
        nb = dims[l] * dims[l + 1] * 6
        fwd.append([im.data_ptr() + off for im in imgs])
        chain.append([im.data_ptr() + off + nb for im in imgs])
        off += 2 * nb
    return fwd, chain


# largest row count the one-launch stack forward serves (rs_mlp_fwd_prec_f32: a workgroup per 32
# rows carries them through every layer, so it fills the chip from ~8K rows per stack down; above
# that the per-layer GEMMs' larger tiles win). 0 turns it off.
MLP_FUSED_MAX_M = 16384


# largest row count the one-launch stack weight gradient serves when the forward / chain run per
# layer (rs_mlp_wgrad_prec_f32 alone: its 64 x 64 tiles x up to 16 row slices); 0 turns it off
MLP_WGRAD_MAX_M = MLP_FUSED_MAX_M


def mlp_fused_ok(M: int, K0: int, Ws, precision: int) -> bool:
    """Whether rs_mlp_fwd_prec_f32 takes this stack (see its header for the shape rules)."""
    if precision not in (PREC_F32_SPLIT6, PREC_F32_SPLIT9) or M > MLP_FUSED_MAX_M or not 1 <= len(Ws) <= 6:
        return False
    if K0 % 32 or not 32 <= K0 <= 256:
        return False
    k = K0
    for W in Ws:
        if W.dim() != 2 or W.shape[0] != k or W.shape[1] not in (64, 128, 256) or not W.is_contiguous():
            return False
        k = W.shape[1]
    return True


# stack-node images built ahead by prepare_mlp_images (one launch for every node of a step), each
# taken (popped) by the node whose weights it holds
_PREPARED_IMAGES = {}
MLP_PREPARE = True


def _image_key(W_lists):
    return tuple((W.data_ptr(), tuple(W.shape)) for Ws in W_lists for W in Ws)


def prepare_mlp_images(nodes):
    """The weight fragment images of several stack nodes (each a list of stacks, each a list of
    Dense kernels) in ONE launch (rs_mlp_weight_images_f32); mlp_weight_image then hands each node
    its own instead of launching. Images not taken by the next prepare are dropped."""
    _PREPARED_IMAGES.clear()
    Ks, Ns, Wp, dst, made = [], [], [], [], []
    for W_lists in nodes:
        L = len(W_lists[0])
        dims = (ctypes.c_int64 * (L + 1))(*[W_lists[0][l].shape[0] for l in range(L)], W_lists[0][L - 1].shape[1])
        nb = query("rs_mlp_weight_image_bytes", L, ctypes.cast(dims, _VP))
        imgs = [torch.empty(nb, dtype=torch.uint8, device=W_lists[0][0].device) for _ in W_lists]
        for Ws, img in zip(W_lists, imgs):
            off = 0
            for W in Ws:
                Ks.append(W.shape[0])
                Ns.append(W.shape[1])
                Wp.append(_dev(W, "W").data_ptr())
                dst.append(img.data_ptr() + off)
                off += 12 * W.shape[0] * W.shape[1]
        made.append((_image_key(W_lists), imgs))
    n = len(Ks)
    if n == 0 or 2 * n > 24:
        return
    arrs = ((ctypes.c_int64 * n)(*Ks), (ctypes.c_int64 * n)(*Ns), (_VP * n)(*Wp), (_VP * n)(*dst))
    call("rs_mlp_weight_images_f32", n, ctypes.cast(arrs[0], _VP), ctypes.cast(arrs[1], _VP),
         ctypes.cast(arrs[2], _VP), ctypes.cast(arrs[3], _VP), _stream())
    for key, imgs in made:
        _PREPARED_IMAGES[key] = imgs


def clear_prepared_images():
    _PREPARED_IMAGES.clear()


def mlp_weight_image(W_lists):
    """Each stack's weight fragment image (rs_mlp_weight_image_f32: every MFMA B fragment of W_l and
    of W_l^T pre-split, for the stack kernels' forward and chain) in one launch (or the one
    prepare_mlp_images built for these weights this step)."""
    ready = _PREPARED_IMAGES.pop(_image_key(W_lists), None)
    if ready is not None:
        return ready
    G, L = len(W_lists), len(W_lists[0])
    dims = (ctypes.c_int64 * (L + 1))(*[W_lists[0][l].shape[0] for l in range(L)], W_lists[0][L - 1].shape[1])
    nb = query("rs_mlp_weight_image_bytes", L, ctypes.cast(dims, _VP))
    dev = W_lists[0][0].device
    imgs = [torch.empty(nb, dtype=torch.uint8, device=dev) for _ in range(G)]
    Wf = [_dev(W_lists[s][l], "W") for s in range(G) for l in range(L)]
    keep = [_ptrs(Wf), _ptrs(imgs)]
    call("rs_mlp_weight_image_f32", G, L, ctypes.cast(dims, _VP), keep[0][1], keep[1][1], _stream())
    return imgs


def mlp_forward(x_list, W_lists, b_lists, relus, precision: int, img=None):
    """Every layer's output of G (1..2) Dense stacks of one architecture in ONE launch
    (rs_mlp_fwd_prec_f32, weights from `img` = mlp_weight_image(W_lists), built here when None):
    returns ys[l][g], layer l's views of one [G, M, N_l] buffer."""
    G, L = len(x_list), len(relus)
    M, K0 = x_list[0].shape
    if img is None:
        img = mlp_weight_image(W_lists)
    xs = [_dev(x, "x").contiguous() for x in x_list]
    dims = (ctypes.c_int64 * (L + 1))(K0, *[W_lists[0][l].shape[1] for l in range(L)])
    outs = [torch.empty((G, M, dims[l + 1]), dtype=torch.float32, device=xs[0].device) for l in range(L)]
    bf = [_dev(b_lists[g][l], "b") if b_lists[g][l] is not None else None for g in range(G) for l in range(L)]
    yf = [outs[l][g] for g in range(G) for l in range(L)]
    keep = [_ptrs(xs), _ptrs(img), _ptrs(bf), _ptrs(yf)]
    rl = (ctypes.c_int * L)(*[1 if r else 0 for r in relus])
    call("rs_mlp_fwd_prec_f32", G, L, ctypes.cast(dims, _VP), M, keep[0][1], keep[1][1], keep[2][1],
         ctypes.cast(rl, _VP), keep[3][1], int(precision), _stream())
    return [[outs[l][g] for g in range(G)] for l in range(L)]


def mlp_chain_ok(M: int, dims, precision: int, want_dx: bool) -> bool:
    """Whether rs_mlp_bwd_chain_prec_f32 takes this stack's input-gradient chain."""
    if precision not in (PREC_F32_SPLIT6, PREC_F32_SPLIT9) or M > MLP_FUSED_MAX_M or not 2 <= len(dims) <= 7:
        return False
    return all(d in (64, 128, 256) for d in dims[1:]) and (not want_dx or dims[0] in (64, 128, 256))


def mlp_backward_chain(g_tops, W_lists, y_lists, relus, precision: int, want_dx: bool, img=None):
    """The input-gradient chain of G (1..2) Dense stacks in ONE launch (rs_mlp_bwd_chain_prec_f32):
    g_tops[s] is dL/d(pre-activation of the top layer) (already masked by its ReLU), y_lists[s][l]
    layer l's forward output. Returns gin[l][s] = dL/d(input of layer l) as the weight gradient of
    layer l - 1 consumes it (masked by y_{l-1} > 0 when layer l - 1 has a ReLU); gin[0] = dL/dx
    (None unless want_dx). Weights from `img` (the forward's mlp_weight_image; built when None)."""
    G, L = len(g_tops), len(relus)
    if img is None:
        img = mlp_weight_image(W_lists)
    M = g_tops[0].shape[0]
    dims = (ctypes.c_int64 * (L + 1))(*[W_lists[0][l].shape[0] for l in range(L)], W_lists[0][L - 1].shape[1])
    gt = [_dev(t, "g_top").contiguous() for t in g_tops]
    outs = [torch.empty((G, M, dims[l]), dtype=torch.float32, device=gt[0].device) if (l > 0 or want_dx) else None
            for l in range(L)]
    yf = [_dev(y_lists[s][l], "y") for s in range(G) for l in range(L)]
    gf = [outs[l][s] if outs[l] is not None else None for s in range(G) for l in range(L)]
    keep = [_ptrs(gt), _ptrs(img), _ptrs(yf), _ptrs(gf)]
    rl = (ctypes.c_int * L)(*[1 if r else 0 for r in relus])
    call("rs_mlp_bwd_chain_prec_f32", G, L, ctypes.cast(dims, _VP), M, keep[0][1], keep[1][1], keep[2][1],
         ctypes.cast(rl, _VP), keep[3][1], int(precision), _stream())
    return [[outs[l][s] for s in range(G)] if outs[l] is not None else [None] * G for l in range(L)]


def mlp_wgrad_ok(dims, precision: int) -> bool:
    return (precision in (PREC_F32_SPLIT6, PREC_F32_SPLIT9) and 2 <= len(dims) <= 7
            and all(d % 64 == 0 and 64 <= d <= 4096 for d in dims))


def mlp_wgrad(x_lists, g_lists, precision: int, W_lists=None, w_scale: float = 0.0, w_dscale=None, queue=None):
    """Every layer's (dW, db) of G (1..2) Dense stacks in ONE launch (rs_mlp_wgrad_prec_f32):
    x_lists[s][l] = layer l's input, g_lists[s][l] = the gradient at its pre-activation; with
    W_lists the folded l2 term w_scale * w_dscale * W. Returns grads[s][l] = (dW, db), views of one
    [K + 1, N] buffer per layer (gemm_wgrad_bias's layout)."""
    G, L = len(x_lists), len(x_lists[0])
    M = x_lists[0][0].shape[0]
    dims = (ctypes.c_int64 * (L + 1))(*[x_lists[0][l].shape[1] for l in range(L)], g_lists[0][L - 1].shape[1])
    dev = x_lists[0][0].device
    bufs = [[torch.empty((dims[l] + 1, dims[l + 1]), dtype=torch.float32, device=dev) for l in range(L)]
            for _ in range(G)]
    xf = [_dev(x_lists[s][l], "x") for s in range(G) for l in range(L)]
    gf = [_dev(g_lists[s][l], "g") for s in range(G) for l in range(L)]
    of = [bufs[s][l] for s in range(G) for l in range(L)]
    keep = [_ptrs(xf), _ptrs(gf), _ptrs(of)]
    if W_lists is not None:
        keep.append(_ptrs([_dev(W_lists[s][l], "W") for s in range(G) for l in range(L)]))
    dp = ctypes.cast(dims, _VP)
    ws = _ws(query("rs_mlp_wgrad_workspace_bytes", G, L, dp, M), dev)
    q, qh = _q(queue)
    call("rs_mlp_wgrad_prec_f32", G, L, dp, M, keep[0][1], keep[1][1], keep[2][1],
         keep[3][1] if W_lists is not None else None, float(w_scale), _p(w_dscale), int(precision), _p(ws),
         ws.numel(), _stream(), qh)
    if q is not None:
        q.keep(ws, w_dscale, *[W_lists[s][l] for s in range(G) for l in range(L)] if W_lists is not None else (),
               *of)
    return [[(bufs[s][l][:dims[l]], bufs[s][l][dims[l]]) for l in range(L)] for s in range(G)]


def gemm_wgrad_bias_group(x_list, g_list, precision: int = 0, queue=None, x_rows=None):
    """[(x_g^T g_g, column sums of g_g) for g] in one split-K launch + one reduction
    (rs_gemm_wgrad_bias_group_prec_f32; each pair bitwise its gemm_wgrad_bias()). x_rows (int32
    [rows of g] per problem): batch row k reads row x_rows[g][k] of x_g (the distinct-row form,
    rs_gemm_wgrad_bias_group_rows_prec_f32: bitwise the sums over the expanded x)."""
    G = len(x_list)
    for t in list(x_list) + list(g_list):
        _dev(t, "operand")
    M = x_list[0].shape[1]
    K = g_list[0].shape[0] if x_rows is not None else x_list[0].shape[0]
    N = g_list[0].shape[1]
    buf = torch.empty((G, M + 1, N), dtype=torch.float32, device=x_list[0].device)
    ws = _ws(query("rs_gemm_wgrad_bias_group_workspace_bytes", G, M, N, K), x_list[0].device)
    px, pg = _ptrs(x_list), _ptrs(g_list)
    q, qh = _q(queue)
    if x_rows is not None:
        pr = _ptrs([_dev(t, "x_rows", torch.int32) for t in x_rows])
        call("rs_gemm_wgrad_bias_group_rows_prec_f32", G, M, N, K, px[1], x_list[0].stride(0), pr[1], pg[1],
             g_list[0].stride(0), _p(buf), int(precision), _p(ws), ws.numel(), _stream(), qh)
    else:
        call("rs_gemm_wgrad_bias_group_prec_f32", G, M, N, K, px[1], x_list[0].stride(0), pg[1],
             g_list[0].stride(0), _p(buf), int(precision), _p(ws), ws.numel(), _stream(), qh)
    if q is not None:
        q.keep(ws, buf)
    return [(buf[g, :M], buf[g, M]) for g in range(G)]


def sum_squares_multi(tensors, scale=1.0):
    """scale * sum_k sum(t_k^2) over 1..8 fp32 tensors in one partial pass (rs_sum_squares_multi_f32)."""
    k = len(tensors)
    for t in tensors:
        _dev(t, "tensor")
    ptrs = (_VP * k)(*[t.data_ptr() for t in tensors])
    ns = (ctypes.c_int64 * k)(*[t.numel() for t in tensors])
    out = torch.empty((), dtype=torch.float32, device=tensors[0].device)
    ws = _ws(query("rs_sum_squares_multi_workspace_bytes", k, ctypes.cast(ns, _VP)), tensors[0].device)
    call("rs_sum_squares_multi_f32", k, ctypes.cast(ptrs, _VP), ctypes.cast(ns, _VP), float(scale), _p(out), _p(ws),
         ws.numel(), _stream())
    return out


def relu_bwd_colsum(dy, y=None, queue=None):
    """g = dy * (y > 0) (identity if y is None) and its column sums (bias gradient)."""
    _dev(dy, "dy")
    M, N = dy.shape
    colsum = torch.empty((N,), dtype=torch.float32, device=dy.device)
    g = torch.empty_like(dy) if y is not None else None
    ws = _ws(query("rs_colsum_workspace_bytes", M, N), dy.device)
    q, qh = _q(queue)
    call("rs_relu_bwd_colsum_f32", _p(dy), _p(y), M, N, _p(g), _p(colsum), _p(ws), ws.numel(), _stream(), qh)
    if q is not None:
        q.keep(ws, colsum)   # written by the queued reduction even when the caller drops it
    return (g if g is not None else dy), colsum


def sum_squares(x, scale=1.0):
    _dev(x, "x")
    out = torch.empty((), dtype=torch.float32, device=x.device)
    ws = _ws(query("rs_sum_squares_workspace_bytes", x.numel()), x.device)
    call("rs_sum_squares_f32", _p(x), x.numel(), float(scale), _p(out), _p(ws), ws.numel(), _stream())
    return out


def dcn_cross_fwd(u, v, w, b):
    _dev(u, "u"), _dev(v, "v"), _dev(w, "w"), _dev(b, "b")
    B, D = u.shape
    L = w.shape[0]
    x0 = torch.empty((B, 2 * D), dtype=torch.float32, device=u.device)
    xl = torch.empty_like(x0)
    s = torch.empty((B, max(L, 1)), dtype=torch.float32, device=u.device)
    call("rs_dcn_cross_vec_fwd_f32", _p(u), _p(v), B, D, L, _p(w), _p(b), _p(x0), _p(xl), _p(s), _stream())
    return x0, xl, s


def dcn_cross_bwd(x0, s, w, b, g_xl, g_x0_extra=None, add_u=None, add_v=None, queue=None):
    """(g_u, g_v, g_w, g_b); add_u / add_v (another consumer's dL/du, dL/dv) are added in the kernel."""
    B, d = x0.shape
    D, L = d // 2, w.shape[0]
    g_u = torch.empty((B, D), dtype=torch.float32, device=x0.device)
    g_v = torch.empty_like(g_u)
    gw = torch.empty_like(w)
    gb = torch.empty_like(b)
    ws = _ws(query("rs_dcn_cross_vec_bwd_workspace_bytes", B, D, L), x0.device)
    q, qh = _q(queue)
    if q is not None:
        q.keep(ws, gw, gb)
    if add_u is not None:
        call("rs_dcn_cross_vec_bwd_add_f32", _p(x0), _p(s), _p(w), _p(b), B, D, L, _p(_dev(g_xl, "g_xl")),
             _p(g_x0_extra), _p(_dev(add_u, "add_u")), _p(_dev(add_v, "add_v")), _p(g_u), _p(g_v), _p(gw), _p(gb),
             _p(ws), ws.numel(), _stream(), qh)
        return g_u, g_v, gw, gb
    call("rs_dcn_cross_vec_bwd_f32", _p(x0), _p(s), _p(w), _p(b), B, D, L, _p(_dev(g_xl, "g_xl")),
         _p(g_x0_extra), _p(g_u), _p(g_v), _p(gw), _p(gb), _p(ws), ws.numel(), _stream(), qh)
    return g_u, g_v, gw, gb


def heads_fwd(xl, h, w_r, b_r, w_c, b_c):
    _dev(xl, "xl"), _dev(h, "h")
    B = xl.shape[0]
    r = torch.empty((B, 1), dtype=torch.float32, device=xl.device)
    p = torch.empty_like(r)
    call("rs_heads_fwd_f32", _p(xl), xl.shape[1], _p(h), h.shape[1], B, _p(w_r), _p(b_r), _p(w_c), _p(b_c),
         _p(r), _p(p), _stream())
    return r, p


def heads_bwd(xl, h, w_r, w_c, p, g_r=None, g_p=None, unit_r=None, unit_c=None, gs_rat=None, gs_ctr=None,
              queue=None):
    B, dx, dh = xl.shape[0], xl.shape[1], h.shape[1]
    g_xl = torch.empty_like(xl)
    g_h = torch.empty_like(h)
    g_wr = torch.empty((dx + dh, 1), dtype=torch.float32, device=xl.device)
    g_wc = torch.empty_like(g_wr)
    g_br = torch.empty((1,), dtype=torch.float32, device=xl.device)
    g_bc = torch.empty_like(g_br)
    ws = _ws(query("rs_heads_bwd_workspace_bytes", B, dx, dh), xl.device)
    q, qh = _q(queue)
    call("rs_heads_bwd_f32", _p(xl), dx, _p(h), dh, B, _p(w_r), _p(w_c), _p(p), _p(g_r), _p(g_p), _p(unit_r),
         _p(unit_c), _p(gs_rat), _p(gs_ctr), _p(g_xl), _p(g_h), _p(g_wr), _p(g_br), _p(g_wc), _p(g_bc),
         _p(ws), ws.numel(), _stream(), qh)
    if q is not None:
        q.keep(ws, g_wr, g_br, g_wc, g_bc)
    return g_xl, g_h, g_wr, g_br, g_wc, g_bc


def ranking_losses(r, p, rating, y_implicit, class_weights=None, ctr_mode=0):
    """Returns (loss[2] = (mse, bce), unit_r, unit_c)."""
    B = r.shape[0]
    loss = torch.empty((2,), dtype=torch.float32, device=r.device)
    unit_r = torch.empty((B,), dtype=torch.float32, device=r.device)
    unit_c = torch.empty_like(unit_r)
    cw0, cw1 = (float(class_weights[0]), float(class_weights[1])) if class_weights else (1.0, 1.0)
    ws = _ws(query("rs_ranking_losses_workspace_bytes", B), r.device)
    call("rs_ranking_losses_f32", _p(r), _p(p), _p(_dev(rating, "rating")), _p(_dev(y_implicit, "y_implicit")),
         B, 1 if class_weights else 0, cw0, cw1, int(ctr_mode), _p(loss), _p(unit_r), _p(unit_c), _p(ws),
         ws.numel(), _stream())
    return loss, unit_r, unit_c


def ranking_losses_combine(r, p, rating, y_implicit, class_weights, ctr_mode, ret, reg, w_ret, w_rat, w_ctr,
                           use_ctr=True):
    """ranking_losses + compute_loss's weighting (+ the regularizer) in one launch sequence
    (rs_ranking_losses_combine_f32): (loss[2], total, total_reg, unit_r, unit_c)."""
    B = r.shape[0]
    dev = r.device
    loss = torch.empty((2,), dtype=torch.float32, device=dev)
    total = torch.empty((), dtype=torch.float32, device=dev)
    total_reg = torch.empty((), dtype=torch.float32, device=dev)
    unit_r = torch.empty((B,), dtype=torch.float32, device=dev)
    unit_c = torch.empty_like(unit_r)
    cw0, cw1 = (float(class_weights[0]), float(class_weights[1])) if class_weights else (1.0, 1.0)
    ws = _ws(query("rs_ranking_losses_workspace_bytes", B), dev)
    call("rs_ranking_losses_combine_f32", _p(r), _p(p), _p(_dev(rating, "rating")), _p(_dev(y_implicit, "y_implicit")),
         B, 1 if class_weights else 0, cw0, cw1, int(ctr_mode), _p(_dev(ret, "ret")), _p(reg), float(w_ret),
         float(w_rat), float(w_ctr), int(bool(use_ctr)), _p(loss), _p(total), _p(total_reg), _p(unit_r), _p(unit_c),
         _p(ws), ws.numel(), _stream())
    return loss, total, total_reg, unit_r, unit_c


def heads_bwd_combine(xl, h, w_r, w_c, p, unit_r, unit_c, g_total, w_ret, w_rat, w_ctr, use_ctr=True, queue=None,
                      relu_h=False):
    """heads_bwd with the loss weighting's backward folded in (rs_heads_bwd_combine_f32):
    (g_xl, g_h, g_wr, g_br, g_wc, g_bc, g_ret). relu_h: h is a ReLU layer's output and g_h comes
    back masked by h > 0 (the gradient at that layer's pre-activation, RS_HEADS_RELU_H)."""
    B, dx, dh = xl.shape[0], xl.shape[1], h.shape[1]
    g_xl = torch.empty_like(xl)
    g_h = torch.empty_like(h)
    g_wr = torch.empty((dx + dh, 1), dtype=torch.float32, device=xl.device)
    g_wc = torch.empty_like(g_wr)
    g_br = torch.empty((1,), dtype=torch.float32, device=xl.device)
    g_bc = torch.empty_like(g_br)
    g_ret = torch.empty((), dtype=torch.float32, device=xl.device)
    ws = _ws(query("rs_heads_bwd_workspace_bytes", B, dx, dh), xl.device)
    q, qh = _q(queue)
    call("rs_heads_bwd_combine_f32", _p(xl), dx, _p(h), dh, B, _p(w_r), _p(w_c), _p(p), _p(unit_r), _p(unit_c),
         _p(_dev(g_total, "g_total")), float(w_ret), float(w_rat), float(w_ctr),
         (RS_HEADS_USE_CTR if use_ctr else 0) | (RS_HEADS_RELU_H if relu_h else 0), _p(g_ret),
         _p(g_xl), _p(g_h), _p(g_wr), _p(g_br), _p(g_wc), _p(g_bc), _p(ws), ws.numel(), _stream(), qh)
    if q is not None:
        q.keep(ws, g_wr, g_br, g_wc, g_bc)
    return g_xl, g_h, g_wr, g_br, g_wc, g_bc, g_ret


# The forward may keep the B x B scores for the backward (half its MFMA work) while they fit this
# budget: 17.2 GB at B = 65536, sized for 288 GB of HBM per GPU.
INBATCH_STORE_SCORES_MAX_BYTES = 48 << 30


_KERNEL_DIMS = (32, 64, 128)   # embedding widths compiled into the in-batch and top-k kernels


def _kernel_dim(D: int) -> int:
    """Narrower embeddings run zero-padded to the next compiled width (zero columns change no
    score, and their gradient columns are dropped)."""
    for d in _KERNEL_DIMS:
        if D <= d:
            return d
    raise NotImplementedError(f"embedding width {D} > {_KERNEL_DIMS[-1]} is not compiled into the "
                              "in-batch / top-k kernels")


def _pad_cols(x: torch.Tensor, Dp: int) -> torch.Tensor:
    if x.shape[1] == Dp:
        return x
    out = torch.zeros((x.shape[0], Dp), dtype=x.dtype, device=x.device)
    out[:, :x.shape[1]] = x
    return out


def inbatch_scores_buffer(B: int, device) -> torch.Tensor:
    return torch.empty((query("rs_inbatch_scores_bytes", B) // 4,), dtype=torch.float32, device=device)


# Contraction precision of the score-storing in-batch pair (include/recsys_hip.h RS_PREC_*):
# 0 = fp32 operands on the f32 MFMA; 9 = exact three-term bf16 split of every fp32 operand, all
# nine cross products (the fp32 products exactly, fp32 accumulation); 6 = the same without the
# three products below 2^-23 of |x.y| (one-fp32-rounding-level error).
PREC_F32, PREC_F32_SPLIT6, PREC_F32_SPLIT9 = 0, 6, 9


def inbatch_softmax_fwd(U, C, weight=1.0, want_grad=True, scores: Optional[torch.Tensor] = None,
                        precision: int = PREC_F32, workspace: Optional[torch.Tensor] = None):
    """Returns (loss_sum fp32 0-dim, row_loss [B], lse [B], dU_unit or None, loss_sum64). With a
    `scores` buffer (inbatch_scores_buffer) the B x B scores are kept for inbatch_softmax_bwd, and
    `precision` selects the contraction kernels (PREC_*). workspace (inbatch_workspace): a buffer
    the caller keeps for the matching inbatch_softmax_bwd (its image of U is then reused)."""
    _dev(U, "U"), _dev(C, "C")
    D0 = U.shape[1]
    if _kernel_dim(D0) != D0:
        tot, row, lse, dU, tot64 = inbatch_softmax_fwd(_pad_cols(U, _kernel_dim(D0)), _pad_cols(C, _kernel_dim(D0)),
                                                      weight, want_grad, scores, precision, workspace)
        return tot, row, lse, (dU[:, :D0].contiguous() if dU is not None else None), tot64
    B, D = U.shape
    row = torch.empty((B,), dtype=torch.float32, device=U.device)
    lse = torch.empty_like(row)
    tot = torch.empty((), dtype=torch.float32, device=U.device)
    tot64 = torch.empty((), dtype=torch.float64, device=U.device)
    dU = torch.empty_like(U) if (want_grad or scores is not None) else None
    ws = workspace if workspace is not None else _ws(query("rs_inbatch_softmax_workspace_bytes", B, D), U.device)
    if scores is not None:
        call("rs_inbatch_softmax_xent_fwd_store_prec_f32", _p(U), _p(C), B, D, float(weight), _p(row), _p(lse),
             _p(tot), _p(tot64), _p(dU), _p(_dev(scores, "scores")), int(precision), _p(ws), ws.numel(), _stream())
    else:
        call("rs_inbatch_softmax_xent_fwd_f32", _p(U), _p(C), B, D, float(weight), _p(row), _p(lse), _p(tot),
             _p(tot64), _p(dU), _p(ws), ws.numel(), _stream())
    return tot, row, lse, dU, tot64


def inbatch_softmax_bwd(U, C, lse, gscale=None, dU_unit=None, weight=1.0, scores: Optional[torch.Tensor] = None,
                        precision: int = PREC_F32, workspace: Optional[torch.Tensor] = None):
    """Returns (dU = g * dU_unit or None, dC); `scores` from a storing forward skips U C^T.
    workspace: the storing forward's (RS_INBATCH_FWD_WS: its image of U is reused)."""
    D0 = U.shape[1]
    if _kernel_dim(D0) != D0:
        Dp = _kernel_dim(D0)
        dU, dC = inbatch_softmax_bwd(_pad_cols(U, Dp), _pad_cols(C, Dp), lse, gscale,
                                     _pad_cols(dU_unit, Dp) if dU_unit is not None else None, weight, scores,
                                     precision, workspace)
        return (dU[:, :D0].contiguous() if dU is not None else None), dC[:, :D0].contiguous()
    B, D = U.shape
    dC = torch.empty_like(C)
    dU = torch.empty_like(U) if dU_unit is not None else None
    ws = workspace if workspace is not None else _ws(query("rs_inbatch_softmax_workspace_bytes", B, D), U.device)
    if scores is not None:
        flags = RS_INBATCH_FWD_WS if workspace is not None else 0
        call("rs_inbatch_softmax_xent_bwd_stored_prec_f32", _p(U), _p(C), B, D, float(weight), _p(lse), _p(scores),
             _p(gscale), _p(dU_unit), _p(dU), _p(dC), int(precision) | flags, _p(ws), ws.numel(), _stream())
    else:
        call("rs_inbatch_softmax_xent_bwd_f32", _p(U), _p(C), B, D, float(weight), _p(lse), _p(gscale),
             _p(dU_unit), _p(dU), _p(dC), _p(ws), ws.numel(), _stream())
    return dU, dC


# Deduplicated pair (rs_inbatch_*_dedup_f32): eligible at D = 128 with the split precisions and
# the kept scores; taken when the batch has at least INBATCH_DEDUP_MIN_B rows and the distinct
# users x distinct items are at most INBATCH_DEDUP_MAX_FRAC of B x B. False turns it off (the
# full B x B pair then runs on every batch; tests only).
INBATCH_DEDUP = True
INBATCH_DEDUP_MIN_B = 16384
INBATCH_DEDUP_MAX_FRAC = 0.8
# device-count plans (no host read: the step stays graph-capturable) for id-keyed batches also
# outside capture; inside a capture they are always used. Round 6: on by default, so an eager step
# (the data-parallel step, the trainer) has no host read in its forward either — a read there drains
# the queue (measured +66 us at C3 one GPU, and it serialises the host behind the GPU in the DP
# step). The device form deduplicates both sides whatever their counts (as the graphed bench step).
INBATCH_DEDUP_DEVICE = True
# GATHER_ORDERED: the embedding gather reads the tables in the id plan's ascending-id order
# when a plan exists (a timing switch; the gathered rows are the same). Off by default: measured
# slower in the C3 step (uniform ids 34-36 vs 33-34 us; Zipf ids 38 vs 28 us, the hot ids' duplicate
# reads then land on one row at once; tools/gpu_r04_p.sh, profiles/r04_gather_order_ab.json)
GATHER_ORDERED = False
# the id plan also writes each distinct slot's id (rs_inbatch_unique_ids_plan_i64), and the
# distinct-row towers gather from those (rs_embedding_gather_tables_ids_f32) instead of through the
# representative rows (rs_embedding_gather_tables_rows_f32)
PLAN_DIDS = True


def inbatch_unique_rows(X):
    """Distinct rows of X [B][D] by content (bitwise): (rep [B] int32, count [ceil(B/32)*32] fp32,
    inv [B] int32, info [2] int64 = (distinct rows, hash-collision rows)), all on the device."""
    X = _dev(X, "X")
    B, D = X.shape
    rep = torch.empty((B,), dtype=torch.int32, device=X.device)
    inv = torch.empty_like(rep)
    count = torch.empty(((B + 31) // 32 * 32,), dtype=torch.float32, device=X.device)
    info = torch.empty((2,), dtype=torch.int64, device=X.device)
    ws = _ws(query("rs_inbatch_unique_rows_workspace_bytes", B), X.device)
    call("rs_inbatch_unique_rows_f32", _p(X), B, D, _p(rep), _p(count), _p(inv), _p(info), _p(ws), ws.numel(),
         _stream())
    return rep, count, inv, info


def inbatch_unique_pair(U, C):
    """inbatch_unique_rows of U and of C in one sequence (rs_inbatch_unique_pair_f32): two
    (rep, count, inv, side info [2], whole info [4]) tuples (one host read covers both sides)."""
    U, C = _dev(U, "U"), _dev(C, "C")
    B, D = U.shape
    reps = torch.empty((2, B), dtype=torch.int32, device=U.device)
    invs = torch.empty_like(reps)
    counts = torch.empty((2, (B + 31) // 32 * 32), dtype=torch.float32, device=U.device)
    info = torch.empty((4,), dtype=torch.int64, device=U.device)
    ws = _ws(query("rs_inbatch_unique_pair_workspace_bytes", B), U.device)
    call("rs_inbatch_unique_pair_f32", _p(U), _p(C), B, D, _p(reps[0]), _p(counts[0]), _p(invs[0]), _p(reps[1]),
         _p(counts[1]), _p(invs[1]), _p(info), _p(ws), ws.numel(), _stream())
    return (reps[0], counts[0], invs[0], info[0:2], info), (reps[1], counts[1], invs[1], info[2:4], info)


def inbatch_unique_ids_pair(user_ids, item_ids, user_rows: int, item_rows: int, order: bool = False,
                            dids: bool = False):
    """The two sides' distinct rows from their ids (rs_inbatch_unique_ids_pair_i64), for tower rows
    that are a function of the id alone; same tuples as inbatch_unique_pair. order: a sixth entry per
    side, the side's batch rows in ascending-id order (rs_inbatch_unique_ids_pair_order_i64: the
    gather reads the tables in that order). dids (with order): a seventh, each distinct slot's id
    (int64 [B], -1 past the count; rs_inbatch_unique_ids_plan_i64), what embedding_gather_tables_ids
    reads, and an eighth, each slot's first position in the order (int32 [B]: the run heads the
    planned sparse update applies)."""
    user_ids, item_ids = _dev(user_ids, "user_ids", torch.int64), _dev(item_ids, "item_ids", torch.int64)
    B = user_ids.shape[0]
    reps = torch.empty((2, B), dtype=torch.int32, device=user_ids.device)
    invs = torch.empty_like(reps)
    counts = torch.empty((2, (B + 31) // 32 * 32), dtype=torch.float32, device=user_ids.device)
    info = torch.empty((6 if order and dids else 4,), dtype=torch.int64, device=user_ids.device)
    ws = _ws(query("rs_inbatch_unique_pair_workspace_bytes", B), user_ids.device)
    if order and dids:
        orders = torch.empty_like(reps)
        starts = torch.empty_like(reps)
        did = torch.empty((2, B), dtype=torch.int64, device=user_ids.device)
        call("rs_inbatch_unique_ids_plan_i64", _p(user_ids), _p(item_ids), B, int(user_rows), int(item_rows),
             _p(reps[0]), _p(counts[0]), _p(invs[0]), _p(orders[0]), _p(did[0]), _p(starts[0]), _p(reps[1]),
             _p(counts[1]), _p(invs[1]), _p(orders[1]), _p(did[1]), _p(starts[1]), _p(info), _p(ws), ws.numel(),
             _stream())
        return ((reps[0], counts[0], invs[0], info[0:2], info, orders[0], did[0], starts[0]),
                (reps[1], counts[1], invs[1], info[2:4], info, orders[1], did[1], starts[1]))
    if order:
        orders = torch.empty_like(reps)
        call("rs_inbatch_unique_ids_pair_order_i64", _p(user_ids), _p(item_ids), B, int(user_rows), int(item_rows),
             _p(reps[0]), _p(counts[0]), _p(invs[0]), _p(orders[0]), _p(reps[1]), _p(counts[1]), _p(invs[1]),
             _p(orders[1]), _p(info), _p(ws), ws.numel(), _stream())
        return ((reps[0], counts[0], invs[0], info[0:2], info, orders[0]),
                (reps[1], counts[1], invs[1], info[2:4], info, orders[1]))
    call("rs_inbatch_unique_ids_pair_i64", _p(user_ids), _p(item_ids), B, int(user_rows), int(item_rows),
         _p(reps[0]), _p(counts[0]), _p(invs[0]), _p(reps[1]), _p(counts[1]), _p(invs[1]), _p(info), _p(ws),
         ws.numel(), _stream())
    return (reps[0], counts[0], invs[0], info[0:2], info), (reps[1], counts[1], invs[1], info[2:4], info)


def _device_counts(users, items):
    """The plan's info array when its sides carry device-resident counts (n_distinct None)."""
    if users is not None and users[3] is None:
        return users[4]
    return None


def inbatch_softmax_fwd_dedup(U, C, users, items, scores, precision: int, weight=1.0, workspace=None):
    """The deduplicated forward. users / items = (rep, count, inv, n_distinct) of
    inbatch_unique_rows, or None for a side that is not deduplicated; with n_distinct None (a
    device-count plan, inbatch_dedup_plan(device_counts=True)) the counts stay on the device
    (rs_inbatch_softmax_xent_fwd_dedup_dev_f32: no host read). Returns (loss_sum, row_loss, lse,
    dU_unit, loss_sum64) for the B batch rows, as inbatch_softmax_fwd."""
    B, D = U.shape
    row = torch.empty((B,), dtype=torch.float32, device=U.device)
    lse = torch.empty_like(row)
    tot = torch.empty((), dtype=torch.float32, device=U.device)
    tot64 = torch.empty((), dtype=torch.float64, device=U.device)
    dU = torch.empty_like(U)
    ws = workspace if workspace is not None else _ws(query("rs_inbatch_dedup_workspace_bytes", B, D), U.device)
    info = _device_counts(users, items)
    if info is not None:
        call("rs_inbatch_softmax_xent_fwd_dedup_dev_f32", _p(U), _p(C), B, D, float(weight), _p(users[0]),
             _p(users[2]), _p(items[0]), _p(items[1]), _p(info), _p(row), _p(lse), _p(tot), _p(tot64), _p(dU),
             _p(_dev(scores, "scores")), int(precision), _p(ws), ws.numel(), _stream())
        return tot, row, lse, dU, tot64
    u_rep, _, u_inv, Bu = users[:4] if users is not None else (None, None, None, B)
    c_rep, c_cnt, _, Bc = items[:4] if items is not None else (None, None, None, B)
    call("rs_inbatch_softmax_xent_fwd_dedup_f32", _p(U), _p(C), B, D, float(weight), _p(u_rep), _p(u_inv), int(Bu),
         _p(c_rep), _p(c_cnt), int(Bc), _p(row), _p(lse), _p(tot), _p(tot64), _p(dU), _p(_dev(scores, "scores")),
         int(precision), _p(ws), ws.numel(), _stream())
    return tot, row, lse, dU, tot64


def inbatch_softmax_bwd_dedup(U, lse, users, items, scores, precision: int, gscale=None, dU_unit=None,
                              weight=1.0, workspace=None):
    """The deduplicated backward (same sides as the forward): (dU = g * dU_unit or None, dC).
    workspace: the forward's (RS_INBATCH_FWD_WS: its image of the distinct users is reused)."""
    B, D = U.shape
    dC = torch.empty_like(U)
    dU = torch.empty_like(U) if dU_unit is not None else None
    ws = workspace if workspace is not None else _ws(query("rs_inbatch_dedup_workspace_bytes", B, D), U.device)
    if workspace is not None:
        precision = int(precision) | RS_INBATCH_FWD_WS
    info = _device_counts(users, items)
    if info is not None:
        call("rs_inbatch_softmax_xent_bwd_dedup_dev_f32", _p(U), B, D, float(weight), _p(lse),
             _p(_dev(scores, "scores")), _p(gscale), _p(dU_unit), _p(dU), _p(dC), _p(users[0]), _p(users[1]),
             _p(items[2]), _p(info), int(precision), _p(ws), ws.numel(), _stream())
        return dU, dC
    u_rep, u_cnt, _, Bu = users[:4] if users is not None else (None, None, None, B)
    _, _, c_inv, Bc = items[:4] if items is not None else (None, None, None, B)
    call("rs_inbatch_softmax_xent_bwd_dedup_f32", _p(U), B, D, float(weight), _p(lse), _p(_dev(scores, "scores")),
         _p(gscale), _p(dU_unit), _p(dU), _p(dC), _p(u_rep), _p(u_cnt), int(Bu), _p(c_inv), int(Bc), int(precision),
         _p(ws), ws.numel(), _stream())
    return dU, dC


RS_INBATCH_FWD_WS = 0x100   # include/recsys_hip.h: the backward is given its forward's workspace


def inbatch_workspace(B: int, D: int, device, dedup: bool = False) -> torch.Tensor:
    """A workspace for one in-batch forward + backward pair (kept by the caller between the two)."""
    n = query("rs_inbatch_dedup_workspace_bytes" if dedup else "rs_inbatch_softmax_workspace_bytes", B, D)
    return torch.empty((n,), dtype=torch.uint8, device=device)


def inbatch_plan_eligible(B: int, config) -> bool:
    """Whether a MultiTaskModel batch of B rows takes the id plan (the deduplicated pair's
    eligibility before the counts are known: D = 128, a split precision, B >= INBATCH_DEDUP_MIN_B)."""
    return (INBATCH_DEDUP and B >= INBATCH_DEDUP_MIN_B and config.embedding_dim == 128
            and config.contraction_precision in (PREC_F32_SPLIT6, PREC_F32_SPLIT9))


def inbatch_dedup_plan(U, C, precision: int, force: bool = False, ids=None, device_counts=None):
    """(users, items) sides for the deduplicated pair, or None when the full pair should run: one
    host synchronisation reads the two distinct-row counts (and the collision counts, which send
    the batch to the full pair). ids = (user_ids, item_ids, user_rows, item_rows[, id plan]) when the
    rows are a function of the id alone (the towers): distinct rows by id, no hashing or verification
    (a fifth entry is the inbatch_unique_ids_pair result already computed for these ids).
    device_counts (default: while the stream is capturing, or INBATCH_DEDUP_DEVICE): an id plan
    whose counts stay on the device — no host read, both sides deduplicated whatever the counts
    (sides (rep, count, inv, None, info))."""
    B, D = U.shape
    if D != 128 or precision not in (PREC_F32_SPLIT6, PREC_F32_SPLIT9):
        return None
    capturing = torch.cuda.is_current_stream_capturing()
    if device_counts is None:   # (the content search's collision count needs the host read)
        device_counts = capturing or (INBATCH_DEDUP_DEVICE and ids is not None)
    if not force and (not INBATCH_DEDUP or B < INBATCH_DEDUP_MIN_B):
        return None
    pre = ids[4] if ids is not None and len(ids) > 4 else None   # an id plan computed before the towers
    if device_counts:
        if ids is None:      # the content search's collision count needs a host read
            return None
        uq, cq = pre if pre is not None else inbatch_unique_ids_pair(*ids[:4])
        return (uq[0], uq[1], uq[2], None, uq[4]), (cq[0], cq[1], cq[2], None, cq[4])
    if capturing:
        return None
    if pre is not None:
        uq, cq = pre
    else:
        uq, cq = inbatch_unique_ids_pair(*ids[:4]) if ids is not None else inbatch_unique_pair(U, C)
    Bu, u_bad, Bc, c_bad = uq[4][:4].tolist()
    if u_bad or c_bad or (not force and Bu * Bc > INBATCH_DEDUP_MAX_FRAC * B * B):
        return None
    users = (uq[0], uq[1], uq[2], Bu) if Bu < B else None
    items = (cq[0], cq[1], cq[2], Bc) if Bc < B else None
    return users, items


def iteration_increment(it):
    call("rs_iteration_increment", _p(_dev(it, "iteration", torch.int64)), _stream())


RS_TOPK_LIST_SCAN = 0x100   # include/recsys_hip.h: the single-pass list scan (checks the bound-first scan)


def topk_ip(queries, items, k, index_base=0, precision: int = 0, list_scan: bool = False):
    """Exact inner-product top-k, ordered by (-score, index) -> (scores [Q,k], index int64 [Q,k]).
    `precision` (PREC_*) selects the scan's contraction for > 64 queries at D = 128; list_scan
    forces the single-pass list scan where the bound-first scan would run (same lists, bitwise)."""
    _dev(queries, "queries"), _dev(items, "items")
    if _kernel_dim(queries.shape[1]) != queries.shape[1]:
        Dp = _kernel_dim(queries.shape[1])
        return topk_ip(_pad_cols(queries, Dp), _pad_cols(items, Dp), k, index_base, precision)
    Q, D = queries.shape
    N = items.shape[0]
    s = torch.empty((Q, k), dtype=torch.float32, device=queries.device)
    i = torch.empty((Q, k), dtype=torch.int64, device=queries.device)
    ws = _ws(query("rs_topk_ip_workspace_bytes", Q, N, D, k), queries.device)
    call("rs_topk_ip_prec_f32", _p(queries), Q, _p(items), N, D, int(k), int(index_base), _p(s), _p(i),
         int(precision) | (RS_TOPK_LIST_SCAN if list_scan else 0), _p(ws), ws.numel(), _stream())
    return s, i


def topk_merge(scores, index, k):
    """[Q, nlists, k] sorted lists -> [Q, k] (the shard exchange's final merge)."""
    _dev(scores, "scores"), _dev(index, "index", torch.int64)
    Q, nl = scores.shape[0], scores.shape[1]
    s = torch.empty((Q, k), dtype=torch.float32, device=scores.device)
    i = torch.empty((Q, k), dtype=torch.int64, device=scores.device)
    ws = _ws(query("rs_topk_merge_workspace_bytes", Q, nl, k), scores.device)
    call("rs_topk_merge_f32", _p(scores), _p(index), Q, nl, int(k), _p(s), _p(i), _p(ws), ws.numel(), _stream())
    return s, i


def rank_metrics(pred: torch.Tensor, truth: torch.Tensor, ks: Sequence[int], n_items: int,
                 lens: Optional[torch.Tensor] = None) -> torch.Tensor:
    """AdvancedMetrics (src/evaluation.py:22-104) over int64 top-K lists [U, K] (optional int32
    lengths [U] for ragged lists) and true rows [U] -> float64 [4*len(ks) + 3]: per k (recall,
    precision, ndcg, map), then mrr, diversity, coverage."""
    _dev(pred, "pred", torch.int64)
    _dev(truth, "truth", torch.int64)
    if lens is not None:
        _dev(lens, "lens", torch.int32)
    U, K = (pred.shape[0], pred.shape[1]) if pred.dim() == 2 else (0, 1)
    ks = [int(k) for k in ks]
    out = torch.empty((4 * len(ks) + 3,), dtype=torch.float64, device=pred.device)
    arr = (ctypes.c_int32 * max(len(ks), 1))(*ks)
    ws = _ws(query("rs_rank_metrics_workspace_bytes", U, len(ks), int(n_items)), pred.device)
    call("rs_rank_metrics_i64", _p(pred), U, K, _p(lens), _p(truth), ctypes.cast(arr, _VP), len(ks), int(n_items),
         _p(out),
         _p(ws), ws.numel(), _stream())
    return out


def l2_normalize_rows(x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """faiss.normalize_L2 on [n, D] rows (zero rows are left as they are)."""
    _dev(x, "x")
    n, D = x.shape
    if out is None:
        out = torch.empty_like(x)
    call("rs_l2_normalize_rows_f32", _p(x), n, D, _p(out), _stream())
    return out


# --------------------------------------------------------------------------------------------
# autograd Functions
# --------------------------------------------------------------------------------------------
class SparseGradSink:
    """Collects IndexedSlices-style (ids, rows) gradients of an embedding table during
    backward (the Keras Embedding gradient is an IndexedSlices, never a dense [V, D] tensor)."""

    def __init__(self):
        self.slices: List[Tuple[torch.Tensor, torch.Tensor]] = []
        # global ||raw rows||^2 set by the data-parallel exchange when the slices it leaves are
        # deduplicated ones (the clip norm is over the raw rows, src/trainer.py:163)
        self.sumsq: Optional[torch.Tensor] = None
        # (ids, order): the stable ascending-id order of these ids (the in-batch id plan's), valid
        # while the sink holds exactly the one slice of those ids; the sparse update then skips its sort
        self.order: Optional[Tuple[torch.Tensor, torch.Tensor]] = None
        # (starts, distinct ids, distinct count): the plan's run heads of that order (optional)
        self.heads: Optional[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]] = None
        # (device int64 [1], event): the plan's deduplicated count of these ids and an event recorded
        # after the plan (optional; valid with the order)
        self.plan_counts = None
        # callables run after a backward adds a slice (the data-parallel exchange starts its sparse
        # collectives from here, as soon as the tables' gradients exist), and a pending finisher the
        # exchange leaves (run by gathered() before the slices are read: the update waits there)
        self.listeners: List = []
        self.pending = None

    def add(self, ids: torch.Tensor, rows: torch.Tensor) -> None:
        """A backward's IndexedSlices for this table."""
        self.slices.append((ids, rows))
        for fn in list(self.listeners):
            fn(self)

    def clear(self):
        self.slices = []
        self.sumsq = None
        self.order = None
        self.heads = None
        self.plan_counts = None
        self.pending = None

    def resolve(self) -> None:
        """Run the pending finisher, if any (it sets slices / sumsq)."""
        fn, self.pending = self.pending, None
        if fn is not None:
            fn()

    def sorted_order(self) -> Optional[torch.Tensor]:
        """The order for gathered()'s ids when it applies (one slice, the same ids), else None."""
        self.resolve()
        if self.order is None or len(self.slices) != 1:
            return None
        ids, order = self.order
        got = self.slices[0][0]
        if got.data_ptr() != ids.data_ptr() or got.numel() != ids.numel() or order.numel() != ids.numel():
            return None
        return order

    def dedupe_plan(self):
        """(order, starts, distinct ids, count) of the id plan of this sink's one slice, or None."""
        o = self.sorted_order()
        if o is None or self.heads is None:
            return None
        return (o,) + tuple(self.heads)

    def early_count(self):
        """(device count, event) of the plan's deduplicated count when the plan describes this
        sink's one slice, else None."""
        return self.plan_counts if self.sorted_order() is not None else None

    def sorted_heads(self):
        """The plan's run heads of sorted_order() when both apply, else None."""
        return self.heads if self.sorted_order() is not None else None

    def gathered(self) -> Optional[Tuple[torch.Tensor, torch.Tensor]]:
        self.resolve()
        if not self.slices:
            return None
        if len(self.slices) == 1:
            return self.slices[0]
        return (torch.cat([s[0] for s in self.slices]), torch.cat([s[1] for s in self.slices]))


class EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, weight, sink):
        ctx.sink = sink
        ctx.save_for_backward(ids)
        return embedding_gather(weight, ids)

    @staticmethod
    def backward(ctx, g):
        (ids,) = ctx.saved_tensors
        ctx.sink.add(ids, g.contiguous())
        return None, None, None


class EmbeddingTablesFn(torch.autograd.Function):
    """Several tables looked up in one launch (the user and item Embeddings of a training step,
    src/models.py:85,89); each table's gradient goes to its own sink as IndexedSlices."""

    @staticmethod
    def forward(ctx, sinks, n_tables, orders, *args):
        # orders: None, or one int32 row order per table (the gather's read order; same result)
        ids, weights = args[:n_tables], args[n_tables:]
        ctx.sinks = sinks
        ctx.save_for_backward(*ids)
        return tuple(embedding_gather_tables(weights, ids, orders))

    @staticmethod
    def backward(ctx, *gs):
        for sink, ids, g in zip(ctx.sinks, ctx.saved_tensors, gs):
            if g is not None:
                sink.add(ids, g.contiguous())
        return (None, None, None) + (None,) * (2 * len(ctx.sinks))


class MultiEmbeddingFn(torch.autograd.Function):
    """x0 = [T_0[ids_0] || ... || dense || 0] (config 5). Each table's gradient is the matching
    column slice of dLoss/dx0, kept as a strided (ids, rows) IndexedSlices in the table's sink."""

    @staticmethod
    def forward(ctx, ids, dense, table_ptrs, num_rows, E, ld, sinks, *tables):
        ctx.sinks, ctx.E = sinks, E
        ctx.save_for_backward(ids)
        return multi_embedding_gather(table_ptrs, num_rows, E, ids, dense, ld)

    @staticmethod
    def backward(ctx, g):
        (ids,) = ctx.saved_tensors
        g = g.contiguous()
        E = ctx.E
        for f, sink in enumerate(ctx.sinks):
            sink.add(ids[f], g[:, f * E:(f + 1) * E])
        return (None,) * (7 + len(ctx.sinks))


DCN2_PLANES = True    # DCNCrossMatFn on the plane-image entry points at precision 6 (DCNCrossMatFn.forward)


class DCNCrossMatFn(torch.autograd.Function):
    """DCN-v2 matrix cross stack x_{l+1} = x0 * (x_l W_l + b_l) + x_l (config-5 extension)."""

    @staticmethod
    def forward(ctx, x0, W, b, precision: int = 0):
        x0 = x0.contiguous()
        # precision 6 runs the stack on the plane-pair GEMM (xgemm images, two cross products per
        # 16x16x32 MFMA, 256 x 256 tiles): 2.05 -> 1.73 ms per 16384 x 3344 x 3344 GEMM, DESIGN §3
        planes = DCN2_PLANES and precision == PREC_F32_SPLIT6 and W.shape[0] > 0
        if planes:   # pre-split operands on the LDS-DMA GEMM (rs_dcn_cross_mat_*_planes_f32)
            xs, us, ximg = dcn_cross_mat_fwd_planes(x0, W, b, precision)
            ctx.save_for_backward(x0, xs, us, W, ximg)
        else:
            xs, us = dcn_cross_mat_fwd(x0, W, b, precision)
            ctx.save_for_backward(x0, xs, us, W)
        ctx.precision, ctx.planes = precision, planes
        return xs[W.shape[0] - 1] if W.shape[0] > 0 else x0.clone()

    @staticmethod
    def backward(ctx, g):
        if ctx.planes:
            x0, xs, us, W, ximg = ctx.saved_tensors
            g_x0, gW, gb = dcn_cross_mat_bwd_planes(x0, xs, us, W, ximg, g.contiguous(), precision=ctx.precision)
        else:
            x0, xs, us, W = ctx.saved_tensors
            g_x0, gW, gb = dcn_cross_mat_bwd(x0, xs, us, W, g.contiguous(), precision=ctx.precision)
        return g_x0, gW, gb, None


class DCN2TrunkFn(torch.autograd.Function):
    """The DCN-v2 ranker's trunk (config 5) as one node at precision 6: the matrix cross stack
    (x_L, rs_dcn_cross_mat_*_planes_f32) and the ReLU deep tower h on x0 (the reference's deep
    net shape, src/models.py:26-29,46-48) with every GEMM on the plane-pair kernel. The tower's
    layer-1 weight gradient reuses the cross stack's image of x0^T, each activation's two images
    come from one read (rs_xgemm_image_dual_f32, the backward's with the ReLU mask and the bias
    gradient folded in), and the tower's dL/dx0 enters the cross backward as its extra term (no
    separate add). apply(x0, W, b, relus, W_1, b_1, ..., W_L, b_L) -> (x_L, h)."""

    @staticmethod
    def forward(ctx, x0, W, b, relus, *deep):
        ctx.set_materialize_grads(False)
        x0 = x0.contiguous()
        B, d = x0.shape
        xs, us, ximg, a_img = dcn_cross_mat_fwd_planes(x0, W, b, PREC_F32_SPLIT6, want_x0_img=True)
        L = len(relus)
        Ws, bs = deep[0::2], deep[1::2]
        hs, himg_t = [], []
        for k in range(L):
            K_in, N_out = Ws[k].shape
            h = xgemm(a_img, xgemm_image(Ws[k], trans=True), B, N_out, K_in, bias=bs[k], relu=relus[k])
            hs.append(h)
            if k + 1 < L:
                a_img, h_t, _ = xgemm_image_dual(h)
                himg_t.append(h_t)
        ctx.relus, ctx.L = tuple(relus), L
        ctx.save_for_backward(x0, xs, us, W, ximg, *hs, *himg_t, *Ws)
        _record_fwd_gates(Ws[0].data_ptr(), hs, relus)   # the masks the backward's images apply (hs > 0)
        return xs[W.shape[0] - 1], hs[-1]

    @staticmethod
    def backward(ctx, g_xl, g_h):
        relus, L = ctx.relus, ctx.L
        x0, xs, us, W, ximg, *rest = ctx.saved_tensors
        hs, himg_t, Ws = rest[:L], rest[L:2 * L - 1], rest[2 * L - 1:]
        B, d = x0.shape
        grads = [None] * (2 * L)
        g = g_h.contiguous() if g_h is not None else torch.zeros_like(hs[-1])
        dx0 = None
        for k in range(L - 1, -1, -1):
            K_in, N_out = Ws[k].shape
            g_img, g_img_t, db = xgemm_image_dual(g, relu_y=hs[k] if relus[k] else None, colsum=True)
            a_t = himg_t[k - 1] if k > 0 else ximg   # input^T images: h_{k-1}^T, or x0^T (the cross stack's)
            grads[2 * k] = xgemm_splitk(a_t, g_img_t, K_in, N_out, B)
            grads[2 * k + 1] = db
            g = xgemm(g_img, xgemm_image(Ws[k]), B, K_in, N_out)   # dL/d(input of layer k)
        dx0 = g
        if g_xl is None:
            g_xl = torch.zeros_like(x0)
        g_x0, gW, gb = dcn_cross_mat_bwd_planes(x0, xs, us, W, ximg, g_xl.contiguous(), g_x0_extra=dx0,
                                                precision=PREC_F32_SPLIT6)
        return (g_x0, gW, gb, None, *grads)


class DenseFn(torch.autograd.Function):
    """y = act(x W + b) (keras Dense, kernel [in, out])."""

    @staticmethod
    def forward(ctx, x, W, b, relu: bool, precision: int = 0):
        x = x.contiguous()
        y = gemm(x, W, bias=b, relu=relu, precision=precision)
        ctx.relu = relu
        ctx.precision = precision
        ctx.rq = _queue_of(W)
        ctx.save_for_backward(x, W, y if relu else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, W, y = ctx.saved_tensors
        g, db = relu_bwd_colsum(dy.contiguous(), y if ctx.relu else None, queue=ctx.rq)
        dx = gemm(g, W, trans_b=True, precision=ctx.precision) if ctx.needs_input_grad[0] else None
        dW = gemm_splitk(x, g, trans_a=True, precision=ctx.precision) if ctx.needs_input_grad[1] else None
        return dx, dW, db, None, None


# ReLU gate recorder (a test instrument): inside `with record_relu_gates() as rec:` every Dense-stack
# node (MLPFn, MLPGroupFn) records, per stack (keyed by its first kernel's address), the gates of its
# ReLU layers exactly as its backward applies them — its saved layer outputs y_k, the mask being
# y_k > 0 in every dX epilogue, chain kernel and column-sum pass — and, in the backward, the support
# of each ReLU layer's pre-activation gradient (which must lie inside that gate). The forward's
# kernels (one-launch stack or per-layer GEMMs) are whatever the node ran: no recomputation.
_GATE_RECORDERS: List[dict] = []


@contextlib.contextmanager
def record_relu_gates():
    """rec = {"fwd": {key: [bool tensor per ReLU layer]}, "bwd": {key: {layer: bool tensor}}},
    key = first_kernel.data_ptr() of the stack."""
    rec = {"fwd": {}, "bwd": {}}
    _GATE_RECORDERS.append(rec)
    try:
        yield rec
    finally:
        _GATE_RECORDERS.remove(rec)


def _record_fwd_gates(key: int, ys, relus):
    if _GATE_RECORDERS:
        _GATE_RECORDERS[-1]["fwd"][key] = [y > 0 for y, r in zip(ys, relus) if r]


def _record_bwd_support(key: int, layer: int, g):
    if _GATE_RECORDERS and g is not None:
        _GATE_RECORDERS[-1]["bwd"].setdefault(key, {})[layer] = g != 0


# attribute on a gradient tensor whose producer already applied the ReLU of the layer it flows
# into (HeadsLossTotalFn with relu_h): that layer's backward does not mask it again
RELU_APPLIED = "_rs_relu_applied"
RS_HEADS_USE_CTR, RS_HEADS_RELU_H = 1, 2   # include/recsys_hip.h


class MLPFn(torch.autograd.Function):
    """A stack of keras Dense layers y_k = act_k(x_k W_k + b_k) (act: ReLU or linear; a Tower,
    src/models.py:76-77, or the DCN deep net, :26-29,46-48) as one autograd node. The backward
    runs two launches per layer instead of the per-layer form's five: the ReLU mask of layer k - 1
    is applied in the epilogue of layer k's dX GEMM (mask = x_k = y_{k-1} > 0, TF's ReluGrad), and
    dW_k and db_k come out of one split-K GEMM (rs_gemm_wgrad_bias: db = the all-ones row of x_k^T
    times g). A ReLU on the top layer is masked by relu_bwd_colsum.
    With l2 > 0 (keras.regularizers.l2 on the kernels, :27) the node also returns the regularizer
    l2 * sum_k ||W_k||^2 (one multi-tensor pass) and folds its gradient 2 l2 g_reg W_k into the
    dW reduction (g_reg read on the device): no separate penalty node, no gradient-accumulation adds."""

    @staticmethod
    def forward(ctx, x, relus, precision, l2, *params):
        ctx.set_materialize_grads(False)
        x = x.contiguous()
        L = len(relus)
        xs = [x]
        if mlp_fused_ok(x.shape[0], x.shape[1], params[0::2], precision) and x.data_ptr() % 16 == 0:
            ctx.img = mlp_weight_image([params[0::2]])
            xs += [ys[0] for ys in mlp_forward([x], [params[0::2]], [params[1::2]], relus, precision, img=ctx.img)]
        else:
            for k in range(L):
                xs.append(gemm(xs[-1], params[2 * k], bias=params[2 * k + 1], relu=relus[k], precision=precision))
        ctx.relus, ctx.precision, ctx.l2 = tuple(relus), precision, float(l2)
        ctx.rq = _queue_of(params[0])
        ctx.gate_key = params[0].data_ptr()
        _record_fwd_gates(ctx.gate_key, xs[1:], relus)
        ctx.save_for_backward(*xs, *params[0::2])
        if l2 > 0:
            return xs[-1], sum_squares_multi(list(params[0::2]), l2)
        return xs[-1]

    @staticmethod
    def backward(ctx, dy, dreg=None):
        relus, prec, l2 = ctx.relus, ctx.precision, ctx.l2
        L = len(relus)
        saved = ctx.saved_tensors
        xs, Ws = saved[: L + 1], saved[L + 1:]
        use_reg = l2 > 0 and dreg is not None
        grads = [None] * (2 * L)
        dx = None
        if dy is None:   # only the regularizer is used
            if use_reg:
                for k in range(L):
                    grads[2 * k] = Ws[k] * (2.0 * l2) * dreg
            return (None, None, None, None, *grads)
        g = dy.contiguous()
        if relus[-1] and not getattr(dy, RELU_APPLIED, False):   # (else its producer masked it)
            g, _ = relu_bwd_colsum(g, xs[L], queue=ctx.rq)
        dims = [Ws[0].shape[0]] + [W.shape[1] for W in Ws]
        if mlp_chain_ok(g.shape[0], dims, prec, ctx.needs_input_grad[0]) and g.data_ptr() % 16 == 0:
            # the whole input-gradient chain in one launch, then the weight gradients
            gin = [t[0] for t in mlp_backward_chain([g], [Ws], [xs[1:]], relus, prec, ctx.needs_input_grad[0],
                                                    img=getattr(ctx, "img", None))]
            gl = [gin[k + 1] for k in range(L - 1)] + [g]
            if _GATE_RECORDERS:
                for k in range(L):
                    if relus[k]:
                        _record_bwd_support(ctx.gate_key, k, gl[k])
            if mlp_wgrad_ok(dims, prec):
                wg = mlp_wgrad([list(xs[:L])], [gl], prec, W_lists=[list(Ws)] if use_reg else None,
                               w_scale=2.0 * l2, w_dscale=dreg.reshape(()) if use_reg else None, queue=ctx.rq)[0]
                for k in range(L):
                    grads[2 * k], grads[2 * k + 1] = wg[k]
                return (gin[0], None, None, None, *grads)
            for k in range(L - 1, -1, -1):
                gk = g if k == L - 1 else gin[k + 1]
                grads[2 * k], grads[2 * k + 1] = gemm_wgrad_bias(
                    xs[k], gk, prec, W=Ws[k] if use_reg else None, w_scale=2.0 * l2,
                    w_dscale=dreg.reshape(()) if use_reg else None, queue=ctx.rq)
            return (gin[0], None, None, None, *grads)
        if g.shape[0] <= MLP_WGRAD_MAX_M and mlp_wgrad_ok(dims, prec):
            # the per-layer dX GEMMs, then every layer's weight gradients in one launch
            gl = [None] * L
            gl[L - 1] = g
            for k in range(L - 1, 0, -1):
                gl[k - 1] = gemm(gl[k], Ws[k], trans_b=True, mask=xs[k] if relus[k - 1] else None, precision=prec)
            if ctx.needs_input_grad[0]:
                dx = gemm(gl[0], Ws[0], trans_b=True, precision=prec)
            if _GATE_RECORDERS:
                for k in range(L):
                    if relus[k]:
                        _record_bwd_support(ctx.gate_key, k, gl[k])
            wg = mlp_wgrad([list(xs[:L])], [gl], prec, W_lists=[list(Ws)] if use_reg else None,
                           w_scale=2.0 * l2, w_dscale=dreg.reshape(()) if use_reg else None, queue=ctx.rq)[0]
            for k in range(L):
                grads[2 * k], grads[2 * k + 1] = wg[k]
            return (dx, None, None, None, *grads)
        for k in range(L - 1, -1, -1):
            if relus[k]:
                _record_bwd_support(ctx.gate_key, k, g)
            dW, db = gemm_wgrad_bias(xs[k], g, prec, W=Ws[k] if use_reg else None, w_scale=2.0 * l2,
                                     w_dscale=dreg.reshape(()) if use_reg else None, queue=ctx.rq)
            grads[2 * k], grads[2 * k + 1] = dW, db
            if k > 0:
                g = gemm(g, Ws[k], trans_b=True, mask=xs[k] if relus[k - 1] else None, precision=prec)
            elif ctx.needs_input_grad[0]:
                dx = gemm(g, Ws[k], trans_b=True, precision=prec)
        return (dx, None, None, None, *grads)


class MLPGroupFn(torch.autograd.Function):
    """G stacks of keras Dense layers with one shape (the user and item towers, src/models.py:76-77,
    86, 90) as one autograd node whose every launch serves all G stacks: per layer one grouped
    GEMM forward, one grouped dW + db GEMM (+ one reduction) and one grouped dX GEMM backward
    (rs_gemm_group / rs_gemm_wgrad_bias_group), each stack's results bitwise its MLPFn's.
    apply(relus, precision, G, x_0 .. x_{G-1}, W/b of stack 0 .., W/b of stack 1 .., ...)."""

    @staticmethod
    def forward(ctx, relus, precision, G, *args):
        ctx.set_materialize_grads(False)
        L = len(relus)
        xs0, params = [x.contiguous() for x in args[:G]], args[G:]
        P = [params[2 * L * g: 2 * L * (g + 1)] for g in range(G)]
        xs = [xs0]
        M, K0 = xs0[0].shape
        if (G <= 2 and all(mlp_fused_ok(M, K0, P[g][0::2], precision) and x.shape == xs0[0].shape
                           and x.data_ptr() % 16 == 0 for g, x in enumerate(xs0))):
            ctx.img = mlp_weight_image([P[g][0::2] for g in range(G)])
            xs += mlp_forward(xs0, [P[g][0::2] for g in range(G)], [P[g][1::2] for g in range(G)], relus, precision,
                              img=ctx.img)
        dims = [K0] + [P[0][2 * k].shape[1] for k in range(L)]
        fimg = cimg = None
        if (len(xs) == 1 and SKINNY_IMG and precision == PREC_F32_SPLIT6 and 1 <= L <= 6
                and all(d % 32 == 0 for d in dims) and M >= 16384):
            ctx.img = mlp_weight_image([P[g][0::2] for g in range(G)])
            fimg, cimg = mlp_layer_images(ctx.img, dims)
        ctx.cimg = cimg
        for k in range(len(xs) - 1, L):
            xs.append(gemm_group(xs[-1], [P[g][2 * k] for g in range(G)], bias=[P[g][2 * k + 1] for g in range(G)],
                                 relu=relus[k], precision=precision, b_img=fimg[k] if fimg else None))
        ctx.relus, ctx.precision, ctx.G = tuple(relus), precision, G
        ctx.rq = _queue_of(params[0])
        ctx.gate_keys = [P[g][0].data_ptr() for g in range(G)]
        for g in range(G):
            _record_fwd_gates(ctx.gate_keys[g], [xs[k + 1][g] for k in range(L)], relus)
        ctx.save_for_backward(*[t for layer in xs for t in layer], *[P[g][2 * k] for g in range(G) for k in range(L)])
        return tuple(xs[-1])

    @staticmethod
    def backward(ctx, *dys):
        relus, prec, G = ctx.relus, ctx.precision, ctx.G
        L = len(relus)
        saved = ctx.saved_tensors
        xs = [list(saved[G * k: G * (k + 1)]) for k in range(L + 1)]
        Ws = [saved[G * (L + 1) + g * L: G * (L + 1) + (g + 1) * L] for g in range(G)]
        grads = [[None] * (2 * L) for _ in range(G)]
        dx = [None] * G
        if any(d is None for d in dys):
            dys = [d if d is not None else torch.zeros_like(xs[L][g]) for g, d in enumerate(dys)]
        gs = [d.contiguous() for d in dys]
        if relus[-1]:
            gs = [relu_bwd_colsum(gs[g], xs[L][g], queue=ctx.rq)[0] for g in range(G)]
        dims = [Ws[0][0].shape[0]] + [W.shape[1] for W in Ws[0]]
        want_dx = any(ctx.needs_input_grad[3: 3 + G])
        if (G <= 2 and mlp_chain_ok(gs[0].shape[0], dims, prec, want_dx)
                and all(t.data_ptr() % 16 == 0 for t in gs)):
            gin = mlp_backward_chain(gs, Ws, [[xs[l + 1][g] for l in range(L)] for g in range(G)],
                                     relus, prec, want_dx, img=getattr(ctx, "img", None))
            if _GATE_RECORDERS:
                for k in range(L):
                    if relus[k]:
                        for g in range(G):
                            _record_bwd_support(ctx.gate_keys[g], k, gs[g] if k == L - 1 else gin[k + 1][g])
            if mlp_wgrad_ok(dims, prec):
                wg = mlp_wgrad([[xs[k][g] for k in range(L)] for g in range(G)],
                               [[gin[k + 1][g] for k in range(L - 1)] + [gs[g]] for g in range(G)], prec,
                               queue=ctx.rq)
                for g in range(G):
                    for k in range(L):
                        grads[g][2 * k], grads[g][2 * k + 1] = wg[g][k]
            for k in range(L - 1, -1, -1):
                if grads[0][2 * k] is not None:
                    break
                gk = gs if k == L - 1 else gin[k + 1]
                for g, (dW, db) in enumerate(gemm_wgrad_bias_group([xs[k][g] for g in range(G)], gk, prec,
                                                                          queue=ctx.rq)):
                    grads[g][2 * k], grads[g][2 * k + 1] = dW, db
            dx = gin[0] if want_dx else dx
            return (None, None, None, *dx, *[t for g in range(G) for t in grads[g]])
        if G <= 2 and gs[0].shape[0] <= MLP_WGRAD_MAX_M and mlp_wgrad_ok(dims, prec):
            # the per-layer dX GEMMs, then every layer's weight gradients in one launch
            gl = [None] * L
            gl[L - 1] = gs
            ci = getattr(ctx, "cimg", None)
            for k in range(L - 1, 0, -1):
                gl[k - 1] = gemm_group(gl[k], [Ws[g][k] for g in range(G)], trans_b=True,
                                       mask=[xs[k][g] for g in range(G)] if relus[k - 1] else None, precision=prec,
                                       b_img=ci[k] if ci else None)
            if want_dx:
                dx = gemm_group(gl[0], [Ws[g][0] for g in range(G)], trans_b=True, precision=prec,
                                b_img=ci[0] if ci else None)
            if _GATE_RECORDERS:
                for k in range(L):
                    if relus[k]:
                        for g in range(G):
                            _record_bwd_support(ctx.gate_keys[g], k, gl[k][g])
            wg = mlp_wgrad([[xs[k][g] for k in range(L)] for g in range(G)],
                           [[gl[k][g] for k in range(L)] for g in range(G)], prec, queue=ctx.rq)
            for g in range(G):
                for k in range(L):
                    grads[g][2 * k], grads[g][2 * k + 1] = wg[g][k]
            return (None, None, None, *dx, *[t for g in range(G) for t in grads[g]])
        for k in range(L - 1, -1, -1):
            if relus[k]:
                for g in range(G):
                    _record_bwd_support(ctx.gate_keys[g], k, gs[g])
            res = gemm_wgrad_bias_group([xs[k][g] for g in range(G)], gs, prec, queue=ctx.rq)
            for g, (dW, db) in enumerate(res):
                grads[g][2 * k], grads[g][2 * k + 1] = dW, db
            ci = getattr(ctx, "cimg", None)
            if k > 0:
                gs = gemm_group(gs, [Ws[g][k] for g in range(G)], trans_b=True,
                                mask=[xs[k][g] for g in range(G)] if relus[k - 1] else None, precision=prec,
                                b_img=ci[k] if ci else None)
            elif any(ctx.needs_input_grad[3: 3 + G]):
                dx = gemm_group(gs, [Ws[g][0] for g in range(G)], trans_b=True, precision=prec,
                                b_img=ci[0] if ci else None)
        return (None, None, None, *dx, *[t for g in range(G) for t in grads[g]])


# The towers over a batch's distinct ids (models.MultiTaskModel with an id plan): a tower row is a
# function of its id alone (src/models.py:85-90), so the lookups and the Dense forward run over the
# plan's distinct ids (the device-side counts bound the rows the kernels touch) and the outputs are
# expanded to the batch rows by the plan's inverse map. Backward per batch row, as autograd would:
# dW over the batch rows with each layer input read through the inverse map, dX with the ReLU masks
# read through it, the embedding gradients per batch row into the tables' sinks. Every value is
# bitwise the per-row towers' (same kernels and per-row arithmetic, the same contraction order).
DISTINCT_TOWERS = True


def distinct_towers_ok(B: int, stacks, precision: int) -> bool:
    """The shapes DistinctTowersFn serves: two identical stacks (linear top), precision 6 / 9, every
    width in {64, 128, 256} and >= 32768 rows over both towers (the weight-stationary kernel), above
    the fused-stack batch limit (so the per-row towers it replaces run the same kernels: the results
    are bitwise theirs)."""
    if not DISTINCT_TOWERS or precision not in (PREC_F32_SPLIT6, PREC_F32_SPLIT9) or 2 * B < 32768:
        return False
    if B <= MLP_FUSED_MAX_M:
        return False
    if stacks and stacks[0] and stacks[0][0].kernel.shape[0] not in GATHER_ROWS_DIMS:
        return False   # the distinct-row gather's compiled widths
    if len(stacks) != 2 or len(stacks[0]) != len(stacks[1]) or not stacks[0]:
        return False
    for a, b in zip(*stacks):
        if a.kernel.shape != b.kernel.shape or a.activation != b.activation or a.precision != precision:
            return False
        if a.kernel.shape[0] not in (64, 128, 256) or a.kernel.shape[1] not in (64, 128, 256):
            return False
    return stacks[0][-1].activation != "relu"


class DistinctTowersFn(torch.autograd.Function):
    """apply(sinks, relus, precision, plans, user_ids, item_ids, user_table, item_table, W/b of the
    user tower ..., W/b of the item tower ...) -> (u, i) [B, D] each. plans = the id plan's two sides
    (rep, count, inv, info side [2], info, ...)."""

    @staticmethod
    def forward(ctx, sinks, relus, precision, plans, uid, iid, utab, itab, *params):
        ctx.set_materialize_grads(False)
        L = len(relus)
        B = uid.shape[0]
        P = [params[:2 * L], params[2 * L:]]
        reps = [plans[0][0], plans[1][0]]
        invs = [plans[0][2], plans[1][2]]
        cnts = [plans[0][3][0:1], plans[1][3][0:1]]   # device int64: the distinct-row counts
        if len(plans[0]) > 6:   # the plan's distinct ids: one dependent load before the row stream
            xs = [embedding_gather_tables_ids([utab, itab], [plans[0][6], plans[1][6]])]
        else:
            xs = [embedding_gather_tables_rows([utab, itab], [uid, iid], reps, cnts)]
        for k in range(L):
            wb = dict(bias=[P[0][2 * k + 1], P[1][2 * k + 1]], relu=relus[k], precision=precision)
            if k < L - 1:   # hidden layers once per distinct id
                xs.append(gemm_group(xs[-1], [P[0][2 * k], P[1][2 * k]], m_dev=cnts, **wb))
            else:           # the top layer per batch row, its input read through the inverse map
                xs.append(gemm_group(xs[-1], [P[0][2 * k], P[1][2 * k]], a_rows=invs, m_rows=B, **wb))
        outs = list(xs[-1])
        ctx.relus, ctx.precision, ctx.sinks = tuple(relus), precision, sinks
        ctx.rq = _queue_of(params[0])
        ctx.gate_keys = [P[0][0].data_ptr(), P[1][0].data_ptr()]
        if _GATE_RECORDERS:
            inv64 = [v.long() for v in invs]
            for g in range(2):
                _record_fwd_gates(ctx.gate_keys[g], [xs[k + 1][g].index_select(0, inv64[g]) if k < L - 1
                                                     else xs[k + 1][g] for k in range(L)], relus)
        ctx.save_for_backward(uid, iid, invs[0], invs[1], *[t for layer in xs for t in layer],
                              *[P[g][2 * k] for g in range(2) for k in range(L)])
        return tuple(outs)

    @staticmethod
    def backward(ctx, du, dc):
        relus, prec = ctx.relus, ctx.precision
        L = len(relus)
        saved = ctx.saved_tensors
        uid, iid, inv_u, inv_c = saved[:4]
        xs = [list(saved[4 + 2 * k: 6 + 2 * k]) for k in range(L + 1)]
        Ws = [saved[6 + 2 * L + g * L: 6 + 2 * L + (g + 1) * L] for g in range(2)]
        invs = [inv_u, inv_c]
        gs = [d.contiguous() if d is not None else torch.zeros_like(xs[L][g]) for g, d in enumerate((du, dc))]
        grads = [[None] * (2 * L) for _ in range(2)]
        for k in range(L - 1, -1, -1):
            if relus[k]:
                for g in range(2):
                    _record_bwd_support(ctx.gate_keys[g], k, gs[g])
            res = gemm_wgrad_bias_group([xs[k][0], xs[k][1]], gs, prec, queue=ctx.rq, x_rows=invs)
            for g, (dW, db) in enumerate(res):
                grads[g][2 * k], grads[g][2 * k + 1] = dW, db
            if k > 0:
                masked = relus[k - 1]
                gs = gemm_group(gs, [Ws[g][k] for g in range(2)], trans_b=True,
                                mask=[xs[k][0], xs[k][1]] if masked else None, precision=prec,
                                mask_rows=invs if masked else None)
            else:
                dx = gemm_group(gs, [Ws[g][0] for g in range(2)], trans_b=True, precision=prec)
                for sink, ids, d in zip(ctx.sinks, (uid, iid), dx):
                    sink.add(ids, d.contiguous())
        return (None, None, None, None, None, None, None, None, *[t for g in range(2) for t in grads[g]])


class LossCombineFn(torch.autograd.Function):
    """compute_loss's w_ret ret + w_rat l_rat + w_ctr l_ctr (src/models.py:147) as one launch
    forward and one backward (rs_loss_combine_f32); l_ctr may be None (no CTR labels, :140)."""

    @staticmethod
    def forward(ctx, ret, l_rat, l_ctr, w_ret: float, w_rat: float, w_ctr: float):
        ctx.w = (float(w_ret), float(w_rat), float(w_ctr))
        ctx.has_ctr = l_ctr is not None
        total = torch.empty((), dtype=torch.float32, device=ret.device)
        call("rs_loss_combine_f32", _p(ret), _p(l_rat), _p(l_ctr), *ctx.w, _p(total), _stream())
        return total

    @staticmethod
    def backward(ctx, g):
        grads = torch.empty(3, dtype=torch.float32, device=g.device)
        call("rs_loss_combine_bwd_f32", _p(g.contiguous()), *ctx.w, _p(grads), _stream())
        return grads[0], grads[1], grads[2] if ctx.has_ctr else None, None, None, None


class DCNCrossFn(torch.autograd.Function):
    """(x0, xL) = concat + vector cross stack (src/models.py:128, 38-44)."""

    @staticmethod
    def forward(ctx, u, v, w, b):
        x0, xl, s = dcn_cross_fwd(u.contiguous(), v.contiguous(), w, b)
        ctx.rq = _queue_of(w)
        ctx.save_for_backward(x0, s, w, b)
        return x0, xl

    @staticmethod
    def backward(ctx, g_x0, g_xl):
        x0, s, w, b = ctx.saved_tensors
        if g_xl is None:
            g_xl = torch.zeros_like(x0)
        g_u, g_v, gw, gb = dcn_cross_bwd(x0, s, w, b, g_xl.contiguous(),
                                         g_x0.contiguous() if g_x0 is not None else None, queue=ctx.rq)
        return g_u, g_v, gw, gb


class HeadsFn(torch.autograd.Function):
    """rating_head / ctr_head on z = [xL || h] (src/models.py:50,119-120,131)."""

    @staticmethod
    def forward(ctx, xl, h, w_r, b_r, w_c, b_c):
        r, p = heads_fwd(xl.contiguous(), h.contiguous(), w_r, b_r, w_c, b_c)
        ctx.rq = _queue_of(w_r)
        ctx.save_for_backward(xl, h, w_r, w_c, p)
        return r, p

    @staticmethod
    def backward(ctx, g_r, g_p):
        xl, h, w_r, w_c, p = ctx.saved_tensors
        outs = heads_bwd(xl.contiguous(), h.contiguous(), w_r, w_c, p,
                         g_r=g_r.contiguous() if g_r is not None else None,
                         g_p=g_p.contiguous() if g_p is not None else None, queue=ctx.rq)
        return outs


class HeadsRankingLossFn(torch.autograd.Function):
    """Heads + Ranking(MSE) + Ranking(BCE, class weights) fused (src/models.py:119-145).
    Outputs (rating [B,1], ctr [B,1], rating_loss, ctr_loss)."""

    @staticmethod
    def forward(ctx, xl, h, w_r, b_r, w_c, b_c, rating, y_implicit, class_weights, ctr_mode):
        ctx.set_materialize_grads(False)   # unused outputs (r, p in compute_loss) cost no zero fills
        xl, h = xl.contiguous(), h.contiguous()
        r, p = heads_fwd(xl, h, w_r, b_r, w_c, b_c)
        loss, unit_r, unit_c = ranking_losses(r, p, rating, y_implicit, class_weights, ctr_mode)
        ctx.rq = _queue_of(w_r)
        ctx.save_for_backward(xl, h, w_r, w_c, p, unit_r, unit_c)
        return r, p, loss[0], loss[1]

    @staticmethod
    def backward(ctx, g_r, g_p, g_lr, g_lc):
        xl, h, w_r, w_c, p, unit_r, unit_c = ctx.saved_tensors
        gs_r = g_lr.contiguous() if g_lr is not None else None
        gs_c = g_lc.contiguous() if g_lc is not None else None
        outs = heads_bwd(xl, h, w_r, w_c, p,
                         g_r=g_r.contiguous() if g_r is not None else None,
                         g_p=g_p.contiguous() if g_p is not None else None,
                         unit_r=unit_r, unit_c=unit_c, gs_rat=gs_r, gs_ctr=gs_c, queue=ctx.rq)
        return (*outs, None, None, None, None)


class HeadsLossTotalFn(torch.autograd.Function):
    """The rating / CTR heads, both Ranking tasks and compute_loss's task weighting — with the train
    step's regularizer added — as one node (src/models.py:119-147; the regularizer is the one
    tfrs.models.Model.train_step adds): outputs (total, total + reg, rating_loss, ctr_loss). Forward:
    heads_fwd + one ranking/combine launch sequence (one launch up to B = 16384); backward: one
    heads launch that also forms g * w_task and the retrieval term's gradient. The per-task losses
    are reported, not differentiated through (mark_non_differentiable). relu_h: h is the output of a
    ReLU layer (the DCN deep net's top, src/models.py:26-29); its gradient then leaves this node
    already masked (the deep net's MLPFn skips its own relu_bwd_colsum launch, RELU_APPLIED)."""

    @staticmethod
    def forward(ctx, xl, h, w_r, b_r, w_c, b_c, ret, reg, rating, y_implicit, class_weights, ctr_mode,
                w_ret, w_rat, w_ctr, use_ctr, relu_h=False):
        ctx.set_materialize_grads(False)
        xl, h = xl.contiguous(), h.contiguous()
        r, p = heads_fwd(xl, h, w_r, b_r, w_c, b_c)
        loss, total, total_reg, unit_r, unit_c = ranking_losses_combine(
            r, p, rating, y_implicit, class_weights, ctr_mode, ret, reg, w_ret, w_rat, w_ctr, use_ctr)
        ctx.rq = _queue_of(w_r)
        ctx.w = (float(w_ret), float(w_rat), float(w_ctr), bool(use_ctr))
        ctx.relu_h = bool(relu_h)
        ctx.has_reg = reg is not None
        ctx.save_for_backward(xl, h, w_r, w_c, p, unit_r, unit_c)
        l_rat, l_ctr = loss[0], loss[1]
        ctx.mark_non_differentiable(l_rat, l_ctr)
        return total, total_reg, l_rat, l_ctr

    @staticmethod
    def backward(ctx, g_total, g_total_reg, _g_lr, _g_lc):
        nones = (None,) * 9
        if g_total is None and g_total_reg is None:
            return (None,) * 8 + nones
        g = g_total if g_total_reg is None else (g_total_reg if g_total is None else g_total + g_total_reg)
        xl, h, w_r, w_c, p, unit_r, unit_c = ctx.saved_tensors
        w_ret, w_rat, w_ctr, use_ctr = ctx.w
        outs = heads_bwd_combine(xl, h, w_r, w_c, p, unit_r, unit_c, g.contiguous(), w_ret, w_rat, w_ctr, use_ctr,
                                 queue=ctx.rq, relu_h=ctx.relu_h)
        if ctx.relu_h:
            setattr(outs[1], RELU_APPLIED, True)
        g_reg = g_total_reg if ctx.has_reg else None
        return (*outs, g_reg) + nones


def _inbatch_forward(ctx, U, C, precision, ids, want):
    """InBatchSoftmaxFn's forward on contiguous U, C; keeps its backward state on ctx."""
    B = U.shape[0]
    scores = None
    if want and query("rs_inbatch_scores_bytes", B) <= INBATCH_STORE_SCORES_MAX_BYTES:
        scores = inbatch_scores_buffer(B, U.device)
    plan = inbatch_dedup_plan(U, C, precision, ids=ids) if scores is not None else None
    # the forward's workspace is kept for the backward when it holds the split image of U the
    # backward's col pass streams (D = 128 at a split precision): one split launch fewer
    keep = scores is not None and want and U.shape[1] == 128 and precision in (PREC_F32_SPLIT6, PREC_F32_SPLIT9)
    ws = inbatch_workspace(B, U.shape[1], U.device, dedup=plan is not None) if keep else None
    if plan is not None:
        tot, row, lse, dU, _ = inbatch_softmax_fwd_dedup(U, C, plan[0], plan[1], scores, precision, workspace=ws)
    else:
        tot, row, lse, dU, _ = inbatch_softmax_fwd(U, C, 1.0, want_grad=want, scores=scores, precision=precision,
                                                   workspace=ws)
    ctx.ib = (lse, dU, scores, precision, plan, ws)
    return tot, row


def _inbatch_backward(ctx, U, C, g):
    lse, dU_unit, scores, precision, plan, ws = ctx.ib
    if plan is not None:
        return inbatch_softmax_bwd_dedup(U, lse, plan[0], plan[1], scores, precision, gscale=g.contiguous(),
                                         dU_unit=dU_unit, workspace=ws)
    return inbatch_softmax_bwd(U, C, lse, gscale=g.contiguous(), dU_unit=dU_unit, scores=scores,
                               precision=precision, workspace=ws)


class InBatchSoftmaxFn(torch.autograd.Function):
    """tfrs.tasks.Retrieval() loss (SUM over the batch) with in-batch negatives."""

    @staticmethod
    def forward(ctx, U, C, precision: int = PREC_F32, ids=None):
        # ids: (user_ids, item_ids, user_rows, item_rows) when U and C are functions of the ids alone
        # (MultiTaskModel's towers): the deduplicated pair then finds distinct rows by id
        ctx.set_materialize_grads(False)   # the per-row losses are non-differentiable
        U, C = U.contiguous(), C.contiguous()
        tot, row = _inbatch_forward(ctx, U, C, precision, ids, ctx.needs_input_grad[0] or ctx.needs_input_grad[1])
        ctx.save_for_backward(U, C)
        ctx.mark_non_differentiable(row)
        return tot, row

    @staticmethod
    def backward(ctx, g, _g_row):
        if g is None:
            return None, None, None, None
        U, C = ctx.saved_tensors
        dU, dC = _inbatch_backward(ctx, U, C, g)
        return dU, dC, None, None


class RetrievalCrossFn(torch.autograd.Function):
    """The retrieval task (src/models.py:137) and the DCN-v1 concat + cross stack (:128, 38-44) on the
    same tower outputs as one node: (loss_sum, row_loss, x0, x_L). Its backward runs the in-batch
    pair first and hands dU, dC to the cross kernel, which adds them last to dL/du, dL/dv
    (rs_dcn_cross_vec_bwd_add_f32) — the same sums as autograd's accumulation of the two consumers,
    without the two [B, D] accumulation passes."""

    @staticmethod
    def forward(ctx, u, v, w, b, precision: int = PREC_F32, ids=None):
        ctx.set_materialize_grads(False)
        u, v = u.contiguous(), v.contiguous()
        tot, row = _inbatch_forward(ctx, u, v, precision, ids, ctx.needs_input_grad[0] or ctx.needs_input_grad[1])
        x0, xl, s = dcn_cross_fwd(u, v, w, b)
        ctx.rq = _queue_of(w)
        ctx.save_for_backward(u, v, x0, s, w, b)
        ctx.mark_non_differentiable(row)
        return tot, row, x0, xl

    @staticmethod
    def backward(ctx, g_tot, _g_row, g_x0, g_xl):
        u, v, x0, s, w, b = ctx.saved_tensors
        dU = dC = None
        if g_tot is not None:
            dU, dC = _inbatch_backward(ctx, u, v, g_tot)
        if g_xl is None:
            g_xl = torch.zeros_like(x0)
        g_u, g_v, gw, gb = dcn_cross_bwd(x0, s, w, b, g_xl.contiguous(),
                                         g_x0.contiguous() if g_x0 is not None else None, add_u=dU, add_v=dC,
                                         queue=ctx.rq)
        return g_u, g_v, gw, gb, None, None


class L2PenaltyFn(torch.autograd.Function):
    """l2 * sum_k ||W_k||^2 (keras.regularizers.l2 on the DCN deep kernels, src/models.py:27)."""

    @staticmethod
    def forward(ctx, l2, *weights):
        ctx.l2 = l2
        ctx.save_for_backward(*weights)
        if len(weights) <= 8:
            return sum_squares_multi(list(weights), l2)
        tot = sum_squares(weights[0], l2)
        for w in weights[1:]:
            tot = tot + sum_squares(w, l2)
        return tot

    @staticmethod
    def backward(ctx, g):
        ws = ctx.saved_tensors
        return (None, *[w * (2.0 * ctx.l2) * g for w in ws])
