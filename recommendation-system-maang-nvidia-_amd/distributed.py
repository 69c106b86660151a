"""Single-node data parallelism: one process per GPU, RCCL over xGMI.

Reference: tf.distribute.MirroredStrategy (src/trainer.py:45-48, variables created under
strategy.scope() at :148) [TF-ext semantics]:
  * every replica gets global_batch / N rows and computes ITS OWN loss — the in-batch softmax
    negatives are per replica — and per-replica losses are not divided by N;
  * dense gradients are all-reduced with SUM;
  * embedding gradients (IndexedSlices) are all-gathered: values and indices concatenated in
    replica order, then clipped / deduplicated / applied identically on every replica.

The exchange (MirroredGradientExchange, an optimizer pre-apply hook):
  * dense gradients: SUM all-reduce in ~32 MB buckets launched from post-accumulate-grad hooks
    DURING the backward (BucketedGradAllReduce: buckets in reverse parameter order, i.e. in the
    order their gradients become ready, launched strictly in bucket order so every rank issues the
    same collective sequence); the step waits only for what has not finished, and the gradients
    become views of the reduced buckets (no copy back). Without hooks: one flat bucket at the end.
  * embedding gradients, "dedupe" mode (default): each replica deduplicates its rows locally
    (rs_sparse_dedupe_f32: ~40 % of the rows remain for Zipf ids), the replicas' raw sums of
    squares are SUM-all-reduced (the Keras clip norm is over the un-deduplicated rows of all
    replicas), and the unique (id, row) pairs of ALL tables go out in one all-gather (plus one
    for the ids) after one tiny all-gather of the per-table counts (the step's one host sync).
    The update then runs with that external norm (rs_sparse_adagrad_sumsq_f32); clip_by_norm is
    linear, so this equals clipping the raw rows up to rounding. "padded" mode: fixed per-rank
    capacity (max_rows), id -1 / zero-row padding, no host sync (graph-capturable); the raw rows
    of every replica are applied as they are.
Every rank then runs the same deterministic update kernels on the same data, so replicas stay
bit-identical without any broadcast. Works with "nccl" (RCCL) and with "gloo" for CPU tests.
"""
from __future__ import annotations

import os
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist


def env_world() -> Tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torchrun environment (defaults: single process)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init_process_group(backend: Optional[str] = None) -> bool:
    """Initialise torch.distributed from env if WORLD_SIZE > 1; returns True when distributed."""
    rank, world, local = env_world()
    if world <= 1:
        return False
    if dist.is_initialized():
        return True
    # RS_DIST_BACKEND=gloo rehearses the multi-rank path with several ranks on one GPU (the 1-GPU
    # box); the product path is RCCL ("nccl"), one rank per GPU
    backend = os.environ.get("RS_DIST_BACKEND", backend)
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend == "nccl":
        torch.cuda.set_device(local)
        dist.init_process_group(backend, rank=rank, world_size=world,
                                device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend, rank=rank, world_size=world)
    return True


def flat_allreduce_(tensors: Sequence[torch.Tensor], group=None, bucket_bytes: int = 64 << 20) -> None:
    """SUM-all-reduce a list of same-device fp32 tensors in place through flat buckets."""
    if not tensors:
        return
    bucket: List[torch.Tensor] = []
    size = 0

    def flush():
        nonlocal bucket, size
        if not bucket:
            return
        flat = torch.cat([t.reshape(-1) for t in bucket])
        dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
        off = 0
        for t in bucket:
            n = t.numel()
            t.copy_(flat[off: off + n].view_as(t))
            off += n
        bucket, size = [], 0

    for t in tensors:
        bucket.append(t)
        size += t.numel() * t.element_size()
        if size >= bucket_bytes:
            flush()
    flush()


class BucketedGradAllReduce:
    """Dense-gradient SUM all-reduce overlapped with the backward.

    Parameters are grouped into buckets of about `bucket_bytes` in REVERSE order (the order the
    backward produces their gradients); a bucket is launched (its gradients copied into one flat
    buffer, then an async all-reduce) as soon as all of its gradients exist and every earlier
    bucket has been launched, so all ranks issue identical collective sequences. ``finish()``
    launches what is left (a gradient the step did not produce contributes zeros), waits, and
    points every .grad at its slice of the reduced buffer."""

    def __init__(self, params: Sequence[torch.nn.Parameter], group=None, bucket_bytes: int = 32 << 20):
        self.group = group
        self.params = [p for p in params if p.requires_grad]
        order = list(reversed(self.params))
        self.buckets: List[List[torch.nn.Parameter]] = []
        cur, size = [], 0
        for p in order:
            cur.append(p)
            size += p.numel() * p.element_size()
            if size >= bucket_bytes:
                self.buckets.append(cur)
                cur, size = [], 0
        if cur:
            self.buckets.append(cur)
        self.where: Dict[int, int] = {id(p): b for b, ps in enumerate(self.buckets) for p in ps}
        self.flats = [torch.empty(sum(p.numel() for p in ps), dtype=ps[0].dtype, device=ps[0].device)
                      for ps in self.buckets]
        self._reset()
        self.active = True
        self.on_all_launched: Optional[Callable[[], None]] = None   # called once the last bucket is out
        self._handles = [p.register_post_accumulate_grad_hook(self._hook) for p in self.params]

    def _reset(self):
        self.ready = [0] * len(self.buckets)
        self.launched = 0
        self.works: List = []

    def begin_step(self):
        """Start a new exchange (the optimizer's zero_grad calls this): collectives still in
        flight from a backward whose step never ran are waited for and dropped, so a diagnostic
        or aborted backward cannot leave stale counters or buffers behind."""
        for w in self.works:
            w.wait()
        self._reset()

    def _hook(self, p):
        if not self.active or not dist.is_initialized():
            return
        b = self.where[id(p)]
        if b < self.launched or self.ready[b] >= len(self.buckets[b]):
            # a second backward before the step (gradient accumulation): the bucket already went
            # out with the first backward's gradients, so this one's would be silently lost
            raise RuntimeError("BucketedGradAllReduce: a gradient arrived for a bucket that was already "
                               "all-reduced; call the optimizer's zero_grad() (begin_step) before every "
                               "backward — accumulating several backward passes per step is not supported")
        self.ready[b] += 1
        self._launch(force=False)

    def _launch(self, force: bool):
        while self.launched < len(self.buckets):
            b = self.launched
            ps = self.buckets[b]
            if not force and self.ready[b] < len(ps):
                return
            grads = [(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1) for p in ps]
            torch.cat(grads, out=self.flats[b])
            self.works.append(dist.all_reduce(self.flats[b], op=dist.ReduceOp.SUM, group=self.group, async_op=True))
            self.launched += 1
            if self.launched == len(self.buckets) and self.on_all_launched is not None:
                self.on_all_launched()

    def all_launched(self) -> bool:
        return self.launched == len(self.buckets)

    def finish(self):
        self._launch(force=True)
        for w in self.works:
            w.wait()
        for ps, flat in zip(self.buckets, self.flats):
            off = 0
            for p in ps:
                n = p.numel()
                p.grad = flat[off: off + n].view_as(p)
                off += n
        self._reset()

    def remove(self):
        for h in self._handles:
            h.remove()
        self._handles = []


def allgather_rows(ids: torch.Tensor, rows: torch.Tensor, group=None,
                   max_rows: Optional[int] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """All-gather (ids [n], rows [n, D]) from every rank, concatenated in rank order.

    With `max_rows` (a bound every rank shares, e.g. the per-rank batch size) each rank pads its
    slice to max_rows with id -1 / zero rows and nothing is read back on the host: the padded
    concatenation goes straight to the sparse update, which skips invalid ids (their zero rows
    add nothing to the clip norm, and the stable sort keeps the real rows in rank order), so
    the result is bitwise the same as the exact concatenation. Without it, ranks may hold
    different n (ragged last batch): sizes are exchanged first (one host read) and the payload
    is padded to the max."""
    world = dist.get_world_size(group)
    if max_rows is not None:
        n, D = ids.numel(), rows.shape[1]
        if n > max_rows:
            raise ValueError(f"allgather_rows: {n} rows exceed max_rows={max_rows}")
        pid = torch.full((max_rows,), -1, dtype=ids.dtype, device=ids.device)
        prow = torch.zeros((max_rows, D), dtype=rows.dtype, device=rows.device)
        pid[:n] = ids
        prow[:n] = rows
        gid = torch.empty((world * max_rows,), dtype=ids.dtype, device=ids.device)
        grow = torch.empty((world * max_rows, D), dtype=rows.dtype, device=rows.device)
        dist.all_gather_into_tensor(gid, pid, group=group)
        dist.all_gather_into_tensor(grow, prow, group=group)
        return gid, grow
    n = torch.tensor([ids.numel()], dtype=torch.int64, device=ids.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s.item()) for s in sizes]
    m = max(sizes)
    D = rows.shape[1]
    pid = torch.zeros((m,), dtype=ids.dtype, device=ids.device)
    prow = torch.zeros((m, D), dtype=rows.dtype, device=rows.device)
    pid[: ids.numel()] = ids
    prow[: ids.numel()] = rows
    gid = [torch.empty_like(pid) for _ in range(world)]
    grow = [torch.empty_like(prow) for _ in range(world)]
    dist.all_gather(gid, pid, group=group)
    dist.all_gather(grow, prow, group=group)
    return (torch.cat([g[:s] for g, s in zip(gid, sizes)]),
            torch.cat([g[:s] for g, s in zip(grow, sizes)]))


def _local_slices(e):
    sl = e.sink.gathered()
    if sl is None:
        dev = e.weight.device
        return (torch.zeros((0,), dtype=torch.int64, device=dev),
                torch.zeros((0, e.weight.shape[1]), dtype=e.weight.dtype, device=dev))
    ids, rows = sl
    return ids.contiguous(), rows


def _hip_dedupe(ids, rows, num_rows, plan=None):
    from . import functional as F
    return F.sparse_dedupe(ids, rows, num_rows, plan=plan)


def _width_groups(embeddings: Sequence) -> List[List[int]]:
    """Table indices grouped by embedding width (first-appearance order): one exchange per width,
    so tables of different widths never share a row buffer."""
    groups: Dict[Tuple[int, torch.dtype], List[int]] = {}
    for t, e in enumerate(embeddings):
        groups.setdefault((int(e.weight.shape[1]), e.weight.dtype), []).append(t)
    return list(groups.values())


def _to_device_async(a: np.ndarray, dev, cache: Optional[dict]) -> torch.Tensor:
    """A host int64 array on the device without draining the stream: a pageable .to(dev) waits for
    every queued kernel before it copies, so the copy goes through one of two cached pinned buffers
    (non_blocking), each reused only after its previous copy's event has passed."""
    if dev.type != "cuda" or cache is None:
        return torch.from_numpy(a).to(dev)
    k = cache.get("pin_turn", 0)
    cache["pin_turn"] = k ^ 1
    buf, ev = cache.get(("pin_idx", k), (None, None))
    if ev is not None:
        ev.synchronize()                      # the copy out of this buffer two uses ago
    if buf is None or buf.numel() < a.size:
        buf = torch.empty((max(a.size, 1 << 16),), dtype=torch.int64, pin_memory=True)
    buf[: a.size].numpy()[:] = a
    out = buf[: a.size].to(dev, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record()
    cache[("pin_idx", k)] = (buf, ev)
    return out


def _hip_merge_order(ids, offs):
    from . import functional as F
    return F.merge_runs_order(ids, offs)


def exchange_sparse_dedupe(embeddings: Sequence, group=None,
                           dedupe_fn: Callable = _hip_dedupe, wait: bool = True,
                           merge_order: Optional[Callable] = _hip_merge_order, count_group=None,
                           cache: Optional[dict] = None):
    """Deduplicate locally, all-reduce the raw norms, all-gather every table's unique (id, row)
    pairs at once (one all-gather of ids and one of rows per embedding width); each sink then
    holds the replica-ordered unique pairs and the global sum of squares of the raw rows
    (sink.sumsq) for the clip. wait=False: only the local deduplication and the small norm / count
    collectives are issued (asynchronously); the returned finisher reads the counts and runs the
    payload all-gathers.
    count_group (a second communicator of the same ranks, MirroredGradientExchange's): the counts
    are all-gathered there on a side stream and copied to pinned host memory, so the finisher's host
    read waits for that copy only, not for the whole step queued on the main stream; when every
    table's sink carries its id plan's deduplicated count (known from the forward on) the side
    stream waits for the plan alone and the counts are on the host long before they are read."""
    if not embeddings:
        return None
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    loc = []
    for e in embeddings:
        ids, rows = _local_slices(e)
        # the step's id plan of these ids (the sink's order and run heads): no sort in the dedupe
        plan = e.sink.dedupe_plan() if dedupe_fn is _hip_dedupe and hasattr(e.sink, "dedupe_plan") else None
        loc.append(dedupe_fn(ids, rows, e.weight.shape[0], plan) if plan is not None
                   else dedupe_fn(ids, rows, e.weight.shape[0]))
    dev = loc[0][0].device
    T = len(loc)
    sumsq = torch.stack([u[3].reshape(()) for u in loc]).to(torch.float32)
    w1 = dist.all_reduce(sumsq, op=dist.ReduceOp.SUM, group=group, async_op=not wait)
    host_counts = None
    if count_group is not None and dev.type == "cuda":
        early = [e.sink.early_count() if hasattr(e.sink, "early_count") else None for e in embeddings]
        use_early = all(x is not None for x in early)
        main = torch.cuda.current_stream(dev)
        side = cache.setdefault("side", torch.cuda.Stream(dev)) if cache is not None else torch.cuda.Stream(dev)
        if use_early:
            for _, ev in early:
                if ev is not None:
                    side.wait_event(ev)
        else:
            side.wait_stream(main)
        with torch.cuda.stream(side):
            src = [x[0] for x in early] if use_early else [u[2].reshape(1) for u in loc]
            counts = torch.cat([c.reshape(1) for c in src]).to(torch.int64)
            allc = torch.empty((world * T,), dtype=torch.int64, device=dev)
            dist.all_gather_into_tensor(allc, counts, group=count_group)
            key = ("pinned", world * T)
            pin = cache.get(key) if cache is not None else None
            if pin is None:
                pin = torch.empty((world * T,), dtype=torch.int64, pin_memory=True)
                if cache is not None:
                    cache[key] = pin
            pin.copy_(allc, non_blocking=True)
            done = torch.cuda.Event()
            done.record(side)
        host_counts = (pin, done)
        w2 = None
    else:
        counts = torch.stack([u[2].reshape(()) for u in loc]).to(torch.int64)
        allc = torch.empty((world * T,), dtype=torch.int64, device=dev)
        w2 = dist.all_gather_into_tensor(allc, counts, group=count_group or group, async_op=not wait)

    def finish():
        for w in (w1, w2):
            if w is not None:
                w.wait()
        if host_counts is not None:
            host_counts[1].synchronize()                      # the side stream's copy only
            C_all = host_counts[0].numpy().reshape(world, T).copy()
        else:
            C_all = allc.cpu().numpy().reshape(world, T)      # the exchange's one host read
        for tabs in _width_groups(embeddings):
            C = C_all[:, tabs]
            D = loc[tabs[0]][1].shape[1]
            cap = max(int(C.sum(axis=1).max()), 1)
            # (no fills: the padding past each rank's rows is never indexed below)
            pid = torch.empty((cap,), dtype=torch.int64, device=dev)
            prow = torch.empty((cap, D), dtype=loc[tabs[0]][1].dtype, device=dev)
            off = 0
            for j, t in enumerate(tabs):
                c = int(C[rank, j])
                if c:
                    pid[off: off + c] = loc[t][0][:c]
                    prow[off: off + c] = loc[t][1][:c]
                off += c
            gid = torch.empty((world * cap,), dtype=torch.int64, device=dev)
            grow = torch.empty((world * cap, D), dtype=prow.dtype, device=dev)
            dist.all_gather_into_tensor(gid, pid, group=group)
            dist.all_gather_into_tensor(grow, prow, group=group)
            # every table's rows of every rank, table-major then rank order, from ONE index_select of
            # the ids and one of the rows; each sink gets a view of its table's span
            offs = np.concatenate([np.zeros((world, 1), np.int64), np.cumsum(C, axis=1)], axis=1)   # [world, n+1]
            idx = np.concatenate([np.arange(r * cap + offs[r, j], r * cap + offs[r, j + 1], dtype=np.int64)
                                  for j in range(len(tabs)) for r in range(world)])
            it = _to_device_async(idx, dev, cache)
            sid, srow = gid.index_select(0, it), grow.index_select(0, it)
            pos = 0
            for j, t in enumerate(tabs):
                n = int(C[:, j].sum())
                tid = sid[pos: pos + n]
                embeddings[t].sink.slices = [(tid, srow[pos: pos + n])]
                embeddings[t].sink.sumsq = sumsq[t]
                # every rank's ids are unique and ascending (the local dedupe's), so the stable order of
                # their rank-ordered concatenation is a merge (binary searches): the update skips its sort
                embeddings[t].sink.heads = None
                embeddings[t].sink.order = None
                if merge_order is not None and n and world <= 64 and tid.is_cuda:
                    offs = np.concatenate([[0], np.cumsum(C[:, j])]).tolist()
                    embeddings[t].sink.order = (tid, merge_order(tid, offs))
                pos += n

    if wait:
        finish()
        return None
    return finish


def exchange_sparse_padded(embeddings: Sequence, max_rows: int, group=None, wait: bool = True):
    """Sync-free: every table's slice padded to max_rows (id -1, zero rows), all tables of one
    width in one all-gather of ids and one of rows; each sink then holds the world * max_rows
    padded concatenation in rank order (the raw rows: the update computes the clip norm itself).
    No host read and static shapes, so the exchange can be captured in a hipGraph with RCCL
    (tests/test_gpu_multirank.py::test_graphed_padded_exchange_step_bitwise_equal_to_eager).
    wait=False: the all-gathers are issued asynchronously and the returned finisher makes the
    current stream wait for them (no host wait) and sets the slices."""
    if not embeddings:
        return None
    world = dist.get_world_size(group)
    loc = [_local_slices(e) for e in embeddings]
    dev = loc[0][0].device
    done = []
    for tabs in _width_groups(embeddings):
        D, T = loc[tabs[0]][1].shape[1], len(tabs)
        pid = torch.full((T, max_rows), -1, dtype=torch.int64, device=dev)
        prow = torch.zeros((T, max_rows, D), dtype=loc[tabs[0]][1].dtype, device=dev)
        for j, t in enumerate(tabs):
            ids, rows = loc[t]
            n = ids.numel()
            if n > max_rows:
                raise ValueError(f"exchange_sparse_padded: {n} rows exceed max_rows={max_rows}")
            pid[j, :n] = ids
            prow[j, :n] = rows
        gid = torch.empty((world, T, max_rows), dtype=torch.int64, device=dev)
        grow = torch.empty((world, T, max_rows, D), dtype=prow.dtype, device=dev)
        works = [dist.all_gather_into_tensor(gid.view(-1), pid.view(-1), group=group, async_op=not wait),
                 dist.all_gather_into_tensor(grow.view(-1), prow.view(-1), group=group, async_op=not wait)]
        done.append((tabs, gid, grow, D, works))

    def finish():
        for tabs, gid, grow, D, works in done:
            for w in works:
                if w is not None:
                    w.wait()
            for j, t in enumerate(tabs):
                embeddings[t].sink.slices = [(gid[:, j].reshape(-1), grow[:, j].reshape(world * max_rows, D))]
                embeddings[t].sink.sumsq = None

    if wait:
        finish()
        return None
    return finish


class MirroredGradientExchange:
    """Optimizer pre-apply hook implementing MirroredStrategy's gradient aggregation.

    `dense_params`: the optimizer's dense parameters — their all-reduce then runs in buckets from
    gradient hooks during the backward (BucketedGradAllReduce); without it, one flat bucket after
    the backward. `sparse`: "dedupe" (default; one host sync per step) or "padded" (sync-free,
    needs `max_rows`, the per-rank bound on any table's gradient rows)."""

    def __init__(self, group=None, max_rows: Optional[int] = None, dense_params=None, sparse: Optional[str] = None,
                 bucket_bytes: int = 32 << 20, dedupe_fn: Callable = _hip_dedupe, force: bool = False,
                 embeddings: Optional[Sequence] = None):
        self.group = group
        self.force = force    # run the collectives even in a one-rank group (capture rehearsal)
        self.max_rows = max_rows
        self.sparse = sparse or "dedupe"
        if self.sparse not in ("dedupe", "padded", "ragged"):
            raise ValueError(f"sparse exchange must be 'dedupe', 'padded' or 'ragged', got {self.sparse!r}")
        if self.sparse == "padded" and max_rows is None:
            raise ValueError("the padded sparse exchange needs max_rows")
        self.dedupe_fn = dedupe_fn
        self.bucketer = None
        active = dist.is_initialized() and (force or dist.get_world_size(group) > 1)
        if dense_params is not None and active:
            self.bucketer = BucketedGradAllReduce(dense_params, group, bucket_bytes)
        # embeddings (the optimizer's tables): the sparse exchange starts from the tables' sinks as
        # soon as the last of them receives its backward slice (the padded all-gathers, or the
        # deduplication and the norm / count collectives), instead of after the whole backward in
        # the optimizer's pre-apply hook; the update waits for it where it reads the slices.
        # Collective order is the same on every rank whether a rank starts early or in the hook (a
        # rank where some table got no slice this step): the sparse collectives always follow the
        # last dense bucket (a start that is ready earlier waits for the bucketer's last launch), so
        # every rank issues [dense buckets in order] then [sparse norm / counts] then [payloads].
        # Without a bucketer (the flat all-reduce runs in the hook) there is no early start.
        early = (embeddings is not None and active and self.sparse != "ragged"
                 and (self.bucketer is not None or dense_params is not None and not list(dense_params)))
        self.embeddings = list(embeddings) if early else None
        self._started = False
        self._seen = None
        # the deduplicating exchange's counts travel on a communicator of their own (a side stream,
        # out of the main stream's collective order: see exchange_sparse_dedupe)
        self.count_group = None
        self._cache = {}
        if active and self.sparse == "dedupe":
            ranks = list(range(dist.get_world_size())) if group is None else dist.get_process_group_ranks(group)
            self.count_group = dist.new_group(ranks=ranks)
        if self.embeddings:
            for e in self.embeddings:
                e.sink.listeners.append(self._on_slice)
            if self.bucketer is not None:
                self.bucketer.on_all_launched = self._try_start

    def _on_slice(self, sink) -> None:
        if self._started:
            if self._seen is not None and [len(e.sink.slices) for e in self.embeddings] != self._seen:
                raise RuntimeError("a table received another gradient slice after its exchange started "
                                   "(a table looked up twice in one step): build MirroredGradientExchange "
                                   "without embeddings= for such a model")
            return
        self._try_start()

    def _try_start(self) -> None:
        if self._started or not all(e.sink.slices for e in self.embeddings):
            return
        if self.bucketer is not None and not self.bucketer.all_launched():
            return   # the bucketer's last launch calls back
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            return   # a captured step keeps the exchange in the pre-apply hook
        self._started = True
        seen = self._seen = [len(e.sink.slices) for e in self.embeddings]
        if self.sparse == "padded":
            fin = exchange_sparse_padded(self.embeddings, self.max_rows, self.group, wait=False)
        else:
            fin = exchange_sparse_dedupe(self.embeddings, self.group, self.dedupe_fn, wait=False,
                                         count_group=self.count_group, cache=self._cache)
        state = {"fin": fin}

        def finish_once():   # shared by every sink: the first read runs it
            f, state["fin"] = state["fin"], None
            if f is None:
                return
            if [len(e.sink.slices) for e in self.embeddings] != seen:
                raise RuntimeError("a table received another gradient slice after its exchange started "
                                   "(a table looked up twice in one step): build MirroredGradientExchange "
                                   "without embeddings= for such a model")
            f()
        for e in self.embeddings:
            e.sink.pending = finish_once

    def begin_step(self) -> None:
        """Called by the optimizer's zero_grad before every backward (resets the bucketer)."""
        self._started = False
        self._seen = None
        if self.bucketer is not None:
            self.bucketer.begin_step()

    def close(self) -> None:
        """Remove the gradient hooks (end of training: later backward passes issue nothing)."""
        if self.bucketer is not None:
            self.bucketer.remove()
            self.bucketer = None
        if self.embeddings:
            for e in self.embeddings:
                if self._on_slice in e.sink.listeners:
                    e.sink.listeners.remove(self._on_slice)
            self.embeddings = None

    def __call__(self, opt) -> None:
        if not dist.is_initialized() or (dist.get_world_size(self.group) == 1 and not self.force):
            return
        if self.bucketer is not None:
            self.bucketer.finish()
        else:
            grads = []
            for p in opt.dense:
                if p.grad is None:   # a replica that did not touch a variable contributes zeros
                    p.grad = torch.zeros_like(p)
                grads.append(p.grad)
            flat_allreduce_(grads, self.group)
        if self._started:   # already issued from the sinks; the update resolves it
            self._started = False
            self._seen = None
            return
        if self.sparse == "dedupe":
            exchange_sparse_dedupe(opt.embeddings, self.group, self.dedupe_fn, count_group=self.count_group,
                                   cache=self._cache)
        elif self.sparse == "padded":
            exchange_sparse_padded(opt.embeddings, self.max_rows, self.group)
        else:
            for e in opt.embeddings:
                ids, rows = _local_slices(e)
                e.sink.slices = [allgather_rows(ids, rows.contiguous(), self.group)]
                e.sink.sumsq = None
