"""Data-parallel exchange (MirroredStrategy semantics) on CPU with gloo, world_size 2.

Checks the host logic of distributed.py — the flat-bucket and the hook-driven bucketed SUM
all-reduce of dense gradients, the ragged / padded / deduplicated (id, row) exchanges of
embedding gradients in rank order, the optimizer hook that combines them — against the
oracle's data_parallel_grads rule (and, for the deduplicated exchange, against one oracle
Adagrad step on the replica-concatenated raw gradients: src/trainer.py:157-163), and the
row-sharded top-K exchange (all-gather of per-shard lists; merge checked with the oracle
ordering). The HIP kernels (deduplication, sparse update) have numpy stand-ins here; their own
parity is in tests/test_gpu_kernels.py."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, fn, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, fn(rank, world)))
    except Exception as e:  # pragma: no cover - surfaced by the parent
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def run(fn, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, fn, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    return out


# ---- workers (module-level so spawn can pickle them) ------------------------------------------
def _allreduce_worker(rank, world):
    from conftest import pkg
    D = pkg("distributed")
    ts = [torch.full((3, 4), float(rank + 1)), torch.arange(5, dtype=torch.float32) * (rank + 1)]
    D.flat_allreduce_(ts, bucket_bytes=16)    # forces several buckets
    return [t.tolist() for t in ts]


def _allgather_worker(rank, world):
    from conftest import pkg
    D = pkg("distributed")
    n = 3 if rank == 0 else 5                 # ragged: last batch of a rank can be shorter
    ids = torch.arange(n, dtype=torch.int64) + 100 * rank
    rows = torch.full((n, 2), float(rank))
    gi, gr = D.allgather_rows(ids, rows)
    return gi.tolist(), gr.tolist()


def _allgather_static_worker(rank, world):
    from conftest import pkg
    D = pkg("distributed")
    n = 3 if rank == 0 else 5
    ids = torch.arange(n, dtype=torch.int64) + 100 * rank
    rows = torch.full((n, 2), float(rank + 1))
    gi, gr = D.allgather_rows(ids, rows, max_rows=6)
    return gi.tolist(), gr.tolist()


def _sharded_topk_worker(rank, world):
    """ShardedBruteForceIndex wiring (row offsets, all-gather order, final merge) with the two
    device kernels stood in by CPU restatements (the kernels themselves are GPU-tested)."""
    from conftest import oracle, pkg
    R = pkg("retrieval")
    F = pkg("functional")
    O = oracle()
    rng = np.random.default_rng(3)
    N, D, Q, k = 90, 8, 5, 7
    items = (rng.integers(-4, 5, (N, D)) / 4).astype(np.float32)   # dyadic: exact scores, ties
    q = (rng.integers(-4, 5, (Q, D)) / 4).astype(np.float32)
    per = N // world

    def cpu_topk(queries, it, kk, index_base=0, precision=0):
        qn = queries.numpy()   # the index holds its rows zero-padded to the kernel width
        qn = np.pad(qn, ((0, 0), (0, it.shape[1] - qn.shape[1])))
        sc, idx = O.topk_ip(qn, it.numpy(), kk)
        return torch.from_numpy(sc.astype(np.float32)), torch.from_numpy(idx + index_base)

    def cpu_merge(scores, index, kk):
        s, i = scores.numpy(), index.numpy()
        out_s, out_i = [], []
        for a in range(s.shape[0]):
            fs, fi = s[a].reshape(-1), i[a].reshape(-1)
            o = np.lexsort((fi, -fs))[:kk]
            out_s.append(fs[o])
            out_i.append(fi[o])
        return torch.from_numpy(np.stack(out_s)), torch.from_numpy(np.stack(out_i))

    F.topk_ip, F.topk_merge = cpu_topk, cpu_merge
    idx = R.ShardedBruteForceIndex(torch.from_numpy(items[rank * per:(rank + 1) * per]), row_offset=rank * per)
    s, i = idx.search(torch.from_numpy(q), k)
    ref_s, ref_i = O.topk_ip(q, items[:per * world], k)
    return bool(np.array_equal(i.numpy(), ref_i) and np.array_equal(s.numpy().astype(np.float64), ref_s))


def _sharded_eval_worker(rank, world):
    """ProductionTrainer._evaluate under data parallelism: every rank scores the
    sampled validation users against its shard of the item rows (ShardedBruteForceIndex) and the
    merged lists give the same recall@k on every rank as the unsharded evaluation and as the
    oracle's np.dot + argpartition restatement (src/trainer.py:195-213). The three device kernels
    (scan, merge, rank metrics) are stood in by CPU restatements; they are GPU-tested themselves."""
    import pandas as pd
    from conftest import oracle, pkg
    R, F, T, L = pkg("retrieval"), pkg("functional"), pkg("trainer"), pkg("lookup")
    cfgm = pkg("config")
    O = oracle()
    rng = np.random.default_rng(5)
    n_items, n_users, D = 203, 40, 16                    # odd: ragged shards
    item_vocab = L.build_vocab([str(i) for i in range(n_items)])
    user_vocab = L.build_vocab([str(i) for i in range(n_users)])
    item_tab = rng.standard_normal((n_items + 1, D)).astype(np.float32)
    user_tab = rng.standard_normal((n_users + 1, D)).astype(np.float32)
    ul, il = L.StringLookup(user_vocab), L.StringLookup(item_vocab)

    class Enc:
        item_lookup = il

        def __call__(self, feats):
            if "movie_id" in feats:
                return {"item_embedding": torch.from_numpy(item_tab[feats["movie_id"].numpy()])}
            return {"user_embedding": torch.from_numpy(user_tab[ul(feats["user_id"])])}

    class Model:
        encoder = Enc()

    def cpu_topk(queries, it, kk, index_base=0, precision=0):
        qn = queries.numpy()   # (an index holds its rows zero-padded to the kernel width)
        qn = np.pad(qn, ((0, 0), (0, it.shape[1] - qn.shape[1])))
        sc, idx = O.topk_ip(qn, it.numpy(), kk)
        return torch.from_numpy(sc.astype(np.float32)), torch.from_numpy(idx + index_base)

    def cpu_merge(scores, index, kk):
        s_, i_ = scores.numpy(), index.numpy()
        out_s, out_i = [], []
        for a in range(s_.shape[0]):
            fs, fi = s_[a].reshape(-1), i_[a].reshape(-1)
            o = np.lexsort((fi, -fs))[:kk]
            out_s.append(fs[o])
            out_i.append(fi[o])
        return torch.from_numpy(np.stack(out_s)), torch.from_numpy(np.stack(out_i))

    def cpu_rank_metrics(pred, truth, ks, n):
        p, t = pred.numpy(), truth.numpy()
        m = np.zeros(4 * len(ks) + 3)
        for j, k in enumerate(ks):
            m[4 * j] = np.mean([t[a] in p[a, :k] for a in range(len(t))])
        return torch.from_numpy(m)

    F.topk_ip, F.topk_merge, F.rank_metrics = cpu_topk, cpu_merge, cpu_rank_metrics
    val_df = pd.DataFrame({"user_id": rng.integers(0, n_users, 300).astype(str),
                           "movie_id": rng.integers(0, n_items + 20, 300).astype(str)})   # some unknown items
    datasets = {"val_df": val_df, "val_ds": object(), "item_vocab": item_vocab}
    out = {}
    for distributed in (True, False):
        tr = T.ProductionTrainer.__new__(T.ProductionTrainer)
        tr.config = cfgm.ModelConfig(embedding_dim=D, eval_topk=[1, 5, 10, 50])
        tr.distributed, tr.rank, tr.world = distributed, rank, world
        tr.device = torch.device("cpu")
        tr.output_dir = __import__("pathlib").Path(__import__("tempfile").mkdtemp())
        out[distributed] = tr._evaluate(Model(), datasets)
    sample = val_df.sample(n=min(1000, len(val_df)), random_state=42)
    ue = user_tab[ul(sample["user_id"].values)].astype(np.float64)
    sims = ue @ item_tab[1:].astype(np.float64).T
    ref = O.recall_at_k(sims, sample["movie_id"].values, item_vocab, [1, 5, 10, 50])
    return out[True], out[False], ref


def _exchange_worker(rank, world):
    """Per-rank oracle gradients -> MirroredGradientExchange -> compare with the oracle rule."""
    from conftest import oracle, pkg
    D = pkg("distributed")
    F = pkg("functional")
    O = oracle()
    cfg = O.OracleConfig(embedding_dim=8, user_tower_dims=[8], item_tower_dims=[8], cross_layers=1, dnn_dims=[8])
    P = O.init_params(cfg, 11, 9, seed=2, bias_scale=0.1)
    rng = np.random.default_rng(0)
    B = 12
    uid, iid = rng.integers(0, 11, B), rng.integers(0, 9, B)
    rating = rng.integers(1, 6, B).astype(np.float64)
    yi = (rating >= 4).astype(np.float64)
    shards = [(uid[:6], iid[:6], rating[:6], yi[:6]), (uid[6:], iid[6:], rating[6:], yi[6:])]
    mine = O.loss_and_grads(P, cfg, *shards[rank])["grads"]
    ref = O.data_parallel_grads(P, cfg, shards)

    class FakeEmb:
        def __init__(self, name):
            self.weight = torch.zeros(P[name].shape)
            self.sink = F.SparseGradSink()

    class FakeOpt:
        pass

    opt = FakeOpt()
    dense_names = [k for k, v in mine.items() if not isinstance(v, tuple)]
    opt.dense = [torch.nn.Parameter(torch.zeros(P[k].shape, dtype=torch.float64)) for k in dense_names]
    for p, k in zip(opt.dense, dense_names):
        p.grad = torch.tensor(mine[k])
    emb_names = [k for k, v in mine.items() if isinstance(v, tuple)]
    opt.embeddings = [FakeEmb(k) for k in emb_names]
    for e, k in zip(opt.embeddings, emb_names):
        e.sink.slices = [(torch.tensor(mine[k][0]), torch.tensor(mine[k][1]))]
    D.MirroredGradientExchange(sparse="ragged")(opt)
    errs = []
    for p, k in zip(opt.dense, dense_names):
        errs.append(float(np.max(np.abs(p.grad.numpy() - ref[k]))))
    for e, k in zip(opt.embeddings, emb_names):
        ids, rows = e.sink.gathered()
        assert np.array_equal(ids.numpy(), ref[k][0])
        errs.append(float(np.max(np.abs(rows.numpy() - ref[k][1]))))
    return max(errs)


def test_flat_allreduce_sums_in_place():
    out = run(_allreduce_worker)
    for r in (0, 1):
        assert out[r][0] == [[3.0] * 4] * 3
        assert out[r][1] == [0.0, 3.0, 6.0, 9.0, 12.0]


def test_allgather_rows_ragged_rank_order():
    out = run(_allgather_worker)
    for r in (0, 1):
        ids, rows = out[r]
        assert ids == [0, 1, 2, 100, 101, 102, 103, 104]
        assert rows == [[0.0, 0.0]] * 3 + [[1.0, 1.0]] * 5


def test_allgather_rows_static_bound_is_padded_in_rank_order():
    """Sync-free path: each rank pads to max_rows with id -1 / zero rows; stripping the padding
    leaves exactly the ragged concatenation (what the sparse update sees)."""
    out = run(_allgather_static_worker)
    for r in (0, 1):
        ids, rows = out[r]
        assert len(ids) == 12 and len(rows) == 12
        assert ids == [0, 1, 2, -1, -1, -1, 100, 101, 102, 103, 104, -1]
        keep = [i for i, v in enumerate(ids) if v >= 0]
        assert [rows[i] for i in keep] == [[1.0, 1.0]] * 3 + [[2.0, 2.0]] * 5
        assert all(rows[i] == [0.0, 0.0] for i in range(12) if ids[i] < 0)


def test_sharded_topk_exchange_matches_global_topk():
    out = run(_sharded_topk_worker)
    assert out[0] is True and out[1] is True, out


def test_mirrored_exchange_matches_oracle_rule():
    out = run(_exchange_worker)
    for r in (0, 1):
        assert isinstance(out[r], float), out[r]
        assert out[r] < 1e-12


# ---- deduplicated / padded sparse exchange, bucketed dense all-reduce ---------------------------
def _np_dedupe(ids, rows, num_rows):
    """CPU stand-in of rs_sparse_dedupe_f32: unique valid ids ascending, rows summed in input
    order, count, raw sum of squares."""
    i = ids.numpy()
    r = rows.numpy()
    ok = (i >= 0) & (i < num_rows)
    u, inv = np.unique(i[ok], return_inverse=True)
    s = np.zeros((len(u), r.shape[1]), r.dtype)
    np.add.at(s, inv, r[ok])
    n = max(len(i), 1)
    out_i = np.full(n, -1, np.int64)
    out_r = np.zeros((n, r.shape[1]), r.dtype)
    out_i[:len(u)] = u
    out_r[:len(u)] = s
    return (torch.from_numpy(out_i), torch.from_numpy(out_r), torch.tensor(len(u), dtype=torch.int64),
            torch.tensor(float(np.sum(r.astype(np.float64) ** 2))))


def _dp_problem(rank, world):
    from conftest import oracle
    O = oracle()
    cfg = O.OracleConfig(embedding_dim=8, user_tower_dims=[8], item_tower_dims=[8], cross_layers=1, dnn_dims=[8])
    P = O.init_params(cfg, 11, 9, seed=2, bias_scale=0.1)
    rng = np.random.default_rng(0)
    B = 24
    uid, iid = rng.integers(0, 11, B), rng.integers(0, 9, B)      # many duplicate ids
    rating = rng.integers(1, 6, B).astype(np.float64)
    yi = (rating >= 4).astype(np.float64)
    h = B // world
    shards = [(uid[r * h:(r + 1) * h], iid[r * h:(r + 1) * h], rating[r * h:(r + 1) * h], yi[r * h:(r + 1) * h])
              for r in range(world)]
    return O, cfg, P, shards


def _fake_opt(P, mine, F):
    class FakeEmb:
        def __init__(self, name):
            self.weight = torch.zeros(P[name].shape, dtype=torch.float64)
            self.sink = F.SparseGradSink()

    class FakeOpt:
        pass

    opt = FakeOpt()
    opt.dense_names = [k for k, v in mine.items() if not isinstance(v, tuple)]
    opt.dense = [torch.nn.Parameter(torch.zeros(P[k].shape, dtype=torch.float64)) for k in opt.dense_names]
    for p, k in zip(opt.dense, opt.dense_names):
        p.grad = torch.tensor(mine[k])
    opt.emb_names = [k for k, v in mine.items() if isinstance(v, tuple)]
    opt.embeddings = [FakeEmb(k) for k in opt.emb_names]
    for e, k in zip(opt.embeddings, opt.emb_names):
        ids, rows = mine[k]
        ok = (ids >= 0)
        e.sink.slices = [(torch.tensor(np.where(ok, ids, -1)), torch.tensor(rows))]
    return opt


def _dedupe_exchange_worker(rank, world):
    """Deduplicated exchange + the update with the exchanged norm (numpy stand-in of
    rs_sparse_adagrad_sumsq_f32) vs one oracle Adagrad step on the replica-concatenated raw
    gradients (MirroredStrategy rule)."""
    from conftest import pkg
    D = pkg("distributed")
    F = pkg("functional")
    O, cfg, P, shards = _dp_problem(rank, world)
    mine = O.loss_and_grads(P, cfg, *shards[rank])["grads"]
    ref = O.data_parallel_grads(P, cfg, shards)
    opt = _fake_opt(P, mine, F)
    D.MirroredGradientExchange(sparse="dedupe", dedupe_fn=_np_dedupe)(opt)
    P1 = {k: v.copy() for k, v in P.items()}
    A1 = O.init_accumulators(P1)
    lr = O.learning_rate(0, 0.05)
    errs = []
    for e, k in zip(opt.embeddings, opt.emb_names):
        ids, rows = e.sink.gathered()
        ids, rows = ids.numpy(), rows.numpy()
        assert np.all(np.diff(ids[:len(ids) // world]) > 0) or world == 1   # rank 0's part: unique ascending
        ss = float(e.sink.sumsq)
        c = 1.0 / max(np.sqrt(ss), 1.0)
        u, inv = np.unique(ids, return_inverse=True)
        gs = np.zeros((len(u), rows.shape[1]))
        np.add.at(gs, inv, rows * c)
        A1[k][u] += gs * gs
        P1[k][u] -= lr * gs / np.sqrt(A1[k][u] + 1e-7)
        raw = np.concatenate([r[1] for r in [ref[k]]])
        errs.append(abs(ss - float(np.sum(raw ** 2))) / max(1.0, float(np.sum(raw ** 2))))
    P2 = {k: v.copy() for k, v in P.items()}
    A2 = O.init_accumulators(P2)
    O.adagrad_apply(P2, A2, {k: ref[k] for k in opt.emb_names}, 0, 0.05, clipnorm=1.0)
    for k in opt.emb_names:
        errs.append(float(np.max(np.abs(P1[k] - P2[k]))))
    for p, k in zip(opt.dense, opt.dense_names):
        errs.append(float(np.max(np.abs(p.grad.numpy() - ref[k]))))
    return max(errs)


def _padded_exchange_worker(rank, world):
    """All tables' padded slices in one all-gather: each sink gets the rank-ordered padded
    concatenation, whose valid rows are exactly the MirroredStrategy concatenation."""
    from conftest import pkg
    D = pkg("distributed")
    F = pkg("functional")
    O, cfg, P, shards = _dp_problem(rank, world)
    mine = O.loss_and_grads(P, cfg, *shards[rank])["grads"]
    ref = O.data_parallel_grads(P, cfg, shards)
    opt = _fake_opt(P, mine, F)
    D.MirroredGradientExchange(sparse="padded", max_rows=16)(opt)
    errs = []
    for e, k in zip(opt.embeddings, opt.emb_names):
        ids, rows = e.sink.gathered()
        assert ids.numel() == world * 16 and e.sink.sumsq is None
        keep = ids.numpy() >= 0
        rid = ref[k][0]
        assert np.array_equal(ids.numpy()[keep], rid[rid >= 0])
        errs.append(float(np.max(np.abs(rows.numpy()[keep] - ref[k][1][rid >= 0]))))
        assert not rows.numpy()[~keep].any()
    return max(errs)


def _early_exchange_worker(rank, world):
    """The sparse exchange started from the tables' sinks (MirroredGradientExchange(embeddings=):
    issued when the last table receives its backward slice, finished where the update reads the
    slices) leaves every sink bitwise what the exchange in the pre-apply hook leaves, for the
    deduplicated and the padded exchanges; a slice arriving after the start is refused."""
    from conftest import pkg
    D = pkg("distributed")
    F = pkg("functional")
    O, cfg, P, shards = _dp_problem(rank, world)
    mine = O.loss_and_grads(P, cfg, *shards[rank])["grads"]
    results = []
    for mode in ("dedupe", "padded"):
        kw = dict(sparse=mode, max_rows=16, dedupe_fn=_np_dedupe)
        ref = _fake_opt(P, mine, F)
        D.MirroredGradientExchange(**kw)(ref)
        opt = _fake_opt(P, mine, F)
        local = [e.sink.slices[0] for e in opt.embeddings]
        for e in opt.embeddings:
            e.sink.clear()
        # dense_params=[]: a bucketer with no buckets (the early start needs one: it orders the
        # sparse collectives after the dense ones on every rank)
        ex = D.MirroredGradientExchange(embeddings=opt.embeddings, dense_params=[], **kw)
        ex.begin_step()
        for e, (ids, rows) in zip(opt.embeddings, local):   # the backward's slices, one table at a time
            assert not ex._started
            e.sink.add(ids, rows)
        assert ex._started and all(e.sink.pending is not None for e in opt.embeddings)
        ex(opt)                                             # the pre-apply hook: nothing left to issue
        for a, b in zip(ref.embeddings, opt.embeddings):
            ia, ra = a.sink.gathered()
            ib, rb = b.sink.gathered()
            results.append(torch.equal(ia, ib) and torch.equal(ra, rb)
                           and (a.sink.sumsq is None) == (b.sink.sumsq is None)
                           and (a.sink.sumsq is None or torch.equal(a.sink.sumsq, b.sink.sumsq)))
        # a second slice for a table after the start: refused where the update reads
        for e in opt.embeddings:
            e.sink.clear()
        ex.begin_step()
        for e, (ids, rows) in zip(opt.embeddings, local):
            e.sink.add(ids, rows)
        try:                                                # refused at the add itself
            opt.embeddings[0].sink.add(*local[0])
            results.append(False)
        except RuntimeError:
            results.append(True)
        try:                                                # and where the update reads
            opt.embeddings[1].sink.gathered()
            results.append(False)
        except RuntimeError:
            results.append(True)
        ex.close()
        assert all(not e.sink.listeners for e in opt.embeddings)
    return all(results)


def _early_exchange_missing_table_worker(rank, world):
    """rank 1 gives table 0 no gradient slice in a step, so only rank 0 can start the
    sparse exchange from the sinks. Every rank must still issue the same collective sequence
    (dense buckets, then the sparse norm / counts, then the payloads): the early start waits for
    the bucketer's last launch, and rank 1 issues the same collectives from the pre-apply hook.
    The sinks then hold exactly what the hook exchange leaves with the same slices, and the dense
    gradients are the SUM over the ranks."""
    from conftest import pkg
    D = pkg("distributed")
    F = pkg("functional")
    O, cfg, P, shards = _dp_problem(rank, world)
    mine = O.loss_and_grads(P, cfg, *shards[rank])["grads"]
    results = []
    for mode in ("dedupe", "padded"):
        kw = dict(sparse=mode, max_rows=16, dedupe_fn=_np_dedupe)
        ref = _fake_opt(P, mine, F)
        if rank == 1:
            ref.embeddings[0].sink.clear()
        D.MirroredGradientExchange(**kw)(ref)
        opt = _fake_opt(P, mine, F)
        local = [e.sink.slices[0] for e in opt.embeddings]
        for e in opt.embeddings:
            e.sink.clear()
        torch.manual_seed(0)
        lin = torch.nn.Linear(3, 2).double()
        dense = list(lin.parameters())
        ex = D.MirroredGradientExchange(embeddings=opt.embeddings, dense_params=dense, bucket_bytes=8, **kw)
        ex.begin_step()
        for t, (e, (ids, rows)) in enumerate(zip(opt.embeddings, local)):   # slices before the dense grads
            if not (rank == 1 and t == 0):
                e.sink.add(ids, rows)
        assert not ex._started                              # the dense buckets have not gone out
        lin(torch.full((4, 3), float(rank + 1), dtype=torch.float64)).sum().backward()
        assert ex._started == (rank == 0)

        class Opt:
            pass
        o = Opt()
        o.dense, o.embeddings = dense, opt.embeddings
        ex(o)
        for a, b in zip(ref.embeddings, opt.embeddings):
            ga, gb = a.sink.gathered(), b.sink.gathered()
            results.append((ga is None) == (gb is None))
            if ga is not None and gb is not None:
                results.append(torch.equal(ga[0], gb[0]) and torch.equal(ga[1], gb[1]))
            results.append((a.sink.sumsq is None) == (b.sink.sumsq is None)
                           and (a.sink.sumsq is None or torch.equal(a.sink.sumsq, b.sink.sumsq)))
        results.append(float(lin.weight.grad.sum()) == 4.0 * (1 + 2) * 6)   # SUM over the 2 ranks
        ex.close()
    return all(results)


def _bucketed_worker(rank, world):
    """Hook-driven buckets launched during the backward: the reduced gradients equal the SUM of
    the replicas' gradients, for several buckets (tiny bucket_bytes) and for a parameter the step
    did not use (zeros)."""
    from conftest import pkg
    D = pkg("distributed")
    torch.manual_seed(0)
    layers = torch.nn.Sequential(torch.nn.Linear(6, 5), torch.nn.ReLU(), torch.nn.Linear(5, 3))
    unused = torch.nn.Parameter(torch.ones(4))
    params = [unused] + list(layers.parameters())     # reverse order: the unused one is bucketed last
    ex = D.MirroredGradientExchange(dense_params=params, sparse="ragged", bucket_bytes=16)
    assert ex.bucketer is not None and len(ex.bucketer.buckets) >= 3

    class Opt:
        dense = params
        embeddings = []

    x = torch.full((4, 6), float(rank + 1))
    layers(x).sum().backward()
    launched_in_backward = ex.bucketer.launched
    ex(Opt)
    got = [p.grad.clone() for p in params]
    ex.close()                 # hooks off: the reference backward passes below issue nothing
    # reference: each rank's own gradients, summed
    ref = []
    for r in range(world):
        for p in params:
            p.grad = None
        layers(torch.full((4, 6), float(r + 1))).sum().backward()
        g = [p.grad.clone() if p.grad is not None else torch.zeros_like(p) for p in params]
        ref = g if not ref else [a + b for a, b in zip(ref, g)]
    return launched_in_backward, max(float((a - b).abs().max()) for a, b in zip(got, ref))


def test_dedupe_exchange_matches_one_oracle_adagrad_step():
    out = run(_dedupe_exchange_worker)
    for r in (0, 1):
        assert isinstance(out[r], float), out[r]
        assert out[r] < 1e-6


def test_padded_exchange_batches_all_tables():
    out = run(_padded_exchange_worker)
    for r in (0, 1):
        assert isinstance(out[r], float), out[r]
        assert out[r] < 1e-12


def test_early_sparse_exchange_matches_hook_exchange():
    out = run(_early_exchange_worker)
    for r in (0, 1):
        assert out[r] is True, out[r]


def test_early_sparse_exchange_same_collective_order_when_a_rank_misses_a_table():
    out = run(_early_exchange_missing_table_worker)
    for r in (0, 1):
        assert out[r] is True, out[r]


def test_bucketed_allreduce_overlaps_backward():
    out = run(_bucketed_worker)
    for r in (0, 1):
        assert isinstance(out[r], tuple), out[r]
        launched, err = out[r]
        assert launched >= 2           # buckets went out during the backward, before the hook
        assert err < 1e-6


def _bucket_state_worker(rank, world):
    """Per-step bucketer state: a second backward before the step raises instead of
    dropping its gradients; zero_grad's begin_step() after an aborted backward (no step) leaves
    nothing stale, so the next real step reduces exactly its own gradients."""
    from conftest import pkg
    D = pkg("distributed")
    torch.manual_seed(0)
    layers = torch.nn.Sequential(torch.nn.Linear(6, 5), torch.nn.ReLU(), torch.nn.Linear(5, 3))
    params = list(layers.parameters())
    ex = D.MirroredGradientExchange(dense_params=params, sparse="ragged", bucket_bytes=16)

    class Opt:
        dense = params
        embeddings = []

    x = torch.full((4, 6), float(rank + 1))
    layers(x).sum().backward()
    raised = False
    try:
        layers(x).sum().backward()          # gradient accumulation: not supported, must be loud
    except RuntimeError as e:
        raised = "already" in str(e)
    # aborted step: new step begins (the optimizer's zero_grad calls begin_step)
    for p in params:
        p.grad = None
    ex.begin_step()
    x2 = torch.full((4, 6), float(2 * rank + 3))
    layers(x2).sum().backward()
    ex(Opt)
    got = [p.grad.clone() for p in params]
    ex.close()
    ref = None
    for r in range(world):
        for p in params:
            p.grad = None
        layers(torch.full((4, 6), float(2 * r + 3))).sum().backward()
        g = [p.grad.clone() for p in params]
        ref = g if ref is None else [a + b for a, b in zip(ref, g)]
    return raised, max(float((a - b).abs().max()) for a, b in zip(got, ref))


def test_bucketed_allreduce_state_is_per_step():
    out = run(_bucket_state_worker)
    for r in (0, 1):
        assert isinstance(out[r], tuple), out[r]
        raised, err = out[r]
        assert raised and err < 1e-6


def _mixed_width_worker(rank, world):
    """Tables of different widths (dedupe and padded modes): one exchange per width, every
    table's rows in rank order, identical on both ranks."""
    from conftest import pkg
    D = pkg("distributed")
    F = pkg("functional")

    class Emb:
        def __init__(self, rows, width):
            self.weight = torch.zeros((rows, width))
            self.sink = F.SparseGradSink()

    res = {}
    for mode in ("dedupe", "padded"):
        embs = [Emb(10, 4), Emb(7, 8), Emb(5, 4)]
        for t, e in enumerate(embs):
            ids = torch.tensor([t, 1 + rank, t], dtype=torch.int64)   # a duplicate id per rank
            rows = torch.full((3, e.weight.shape[1]), float(10 * rank + t))
            e.sink.slices = [(ids, rows)]

        class Opt:
            dense = []
            embeddings = embs

        D.MirroredGradientExchange(sparse=mode, max_rows=4, dedupe_fn=_np_dedupe)(Opt)
        out = []
        for e in embs:
            ids, rows = e.sink.gathered()
            keep = ids >= 0
            out.append((ids[keep].tolist(), rows[keep].tolist()))
        res[mode] = out
    return res


def test_mixed_width_tables_exchange():
    out = run(_mixed_width_worker)
    assert out[0] == out[1], (out[0], out[1])
    dd, pd_ = out[0]["dedupe"], out[0]["padded"]
    for t, width in enumerate((4, 8, 4)):
        # dedupe: rank-local unique ids ascending, duplicates summed, ranks concatenated
        u0 = sorted({t, 1})
        u1 = sorted({t, 2})
        assert dd[t][0] == u0 + u1
        for j, i in enumerate(u0 + u1):
            r = 0 if j < len(u0) else 1
            n = 2 if i == t and t != 1 + r else (3 if i == t == 1 + r else 1)
            assert dd[t][1][j] == [float(10 * r + t) * n] * width
        # padded: the raw rows, rank order
        assert pd_[t][0] == [t, 1, t, t, 2, t]
        assert [row[0] for row in pd_[t][1]] == [float(t)] * 3 + [float(10 + t)] * 3


def test_sharded_eval_recall_matches_unsharded_and_oracle():
    out = run(_sharded_eval_worker)
    for r in (0, 1):
        sharded, whole, ref = out[r]
        assert sharded == whole, (r, sharded, whole)
        for k, v in ref.items():
            assert abs(sharded[k] - v) < 1e-12, (r, k, sharded[k], v)
    assert out[0][0] == out[1][0]
