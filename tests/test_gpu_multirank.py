"""The data-parallel path with the real HIP kernels: 2 ranks, both on the box's one GPU.

Reference: tf.distribute.MirroredStrategy (src/trainer.py:45-48, variables under strategy.scope()
at :148) — each replica trains on its slice of the global batch with its own in-batch negatives,
dense gradients are SUM-all-reduced, embedding IndexedSlices are gathered in replica order, and
every replica applies the same update.

The ranks are fresh child processes (a spawn context: the parent never execs; each child imports
torch and the HIP library itself) joined by torch.distributed over gloo (RS_DIST_BACKEND=gloo —
two RCCL ranks cannot share one GPU); the exchange code is the product path
(distributed.MirroredGradientExchange: hook-driven bucketed dense all-reduce, the HIP
deduplication kernel rs_sparse_dedupe_f32 or the padded exchange, the multi-table sparse Adagrad).
Checked against the oracle's MirroredStrategy rule (oracle.data_parallel_grads + adagrad_apply)
in float64 at 1e-4, and the two replicas' parameters must be bitwise equal after every run."""
import os
import socket

import numpy as np
import pytest

from conftest import ROOT, assert_close, oracle, pkg

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, fn, args, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    backend = os.environ.get("RS_TEST_BACKEND", "gloo")
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", RS_DIST_BACKEND=backend)
    try:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(0)
        D = pkg("distributed")
        if world == 1:   # init_process_group() leaves a one-process job undistributed
            dist.init_process_group(backend, rank=0, world_size=1,
                                    **({"device_id": torch.device("cuda", 0)} if backend == "nccl" else {}))
        else:
            assert D.init_process_group()
        assert dist.get_backend() == backend
        pkg("_native").load()
        try:
            q.put((rank, fn(rank, world, *args)))
        finally:
            torch.cuda.synchronize()
            dist.destroy_process_group()
    except BaseException as e:  # surfaced by the parent
        import traceback
        q.put((rank, "ERROR: " + repr(e) + "\n" + traceback.format_exc()))


def run_ranks(fn, *args, world=2, timeout=150):
    # (timeout: a rank that has not reported by then fails the test, with its ranks killed, well
    # inside the 180 s a GPU runner waits for output before it takes a run to be hung)
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank_main, args=(r, world, port, fn, args, q)) for r in range(world)]
    for p in ps:
        p.start()
    try:
        out = dict(q.get(timeout=timeout) for _ in ps)
    finally:
        for p in ps:
            p.join(timeout=15)
            if p.is_alive():
                p.kill()
    for r, v in out.items():
        if isinstance(v, str) and v.startswith("ERROR"):
            raise AssertionError(f"rank {r}: {v}")
    return out


# ---------------------------------------------------------------------------------------------
# MultiTaskModel at the reference dims (D = 128, towers 256-128-64, 3 cross layers, deep 256-128)
# ---------------------------------------------------------------------------------------------
LR = 0.01
CW = {0: 1.6, 1: 0.73}
NU, NI = 6040, 3706          # ML-1M-shaped tables (the graph-capture test below)
# "ml1m": ML-1M-shaped tables, per-rank B = 2048, item ids with hot duplicates (a fifth from 40
# rows); "zipf": config 3's id law, Zipf(1.05) over 200k users / 50k items (the hot ids are the
# same as over 10M / 1M: the law's head does not depend on the vocabulary), per-rank B = 8192 with
# the deduplicated in-batch pair switched on from that batch (functional.INBATCH_DEDUP_MIN_B; the
# ranks assert it ran), one item filling several percent of the batch
PROBLEMS = {"ml1m": dict(nu=6040, ni=3706, B=2048, steps=3, zipf=False),
            "zipf": dict(nu=200_000, ni=50_000, B=8192, steps=2, zipf=True),
            # per-rank B above the fused-stack limit: the towers run over the id plan's distinct rows
            "zipf_big": dict(nu=200_000, ni=50_000, B=20000, steps=2, zipf=True, gates=False)}


def _dup_ids(rng, n, rows):
    """Ids with duplicates inside and across the ranks' slices (a fifth drawn from 40 hot rows,
    ~10 copies each; the rest uniform), so the deduplicating exchange has work."""
    hot = rng.choice(rows, 40, replace=False)
    ids = rng.integers(0, rows, n)
    pick = rng.random(n) < 0.2
    ids[pick] = hot[rng.integers(0, 40, int(pick.sum()))]
    return ids.astype(np.int64)


def _zipf_ids(rng, n, vocab, a=1.05):
    """bench.py zipf_ids: Zipf(a) ranks over [1, vocab], scattered by a multiplicative permutation."""
    ranks = rng.zipf(a, size=n * 2)
    ranks = ranks[ranks <= vocab][:n]
    while ranks.size < n:
        extra = rng.zipf(a, size=n)
        ranks = np.concatenate([ranks, extra[extra <= vocab]])[:n]
    return ((ranks.astype(np.int64) * (2654435761 % vocab or 1)) % vocab) + 1


def _mt_problem(world, name):
    O = oracle()
    pr = PROBLEMS[name]
    ocfg = O.OracleConfig(embedding_dim=128, cross_layers=3, learning_rate_retrieval=LR)
    P = O.init_params(ocfg, pr["nu"] + 1, pr["ni"] + 1, seed=21, dtype=np.float32, bias_scale=0.05)
    rng = np.random.default_rng(2024)
    batches = []
    for _ in range(pr["steps"]):
        Bg = pr["B"] * world
        if pr["zipf"]:
            uid, iid = _zipf_ids(rng, Bg, pr["nu"]), _zipf_ids(rng, Bg, pr["ni"])
        else:
            uid, iid = rng.integers(0, pr["nu"] + 1, Bg), _dup_ids(rng, Bg, pr["ni"] + 1)
        rating = rng.integers(1, 6, Bg).astype(np.float32)
        batches.append((uid, iid, rating, (rating >= 4).astype(np.float32)))
    return O, ocfg, P, batches


def _snapshot(model, opt):
    """parameters and Adagrad accumulators by parameter name (numpy copies)."""
    names = {id(p): n for n, p in model.named_parameters()}
    P = {n: p.detach().cpu().numpy().copy() for n, p in model.named_parameters()}
    A = {names[id(p)]: a.cpu().numpy().copy() for p, a in zip(opt.dense, opt.accum)}
    for e, a in zip(opt.embeddings, opt.emb_accum):
        A[names[id(e.weight)]] = a.cpu().numpy().copy()
    return P, A


def _pack(masks):
    return {k: [(np.packbits(m), m.shape) for m in v] for k, v in masks.items()}


def _unpack(packed):
    return {k: [np.unpackbits(b, count=int(np.prod(shp))).reshape(shp).astype(bool) for b, shp in v]
            for k, v in packed.items()}


def _mt_rank(rank, world, mode, name):
    import torch
    from conftest import gpu_relu_masks
    cfgm, models, optim, tr, D = pkg("config"), pkg("models"), pkg("optim"), pkg("trainer"), pkg("distributed")
    F = pkg("functional")
    dev = torch.device("cuda", 0)
    pr = PROBLEMS[name]
    O, ocfg, P, batches = _mt_problem(world, name)
    B = pr["B"]
    cfg = cfgm.ModelConfig(embedding_dim=128, cross_layers=3, batch_size=B * world, learning_rate_retrieval=LR,
                           distributed_strategy="mirrored")
    model = models.MultiTaskModel(cfg, pr["nu"], pr["ni"], {}, class_weights=CW, device=dev)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in P.items()})
    opt = optim.Adagrad(model.dense_parameters(), model.embedding_modules(),
                        optim.ExponentialDecay(LR, 1000, 0.96, True), clipnorm=1.0)
    parts = mode.split("-")
    early = "early" in parts                  # the sparse exchange started from the tables' sinks
    if "rows" in parts:                       # the per-row towers (no distinct-row towers)
        F.DISTINCT_TOWERS = False
    mode = parts[0]
    distinct = []
    real_ok = F.distinct_towers_ok

    def ok_spy(*a, **k):                      # record whether the distinct-row towers ran
        r_ = real_ok(*a, **k)
        distinct.append(r_)
        return r_
    F.distinct_towers_ok = ok_spy
    ex = D.MirroredGradientExchange(max_rows=B, dense_params=opt.dense, sparse=mode,
                                    embeddings=opt.embeddings if early else None)
    assert ex.bucketer is not None            # dense all-reduce from the backward's grad hooks
    opt.pre_apply_hooks.append(ex)
    plans = []
    real_plan = F.inbatch_dedup_plan

    def spy(*a, **k):                         # record whether the deduplicated pair ran
        p_ = real_plan(*a, **k)
        plans.append(p_ is not None)
        return p_
    F.inbatch_dedup_plan = spy
    if pr["zipf"]:
        F.INBATCH_DEDUP_MIN_B = B
    losses, snaps, masks = [], [], []
    sl = slice(rank * B, (rank + 1) * B)
    for uid, iid, rating, yi in batches:
        if rank == 0:
            snaps.append(_snapshot(model, opt))
        data = ({"user_id": torch.from_numpy(uid[sl]).to(dev), "movie_id": torch.from_numpy(iid[sl]).to(dev)},
                {"rating": torch.from_numpy(rating[sl]).to(dev), "y_implicit": torch.from_numpy(yi[sl]).to(dev)})
        if pr.get("gates", True):
            with F.record_relu_gates() as rec:     # the step's own gates, checked against its backward
                losses.append(float(tr.ProductionTrainer.train_step(model, opt, data)["loss"]))
            masks.append(_pack(gpu_relu_masks(model, rec)))
        else:
            losses.append(float(tr.ProductionTrainer.train_step(model, opt, data)["loss"]))
    F.inbatch_dedup_plan = real_plan
    F.distinct_towers_ok = real_ok
    ex.close()
    torch.cuda.synchronize()
    return {"losses": losses, "snaps": snaps if pr.get("gates", True) else [], "final": _snapshot(model, opt)[0],
            "masks": masks, "plans": plans, "distinct": distinct}


def _check_against_oracle(name, mode, out):
    """Every step against the oracle's MirroredStrategy step taken from the same parameters and
    accumulators (rank 0's snapshot before the step), in float64, under the GPU ranks' ReLU gates
    (recorded from each step's own forward, conftest.gpu_relu_masks; every gate that differs from the float64 sign must sit within fp32
    rounding of zero): the per-replica losses and the updated parameters at 1e-4."""
    from conftest import assert_flips_are_rounding, mask_flips
    O, ocfg, _, batches = _mt_problem(2, name)
    B = PROBLEMS[name]["B"]
    snaps = out[0]["snaps"] + [(out[0]["final"], None)]
    report = []
    for s, (uid, iid, rating, yi) in enumerate(batches):
        P = {k: v.astype(np.float64) for k, v in snaps[s][0].items()}
        A = {k: v.astype(np.float64) for k, v in snaps[s][1].items()}
        shards = [(uid[r * B:(r + 1) * B], iid[r * B:(r + 1) * B], rating[r * B:(r + 1) * B].astype(np.float64),
                   yi[r * B:(r + 1) * B].astype(np.float64)) for r in range(2)]
        masks = [_unpack(out[r]["masks"][s]) for r in range(2)]
        for r in (0, 1):                            # each replica's own loss (per-replica negatives)
            flips = mask_flips(O, P, ocfg, shards[r][0], shards[r][1], masks[r])
            assert_flips_are_rounding(flips)
            report.append((s, r, sum(n for layers in flips.values() for n, _ in layers)))
            want = O.loss_and_grads(P, ocfg, *shards[r], CW, with_grads=False)["loss"]
            got = out[r]["losses"][s]
            assert abs(got - want) <= 1e-4 * max(1.0, abs(want)), (mode, r, s, got, want)
        G = O.data_parallel_grads(P, ocfg, shards, CW, masks=masks)
        O.adagrad_apply(P, A, G, s, LR, clipnorm=1.0)
        for k, v in P.items():
            assert_close(snaps[s + 1][0][k], v, 1e-4, f"{name} {mode} step {s}: {k}")
    print(f"{name} {mode}: flipped gates per (step, rank):", report)


@pytest.mark.parametrize("mode", ["dedupe", "padded"])
def test_multitask_two_ranks_match_oracle_and_each_other(cuda, mode):
    """ML-1M-shaped: 3 steps, each against the oracle's MirroredStrategy step at 1e-4 (no relaxed
    branch); the two replicas' parameters bitwise equal after the run."""
    out = run_ranks(_mt_rank, mode, "ml1m")
    a, b = out[0]["final"], out[1]["final"]
    for k in a:                                     # replicas stay bit-identical (no broadcast)
        assert np.array_equal(a[k], b[k]), k
    _check_against_oracle("ml1m", mode, out)


@pytest.mark.parametrize("mode", ["dedupe", "padded"])
def test_early_sparse_exchange_bitwise_equal_to_hook_exchange(cuda, mode):
    """The sparse exchange issued from the tables' sinks as the backward delivers their slices
    (MirroredGradientExchange(embeddings=)) against the same exchange in the pre-apply hook: every
    loss and the final parameters and accumulators bitwise equal, on both ranks."""
    base = run_ranks(_mt_rank, mode, "ml1m")
    early = run_ranks(_mt_rank, mode + "-early", "ml1m")
    for r in (0, 1):
        assert base[r]["losses"] == early[r]["losses"], r
        for k in base[r]["final"]:
            assert np.array_equal(base[r]["final"][k], early[r]["final"][k]), (r, k)


def test_distinct_row_towers_two_ranks_bitwise_equal_to_per_row(cuda):
    """Per-rank B = 20000 on Zipf ids (above the fused-stack limit): the towers over the id plan's
    distinct rows, with the sparse exchange started from the sinks they feed, give every loss and the
    final parameters bitwise those of the per-row towers, on both ranks, replicas bitwise equal."""
    rows = run_ranks(_mt_rank, "dedupe-early-rows", "zipf_big", timeout=160)
    dist_ = run_ranks(_mt_rank, "dedupe-early", "zipf_big", timeout=160)
    for r in (0, 1):
        assert dist_[r]["distinct"] and all(dist_[r]["distinct"]), dist_[r]["distinct"]
        assert not any(rows[r]["distinct"]), rows[r]["distinct"]
        assert all(dist_[r]["plans"]), dist_[r]["plans"]
        assert rows[r]["losses"] == dist_[r]["losses"], r
        for k in rows[r]["final"]:
            assert np.array_equal(rows[r]["final"][k], dist_[r]["final"][k]), (r, k)
    for k in dist_[0]["final"]:
        assert np.array_equal(dist_[0]["final"][k], dist_[1]["final"][k]), k


def test_multitask_two_ranks_zipf_c3_law(cuda):
    """Config 3's Zipf(1.05) id law at per-rank B = 8192 with the deduplicated in-batch pair on
    (asserted on both ranks), both exchange modes: 2 steps each against the oracle at 1e-4 under
    the GPU's gates, replicas bitwise equal; and the two modes against each other, independent of
    the oracle: the deduplicating exchange sums each replica's duplicate rows before the gather and
    the padded one after it, so the results differ only by the order of fp32 additions (1e-5)."""
    finals = {}
    for mode in ("dedupe", "padded"):
        out = run_ranks(_mt_rank, mode, "zipf")
        for r in (0, 1):
            assert out[r]["plans"] and all(out[r]["plans"]), (mode, r, out[r]["plans"])
        a, b = out[0]["final"], out[1]["final"]
        for k in a:
            assert np.array_equal(a[k], b[k]), k
        _check_against_oracle("zipf", mode, out)
        finals[mode] = a
    for k in finals["dedupe"]:
        assert_close(finals["padded"][k], finals["dedupe"][k], 1e-5, f"padded vs dedupe: {k}")
# ---------------------------------------------------------------------------------------------
# DCN-v2 ranker (config 5 extension) with 6 tables
# ---------------------------------------------------------------------------------------------
NF, E, ND, L2_, BD = 6, 128, 13, 2, 512
DEEP = [256, 128]
VOCAB = [501 + 37 * f for f in range(NF)]


def _dcn2_data(world, steps=2):
    rng = np.random.default_rng(77)
    out = []
    for _ in range(steps):
        Bg = BD * world
        ids = np.stack([_dup_ids(rng, Bg, v + 1) for v in VOCAB])
        dense = rng.standard_normal((Bg, ND)).astype(np.float32)
        y = (rng.random(Bg) < 0.3).astype(np.float32)
        out.append((ids, dense, y))
    return out


def _dcn2_rank(rank, world, mode):
    import torch
    models, optim, D = pkg("models"), pkg("optim"), pkg("distributed")
    dev = torch.device("cuda", 0)
    m = models.DCNv2Ranker(VOCAB, embedding_dim=E, num_dense=ND, cross_layers=L2_, deep_layers=DEEP, device=dev,
                           precision=6, seed=5)
    with torch.no_grad():
        g = torch.Generator(device="cpu").manual_seed(9)
        m.cross_b.copy_((torch.rand(m.cross_b.shape, generator=g) - 0.5) * 0.02)
        m.cross_b[:, m.d_raw:] = 0
    opt = optim.Adagrad(m.dense_parameters(), m.embedding_modules(), 1e-2, clipnorm=1.0)
    ex = D.MirroredGradientExchange(max_rows=BD, dense_params=opt.dense, sparse=mode)
    opt.pre_apply_hooks.append(ex)
    sl = slice(rank * BD, (rank + 1) * BD)
    snaps = []
    for ids, dense, y in _dcn2_data(world):
        if rank == 0:
            snaps.append(_snapshot(m, opt))
        opt.zero_grad()
        loss = m.compute_loss(torch.from_numpy(np.ascontiguousarray(ids[:, sl])).to(dev),
                              torch.from_numpy(dense[sl]).to(dev), torch.from_numpy(y[sl]).to(dev))
        loss.backward()
        opt.step()
    ex.close()
    torch.cuda.synchronize()
    return {"snaps": snaps, "final": _snapshot(m, opt)[0], "d": m.d}


@pytest.mark.parametrize("mode", ["dedupe", "padded"])
def test_dcn2_two_ranks_match_oracle_and_each_other(cuda, mode):
    """Each step against the oracle's data-parallel step from rank 0's snapshot (6 tables, ids with
    duplicates): dense gradients summed over the replicas, table rows gathered in replica order."""
    O = oracle()
    out = run_ranks(_dcn2_rank, mode)
    a, b = out[0]["final"], out[1]["final"]
    for k in a:
        assert np.array_equal(a[k], b[k]), k
    d = out[0]["d"]
    snaps = out[0]["snaps"] + [(out[0]["final"], None)]
    for step, (ids, dense, y) in enumerate(_dcn2_data(2)):
        P = {k: v.astype(np.float64) for k, v in snaps[step][0].items()}
        A = {k: v.astype(np.float64) for k, v in snaps[step][1].items()}
        tot = None
        for r in range(2):
            sl = slice(r * BD, (r + 1) * BD)
            g = O.dcn2_ranker_loss_and_grads(P, NF, E, d, DEEP, ids[:, sl], dense[sl].astype(np.float64),
                                            y[sl].astype(np.float64))["grads"]
            if tot is None:
                tot = g
                continue
            for k, v in g.items():
                tot[k] = ((np.concatenate([tot[k][0], v[0]]), np.concatenate([tot[k][1], v[1]]))
                          if isinstance(v, tuple) else tot[k] + v)
        O.adagrad_apply(P, A, tot, step, 1e-2, clipnorm=1.0)
        for k, v in P.items():
            assert_close(snaps[step + 1][0][k], v, 1e-4, f"{mode} step {step}: {k}")


# ---------------------------------------------------------------------------------------------
# Row-sharded exact top-K (config 4): the HIP scan per rank, gloo all-gather, the HIP merge
# ---------------------------------------------------------------------------------------------
def _topk_problem(Q):
    rng = np.random.default_rng(31)
    N, Dm = 200_000, 128
    items = (rng.integers(-8, 9, (N, Dm)) / 16).astype(np.float32)
    q = (rng.integers(-8, 9, (Q, Dm)) / 16).astype(np.float32)
    items[N - 5:] = items[7]                 # equal rows on both shards: the global index decides
    return items, q


def _topk_rank(rank, world, Q, prec):
    import torch
    R = pkg("retrieval")
    dev = torch.device("cuda", 0)
    items, q = _topk_problem(Q)
    per = items.shape[0] // world
    idx = R.ShardedBruteForceIndex(torch.from_numpy(items[rank * per:(rank + 1) * per]).to(dev),
                                   row_offset=rank * per, precision=prec)
    s, i = idx.search(torch.from_numpy(q).to(dev), 100)
    return s.cpu().numpy().astype(np.float64), i.cpu().numpy()


@pytest.mark.parametrize("Q,prec", [(10, 6), (300, 6), (300, 0)])
def test_sharded_topk_two_ranks_bitexact(cuda, Q, prec):
    O = oracle()
    out = run_ranks(_topk_rank, Q, prec)
    s0, i0 = out[0]
    s1, i1 = out[1]
    items, q = _topk_problem(Q)
    assert np.array_equal(i0, i1) and np.array_equal(s0, s1)
    sc, idx = O.topk_ip(q, items, 100)
    assert np.array_equal(i0, idx)
    assert np.array_equal(s0, sc)


def _eval_rank(rank, world):
    """ProductionTrainer._evaluate on a mirrored MultiTaskModel: sharded over the ranks (each rank's
    item-tower rows only, ShardedBruteForceIndex) and unsharded, plus the embeddings for the oracle."""
    import pathlib
    import tempfile

    import pandas as pd
    import torch
    cfgm, models, T, L = pkg("config"), pkg("models"), pkg("trainer"), pkg("lookup")
    dev = torch.device("cuda", 0)
    n_users, n_items = 700, 3001                    # odd: ragged item shards
    uv = L.build_vocab([str(i) for i in range(n_users)])
    iv = L.build_vocab([str(i) for i in range(n_items)])
    cfg = cfgm.ModelConfig(embedding_dim=64, cross_layers=2, eval_topk=[5, 10, 20, 50])
    model = models.MultiTaskModel(cfg, uv, iv, {}, seed=9, device=dev)     # same seed: identical replicas
    rng = np.random.default_rng(3)
    val_df = pd.DataFrame({"user_id": rng.integers(0, n_users, 1500).astype(str),
                           "movie_id": rng.integers(0, n_items + 40, 1500).astype(str)})
    datasets = {"val_df": val_df, "val_ds": object(), "item_vocab": iv}
    out = {}
    for distributed in (True, False):
        tr = T.ProductionTrainer.__new__(T.ProductionTrainer)
        tr.config, tr.device = cfg, dev
        tr.distributed, tr.rank, tr.world = distributed, rank, world
        tr.output_dir = pathlib.Path(tempfile.mkdtemp())
        out[distributed] = tr._evaluate(model, datasets)
    with torch.no_grad():
        ids = torch.arange(1, n_items + 1, device=dev)
        items = model.encoder({"movie_id": ids})["item_embedding"].double().cpu().numpy()
        sample = val_df.sample(n=1000, random_state=42)
        users = model.encoder({"user_id": sample["user_id"].values})["user_embedding"].double().cpu().numpy()
    return out[True], out[False], users, items, list(sample["movie_id"].values), iv


def test_sharded_eval_two_ranks_matches_unsharded_and_oracle(cuda):
    """_evaluate under data parallelism scores the items sharded over the ranks
    with the HIP scan, the all-gather and the HIP merge; every rank gets the unsharded evaluation's
    recall@k exactly, which equals the oracle's np.dot + argpartition (src/trainer.py:195-213) on
    the same embeddings."""
    O = oracle()
    out = run_ranks(_eval_rank)
    for r in (0, 1):
        sharded, whole, users, items, truth, iv = out[r]
        assert sharded == whole, (r, sharded, whole)
        ref = O.recall_at_k(users @ items.T, truth, iv, [5, 10, 20, 50])
        for k, v in ref.items():
            assert abs(sharded[k] - v) < 1e-12, (r, k, sharded[k], v)
    assert out[0][0] == out[1][0]


# ---------------------------------------------------------------------------------------------
# hipGraph capture of the data-parallel step with RCCL collectives (one rank: RCCL refuses two
# ranks on one GPU, so the collectives run in a one-rank group, forced through the exchange)
# ---------------------------------------------------------------------------------------------
def _graph_rank(rank, world):
    import torch
    cfgm, models, optim, tr, D, graphs = (pkg("config"), pkg("models"), pkg("optim"), pkg("trainer"),
                                          pkg("distributed"), pkg("graphs"))
    dev = torch.device("cuda", 0)
    O = oracle()
    B = 1024
    ocfg = O.OracleConfig(embedding_dim=128, cross_layers=3, learning_rate_retrieval=LR)
    P = O.init_params(ocfg, NU + 1, NI + 1, seed=5, dtype=np.float32, bias_scale=0.05)
    rng = np.random.default_rng(8)
    batches = []
    for _ in range(4):
        uid = torch.from_numpy(rng.integers(0, NU + 1, B)).to(dev)
        iid = torch.from_numpy(_dup_ids(rng, B, NI + 1)).to(dev)
        rating = torch.from_numpy(rng.integers(1, 6, B).astype(np.float32)).to(dev)
        batches.append(graphs.pack_batch(({"user_id": uid, "movie_id": iid},
                                          {"rating": rating, "y_implicit": (rating >= 4).float()})))
    finals = []
    for graphed in (False, True):
        cfg = cfgm.ModelConfig(embedding_dim=128, cross_layers=3, batch_size=B, learning_rate_retrieval=LR)
        model = models.MultiTaskModel(cfg, NU, NI, {}, class_weights=CW, device=dev)
        model.load_state_dict({k: torch.from_numpy(v) for k, v in P.items()})
        opt = optim.Adagrad(model.dense_parameters(), model.embedding_modules(),
                            optim.ExponentialDecay(LR, 1000, 0.96, True), clipnorm=1.0)
        ex = D.MirroredGradientExchange(max_rows=B, dense_params=opt.dense, sparse="padded", force=True)
        assert ex.bucketer is not None
        opt.pre_apply_hooks.append(ex)

        def step(batch, model=model, opt=opt):
            return tr.ProductionTrainer.train_step(model, opt, batch)["loss"]

        runner = graphs.GraphedTrainStep(step, batches[0]) if graphed else step
        for i in range(4):
            runner(batches[i])
        torch.cuda.synchronize()
        ex.close()
        finals.append({k: v.detach().cpu().numpy() for k, v in model.state_dict().items()})
    return finals


def test_graphed_padded_exchange_step_bitwise_equal_to_eager(cuda):
    """The padded exchange (no host read, static shapes) and the hook-driven bucketed all-reduce
    captured in a hipGraph with their RCCL collectives: 4 steps (1 eager + capture + 3 replays)
    bitwise equal to 4 eager steps."""
    import os as _os
    _os.environ["RS_TEST_BACKEND"] = "nccl"
    try:
        out = run_ranks(_graph_rank, world=1)
    finally:
        _os.environ.pop("RS_TEST_BACKEND", None)
    eager, graphed = out[0]
    for k in eager:
        assert np.array_equal(eager[k], graphed[k]), k
