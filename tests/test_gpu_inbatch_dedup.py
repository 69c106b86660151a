"""The deduplicated in-batch pair (rs_inbatch_unique_rows_f32 + rs_inbatch_softmax_xent_*_dedup_f32)
against the oracle's full B x B retrieval loss (oracle/recsys_oracle.py retrieval_loss /
retrieval_grads, restating src/models.py:116,137 + tfrs.tasks.Retrieval): batches whose tower
rows repeat (few distinct users and/or items, skewed multiplicities) must give every batch row the
loss, lse, dU and dC of the full pair, within the north-star 1e-4."""
import numpy as np
import pytest

from conftest import assert_close, oracle, pkg

pytestmark = pytest.mark.gpu


def _t(x, dev):
    import torch
    t = torch.from_numpy(np.ascontiguousarray(x))
    return (t.float() if t.dtype == torch.float64 else t).to(dev)


def _n(t):
    return t.detach().double().cpu().numpy() if t.dtype.is_floating_point else t.detach().cpu().numpy()


def _batch(rng, B, n_distinct, D, skew):
    """B rows drawn from n_distinct pool rows (Zipf-skewed picks when skew > 0)."""
    pool = rng.standard_normal((n_distinct, D)) * 0.4
    if skew > 0:
        idx = (rng.zipf(skew, B) - 1) % n_distinct
    else:
        idx = rng.integers(0, n_distinct, B)
    return pool[idx].astype(np.float32)


@pytest.mark.parametrize("B,D,nd", [(1, 128, 1), (31, 128, 3), (1000, 128, 250), (1000, 32, 1000), (4099, 36, 40),
                                    (70001, 128, 5000)])
def test_unique_rows_match_numpy(cuda, B, D, nd):
    import torch
    F = pkg("functional")
    rng = np.random.default_rng(B + D)
    X = _batch(rng, B, nd, D, 1.2)
    if B > 2:
        X[1] = -0.0 * np.abs(X[1])      # -0.0 and +0.0 rows are distinct bitwise
        X[2] = 0.0 * np.abs(X[2])
    rep, count, inv, info = F.inbatch_unique_rows(_t(X, cuda))
    torch.cuda.synchronize()
    bits = X.view(np.uint32)
    _, first, np_inv, np_cnt = np.unique(bits, axis=0, return_index=True, return_inverse=True, return_counts=True)
    np_inv = np_inv.reshape(-1)
    nu, bad = _n(info).tolist()
    assert bad == 0 and nu == len(first)
    rep, count, inv = _n(rep), _n(count), _n(inv)
    assert inv.min() >= 0 and inv.max() < nu
    assert np.array_equal(rep[inv], first[np_inv])          # each row's representative = its first occurrence
    assert np.array_equal(count[inv], np_cnt[np_inv].astype(np.float64))
    assert count[nu:].sum() == 0 and count.shape[0] == (B + 31) // 32 * 32


@pytest.mark.parametrize("prec", [6, 9])
@pytest.mark.parametrize("B,nu,nc,skew", [(1000, 37, 300, 1.3), (2001, 2001, 150, 1.2), (2001, 400, 2001, 0.0),
                                          (4100, 64, 64, 1.1), (777, 1, 5, 0.0), (3000, 1500, 700, 0.0)])
def test_dedup_pair_matches_oracle(cuda, B, nu, nc, skew, prec):
    import torch
    F = pkg("functional")
    O = oracle()
    D = 128
    rng = np.random.default_rng(B + nu + 7 * nc + prec)
    U = _batch(rng, B, nu, D, skew)
    C = _batch(rng, B, nc, D, skew)
    tU, tC = _t(U, cuda), _t(C, cuda)
    plan = F.inbatch_dedup_plan(tU, tC, prec, force=True)
    assert plan is not None
    users, items = plan
    n_u, n_c = len(np.unique(U, axis=0)), len(np.unique(C, axis=0))
    assert (users[3] if users else B) == n_u and (items[3] if items else B) == n_c
    U64, C64 = U.astype(np.float64), C.astype(np.float64)
    row, tot, lse = O.retrieval_loss(U64, C64)
    dU, dC = O.retrieval_grads(U64, C64, lse)
    S = F.inbatch_scores_buffer(B, cuda)
    T, ROW, LSE, DU, T64 = F.inbatch_softmax_fwd_dedup(tU, tC, users, items, S, prec)
    g = torch.tensor(1.25, device=cuda)
    DUs, DC = F.inbatch_softmax_bwd_dedup(tU, LSE, users, items, S, prec, gscale=g, dU_unit=DU)
    assert_close(_n(ROW), row, 1e-4, "row loss")
    assert_close(_n(LSE), lse, 1e-4, "lse")
    assert abs(float(T64.item()) - tot) <= 1e-4 * max(1.0, abs(tot))
    assert_close(_n(DU), dU, 1e-4, "dU (unit)")
    assert_close(_n(DUs), 1.25 * dU, 1e-4, "dU")
    assert_close(_n(DC), 1.25 * dC, 1e-4, "dC")


def test_dedup_pair_matches_full_pair_at_c3_like_skew(cuda):
    """B = 20000 rows from Zipf(1.05) ids (the C3 id law) over 10M users / 1M items:
    the deduplicated pair against the full B x B split pair (itself oracle-checked above)."""
    import torch
    F = pkg("functional")
    B, D, prec = 20000, 128, 6
    rng = np.random.default_rng(1234)

    def zipf_rows(V, n):
        r = rng.zipf(1.05, n * 3)
        r = r[r <= V][:n].astype(np.int64)
        return (r * 2654435761) % V
    uid, iid = zipf_rows(10_000_000, B), zipf_rows(1_000_000, B)
    U = np.zeros((B, D), np.float32)
    C = np.zeros((B, D), np.float32)
    _, ui = np.unique(uid, return_inverse=True)
    _, ii = np.unique(iid, return_inverse=True)
    U[:] = (rng.standard_normal((ui.max() + 1, D)) * 0.3).astype(np.float32)[ui]
    C[:] = (rng.standard_normal((ii.max() + 1, D)) * 0.3).astype(np.float32)[ii]
    tU, tC = _t(U, cuda), _t(C, cuda)
    plan = F.inbatch_dedup_plan(tU, tC, prec)
    assert plan is not None and plan[0] is not None and plan[1] is not None
    assert plan[0][3] == ui.max() + 1 and plan[1][3] == ii.max() + 1
    g = torch.tensor(0.5, device=cuda)
    S = F.inbatch_scores_buffer(B, cuda)
    full = F.inbatch_softmax_fwd(tU, tC, scores=S, precision=prec)
    full_b = F.inbatch_softmax_bwd(tU, tC, full[2], gscale=g, dU_unit=full[3], scores=S, precision=prec)
    S2 = F.inbatch_scores_buffer(B, cuda)
    dd = F.inbatch_softmax_fwd_dedup(tU, tC, plan[0], plan[1], S2, prec)
    dd_b = F.inbatch_softmax_bwd_dedup(tU, dd[2], plan[0], plan[1], S2, prec, gscale=g, dU_unit=dd[3])
    for name, a, b in (("row loss", dd[1], full[1]), ("lse", dd[2], full[2]), ("dU", dd_b[0], full_b[0]),
                       ("dC", dd_b[1], full_b[1])):
        assert_close(_n(a), _n(b), 1e-4, name)
    assert abs(float(dd[4].item()) - float(full[4].item())) <= 1e-4 * abs(float(full[4].item()))


def test_autograd_function_takes_dedup_path_and_matches(cuda, monkeypatch):
    """InBatchSoftmaxFn (the model's retrieval loss, models.py) at B = 16384 with repeated rows:
    the deduplicated pair runs (plan taken) and its loss / gradients match the full pair's."""
    import torch
    F = pkg("functional")
    B, D = 16384, 128
    rng = np.random.default_rng(5)
    U = _batch(rng, B, 3000, D, 1.1)
    C = _batch(rng, B, 900, D, 1.1)
    res = {}
    taken = []
    real_plan = F.inbatch_dedup_plan

    def spy(*a, **k):
        p = real_plan(*a, **k)
        taken.append(p is not None)
        return p
    monkeypatch.setattr(F, "inbatch_dedup_plan", spy)
    for on in (True, False):
        monkeypatch.setattr(F, "INBATCH_DEDUP", on)
        tU = _t(U, cuda).requires_grad_(True)
        tC = _t(C, cuda).requires_grad_(True)
        tot, row = F.InBatchSoftmaxFn.apply(tU, tC, 6)
        (0.25 * tot).backward()
        res[on] = (_n(tot), _n(row), _n(tU.grad), _n(tC.grad))
    assert taken == [True, False]
    for j, name in enumerate(("loss", "row loss", "dU", "dC")):
        assert_close(res[True][j], res[False][j], 1e-4, name)


@pytest.mark.parametrize("B,nu,nc", [(1, 1, 1), (1000, 300, 1000), (70001, 5000, 800)])
def test_unique_pair_equals_two_single_calls(cuda, B, nu, nc):
    """rs_inbatch_unique_pair_f32 (both sides in one sort) gives each side exactly the outputs of
    its own rs_inbatch_unique_rows_f32 call (same key order within a side)."""
    import torch
    F = pkg("functional")
    rng = np.random.default_rng(B + nu)
    U = _t(_batch(rng, B, nu, 128, 1.1), cuda)
    C = _t(_batch(rng, B, nc, 128, 0.0), cuda)
    pu, pc = F.inbatch_unique_pair(U, C)
    su, sc = F.inbatch_unique_rows(U), F.inbatch_unique_rows(C)
    torch.cuda.synchronize()
    for p, q in ((pu, su), (pc, sc)):
        nd = int(q[3][0])
        assert torch.equal(p[3], q[3])
        assert torch.equal(p[0][:nd], q[0][:nd]) and torch.equal(p[2], q[2]) and torch.equal(p[1], q[1])


@pytest.mark.parametrize("B,nu,nc,urows,crows", [(1, 1, 1, 10, 10), (1000, 300, 1000, 5000, 1001),
                                                 (70001, 5000, 800, 10_000_001, 1_000_001),
                                                 # one id per side: every key in one bucket of the id
                                                 # sort (its > 2048-key path), small and large tables
                                                 (50000, 1, 1, 10, 10), (30001, 1, 2, 10_000_001, 1_000_001)])
def test_unique_ids_pair_matches_numpy(cuda, B, nu, nc, urows, crows):
    """rs_inbatch_unique_ids_pair_i64: rows grouped by id, distinct index = ascending id order,
    representative = first occurrence, counts = multiplicities; ids outside [0, rows) (the gather's
    zero rows) form one group per side; no collision counts."""
    import torch
    F = pkg("functional")
    rng = np.random.default_rng(B + nu + nc)
    uid = rng.choice(urows, nu, replace=False)[(rng.zipf(1.2, B) - 1) % nu].astype(np.int64)
    cid = rng.choice(crows, nc, replace=False)[rng.integers(0, nc, B)].astype(np.int64)
    if B > 4:
        uid[[1, 3]] = [-5, urows + 7]      # out of range: one group with key "no row"
        cid[2] = crows
    pu, pc = F.inbatch_unique_ids_pair(_t(uid, cuda), _t(cid, cuda), urows, crows)
    torch.cuda.synchronize()
    for ids, rows, (rep, count, inv, side, _) in ((uid, urows, pu), (cid, crows, pc)):
        key = np.where((ids < 0) | (ids >= rows), np.int64(2 ** 62), ids)
        _, first, np_inv, np_cnt = np.unique(key, return_index=True, return_inverse=True, return_counts=True)
        nd, bad = _n(side).tolist()
        assert bad == 0 and nd == len(first)
        rep, count, inv = _n(rep), _n(count), _n(inv)
        assert np.array_equal(inv, np_inv.reshape(-1))
        assert np.array_equal(rep[:nd], first)
        assert np.array_equal(count[:nd], np_cnt.astype(np.float64)) and count[nd:].sum() == 0


def test_model_retrieval_loss_dedups_by_id(cuda, monkeypatch):
    """MultiTaskModel.compute_loss hands the ids to InBatchSoftmaxFn: the id plan is taken, and the
    loss (1e-5) and every gradient (the north-star 1e-4; the two plans order the distinct rows
    differently, so the fp32 sums over 16384 rows differ at ~1e-5) equal those of the same step on
    the content plan."""
    import torch
    F = pkg("functional")
    M = pkg("models")
    C = pkg("config")
    cfg = C.ModelConfig(embedding_dim=128)
    rng = np.random.default_rng(3)
    B = 16384
    feats = {"user_id": torch.from_numpy(((rng.zipf(1.1, B) * 7919) % 5000 + 1).astype(np.int64)).to(cuda),
             "movie_id": torch.from_numpy(((rng.zipf(1.1, B) * 104729) % 3000 + 1).astype(np.int64)).to(cuda)}
    labels = {"rating": torch.from_numpy(rng.integers(1, 6, B).astype(np.float32)).to(cuda),
              "y_implicit": torch.from_numpy((rng.random(B) < 0.3).astype(np.float32)).to(cuda)}
    used = []
    real_ids, real_rows, real_plan = F.inbatch_unique_ids_pair, F.inbatch_unique_pair, F.inbatch_dedup_plan
    monkeypatch.setattr(F, "inbatch_unique_ids_pair", lambda *a, **k: used.append("ids") or real_ids(*a, **k))
    monkeypatch.setattr(F, "inbatch_unique_pair", lambda *a, **k: used.append("rows") or real_rows(*a, **k))
    res = []
    for by_id in (True, False):
        if not by_id:   # the same step with the ids withheld from the plan: distinct rows by content
            monkeypatch.setattr(F, "inbatch_plan_eligible", lambda B, config: False)   # no id plan up front
            monkeypatch.setattr(F, "inbatch_dedup_plan",
                                lambda U, C_, precision, force=False, ids=None: real_plan(U, C_, precision, force))
        model = M.MultiTaskModel(cfg, 5000, 3000, {}, seed=11, device=cuda)
        loss = model.compute_loss((feats, labels), training=True)
        loss.backward()
        g = {n: p.grad.detach().double().cpu().numpy() for n, p in model.named_parameters() if p.grad is not None}
        sl = [e.sink.gathered()[1].detach().double().cpu().numpy() for e in model.embedding_modules()]
        res.append((float(loss), g, sl))
    assert used == ["ids", "rows"]
    assert abs(res[0][0] - res[1][0]) <= 1e-5 * abs(res[1][0])
    for n in res[1][1]:
        assert_close(res[0][1][n], res[1][1][n], 1e-4, n)
    for a_, b_ in zip(res[0][2], res[1][2]):
        assert_close(a_, b_, 1e-4, "embedding slices")


def _zipf_ids(rng, n, vocab, a=1.05):
    ranks = rng.zipf(a, size=n * 2)
    ranks = ranks[ranks <= vocab][:n]
    while ranks.size < n:
        extra = rng.zipf(a, size=n)
        ranks = np.concatenate([ranks, extra[extra <= vocab]])[:n]
    return ((ranks.astype(np.int64) * (2654435761 % vocab or 1)) % vocab) + 1


@pytest.mark.parametrize("B,urows,crows", [(20000, 10_000_000, 1_000_000), (1000, 50, 3000), (4099, 5000, 7)])
def test_device_count_pair_bitwise_equals_host_count_pair(cuda, B, urows, crows):
    """rs_inbatch_softmax_xent_{fwd,bwd}_dedup_dev_f32 (counts read on the device, grids sized for
    B: the graph-capturable form) against the host-count entries on the same id plan: the same
    stream-K shape is derived on the device, so every output is bitwise equal."""
    import torch
    F = pkg("functional")
    rng = np.random.default_rng(B + urows)
    uid, iid = _zipf_ids(rng, B, urows - 1), _zipf_ids(rng, B, crows - 1)
    _, ui = np.unique(uid, return_inverse=True)
    _, ii = np.unique(iid, return_inverse=True)
    U = (rng.standard_normal((ui.max() + 1, 128)) * 0.3).astype(np.float32)[ui]
    C = (rng.standard_normal((ii.max() + 1, 128)) * 0.3).astype(np.float32)[ii]
    tU, tC = _t(U, cuda), _t(C, cuda)
    ids = (_t(uid, cuda), _t(iid, cuda), urows, crows)
    host = F.inbatch_dedup_plan(tU, tC, 6, force=True, ids=ids, device_counts=False)
    dev = F.inbatch_dedup_plan(tU, tC, 6, force=True, ids=ids, device_counts=True)
    assert host is not None and dev is not None and dev[0][3] is None
    if host[0] is None or host[1] is None:    # a side without duplicates: the host plan keeps it whole
        pytest.skip("both sides must be deduplicated for a like-for-like comparison")
    g = torch.tensor(0.75, device=cuda)
    outs = []
    for plan in (host, dev):
        S = F.inbatch_scores_buffer(B, cuda)
        tot, row, lse, dU, tot64 = F.inbatch_softmax_fwd_dedup(tU, tC, plan[0], plan[1], S, 6)
        dUs, dC = F.inbatch_softmax_bwd_dedup(tU, lse, plan[0], plan[1], S, 6, gscale=g, dU_unit=dU)
        torch.cuda.synchronize()
        outs.append([tot, row, lse, dU, tot64, dUs, dC])
    for j, (a, b) in enumerate(zip(*outs)):
        assert torch.equal(a, b), j


@pytest.mark.parametrize("eager_device", [True, False])
def test_graphed_c3_like_step_with_dedup_bitwise_equal_to_eager(cuda, eager_device, monkeypatch):
    """A MultiTaskModel training step at B = 16384 on Zipf ids (the deduplicated pair on) captured
    in a hipGraph: the captured plan keeps its counts on the device (no host read), and 1 eager step
    + capture + 3 replays end bitwise equal to 4 eager steps — with the eager steps on device-count
    plans (the default since round 6) and on host-count plans."""
    import torch
    cfgm, models, optim, tr, graphs = pkg("config"), pkg("models"), pkg("optim"), pkg("trainer"), pkg("graphs")
    F = pkg("functional")
    monkeypatch.setattr(F, "INBATCH_DEDUP_DEVICE", eager_device)
    B, NU, NI = 16384, 200_000, 50_000
    rng = np.random.default_rng(17)
    batches = []
    for _ in range(4):
        rating = torch.from_numpy(rng.integers(1, 6, B).astype(np.float32)).to(cuda)
        batches.append(graphs.pack_batch(({"user_id": _t(_zipf_ids(rng, B, NU), cuda),
                                           "movie_id": _t(_zipf_ids(rng, B, NI), cuda)},
                                          {"rating": rating, "y_implicit": (rating >= 4).float()})))
    finals, plans = [], []
    real_plan = F.inbatch_dedup_plan

    def spy(*a, **k):
        p_ = real_plan(*a, **k)
        plans.append(None if p_ is None else ("device" if p_[0][3] is None else "host"))
        return p_
    F.inbatch_dedup_plan = spy
    try:
        for graphed in (False, True):
            cfg = cfgm.ModelConfig(embedding_dim=128, batch_size=B)
            model = models.MultiTaskModel(cfg, NU, NI, {}, class_weights={0: 1.6, 1: 0.73}, seed=4, device=cuda)
            opt = optim.Adagrad(model.dense_parameters(), model.embedding_modules(),
                                optim.ExponentialDecay(0.05, 1000, 0.96, True), clipnorm=1.0, defer_reductions=True)
            step = lambda b, model=model, opt=opt: tr.ProductionTrainer.train_step(model, opt, b)["loss"]  # noqa: E731
            runner = graphs.GraphedTrainStep(step, batches[0]) if graphed else step
            for b in batches:
                runner(b)
            torch.cuda.synchronize()
            finals.append({k: v.detach().clone() for k, v in model.state_dict().items()})
    finally:
        F.inbatch_dedup_plan = real_plan
    # eager: 4 plans of the eager kind; graphed: the eager first step, then the capture's device-count plan
    ek = "device" if eager_device else "host"
    assert plans == [ek] * 4 + [ek, "device"], plans
    for k in finals[0]:
        assert torch.equal(finals[0][k], finals[1][k]), k


def test_sparse_update_takes_the_id_plan_order_bitwise(cuda, monkeypatch):
    """The tables' sparse Adagrad takes the step's id-plan order (each side's stable ascending-id
    order, carried by the embedding sinks) instead of sorting the ids again: two eager steps at
    B = 16384 on Zipf ids end bitwise equal with and without it, and the ordered entry is the one
    that ran."""
    import torch
    cfgm, models, optim, tr = pkg("config"), pkg("models"), pkg("optim"), pkg("trainer")
    F = pkg("functional")
    B, NU, NI = 16384, 200_000, 50_000
    rng = np.random.default_rng(23)
    batches = []
    for _ in range(2):
        rating = torch.from_numpy(rng.integers(1, 6, B).astype(np.float32)).to(cuda)
        batches.append(({"user_id": _t(_zipf_ids(rng, B, NU), cuda), "movie_id": _t(_zipf_ids(rng, B, NI), cuda)},
                        {"rating": rating, "y_implicit": (rating >= 4).float()}))
    real = F.sparse_adagrad_multi
    seen = []

    def spy(*a, **k):
        seen.append((k.get("orders") is not None, k.get("heads") is not None))
        return real(*a, **k)
    monkeypatch.setattr(F, "sparse_adagrad_multi", spy)
    finals = []
    for use, heads in ((False, False), (True, False), (True, True)):
        monkeypatch.setattr(optim, "SPARSE_USE_PLAN_ORDER", use)
        monkeypatch.setattr(optim, "SPARSE_USE_PLAN_HEADS", heads)
        cfg = cfgm.ModelConfig(embedding_dim=128, batch_size=B)
        model = models.MultiTaskModel(cfg, NU, NI, {}, class_weights={0: 1.6, 1: 0.73}, seed=4, device=cuda)
        opt = optim.Adagrad(model.dense_parameters(), model.embedding_modules(),
                            optim.ExponentialDecay(0.05, 1000, 0.96, True), clipnorm=1.0, defer_reductions=True)
        for b in batches:
            tr.ProductionTrainer.train_step(model, opt, b)
        torch.cuda.synchronize()
        finals.append({k: v.detach().clone() for k, v in model.state_dict().items()})
    assert seen == [(False, False)] * 2 + [(True, False)] * 2 + [(True, True)] * 2, seen
    for k in finals[0]:
        assert torch.equal(finals[0][k], finals[1][k]), k
        assert torch.equal(finals[0][k], finals[2][k]), k


@pytest.mark.parametrize("B,urows,crows", [(3, 10, 10), (5000, 300, 70000), (65536, 10_000_001, 1_000_001)])
def test_planned_sparse_update_bitwise_equal_to_sorting_update(cuda, B, urows, crows):
    """rs_sparse_adagrad_multi_step_planned_f32 (the apply pass over the plan's run heads: one slice
    per distinct id) leaves both tables, both accumulators and the step counter bitwise what the
    sorting update (rs_sparse_adagrad_multi_step_f32) leaves: Zipf-hot runs spanning many windows,
    out-of-range ids (the skipped group), clip-norm on."""
    import torch
    F = pkg("functional")
    rng = np.random.default_rng(B + 7)
    uid = _zipf_ids(rng, B, urows - 1)
    iid = _zipf_ids(rng, B, crows - 1)
    if B > 4:
        uid[1], uid[4], iid[2] = -3, urows + 9, crows
    tu, ti = _t(uid, cuda), _t(iid, cuda)
    plan = F.inbatch_unique_ids_pair(tu, ti, urows, crows, order=True, dids=True)
    g = [torch.randn((B, 128), device=cuda) * 0.1, torch.randn((B, 128), device=cuda) * 0.1]
    out = []
    for mode in ("sort", "order", "heads"):
        tabs = [torch.randn((urows, 128), device=cuda, generator=torch.Generator(cuda).manual_seed(1)),
                torch.randn((crows, 128), device=cuda, generator=torch.Generator(cuda).manual_seed(2))]
        accs = [torch.full_like(t, 0.1) for t in tabs]
        it = torch.zeros((), dtype=torch.int64, device=cuda)
        orders = [plan[0][5], plan[1][5]] if mode != "sort" else None
        heads = [(plan[0][7], plan[0][6], plan[0][3][0:1]), (plan[1][7], plan[1][6], plan[1][3][0:1])] \
            if mode == "heads" else None
        F.sparse_adagrad_multi(tabs, accs, [tu, ti], g, it, 0.05, 0.96, 1000, 1.0, 1e-7, increment=True,
                               orders=orders, heads=heads)
        torch.cuda.synchronize()
        out.append((tabs, accs, int(it)))
    for m in (1, 2):
        assert out[m][2] == out[0][2] == 1
        for j in range(2):
            assert torch.equal(out[m][0][j], out[0][0][j]), (m, j)
            assert torch.equal(out[m][1][j], out[0][1][j]), (m, j)


@pytest.mark.parametrize("B,urows,crows", [(1, 10, 10), (5000, 300, 70000), (70001, 10_000_001, 1_000_001)])
def test_id_plan_orders_and_ordered_gather(cuda, B, urows, crows):
    """rs_inbatch_unique_ids_pair_order_i64: each side's rows in ascending-id order (stable, ids
    outside the table last as one group) with the same plan as the unordered call; the gather that
    reads the tables in that order (rs_embedding_gather_tables_ordered_f32) writes exactly the
    unordered gather's rows."""
    import torch
    F = pkg("functional")
    rng = np.random.default_rng(B)
    uid = _zipf_ids(rng, B, urows - 1)
    iid = rng.integers(0, crows, B).astype(np.int64)
    if B > 4:
        uid[2], iid[3] = -1, crows + 5          # invalid ids: the "no row" group, zero rows
    tu, ti = _t(uid, cuda), _t(iid, cuda)
    po = F.inbatch_unique_ids_pair(tu, ti, urows, crows, order=True)
    pp = F.inbatch_unique_ids_pair(tu, ti, urows, crows)
    torch.cuda.synchronize()
    for side, ids, rows in ((0, uid, urows), (1, iid, crows)):
        nd = int(pp[side][3][0])                 # rep / count past the distinct count are scratch
        assert torch.equal(po[side][3], pp[side][3]), side
        assert torch.equal(po[side][2], pp[side][2]), side
        assert torch.equal(po[side][0][:nd], pp[side][0][:nd]), side
        assert torch.equal(po[side][1][:nd], pp[side][1][:nd]), side
        key = np.where((ids < 0) | (ids >= rows), np.int64(2 ** 62), ids)
        assert np.array_equal(_n(po[side][5]), np.argsort(key, kind="stable"))
    tabs = [torch.randn((urows, 128), device=cuda), torch.randn((crows, 128), device=cuda)]
    a = F.embedding_gather_tables(tabs, [tu, ti])
    b = F.embedding_gather_tables(tabs, [tu, ti], orders=[po[0][5], po[1][5]])
    torch.cuda.synchronize()
    for x, y in zip(a, b):
        assert torch.equal(x, y)


@pytest.mark.parametrize("B,urows,crows", [(1, 10, 10), (5000, 300, 70000), (65536, 10_000_001, 1_000_001)])
def test_id_plan_distinct_ids_and_ids_gather(cuda, B, urows, crows):
    """rs_inbatch_unique_ids_plan_i64: the same plan as the ordered call, plus each distinct slot's
    id (ascending; the out-of-range group -> the table's row count; -1 from the distinct count on);
    rs_embedding_gather_tables_ids_f32 from those ids writes exactly the rows the representative-row
    gather (rs_embedding_gather_tables_rows_f32) writes, zero rows for the out-of-range group, and
    leaves every position past the count untouched."""
    import torch
    F = pkg("functional")
    rng = np.random.default_rng(B + 1)
    uid = _zipf_ids(rng, B, urows - 1)
    iid = rng.integers(0, crows, B).astype(np.int64)
    if B > 4:
        uid[2], iid[3], iid[4] = -1, crows + 5, -7   # invalid ids: the "no row" group, zero rows
    tu, ti = _t(uid, cuda), _t(iid, cuda)
    pd = F.inbatch_unique_ids_pair(tu, ti, urows, crows, order=True, dids=True)
    po = F.inbatch_unique_ids_pair(tu, ti, urows, crows, order=True)
    torch.cuda.synchronize()
    assert len(pd[0]) == 8 and len(po[0]) == 6
    for side, ids, rows in ((0, uid, urows), (1, iid, crows)):
        nd = int(po[side][3][0])
        assert torch.equal(pd[side][3], po[side][3]) and torch.equal(pd[side][2], po[side][2]), side
        assert torch.equal(pd[side][5], po[side][5]), side
        assert torch.equal(pd[side][0][:nd], po[side][0][:nd]), side
        assert torch.equal(pd[side][1][:nd], po[side][1][:nd]), side
        did = _n(pd[side][6])
        rep = _n(pd[side][0])[:nd]
        want = ids[rep]
        want = np.where((want < 0) | (want >= rows), rows, want)
        assert np.array_equal(did[:nd], want), side
        assert np.all(did[nd:] == -1), side
        assert np.all(np.diff(did[:nd]) > 0), side        # ascending, distinct
        # run heads: slot p's first position in the order holds its representative row
        st = _n(pd[side][7])[:nd]
        order = _n(pd[side][5])
        assert st[0] == 0 and np.all(np.diff(st) > 0), side
        assert np.array_equal(order[st], rep), side
        assert np.array_equal(np.diff(np.append(st, B)), _n(pd[side][1])[:nd].astype(np.int64)), side
    tabs = [torch.randn((urows, 128), device=cuda), torch.randn((crows, 128), device=cuda)]
    cnts = [po[0][3][0:1], po[1][3][0:1]]
    a = F.embedding_gather_tables_rows(tabs, [tu, ti], [po[0][0], po[1][0]], cnts)
    sentinel = [torch.full((B, 128), 7.0, device=cuda) for _ in range(2)]
    b = F.embedding_gather_tables_ids(tabs, [pd[0][6], pd[1][6]], out=sentinel)
    torch.cuda.synchronize()
    for side, ids, rows in ((0, uid, urows), (1, iid, crows)):
        nd = int(po[side][3][0])
        assert torch.equal(a[side][:nd], b[side][:nd]), side
        assert bool((b[side][nd:] == 7.0).all()), side
        bad = _n(pd[side][6])[:nd] >= rows
        if bad.any():
            assert not _n(b[side])[:nd][bad].any(), side


@pytest.mark.parametrize("dedup", [False, True])
def test_backward_reuses_forward_workspace_bitwise(cuda, dedup):
    """RS_INBATCH_FWD_WS: a backward given its storing forward's workspace skips splitting U again
    (the forward's image is reused) — dU and dC bitwise those of a backward on a fresh workspace,
    for the full split pair and for the deduplicated pair (host and device counts)."""
    import torch
    F = pkg("functional")
    rng = np.random.default_rng(5 + dedup)
    B, D = 3000, 128
    if dedup:
        uid = rng.integers(0, 400, B)
        iid = rng.integers(0, 900, B)
        Ud = rng.standard_normal((400, D)).astype(np.float32) * 0.3
        Cd = rng.standard_normal((900, D)).astype(np.float32) * 0.3
        U32, C32 = Ud[uid], Cd[iid]
    else:
        U32 = rng.standard_normal((B, D)).astype(np.float32) * 0.3
        C32 = rng.standard_normal((B, D)).astype(np.float32) * 0.3
    tU, tC = torch.from_numpy(U32).to(cuda), torch.from_numpy(C32).to(cuda)
    g = torch.tensor(0.5, device=cuda)
    variants = [None] if not dedup else [False, True]
    for dev_counts in variants:
        outs = []
        for reuse in (False, True):
            S = F.inbatch_scores_buffer(B, cuda)
            ws = F.inbatch_workspace(B, D, cuda, dedup=dedup) if reuse else None
            if dedup:
                ids = (torch.from_numpy(uid).to(cuda), torch.from_numpy(iid).to(cuda), 400, 900)
                plan = F.inbatch_dedup_plan(tU, tC, 6, force=True, ids=ids, device_counts=dev_counts)
                tot, row, lse, dU, _ = F.inbatch_softmax_fwd_dedup(tU, tC, plan[0], plan[1], S, 6, workspace=ws)
                dUs, dC = F.inbatch_softmax_bwd_dedup(tU, lse, plan[0], plan[1], S, 6, gscale=g, dU_unit=dU,
                                                      workspace=ws)
            else:
                tot, row, lse, dU, _ = F.inbatch_softmax_fwd(tU, tC, scores=S, precision=6, workspace=ws)
                dUs, dC = F.inbatch_softmax_bwd(tU, tC, lse, gscale=g, dU_unit=dU, scores=S, precision=6,
                                                workspace=ws)
            torch.cuda.synchronize()
            outs.append((dUs.cpu(), dC.cpu(), lse.cpu()))
        for a, b in zip(outs[0], outs[1]):
            assert torch.equal(a, b)
