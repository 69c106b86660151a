"""The deduplicated in-batch pair at the size the bench times it (BASELINE config 3): B = 65536,
D = 128, contraction precision 6, the first batch of bench.py's C3 Zipf(1.05) ids over the 10M-user /
1M-item tables, routed through the model's id plan (rs_inbatch_unique_ids_pair_i64) exactly as
MultiTaskModel.compute_loss does (functional.inbatch_dedup_plan with ids).

Tower rows are functions of the id alone (src/models.py:85-90), so U / C here are one random row
per distinct id, repeated wherever the id repeats. Checked, always including the last rows,
columns and tiles (the largest byte offsets):
* the plan: distinct counts and inverse maps against numpy;
* lse, row loss and dU on sampled rows, dC on sampled columns, against float64 (truth over all B
  columns: the full definition, no counts involved);
* the fp64-accumulated total against sum(lse) - sum(diag);
* kept-score tiles, including the last one past 2^31 bytes of the ~2.3 GB kept-score region;
* every batch row's loss, lse, dU and dC against the full B x B split pair on the same batch.
Reference: tfrs.tasks.Retrieval (src/models.py:116,137), SURVEY Appendix A.6. Tolerance: the
north-star 1e-4 (conftest.assert_close).
"""
import os

import numpy as np
import pytest

from conftest import assert_close, pkg, score_tiles

pytestmark = pytest.mark.gpu

B, D, PREC = 65536, 128, 6
USERS, ITEMS = 10_000_000, 1_000_000


def zipf_ids(rng, n, vocab, a=1.05):
    """bench.py zipf_ids: Zipf(a) ranks over [1, vocab], scattered by a multiplicative permutation."""
    ranks = rng.zipf(a, size=n * 2)
    ranks = ranks[ranks <= vocab][:n]
    while ranks.size < n:
        extra = rng.zipf(a, size=n)
        ranks = np.concatenate([ranks, extra[extra <= vocab]])[:n]
    perm_mult = 2654435761 % vocab or 1
    return ((ranks.astype(np.int64) * perm_mult) % vocab) + 1


def _n(t):
    return t.detach().double().cpu().numpy() if t.dtype.is_floating_point else t.detach().cpu().numpy()


def _lse_rows(Q32, K32, chunk=1024):
    """log sum_j exp(Q_i . K_j) over every K row: fp32 host GEMM per chunk, float64 exp-sum."""
    import torch
    Qt, Kt = torch.from_numpy(Q32), torch.from_numpy(K32)
    out = np.empty(Q32.shape[0], np.float64)
    for r0 in range(0, Q32.shape[0], chunk):
        S = Qt[r0:r0 + chunk] @ Kt.T
        m = S.max(dim=1, keepdim=True).values
        s = torch.exp(S - m).sum(dim=1, dtype=torch.float64)
        out[r0:r0 + chunk] = (m[:, 0].double() + torch.log(s)).numpy()
    return out


def _tile(S_buf, NT, it, ut):
    """32 x 32 kept-score tile (item tile it, user tile ut) -> M[user_local, item_local]
    (conftest.score_tiles)."""
    off = (it * NT + ut) * 1024
    return score_tiles(S_buf[off:off + 1024].cpu().numpy())


def test_dedup_pair_c3_size_through_id_plan(cuda):
    import torch
    torch.set_num_threads(max(1, min(16, os.cpu_count() or 1)))
    F = pkg("functional")
    rng = np.random.default_rng(1234)          # bench.py setup_two_tower, rank 0: the first batch
    uid = zipf_ids(rng, B, USERS)
    iid = zipf_ids(rng, B, ITEMS)
    u_keys, u_first, u_inv, u_cnt = np.unique(uid, return_index=True, return_inverse=True, return_counts=True)
    c_keys, c_first, c_inv, c_cnt = np.unique(iid, return_index=True, return_inverse=True, return_counts=True)
    nu, nc = len(u_keys), len(c_keys)
    assert 20_000 < nu < 35_000 and 15_000 < nc < 30_000, (nu, nc)     # the C3 shape (~26.5k x ~21.3k)
    vr = np.random.default_rng(99)
    Ud = (vr.standard_normal((nu, D)) * 0.35).astype(np.float32)       # one tower row per distinct id
    Cd = (vr.standard_normal((nc, D)) * 0.35).astype(np.float32)
    U32, C32 = Ud[u_inv], Cd[c_inv]
    U, C = U32.astype(np.float64), C32.astype(np.float64)
    tU, tC = torch.from_numpy(U32).to(cuda), torch.from_numpy(C32).to(cuda)
    tuid, tiid = torch.from_numpy(uid).to(cuda), torch.from_numpy(iid).to(cuda)

    # the host-count form (its counts are checked here; the device-count form, the eager default since
    # round 6, is bitwise this one: test_gpu_inbatch_dedup.py::test_device_count_pair_bitwise_equals_host_count_pair)
    plan = F.inbatch_dedup_plan(tU, tC, PREC, ids=(tuid, tiid, USERS + 1, ITEMS + 1), device_counts=False)
    assert plan is not None and plan[0] is not None and plan[1] is not None, "the dedup pair must be taken"
    users, items = plan
    assert users[3] == nu and items[3] == nc
    # distinct index = ascending id order, representative = first occurrence, counts = multiplicities
    assert np.array_equal(_n(users[2]), u_inv) and np.array_equal(_n(items[2]), c_inv)
    assert np.array_equal(_n(users[0])[:nu], u_first) and np.array_equal(_n(items[0])[:nc], c_first)
    assert np.array_equal(_n(users[1])[:nu], u_cnt) and np.array_equal(_n(items[1])[:nc], c_cnt)

    S_dd = F.inbatch_scores_buffer(B, cuda)
    T, ROW, LSE, DU, T64 = F.inbatch_softmax_fwd_dedup(tU, tC, users, items, S_dd, PREC)
    g = 0.75
    DUs, DC = F.inbatch_softmax_bwd_dedup(tU, LSE, users, items, S_dd, PREC, gscale=torch.tensor(g, device=cuda),
                                          dU_unit=DU)
    torch.cuda.synchronize()

    # sampled rows (first, random, last): lse, row loss, dU against float64 over all B columns
    rows = np.unique(np.concatenate([np.arange(64), rng.choice(B, 192, replace=False), np.arange(B - 64, B),
                                     u_first[np.argsort(-u_cnt)[:8]]]))        # the hottest users too
    S_r = U[rows] @ C.T
    m = S_r.max(1, keepdims=True)
    lse_r = (m + np.log(np.exp(S_r - m).sum(1, keepdims=True)))[:, 0]
    P_r = np.exp(S_r - lse_r[:, None])
    dU_r = P_r @ C - C[rows]
    assert_close(_n(LSE)[rows], lse_r, 1e-4, "lse")
    assert_close(_n(ROW)[rows], lse_r - np.einsum("ij,ij->i", U[rows], C[rows]), 1e-4, "row loss")
    assert_close(_n(DU)[rows], dU_r, 1e-4, "dU (unit)", floor=0.0)
    assert_close(_n(DUs)[rows], g * dU_r, 1e-4, "dU", floor=0.0)

    # sampled columns: dC_j = g (sum_i P_ij U_i - U_j) needs every row's lse (a row's lse is its
    # distinct user's lse over all B columns: host fp32 GEMM of the distinct users against C)
    lse_d = _lse_rows(Ud, C32)
    lse_all = lse_d[u_inv]
    assert np.abs(lse_all[rows] - lse_r).max() < 1e-5
    cols = np.unique(np.concatenate([np.arange(64), rng.choice(B, 192, replace=False), np.arange(B - 64, B),
                                     c_first[np.argsort(-c_cnt)[:8]]]))
    P_c = np.exp(U @ C[cols].T - lse_all[:, None])
    dC_c = g * (P_c.T @ U - U[cols])
    assert_close(_n(DC)[cols], dC_c, 1e-4, "dC", floor=0.0)

    tot = float(lse_all.sum() - np.einsum("ij,ij->i", U, C).sum())
    assert abs(float(T64.item()) - tot) <= 1e-4 * max(1.0, abs(tot)), (float(T64.item()), tot)
    assert abs(float(T.item()) - tot) <= 1e-4 * max(1.0, abs(tot))

    # kept scores of the distinct pairs: tile (item tile it, user tile ut) holds
    # U[u_first[32 ut + a]] . C[c_first[32 it + b]]; the last tile sits past 2^31 bytes
    NTu, NTc = (nu + 31) // 32, (nc + 31) // 32
    last_off = ((NTc - 1) * NTu + NTu - 1) * 4096
    assert last_off > (1 << 31), last_off
    for it, ut in ((0, 0), (NTc - 1, 0), (0, NTu - 1), (NTc - 1, NTu - 1), (NTc - 2, NTu - 2),
                   (NTc // 2, NTu // 3)):
        M = _tile(S_dd, NTu, it, ut)
        ur = np.arange(32 * ut, min(32 * ut + 32, nu))
        cr = np.arange(32 * it, min(32 * it + 32, nc))
        ref = Ud[ur].astype(np.float64) @ Cd[cr].astype(np.float64).T
        got = M[:len(ur), :len(cr)]
        assert np.abs(got - ref).max() <= 1e-5 * max(1.0, np.abs(ref).max()), (it, ut)

    # the entry the bench's graphed C3 step runs (the plan's counts stay on the device, grids sized
    # for B: rs_inbatch_softmax_xent_{fwd,bwd}_dedup_dev_f32) on the same batch, into a fresh score
    # buffer: every output and the whole kept-score region (to its last tile past 2^31 bytes) bitwise
    # the host-count pair's just checked against float64
    plan_d = F.inbatch_dedup_plan(tU, tC, PREC, ids=(tuid, tiid, USERS + 1, ITEMS + 1), device_counts=True)
    assert plan_d is not None and plan_d[0][3] is None and plan_d[1][3] is None, "device-count plan expected"
    S_dv = F.inbatch_scores_buffer(B, cuda)
    S_dv.fill_(float("nan"))          # a tile the device form skipped would stay NaN
    Td, ROWd, LSEd, DUd, T64d = F.inbatch_softmax_fwd_dedup(tU, tC, plan_d[0], plan_d[1], S_dv, PREC)
    DUsd, DCd = F.inbatch_softmax_bwd_dedup(tU, LSEd, plan_d[0], plan_d[1], S_dv, PREC,
                                            gscale=torch.tensor(g, device=cuda), dU_unit=DUd)
    torch.cuda.synchronize()
    for name, a_, b_ in (("total", Td, T), ("row loss", ROWd, ROW), ("lse", LSEd, LSE), ("dU unit", DUd, DU),
                         ("total64", T64d, T64), ("dU", DUsd, DUs), ("dC", DCd, DC)):
        assert torch.equal(a_, b_), f"device-count {name} differs from the host-count pair"
    used = NTu * NTc * 1024
    assert torch.equal(S_dv[:used], S_dd[:used]), "kept scores differ between the device- and host-count pairs"
    assert (used - 1) * 4 > (1 << 31)
    del S_dd, S_dv

    # the full B x B split pair on the same batch (itself fp64-checked at this size in
    # test_gpu_production_sizes.py): every batch row, 1e-4
    S_full = F.inbatch_scores_buffer(B, cuda)
    full = F.inbatch_softmax_fwd(tU, tC, scores=S_full, precision=PREC)
    full_b = F.inbatch_softmax_bwd(tU, tC, full[2], gscale=torch.tensor(g, device=cuda), dU_unit=full[3],
                                   scores=S_full, precision=PREC)
    torch.cuda.synchronize()
    for name, a, b in (("row loss", ROW, full[1]), ("lse", LSE, full[2]), ("dU", DUs, full_b[0]),
                       ("dC", DC, full_b[1])):
        assert_close(_n(a), _n(b), 1e-4, f"{name} vs full pair")
    assert abs(float(T64.item()) - float(full[4].item())) <= 1e-4 * abs(float(full[4].item()))
    del S_full
    torch.cuda.empty_cache()


def test_graphed_c3_step_bitwise_equal_to_eager(cuda):
    """The bench's C3 step at its size (B = 65536, Zipf(1.05) ids over the 10M-user / 1M-item tables,
    reference model dims, deferred reductions) captured in a hipGraph: the captured id plan keeps its
    counts on the device (the *_dedup_dev_f32 pair), and 1 eager step + capture + 2 replays end
    bitwise equal to 3 eager steps (every parameter, accumulator and loss)."""
    import torch
    cfgm, models, optim, tr, graphs = pkg("config"), pkg("models"), pkg("optim"), pkg("trainer"), pkg("graphs")
    F = pkg("functional")
    rng = np.random.default_rng(1234)
    batches = []
    for _ in range(3):
        uid = torch.from_numpy(zipf_ids(rng, B, USERS)).to(cuda)
        iid = torch.from_numpy(zipf_ids(rng, B, ITEMS)).to(cuda)
        rating = torch.from_numpy(rng.integers(1, 6, B).astype(np.float32)).to(cuda)
        batches.append(graphs.pack_batch(({"user_id": uid, "movie_id": iid},
                                          {"rating": rating, "y_implicit": (rating >= 4).float()})))
    plans, finals = [], []
    real_plan = F.inbatch_dedup_plan

    def spy(*a, **k):
        p_ = real_plan(*a, **k)
        plans.append(None if p_ is None else ("device" if p_[0][3] is None else "host"))
        return p_
    F.inbatch_dedup_plan = spy
    try:
        for graphed in (False, True):
            cfg = cfgm.ModelConfig(embedding_dim=D, batch_size=B)
            model = models.MultiTaskModel(cfg, USERS, ITEMS, {}, class_weights={0: 1.6, 1: 0.73}, seed=4,
                                          device=cuda)
            opt = optim.Adagrad(model.dense_parameters(), model.embedding_modules(),
                                optim.ExponentialDecay(0.05, 1000, 0.96, True), clipnorm=1.0, defer_reductions=True)
            step = lambda b, model=model, opt=opt: tr.ProductionTrainer.train_step(model, opt, b)["loss"]  # noqa: E731
            runner = graphs.GraphedTrainStep(step, batches[0]) if graphed else step
            losses = [runner(b).detach().clone() for b in batches]
            torch.cuda.synchronize()
            finals.append(({k: v.detach().clone() for k, v in model.state_dict().items()},
                           [a.clone() for a in opt.emb_accum], losses))
            del model, opt, runner, step
            torch.cuda.empty_cache()
    finally:
        F.inbatch_dedup_plan = real_plan
    ek = "device" if F.INBATCH_DEDUP_DEVICE else "host"   # (the eager steps' plans: device since round 6)
    assert plans == [ek] * 3 + [ek, "device"], plans
    (sd0, acc0, l0), (sd1, acc1, l1) = finals
    for a_, b_ in zip(l0, l1):
        assert torch.equal(a_, b_)
    for k in sd0:
        assert torch.equal(sd0[k], sd1[k]), k
    for a_, b_ in zip(acc0, acc1):
        assert torch.equal(a_, b_)


@pytest.mark.parametrize("b,users,items", [(B, USERS, ITEMS), (20000, 300_000, 60_000)])
def test_distinct_row_towers_bitwise_equal_to_per_row_towers(cuda, monkeypatch, b, users, items):
    """The towers over the id plan's distinct ids (functional.DistinctTowersFn: lookups and Dense
    forward once per distinct id on the weight-stationary kernel with device-side row counts, outputs
    expanded by the inverse map; dW over the batch rows with each layer input read through the map,
    dX with the ReLU masks read through it) against the per-row towers: 2 eager C3-law training steps
    (B = 65536 over the 10M / 1M tables, and a ragged B = 20000), every loss, parameter and Adagrad
    accumulator bitwise equal."""
    import torch
    cfgm, models, optim, tr = pkg("config"), pkg("models"), pkg("optim"), pkg("trainer")
    F = pkg("functional")
    rng = np.random.default_rng(77)
    batches = []
    for _ in range(2):
        uid = torch.from_numpy(zipf_ids(rng, b, users)).to(cuda)
        iid = torch.from_numpy(zipf_ids(rng, b, items)).to(cuda)
        rating = torch.from_numpy(rng.integers(1, 6, b).astype(np.float32)).to(cuda)
        batches.append(({"user_id": uid, "movie_id": iid}, {"rating": rating, "y_implicit": (rating >= 4).float()}))
    monkeypatch.setattr(F, "INBATCH_DEDUP_MIN_B", min(F.INBATCH_DEDUP_MIN_B, b))
    calls = []
    real = F.DistinctTowersFn.apply

    def spy(*a):
        calls.append(1)
        return real(*a)
    monkeypatch.setattr(F.DistinctTowersFn, "apply", spy)
    finals = []
    for distinct in (False, True):
        monkeypatch.setattr(F, "DISTINCT_TOWERS", distinct)
        cfg = cfgm.ModelConfig(embedding_dim=D, batch_size=b)
        model = models.MultiTaskModel(cfg, users, items, {}, class_weights={0: 1.6, 1: 0.73}, seed=4, device=cuda)
        opt = optim.Adagrad(model.dense_parameters(), model.embedding_modules(),
                            optim.ExponentialDecay(0.05, 1000, 0.96, True), clipnorm=1.0, defer_reductions=True)
        losses = [tr.ProductionTrainer.train_step(model, opt, bt)["loss"].detach().clone() for bt in batches]
        torch.cuda.synchronize()
        finals.append(({k: v.detach().clone() for k, v in model.state_dict().items()},
                       [a.clone() for a in opt.accum], [a.clone() for a in opt.emb_accum], losses))
        del model, opt
        torch.cuda.empty_cache()
    assert len(calls) == 2, calls                   # the distinct path ran on both steps of the second run
    (sd0, ad0, ae0, l0), (sd1, ad1, ae1, l1) = finals
    for x_, y_ in zip(l0, l1):
        assert torch.equal(x_, y_), (x_, y_)
    for k in sd0:
        assert torch.equal(sd0[k], sd1[k]), k
    for x_, y_ in zip(ad0 + ae0, ad1 + ae1):
        assert torch.equal(x_, y_)
