#!/usr/bin/env python3
"""Benchmark: the reference's training step (MultiTaskModel two-tower retrieval + DCN ranking,
forward + backward + Adagrad) on the MI355X HIP path.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|c4|c5] [--no-cpu-baseline]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json configs): default `c3` = synthetic 10M users x 1M items, emb_dim 128,
in-batch negatives, batch 65536 per GPU (weak scaling: global batch = 65536 N), with the
reference model defaults (towers 128->256->128->64->128, 3 vector-cross layers, deep 256->128,
rating + CTR heads, Adagrad + clipnorm). `c2` = the MovieLens-1M-shaped DCN ranker (6,040 x
3,706, D=128, 3 cross layers, batch 4096). Ids are Zipf(1.05) over the tables (seed 1234),
ratings uniform 1..5; all inputs are resident in HBM before timing. A "step" is one full
training step over one batch. value = ranked (user, item) pairs trained per second, whole job.

One JSON line on rank 0 also carries: in-batch user x item dots/s, the roofline of the dominant
kernel (the in-batch softmax passes, timed live with HIP events on the launch stream) and the
CPU baseline (the oracle's numpy fp32 train step on a bounded sample, rank 0 only).
"""
import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import importlib  # noqa: E402

PKG = "recommendation-system-maang-nvidia-_amd"
cfgmod = importlib.import_module(PKG + ".config")
models = importlib.import_module(PKG + ".models")
optim = importlib.import_module(PKG + ".optim")
F = importlib.import_module(PKG + ".functional")
distributed = importlib.import_module(PKG + ".distributed")
graphs = importlib.import_module(PKG + ".graphs")

FP32_MFMA_PEAK_TFLOPS = 157.3      # MI355X_MICROARCH.md: fp32 MFMA (no xf32) dense peak
BF16_MFMA_PEAK_TFLOPS = 2500.0     # MI355X_MICROARCH.md: bf16 MFMA dense peak (no sparsity)
HBM_PEAK_GBS = 8000.0


def contraction_peak(precision):
    """Peak fp32-product rate of the in-batch contractions at a contraction precision: the f32
    MFMA peak, or the bf16 MFMA peak shared by the 6 / 9 bf16 products of each fp32 product."""
    if precision in (6, 9):
        return round(BF16_MFMA_PEAK_TFLOPS / precision, 1), (
            f"bf16 MFMA dense peak {BF16_MFMA_PEAK_TFLOPS:.0f} TF/s / {precision} bf16 products per fp32 product")
    return FP32_MFMA_PEAK_TFLOPS, "f32 MFMA dense peak"

CONFIGS = {
    "c3": dict(workload="synthetic-10Mx1M-two-tower+dcn-train-step", users=10_000_000, items=1_000_000,
               D=128, B=65536, cross=3),
    "c2": dict(workload="movielens1m-shaped-dcn-ranker-train-step", users=6040, items=3706, D=128, B=4096,
               cross=3),
    # config 5 (extension model): 26 sparse x 1M-row tables + 13 dense, E=128 -> d = 3,341 (padded
    # 3,344), 4 matrix cross layers + 3x1024 deep; 131,072 global = 16,384 per GPU at 8 GPUs
    # config 4: 100M x 128 items row-sharded over 8 GPUs = 12.5M rows per GPU, exact top-100
    "c4": dict(workload="synthetic-100M-item-bruteforce-top100 (12.5M-row shard per GPU)", rows=12_500_000,
               D=128, k=100, Q=1024, B=1024),
    "c5": dict(workload="criteo-shaped-dcn-v2-train-step", tables=26, rows=1_000_000, dense=13, D=128,
               B=16384, cross=4, deep=[1024, 1024, 1024]),
}


def _r02_traffic():
    try:
        with open(os.path.join(ROOT, "profiles", "r02_pmc_traffic.json")) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def _r03_traffic(key, field="traffic_bytes"):
    """A per-launch figure from the newest profiles/r0*_pmc_traffic.json (tools/gpu_pmc_traffic.sh: the
    dispatches of N launches of one entry point between two marker kernels, one counter per rocprofv3
    pass)."""
    rec = None
    for name in ("r05_pmc_traffic.json", "r03_pmc_traffic.json"):
        try:
            with open(os.path.join(ROOT, "profiles", name)) as f:
                rec = json.load(f).get(key)
        except (OSError, ValueError):
            continue
        if rec:
            break
    rec = rec or {}
    v = rec.get(field)
    return v if v is None or field != "traffic_bytes" else int(v)


def dedup_pair_traffic(B, D, precision):
    """Per-launch HBM-side bytes of the deduplicated pair's row and col passes (mean of the two,
    like pmc_traffic) from the newest profiles/r0*_pmc_ibdedup_traffic.json (tools/gpu_pmc_dedup.sh: the
    C3 shape, B = 65536, D = 128, Zipf(1.05) ids, precision 6), else None."""
    if (B, D, precision) != (65536, 128, 6):
        return None
    rec = None
    for name in ("r05_pmc_ibdedup_traffic.json", "r04_pmc_ibdedup_traffic.json",
                 "r03_pmc_ibdedup_traffic.json"):   # the newest record
        try:
            with open(os.path.join(ROOT, "profiles", name)) as f:
                rec = json.load(f)["ib_dedup"]
            break
        except (OSError, ValueError, KeyError):
            continue
    if rec is None:
        return None
    fe, wr = rec.get("kernels_fetch_KB", {}), rec.get("kernels_write_KB", {})
    ks = [k for k in fe if "inbatch_row_m16_kernel<6" in k or "inbatch_col_m16_kernel<6" in k]
    if len(ks) != 2:
        return None
    return int(sum((2 * fe[k] + wr.get(k, 0.0)) * 1024 for k in ks) / 2)


def pmc_traffic(B, D, stored=False, precision=0):
    """Per-launch HBM-side bytes of the in-batch passes from the committed PMC passes: the round-2
    kernels (profiles/r02_pmc_traffic.json: the stored split pair at B = 65536, D = 128, written by
    round 2's PMC driver, in git history), else profiles/r01_pmc.json, or None for other shapes."""
    r2 = _r02_traffic()
    if r2 and stored and precision == 6 and D == 128 and B == 65536:
        ks = [k for k in r2["ib"] if "inbatch_row_m16_kernel<6" in k or "inbatch_col_m16_kernel<6" in k]
        if len(ks) == 2:
            return int(sum(r2["ib"][k]["traffic_bytes"] for k in ks) / 2)
    key = "inbatch_stored_pair" if stored else "inbatch_pass_kernel"
    if stored and precision in (6, 9) and D == 128:
        key = f"inbatch_stored_pair_split{precision}"
    try:
        with open(os.path.join(ROOT, "profiles", "r01_pmc.json")) as f:
            rec = json.load(f)[key].get(f"B{B}_D{D}")
        return int(rec["traffic_bytes_per_launch_mean"]) if rec else None
    except (OSError, KeyError, ValueError):
        return None


def zipf_ids(rng, n, vocab, a=1.05):
    """Zipf(a) ranks over [1, vocab] (row 0 is the OOV row), permuted so hot rows are scattered."""
    ranks = rng.zipf(a, size=n * 2)
    ranks = ranks[ranks <= vocab][:n]
    while ranks.size < n:
        extra = rng.zipf(a, size=n)
        ranks = np.concatenate([ranks, extra[extra <= vocab]])[:n]
    perm_mult = 2654435761 % vocab or 1
    return ((ranks.astype(np.int64) * perm_mult) % vocab) + 1


class LaunchTimer:
    """Brackets every call of the given functional.* entry points with HIP events on the launch
    stream (the current torch stream, which is the stream our kernels are launched on).
    `sizes` (optional) maps an entry point name to f(args) -> a per-call size kept in .sizes.
    pre_roll_us: before the start event, a GPU spin of about that long (torch.cuda._sleep), so that
    the host's Python and launch work for the call overlaps the spin instead of sitting between the
    start event and the kernel: on an eager step whose queue has drained, the bracket then holds
    the kernels alone (the 25-30 us gather measured 60 us without it, rocprofv3 26 us)."""

    def __init__(self, names, sizes=None, pre_roll_us=0):
        self.names = names
        self.size_fns = sizes or {}
        self.pairs = []
        self.names_of = []   # the entry point of each pair
        self.sizes = []
        self.active = False
        self._orig = {}
        self.pre_roll_cycles = int(pre_roll_us * 2400)   # cycles at <= 2.4 GHz

    def install(self):
        timer = self
        for name in self.names:
            fn = getattr(F, name)
            self._orig[name] = fn
            size_fn = self.size_fns.get(name)

            def wrapped(*a, __fn=fn, __size=size_fn, __name=name, **k):
                if not timer.active:
                    return __fn(*a, **k)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                if timer.pre_roll_cycles and not torch.cuda.is_current_stream_capturing():
                    torch.cuda._sleep(timer.pre_roll_cycles)
                s.record()
                out = __fn(*a, **k)
                e.record()
                timer.pairs.append((s, e))
                timer.names_of.append(__name)
                if __size is not None:
                    timer.sizes.append(__size(*a, **k))
                return out

            setattr(F, name, wrapped)

    def uninstall(self):
        for name, fn in self._orig.items():
            setattr(F, name, fn)
        self._orig = {}

    def mean_ms(self):
        if not self.pairs:
            return float("nan")
        return float(np.mean([s.elapsed_time(e) for s, e in self.pairs]))

    def total_ms(self):
        return float(np.sum([s.elapsed_time(e) for s, e in self.pairs])) if self.pairs else float("nan")

    def per_entry_ms(self):
        """{entry point: mean launch ms} (e.g. the in-batch forward = row pass, backward = col pass)."""
        out = {}
        for n, (s, e) in zip(self.names_of, self.pairs):
            out.setdefault(n, []).append(s.elapsed_time(e))
        return {n: round(float(np.mean(v)), 4) for n, v in out.items()}


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def gather_bytes(n, D):
    """Algorithmic HBM bytes of one embedding gather of n rows: read the row,
    write the row, read the int64 id."""
    return n * (2 * D * 4 + 8)


def gather_roofline(pairs, nbytes):
    """{achieved GB/s, frac of 8 TB/s, avg launch ms} over HIP-event-timed gathers moving
    `nbytes[i]` algorithmic bytes each."""
    if not pairs:
        return None
    ms = [s.elapsed_time(e) for s, e in pairs]
    byts = float(sum(nbytes))
    gbs = byts / (sum(ms) * 1e-3) / 1e9
    return {"achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
            "avg_launch_ms": round(float(np.mean(ms)), 5), "bytes_per_launch": int(byts / len(ms)), "launches": len(ms)}


def uniform_gather_roofline(tables, B, D, dev, reps=20):
    """The same gather launch (all tables at once) with uniform ids (SURVEY §8d C3 asks for Zipf
    and uniform), a fresh id batch per launch, timed with HIP events on the launch stream after
    the timed region. The launches are captured in one hipGraph and its replay is bracketed by
    HIP events, so no host enqueue gap enters the time (the graph's own launch gaps do: the
    per-launch figure is an upper bound)."""
    g = torch.Generator(device=dev)
    g.manual_seed(99)
    batches = [[torch.randint(1, w.shape[0], (B,), device=dev, generator=g) for w in tables] for _ in range(reps)]
    F.embedding_gather_tables(tables, batches[0])           # warm
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for ids in batches:
            F.embedding_gather_tables(tables, ids)
    graph.replay()                                          # warm replay
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    graph.replay()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / reps
    byts = gather_bytes(B, D) * len(tables)
    gbs = byts / (ms * 1e-3) / 1e9
    return {"achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
            "avg_launch_ms": round(ms, 5), "bytes_per_launch": int(byts), "launches": reps,
            "timing": "one hipGraph replay of the launches (fresh uniform ids each) between two HIP events"}


def cpu_baseline(conf, seconds=15.0):
    """The oracle's numpy fp32 train step on a bounded sample of the same workload: same table
    shapes and model, batch 4096 (SURVEY §8d / BASELINE.md scaled CPU batch)."""
    O = importlib.import_module("oracle.recsys_oracle")
    try:
        from threadpoolctl import threadpool_info
        cores = max([i.get("num_threads", 1) for i in threadpool_info()] or [1])
    except Exception:  # pragma: no cover
        cores = os.cpu_count() or 1
    B = min(conf["B"], 4096)
    ocfg = O.OracleConfig(embedding_dim=conf["D"], cross_layers=conf["cross"])
    rng = np.random.default_rng(7)
    P = {}
    for name, shp in O.param_shapes(ocfg, conf["users"] + 1, conf["items"] + 1).items():
        if name.endswith("embedding.weight"):
            P[name] = np.full(shp, 0.01, dtype=np.float32)       # content irrelevant for timing
        else:
            P[name] = (rng.standard_normal(shp) * 0.05).astype(np.float32)
    A = {k: np.full_like(v, 0.1) for k, v in P.items()}
    uid = zipf_ids(rng, B, conf["users"])
    iid = zipf_ids(rng, B, conf["items"])
    rating = rng.integers(1, 6, B).astype(np.float32)
    yi = (rating >= 4).astype(np.float32)
    cw = {0: 1.0, 1: 1.0}
    O.train_step(P, A, ocfg, 0, uid, iid, rating, yi, cw)  # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        O.train_step(P, A, ocfg, n + 1, uid, iid, rating, yi, cw)
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds or n >= 50:
            break
    return {"value": round(B * n / el, 2), "unit": "ranked pairs/s", "cores": int(cores), "kind": "port",
            "cpu": cpu_model(),
            "sample": f"{n} numpy-fp32 oracle train steps at batch {B} on the full "
                      f"{conf['users']}x{conf['items']} tables ({el:.1f} s)"}


def setup_two_tower(conf, dev, rank, is_dist, precision=6, padded=False, exchange=None):
    """BASELINE configs 2/3: the reference MultiTaskModel training step. exchange ("dedupe" /
    "padded", one GPU): the data-parallel exchange forced on in a one-rank RCCL group (the N-
    independent costs of the DP step: local dedupe, the host read, the collectives' launch)."""
    B, D = conf["B"], conf["D"]
    cfg = cfgmod.ModelConfig(embedding_dim=D, cross_layers=conf["cross"], batch_size=B,
                             contraction_precision=precision)
    torch.manual_seed(0)
    model = models.MultiTaskModel(cfg, conf["users"], conf["items"], {}, class_weights={0: 1.6, 1: 0.73},
                                  device=dev)
    opt = optim.Adagrad(model.dense_parameters(), model.embedding_modules(),
                        optim.ExponentialDecay(cfg.learning_rate_retrieval, 1000, 0.96, True), clipnorm=1.0,
                        defer_reductions=not is_dist)
    if is_dist or exchange:   # padded: the sync-free exchange (graph-capturable); default: deduplicated, one host read
        padded = padded or exchange == "padded"
        opt.pre_apply_hooks.append(distributed.MirroredGradientExchange(
            max_rows=B, dense_params=opt.dense, sparse="padded" if padded else None, embeddings=opt.embeddings,
            force=bool(exchange)))
    rng = np.random.default_rng(1234 + rank)          # each rank: its share of the global batch
    # Zipf(1.05) ids (default) and uniform ids (RS_BENCH_IDS=uniform: the main line on
    # uniform ids, a timing switch for A/Bs of the uniform-id step)
    uniform = conf.get("ids", os.environ.get("RS_BENCH_IDS", "zipf")) == "uniform"

    def ids(vocab):
        return rng.integers(1, vocab + 1, B).astype(np.int64) if uniform else zipf_ids(rng, B, vocab)
    batches = []
    for _ in range(4):
        uid = torch.from_numpy(ids(conf["users"])).to(dev)
        iid = torch.from_numpy(ids(conf["items"])).to(dev)
        rating = torch.from_numpy(rng.integers(1, 6, B).astype(np.float32)).to(dev)
        batches.append(graphs.pack_batch(({"user_id": uid, "movie_id": iid},
                                          {"rating": rating, "y_implicit": (rating >= 4).float()})))

    def train_step(batch):
        opt.zero_grad()
        # loss + sum(model.losses) from the loss node itself (no add launch)
        loss, total, _ = model.compute_loss(batch, with_regularization=True)
        total.backward(F.backward_seed(total))                    # (no ones_like fill launch)
        opt.step()
        return loss.detach()

    # the forward keeps the B x B scores when they fit F.INBATCH_STORE_SCORES_MAX_BYTES, and the
    # backward then only does P^T.U (2 B^2 D) instead of recomputing S (4 B^2 D)
    stored = F._native.query("rs_inbatch_scores_bytes", B) <= F.INBATCH_STORE_SCORES_MAX_BYTES
    split = stored and D == 128 and precision in (6, 9)
    if split:
        kernel = (f"inbatch_row_m16_kernel<{precision}> (rs_inbatch_softmax_xent_fwd_store_prec: S = U C^T, online "
                  f"softmax, P.C, S kept) + inbatch_col_m16_kernel<{precision}> "
                  "(rs_inbatch_softmax_xent_bwd_stored_prec: P^T.U from the kept S); fp32 operands as exact "
                  f"3-term bf16 splits, {precision} v_mfma_f32_16x16x32_bf16 products per fp32 product")
    elif stored:
        kernel = ("inbatch_pass_kernel<D,1> (rs_inbatch_softmax_xent_fwd_store: S = U C^T, online softmax, "
                  "P.C, S kept) + inbatch_col_stored_kernel (rs_inbatch_softmax_xent_bwd_stored: P^T.U "
                  "from the kept S)")
    else:
        kernel = "inbatch_pass_kernel (rs_inbatch_softmax_xent_fwd/bwd): S = U C^T + P.V per pass"

    def set_precision(prec):
        models.set_contraction_precision(model, prec)

    def _scaled(v, f):
        return (lambda: f * v()) if callable(v) else f * v

    # algorithmic FLOPs of each timed call: the full pair does B x B pairs, the deduplicated pair
    # (functional.inbatch_dedup_plan) Bu x Bc distinct users x distinct items; the executed pairs
    # of the forwards are kept for the dots_computed figure
    pairs_done = []

    def _pairs(users, items, n):
        if users is not None and users[3] is None:   # a device-count plan: read after the timing
            info = users[4]
            return lambda: int(info[0]) * int(info[2])
        return (users[3] if users is not None else n) * (items[3] if items is not None else n)

    def _fwd_dedup_flops(U, C, users, items, *a, **k):
        pairs_done.append(_pairs(users, items, U.shape[0]))
        pd, D_ = pairs_done[-1], U.shape[1]
        return (lambda: 4.0 * pd() * D_) if callable(pd) else 4.0 * pd * D_

    def _fwd_flops(U, C, *a, **k):
        pairs_done.append(U.shape[0] ** 2)
        return 4.0 * U.shape[0] ** 2 * U.shape[1]
    timed_flops = {
        "inbatch_softmax_fwd": _fwd_flops,
        "inbatch_softmax_bwd": lambda U, C, *a, **k: (2.0 if k.get("scores") is not None else 4.0) * U.shape[0] ** 2
        * U.shape[1],
        "inbatch_softmax_fwd_dedup": _fwd_dedup_flops,
        "inbatch_softmax_bwd_dedup": lambda U, lse, users, items, *a, **k: _scaled(
            _pairs(users, items, U.shape[0]), 2.0 * U.shape[1]),
    }

    def extra(el, world, steps):
        # dots_per_sec = the user x item dots the step actually evaluates (the deduplicated pair:
        # distinct users x distinct items); the B^2 figure is an equivalence (the reference's full
        # matrix, whose repeated rows this build scores once), reported beside it, not as throughput
        eq = round(B * B * world * steps / el, 1)
        out = {"dots_per_sec": eq, "dots_per_sec_basis": "B^2 user x item dots per step per GPU (full pair ran)",
               "dots_equivalent_per_sec": eq,
               "dots_equivalent_basis": "B^2 user x item dots per step per GPU (the reference's full in-batch "
                                        "matrix); an equivalence, not executed work"}
        if pairs_done:
            pairs_done[:] = [v() if callable(v) else v for v in pairs_done]
            n = len(pairs_done)
            out["dots_per_sec"] = round(sum(pairs_done) / n * world * steps / el, 1)
            out["dots_per_sec_basis"] = "executed (user, item) dots per step per GPU: distinct users x distinct items"
            out["inbatch_pairs_computed_per_step"] = int(sum(pairs_done) / n)
        return out

    return dict(train_step=train_step, batches=batches, timed=list(timed_flops), timed_flops=timed_flops,
                prepass=["inbatch_unique_rows", "inbatch_unique_pair", "inbatch_unique_ids_pair"],
                gather=dict(names=["embedding_gather", "embedding_gather_tables", "embedding_gather_tables_rows",
                                   "embedding_gather_tables_ids"],
                            bytes={"embedding_gather": lambda t, ids, *a, **k: gather_bytes(ids.numel(), t.shape[1]),
                                   "embedding_gather_tables": lambda ts, ids, *a, **k: sum(
                                       gather_bytes(i.numel(), t.shape[1]) for t, i in zip(ts, ids)),
                                   # the distinct-row towers' lookups: the distinct ids only (device
                                   # counts, read after the bracket), + the int32 representative index
                                   "embedding_gather_tables_rows": lambda ts, ids, reps, counts, *a, **k: sum(
                                       gather_bytes(int(c.item()), t.shape[1]) + 4 * int(c.item())
                                       for t, c in zip(ts, counts)),
                                   # straight from the plan's distinct ids (round 6): the rows of the
                                   # ids >= 0 (read after the bracket), each with its int64 id
                                   "embedding_gather_tables_ids": lambda ts, dids, *a, **k: sum(
                                       gather_bytes(int((d >= 0).sum().item()), t.shape[1])
                                       for t, d in zip(ts, dids))},
                            tables=[model.encoder.user_embedding.weight, model.encoder.item_embedding.weight],
                            kernel="gather_tables_wave_kernel (rs_embedding_gather_tables_ids_f32 / _tables_f32: "
                                   "the user and item lookups of a step in one launch; above the fused-stack batch "
                                   "limit over the id plan's distinct ids only, read straight from the plan)",
                            bytes_basis="rows gathered (2 D 4 + 8) per table: row read + row write + int64 id "
                                        "(the distinct-id form: the plan's int64 distinct id)"),
                flops_per_launch=[4.0 * B * B * D, (2.0 if stored else 4.0) * B * B * D],
                kernel=kernel, precision=precision if split else 0, set_precision=set_precision,
                model="MultiTaskModel(two-tower + DCN-v1 cross + deep)",
                config={"users": conf["users"], "items": conf["items"], "embedding_dim": D,
                        "cross_layers": conf["cross"]},
                extra=extra,
                # the committed PMC passes: the full B x B pair (r02), the deduplicated pair at the C3
                # Zipf shape (tools/gpu_pmc_dedup.sh)
                traffic=lambda: (pmc_traffic(B, D, stored, precision)
                                 if all(p == B * B for p in pairs_done)
                                 else dedup_pair_traffic(B, D, precision) if not uniform else None),
                data=("synthetic (uniform ids" if uniform else "synthetic (Zipf(1.05) ids")
                + ", random-init weights of the model architecture)")


def setup_dcn2(conf, dev, rank, is_dist, precision=6):
    """BASELINE config 5 (extension): Criteo-shaped DCN-v2 ranker training step."""
    B, E, L = conf["B"], conf["D"], conf["cross"]
    torch.manual_seed(0)
    model = models.DCNv2Ranker([conf["rows"]] * conf["tables"], embedding_dim=E, num_dense=conf["dense"],
                               cross_layers=L, deep_layers=conf["deep"], device=dev, precision=precision)
    opt = optim.Adagrad(model.dense_parameters(), model.embedding_modules(), 1e-3, clipnorm=1.0,
                        defer_reductions=not is_dist)
    if is_dist:
        opt.pre_apply_hooks.append(distributed.MirroredGradientExchange(max_rows=B, dense_params=opt.dense,
                                                                        embeddings=opt.embeddings))
    rng = np.random.default_rng(4321 + rank)
    batches = []
    for _ in range(2):
        ids = torch.from_numpy(np.stack([zipf_ids(rng, B, conf["rows"]) for _ in range(conf["tables"])])).to(dev)
        dense = torch.from_numpy(rng.standard_normal((B, conf["dense"])).astype(np.float32)).to(dev)
        y = torch.from_numpy((rng.random(B) < 0.25).astype(np.float32)).to(dev)
        batches.append(({"user_id": ids, "dense": dense}, {"y": y}))

    def train_step(batch):
        opt.zero_grad()
        loss = model.compute_loss(batch[0]["user_id"], batch[0]["dense"], batch[1]["y"])
        loss.backward(F.backward_seed(loss))
        opt.step()
        return loss.detach()

    d = model.d
    planes = F.DCN2_PLANES and precision == 6
    kern = ("xgemm_kernel (operands split once into exact 3-term bf16 plane images, streamed by LDS-DMA into a "
            "3-slot ring; two cross products per v_mfma_f32_16x16x32_bf16, 6 bf16 products per fp32 product) + the "
            "image builds, elementwise passes and column sums" if planes else
            (f"gemm_x3_kernel<..., {precision}> (fp32 operands split into 3 bf16 terms at LDS staging)" if precision
             else "gemm_f32_kernel"))
    def mg_bytes(table_ptrs, num_rows, E_, ids, dense, ld, *a, **k):
        Bb = ids.shape[1]
        return ids.numel() * (E_ * 4 + 8) + Bb * ld * 4 + (dense.numel() * 4 if dense is not None else 0)

    return dict(train_step=train_step, batches=batches,
                timed=(["dcn_cross_mat_fwd_planes", "dcn_cross_mat_bwd_planes"] if planes
                       else ["dcn_cross_mat_fwd", "dcn_cross_mat_bwd"]),
                gather=dict(names=["multi_embedding_gather"], bytes={"multi_embedding_gather": mg_bytes}, tables=None,
                            kernel="multi_gather_kernel (rs_multi_embedding_gather_f32)",
                            bytes_basis="26 B (E 4 + 8) rows + ids read, B d 4 x0 written, B 13 4 dense read"),
                flops_per_launch=[2.0 * B * d * d * L, 4.0 * B * d * d * L],
                kernel=f"{kern} in the DCN-v2 cross stack (rs_dcn_cross_mat_fwd/bwd{'_planes' if planes else '_prec'}: "
                       "x W fwd, t W^T and x^T t bwd)", precision=precision,
                set_precision=lambda prec: models.set_contraction_precision(model, prec),
                model=f"DCNv2Ranker({conf['tables']} sparse x {conf['rows']} rows + {conf['dense']} dense, "
                      f"E={E}, d={d}, {L} matrix cross, deep {conf['deep']})",
                config={"tables": conf["tables"], "rows_per_table": conf["rows"], "dense_features": conf["dense"],
                        "embedding_dim": E, "cross_dim": d, "cross_layers": L, "deep": conf["deep"]},
                extra=lambda el, world, steps: {}, traffic=dcn2_traffic(B, L) if planes else None)


def dcn2_traffic(B, L):
    """Mean HBM-side bytes per timed launch (the cross stack's forward call, its backward call):
    half of the measured forward + backward pair at this batch (profiles/r03_pmc_traffic.json,
    d = 3344, L = 4), else the round-2 per-kernel sum (B = 16384)."""
    if L == 4:
        pair = _r03_traffic(f"c5_b{B}")
        if pair:
            return int(pair / 2)
    return dcn2_traffic_r02(B, L)


def dcn2_traffic_r02(B, L):
    """Mean HBM-side bytes per timed launch (the cross stack's forward call, its backward call) from
    profiles/r02_pmc_traffic.json (B = 16384 only): forward = L x (dual image of x_l, W^T image,
    xgemm), backward = L x (dual prep, split-K dW, W image, xgemm dX); per-kernel means."""
    r2 = _r02_traffic()
    if not r2 or B != 16384:
        return None
    t = {}
    for k, v in r2.get("xg", {}).items():
        t[k.replace("void rs::", "").strip()] = v["traffic_bytes"]
    try:
        fwd = L * (t["ximg_dual_kernel<0>"] + t["ximg_kernel<true>"] + t["xgemm_kernel<false, 0>"])
        bwd = L * (t["ximg_dual_kernel<1>"] + t["xgemm_kernel<true, 0>"] + t["ximg_kernel<false>"]
                   + t["xgemm_kernel<false, 0>"])
    except KeyError:
        return None
    return int((fwd + bwd) / 2)


def cpu_baseline_dcn2(conf, seconds=15.0):
    """The oracle's numpy fp32 DCN-v2 ranker step (+ Adagrad) on a bounded sample: batch 1024,
    full-size cross/deep weights, 26 tables of 100k rows (row count only affects the gather)."""
    O = importlib.import_module("oracle.recsys_oracle")
    try:
        from threadpoolctl import threadpool_info
        cores = max([i.get("num_threads", 1) for i in threadpool_info()] or [1])
    except Exception:  # pragma: no cover
        cores = os.cpu_count() or 1
    B, E, L, nf, nd = 1024, conf["D"], conf["cross"], conf["tables"], conf["dense"]
    d = (nf * E + nd + 15) // 16 * 16
    rows = 100_000
    rng = np.random.default_rng(5)
    P = {f"tables.{f}.weight": np.full((rows + 1, E), 0.01, np.float32) for f in range(nf)}
    P["cross_W"] = (rng.standard_normal((L, d, d)) / np.sqrt(d)).astype(np.float32)
    P["cross_b"] = np.zeros((L, d), np.float32)
    prev = d
    for j, u in enumerate(conf["deep"]):
        P[f"deep_nets.{j}.kernel"] = (rng.standard_normal((prev, u)) * 0.02).astype(np.float32)
        P[f"deep_nets.{j}.bias"] = np.zeros(u, np.float32)
        prev = u
    P["ctr_head.kernel"] = (rng.standard_normal((d + prev, 1)) * 0.02).astype(np.float32)
    P["ctr_head.bias"] = np.zeros(1, np.float32)
    A = {k: np.full_like(v, 0.1) for k, v in P.items()}
    ids = np.stack([zipf_ids(rng, B, rows) for _ in range(nf)])
    dense = rng.standard_normal((B, nd)).astype(np.float32)
    y = (rng.random(B) < 0.25).astype(np.float32)
    n, t0 = 0, time.perf_counter()
    while True:
        out = O.dcn2_ranker_loss_and_grads(P, nf, E, d, conf["deep"], ids, dense, y)
        O.adagrad_apply(P, A, out["grads"], n, 1e-3, clipnorm=1.0)
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds or n >= 20:
            break
    return {"value": round(B * n / el, 2), "unit": "ranked pairs/s", "cores": int(cores), "kind": "port",
            "cpu": cpu_model(),
            "sample": f"{n} numpy-fp32 oracle DCN-v2 train steps at batch {B} (d={d}, {L} cross, "
                      f"deep {conf['deep']}; 26 tables of {rows} rows) ({el:.1f} s)"}


def setup_topk(conf, dev, rank, is_dist, precision=6):
    """BASELINE config 4: exact top-k over this rank's 12.5M-row shard of a 100M x 128 item table
    (ShardedBruteForceIndex: local scan + RCCL all-gather of the per-rank top-k + device merge)."""
    retrieval = importlib.import_module(PKG + ".retrieval")
    N, D, Q, k = conf["rows"], conf["D"], conf["Q"], conf["k"]
    g = torch.Generator(device=dev)
    g.manual_seed(1000 + rank)
    items = torch.randn((N, D), device=dev, generator=g)
    g.manual_seed(7)
    queries = torch.randn((Q, D), device=dev, generator=g)
    index = retrieval.ShardedBruteForceIndex(items, row_offset=rank * N, metric="ip", precision=precision)
    del items
    split = precision in (6, 9) and D == 128 and Q > 64

    def set_precision(prec):
        index.local.precision = prec

    def step(_batch):
        s, i = index.search(queries, k)
        return s[0, 0]

    return dict(train_step=step, batches=[None], timed=["topk_ip"], flops_per_launch=[2.0 * Q * N * D],
                kernel=(f"topk_thr_kernel<{precision if split else 0},8 waves,64-row tiles> + topk_select_kernel "
                        "(rs_topk_ip_prec_f32, bound-first: geometric row ranges [0, 2048), [2048, 8192), ... "
                        "(ratio 4), each scanned against the k-th score of the exact list of all earlier ranges "
                        "(-inf for the first), then sorted with that list by a select; scores = items . Q^T)"
                        + (f"; fp32 operands as exact 3-term bf16 splits, {precision} bf16 MFMA products per fp32 "
                           "product" if split else "")),
                precision=precision if split else 0, set_precision=set_precision,
                model=f"ShardedBruteForceIndex(ip, {N} rows x {D} per GPU, top-{k})",
                config={"rows_per_gpu": N, "embedding_dim": D, "queries": Q, "k": k},
                extra=lambda el, world, steps: {"queries_per_sec": round(Q * steps / el, 1)},
                traffic=_r03_traffic("c4") if (Q, N, D, k) == (1024, 12_500_000, 128, 100) else None,
                units=lambda el, world, steps: Q * N * world * steps,
                data="synthetic N(0,1) item rows and queries (seeded per rank), resident in HBM",
                unit="user x item dots/s (exact top-100 search over the whole sharded table)")


def cpu_baseline_topk(conf, seconds=15.0):
    """The oracle's numpy top-k (float64 scores + stable (-score, index) sort) on a bounded
    sample: 16 queries against 1M rows of the same shape."""
    O = importlib.import_module("oracle.recsys_oracle")
    try:
        from threadpoolctl import threadpool_info
        cores = max([i.get("num_threads", 1) for i in threadpool_info()] or [1])
    except Exception:  # pragma: no cover
        cores = os.cpu_count() or 1
    rng = np.random.default_rng(3)
    n, Q = 1_000_000, 16
    items = rng.standard_normal((n, conf["D"])).astype(np.float32)
    q = rng.standard_normal((Q, conf["D"])).astype(np.float32)
    reps, t0 = 0, time.perf_counter()
    while True:
        O.topk_ip(q, items, conf["k"])
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds or reps >= 5:
            break
    return {"value": round(Q * n * reps / el, 1), "unit": "user x item dots/s", "cores": int(cores), "kind": "port",
            "cpu": cpu_model(), "sample": f"{reps} oracle top-{conf['k']} searches of {Q} queries over {n} rows ({el:.1f} s)"}


SETUPS = {"c2": "two_tower", "c3": "two_tower", "c4": "topk", "c5": "dcn2"}
CPU_BASELINES = {"c5": "cpu_baseline_dcn2", "c4": "cpu_baseline_topk"}


def setup(name, conf, dev, rank, is_dist, precision, padded=False, exchange=None):
    if SETUPS[name] == "two_tower":
        return setup_two_tower(conf, dev, rank, is_dist, precision, padded, exchange)
    fn = {"topk": setup_topk, "dcn2": setup_dcn2}[SETUPS[name]]
    return fn(conf, dev, rank, is_dist, precision)


def measure(name, conf, dev, rank, world, is_dist, steps, warmup, *, eager=False, graph=False, f32_compare=True,
            cpu_seconds=15.0, cpu=True, precision=6, exchange=None):
    """Set up one workload, run `warmup` untimed steps, time exactly `steps` steps between a
    barrier + synchronize on both sides (max over ranks), then the roofline (HIP events on the
    launch stream around every measured launch), the gather roofline, the optional f32-MFMA
    comparison and the CPU baseline. Returns (record, wall seconds) — the record on rank 0."""
    if graph and is_dist and name not in ("c2", "c3"):
        raise SystemExit(f"bench.py: --graph with more than one rank is supported for c2 / c3 only")
    # a captured data-parallel step uses the padded exchange (no host read; RCCL collectives captured)
    wl = setup(name, conf, dev, rank, is_dist, precision, padded=graph and is_dist, exchange=exchange)
    if exchange == "dedupe":
        eager = True   # the deduplicating exchange reads its counts on the host: not capturable
    B = conf["B"]
    batches, train_step = wl["batches"], wl["train_step"]
    nb = len(batches)
    # One-GPU c2 / c3 steps are one hipGraph replay each: no host read inside the step (the
    # deduplicated pair's id plan keeps its counts on the device while the stream captures), and
    # no Python between launches (measured at C3: 3.85 ms graphed vs 4.0-4.1 ms eager, the eager
    # step host-bound around the id plan). Data-parallel steps stay eager by default (the
    # deduplicating exchange reads its counts on the host); --graph selects the padded exchange.
    use_graph = (not eager and not is_dist and name in ("c2", "c3")) or graph
    if use_graph and is_dist and dist.get_backend() == "gloo":
        # CPU collectives cannot be captured into a hipGraph (RCCL's can): the gloo rehearsal of
        # the multi-rank path runs eager
        use_graph = False
    runner = graphs.GraphedTrainStep(train_step, batches[0]) if use_graph else train_step

    def step(i):
        return runner(batches[i % nb])

    timer = LaunchTimer(wl["timed"], wl.get("timed_flops"))
    timer.install()
    ptimer = LaunchTimer(wl["prepass"]) if wl.get("prepass") else None
    if ptimer:
        ptimer.install()
    gw = wl.get("gather")
    gtimer = LaunchTimer(gw["names"], gw["bytes"], pre_roll_us=150) if gw else None
    if gtimer:
        gtimer.install()
    try:
        for i in range(warmup):
            step(i)
        torch.cuda.synchronize()
        if is_dist:
            dist.barrier()
        torch.cuda.synchronize()
        timer.active = True
        if ptimer:
            ptimer.active = True
        t0 = time.perf_counter()
        for i in range(steps):
            loss = step(i)
        torch.cuda.synchronize()
        if is_dist:
            dist.barrier()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        timer.active = False
        if ptimer:
            ptimer.active = False
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        if is_dist:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
        last_loss = float(loss.item())
        roofline_timing = "HIP events around every measured launch of the timed steps"
        if use_graph or gtimer:
            # graph replays run no Python: time the same launches in 3 eager steps right after; the
            # gathers are always timed there, each behind a GPU pre-roll (LaunchTimer) that keeps
            # the host's launch work out of their brackets — not inside the timed region
            timer.active = use_graph
            timer.pre_roll_cycles = LaunchTimer([], pre_roll_us=150).pre_roll_cycles   # (outside the timed region)
            if gtimer:
                gtimer.active = True
            for i in range(3):
                train_step(batches[i % nb])
            torch.cuda.synchronize()
            timer.active = False
            if gtimer:
                gtimer.active = False
            if use_graph:
                roofline_timing = ("HIP events around the measured launches of 3 eager steps after the graphed timed "
                               "region, each behind a ~150 us GPU pre-roll (the host's launch work outside the bracket)")
        f32_cmp = None
        if wl.get("precision") and not use_graph and f32_compare:
            # the same steps with the f32-MFMA contraction kernels, for comparison (not the value)
            wl["set_precision"](0)
            for i in range(2):
                train_step(batches[i % nb])
            torch.cuda.synchronize()
            if is_dist:
                dist.barrier()
            n_cmp = min(steps, 20)   # a reported comparison, not the value: a bounded sample
            t1 = time.perf_counter()
            for i in range(n_cmp):
                train_step(batches[i % nb])
            torch.cuda.synchronize()
            if is_dist:
                dist.barrier()
            tt = torch.tensor([(time.perf_counter() - t1) * steps / n_cmp], dtype=torch.float64, device=dev)
            if is_dist:
                dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            f32_cmp = float(tt.item())
            wl["set_precision"](wl["precision"])
        nk = len(wl["timed"])
        n_calls = len(timer.pairs)
        if wl.get("timed_flops"):   # (sizes of device-count calls are read now, after the timing)
            flops = float(sum(v() if callable(v) else v for v in timer.sizes))
        else:
            flops = sum(wl["flops_per_launch"][j % nk] for j in range(n_calls))
        tot_ms = timer.total_ms()
        achieved = flops / (tot_ms * 1e-3) / 1e12 if n_calls and tot_ms == tot_ms else None
        gather_line = None
        if gw:
            # the step's own gathers, keyed by the id law of the timed batches ("in_step"); beside
            # them the same launch on fresh uniform ids as a standalone graph replay
            law = conf.get("ids", os.environ.get("RS_BENCH_IDS", "zipf"))
            gather_line = {"kernel": gw["kernel"], "bound": "hbm", "bytes_basis": gw["bytes_basis"],
                           "in_step": dict(gather_roofline(gtimer.pairs, gtimer.sizes) or {}, ids=law,
                                           timing="HIP events around the step's gather launches in 3 eager steps "
                                                  "after the timed region, each behind a ~150 us GPU pre-roll "
                                                  "(the host's launch work outside the bracket)")}
            if gw.get("tables"):
                gather_line["uniform_standalone"] = uniform_gather_roofline(gw["tables"], B,
                                                                            gw["tables"][0].shape[1], dev)
                if B == 65536 and name == "c3":   # the C3 gather's PMC passes (Zipf and uniform ids)
                    # (committed passes of the full-B lookup of the same id law; the step's own launch
                    # gathers the distinct ids only when the distinct-row towers run)
                    gather_line["in_step"]["traffic_full_b_gather"] = _r03_traffic(f"gather_{law}")
                    gather_line["in_step"]["l2_hit_rate_full_b_gather"] = _r03_traffic(f"gather_{law}",
                                                                                       "l2_hit_rate")
                    gather_line["uniform_standalone"]["traffic"] = _r03_traffic("gather_uniform")
    finally:
        timer.uninstall()
        if gtimer:
            gtimer.uninstall()
        if ptimer:
            ptimer.uninstall()
    if rank != 0:
        return None, el
    peak, peak_basis = contraction_peak(wl.get("precision", 0))
    units = wl["units"](el, world, steps) if "units" in wl else B * world * steps
    rec = {
        "value": round(units / el, 1),
        "unit": wl.get("unit", "ranked pairs/s (full train step: fwd+bwd+Adagrad)"),
        "ms_per_step": round(el / steps * 1e3, 3),
        "steps": steps,
        "warmup": warmup,
        "data": wl.get("data", "synthetic (Zipf(1.05) ids, random-init weights of the model architecture)"),
        "config": dict(workload=conf["workload"], model=wl["model"], global_batch=B * world, per_gpu_batch=B,
                       parallelism=f"dp{world}", hipgraph=use_graph, **wl["config"],
                       **({"exchange_rehearsal": f"{exchange} exchange forced on in a one-rank RCCL group"}
                          if exchange else {})),
        **wl["extra"](el, world, steps),
        "loss": last_loss,
        "roofline": {"kernel": wl["kernel"], "bound": "mfma",
                     "achieved": round(achieved, 2) if achieved else None, "peak": peak,
                     "unit": "TFLOP/s", "frac": round(achieved / peak, 4) if achieved else None,
                     "traffic": wl["traffic"]() if callable(wl["traffic"]) else wl["traffic"],
                     "avg_launch_ms": round(timer.mean_ms(), 4), "per_entry_ms": timer.per_entry_ms(),
                     "flop_per_launch": (round(flops / n_calls) if wl.get("timed_flops") and n_calls
                                         else wl["flops_per_launch"]), "peak_basis": peak_basis,
                     "timing": roofline_timing},
    }
    if wl.get("roofline_note"):
        rec["roofline"]["note"] = wl["roofline_note"]
    if ptimer is not None and ptimer.pairs:
        # the deduplicated pair's pre-pass (distinct rows by content: hash, sort, verify), outside
        # the roofline's launches; the plan's one host read of the two counts is in ms_per_step
        rec["roofline"]["dedup_prepass_ms_per_step"] = round(ptimer.total_ms() / steps, 4)
    if gather_line:
        rec["roofline"]["gather"] = gather_line
    if wl.get("precision"):
        rec["precision"] = (f"fp32 operands and fp32 accumulation; GEMM-shaped contractions (in-batch softmax, "
                            f"Dense layers, DCN-v2 cross, top-K scan) on the bf16 MFMA with every fp32 operand split "
                            f"exactly into 3 bf16 terms, {wl['precision']} cross products per fp32 product "
                            "(ModelConfig.contraction_precision; 0 = f32 MFMA)")
        if f32_cmp is not None:
            cmp_units = wl["units"](f32_cmp, world, steps) if "units" in wl else B * world * steps
            rec["f32_mfma_compare"] = {"ms_per_step": round(f32_cmp / steps * 1e3, 3),
                                       "value": round(cmp_units / f32_cmp, 1),
                                       "note": "same steps with contraction_precision=0 (f32 MFMA), after the "
                                               "timed region"}
    del wl, batches, train_step, runner
    if cpu and world == 1:
        rec["cpu_baseline"] = globals()[CPU_BASELINES.get(name, "cpu_baseline")](conf, cpu_seconds)
    return rec, el


def free_device_memory():
    import gc
    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100, help="timed steps (default 100: a timed region of ~1.7 s at c3, long enough for an external utilisation sampler)")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="c3")
    ap.add_argument("--batch", type=int, default=0, help="override per-GPU batch")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--eager", action="store_true", help="do not capture the step in a hipGraph")
    ap.add_argument("--graph", action="store_true",
                    help="force hipGraph capture of the step (with more than one rank: the padded exchange)")
    ap.add_argument("-o", "--out", default=None, help="also write the JSON line to this file")
    ap.add_argument("--precision", type=int, choices=(0, 6, 9), default=6,
                    help="in-batch contraction precision (ModelConfig.contraction_precision)")
    ap.add_argument("--no-f32-compare", action="store_true",
                    help="skip the extra timed steps at precision 0 reported beside the value")
    ap.add_argument("--exchange", choices=("dedupe", "padded"), default=None,
                    help="one GPU: run the data-parallel exchange anyway in a one-rank RCCL group (the DP step's "
                         "N-independent costs; dedupe runs eager, padded captured)")
    ap.add_argument("--extras", choices=("auto", "on", "off"), default="auto",
                    help="also time configs 5 (B = 16384 and 65536) and 4 as sub-records of the c3 line "
                         "(auto: on one GPU only)")
    args = ap.parse_args()

    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # one process per GPU: this parent touches no GPU; it starts the N rank processes under
        # torch.distributed.run (RCCL rendezvous on 127.0.0.1) and exits with their status
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
        sys.exit(subprocess.call(cmd))
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world_env}: refusing to report a mislabelled "
              "measurement", file=sys.stderr)
        sys.exit(2)

    is_dist = distributed.init_process_group("nccl")
    rank = dist.get_rank() if is_dist else 0
    world = dist.get_world_size() if is_dist else 1
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if args.exchange and world == 1 and not dist.is_initialized():
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                device_id=dev)

    conf = dict(CONFIGS[args.config])
    if args.batch:
        conf["B"] = args.batch
    rec, _ = measure(args.config, conf, dev, rank, world, is_dist, args.steps, args.warmup, eager=args.eager,
                     graph=args.graph, f32_compare=not args.no_f32_compare, cpu_seconds=args.cpu_seconds,
                     cpu=not args.no_cpu_baseline, precision=args.precision, exchange=args.exchange)
    extras = {}
    if args.config == "c3" and not args.exchange and (args.extras == "on" or (args.extras == "auto" and world == 1)):
        # configs 5 and 4 ride along as sub-records (the driver's one command times all three)
        cpu_s = min(args.cpu_seconds, 8.0)
        for key, cname, over, steps, warm in (("c3_uniform_ids", "c3", {"ids": "uniform"}, 10, 3),
                                              ("c5", "c5", {}, 10, 3), ("c5_b65536", "c5", {"B": 65536}, 3, 1),
                                              ("c4", "c4", {}, 10, 2)):
            free_device_memory()
            c = dict(CONFIGS[cname], **over)
            t0 = time.perf_counter()
            r, _ = measure(cname, c, dev, rank, world, is_dist, steps, warm, f32_compare=False, cpu_seconds=cpu_s,
                           cpu=not args.no_cpu_baseline and key not in ("c5_b65536", "c3_uniform_ids"),
                           precision=args.precision)
            if r is not None:
                r["wall_s"] = round(time.perf_counter() - t0, 1)
                extras[key] = r
    if rank == 0:
        out = {"metric": "ranked pairs/sec (DCN fwd) + user×item dots/sec (retrieval), 1/2/4/8 MI355X",
               "value": rec.pop("value"), "unit": rec.pop("unit"), "n_gpus": world, "steps": rec.pop("steps"),
               "warmup": rec.pop("warmup"), "ms_per_step": rec.pop("ms_per_step"), "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": "f32", **rec}
        if extras:
            out["extra"] = extras
        line = json.dumps(out)
        print(line, flush=True)
        if args.out:
            with open(args.out, "w") as f:
                f.write(line + "\n")
    if is_dist:
        dist.barrier()
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
