#!/usr/bin/env python3
"""Benchmark: the reference's training step (MultiTaskModel two-tower retrieval + DCN ranking,
forward + backward + Adagrad) on the MI355X HIP path.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2] [--no-cpu-baseline]
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
HBM_PEAK_GBS = 8000.0

CONFIGS = {
    "c3": dict(workload="synthetic-10Mx1M-two-tower+dcn-train-step", users=10_000_000, items=1_000_000,
               D=128, B=65536, cross=3),
    "c2": dict(workload="movielens1m-shaped-dcn-ranker-train-step", users=6040, items=3706, D=128, B=4096,
               cross=3),
}


def pmc_traffic(B, D):
    """Per-launch HBM-side bytes of the in-batch passes from the committed PMC passes
    (profiles/r01_pmc.json, collected with tools/gpu_pmc.sh), or None for other shapes."""
    try:
        with open(os.path.join(ROOT, "profiles", "r01_pmc.json")) as f:
            rec = json.load(f)["inbatch_pass_kernel"].get(f"B{B}_D{D}")
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


class InbatchTimer:
    """Brackets every in-batch softmax pass with HIP events on the launch stream."""

    def __init__(self):
        self.pairs = []
        self.active = False

    def install(self):
        timer = self
        fwd, bwd = F.inbatch_softmax_fwd, F.inbatch_softmax_bwd

        def fwd_t(*a, **k):
            if not timer.active:
                return fwd(*a, **k)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            out = fwd(*a, **k)
            e.record()
            timer.pairs.append((s, e))
            return out

        def bwd_t(*a, **k):
            if not timer.active:
                return bwd(*a, **k)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            out = bwd(*a, **k)
            e.record()
            timer.pairs.append((s, e))
            return out

        F.inbatch_softmax_fwd, F.inbatch_softmax_bwd = fwd_t, bwd_t

    def mean_ms(self):
        if not self.pairs:
            return float("nan")
        return float(np.mean([s.elapsed_time(e) for s, e in self.pairs]))


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
            "sample": f"{n} numpy-fp32 oracle train steps at batch {B} on the full "
                      f"{conf['users']}x{conf['items']} tables ({el:.1f} s)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="c3")
    ap.add_argument("--batch", type=int, default=0, help="override per-GPU batch")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--eager", action="store_true", help="do not capture the step in a hipGraph")
    ap.add_argument("--graph", action="store_true", help="force hipGraph capture of the step")
    ap.add_argument("-o", "--out", default=None, help="also write the JSON line to this file")
    args = ap.parse_args()

    is_dist = distributed.init_process_group("nccl")
    rank = dist.get_rank() if is_dist else 0
    world = dist.get_world_size() if is_dist else 1
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    conf = dict(CONFIGS[args.config])
    if args.batch:
        conf["B"] = args.batch
    B, D = conf["B"], conf["D"]
    cfg = cfgmod.ModelConfig(embedding_dim=D, cross_layers=conf["cross"], batch_size=B)
    torch.manual_seed(0)
    model = models.MultiTaskModel(cfg, conf["users"], conf["items"], {}, class_weights={0: 1.6, 1: 0.73},
                                  device=dev)
    opt = optim.Adagrad(model.dense_parameters(), model.embedding_modules(),
                        optim.ExponentialDecay(cfg.learning_rate_retrieval, 1000, 0.96, True), clipnorm=1.0)
    if is_dist:
        opt.pre_apply_hooks.append(distributed.MirroredGradientExchange())

    # synthetic batches resident in HBM (different per rank: the global batch is split)
    rng = np.random.default_rng(1234 + rank)
    nb = 4
    batches = []
    for _ in range(nb):
        uid = torch.from_numpy(zipf_ids(rng, B, conf["users"])).to(dev)
        iid = torch.from_numpy(zipf_ids(rng, B, conf["items"])).to(dev)
        rating = torch.from_numpy(rng.integers(1, 6, B).astype(np.float32)).to(dev)
        yi = (rating >= 4).float()
        batches.append(({"user_id": uid, "movie_id": iid}, {"rating": rating, "y_implicit": yi}))

    def train_step(batch):
        opt.zero_grad()
        loss = model.compute_loss(batch)
        total = loss + sum(model.losses)
        total.backward()
        opt.step()
        return loss.detach()

    # Small batches are launch-bound: the whole step becomes one hipGraph replay. Large batches
    # (C3) are GPU-bound, so they run eagerly and the in-batch launches are bracketed with HIP
    # events inside the timed region itself. Data-parallel runs keep the RCCL exchange eager.
    use_graph = (not args.eager and not is_dist and B <= 16384) or args.graph
    runner = graphs.GraphedTrainStep(train_step, batches[0]) if use_graph else train_step

    def step(i):
        return runner(batches[i % nb])

    timer = InbatchTimer()
    timer.install()
    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    if is_dist:
        dist.barrier()
    torch.cuda.synchronize()
    timer.active = True
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = step(i)
    torch.cuda.synchronize()
    if is_dist:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    timer.active = False
    t = torch.tensor([el], dtype=torch.float64, device=dev)
    if is_dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())
    last_loss = float(loss.item())
    ib_ms = timer.mean_ms()
    roofline_timing = "HIP events around every in-batch launch of the timed steps"
    if use_graph:
        # graph replays run no Python: time the same launches in 3 eager steps right after
        timer.active = True
        for i in range(3):
            train_step(batches[i % nb])
        torch.cuda.synchronize()
        timer.active = False
        ib_ms = timer.mean_ms()
        roofline_timing = "HIP events around the in-batch launches of 3 eager steps after the graphed timed region"

    if rank != 0:
        if is_dist:
            dist.barrier()
            dist.destroy_process_group()
        return
    pairs = B * world * args.steps
    ms_step = el / args.steps * 1e3
    ib_flops = 4.0 * B * B * D            # S = U C^T and P.V products (2 x 2 B^2 D) per pass
    ib_tf = ib_flops / (ib_ms * 1e-3) / 1e12 if ib_ms == ib_ms else None
    out = {
        "metric": "ranked pairs/sec (DCN fwd) + user×item dots/sec (retrieval), 1/2/4/8 MI355X",
        "value": round(pairs / el, 1),
        "unit": "ranked pairs/s (full train step: fwd+bwd+Adagrad)",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (Zipf(1.05) ids, random-init weights of the reference architecture)",
        "config": {"workload": conf["workload"], "model": "MultiTaskModel(two-tower + DCN-v1 cross + deep)",
                   "users": conf["users"], "items": conf["items"], "embedding_dim": D,
                   "cross_layers": conf["cross"], "global_batch": B * world, "per_gpu_batch": B,
                   "parallelism": f"dp{world}", "hipgraph": use_graph},
        "dots_per_sec": round(B * B * world * args.steps / el, 1),
        "loss": last_loss,
        "roofline": {"kernel": "inbatch_pass_kernel (rs_inbatch_softmax_xent_fwd/bwd)", "bound": "mfma",
                     "achieved": round(ib_tf, 2) if ib_tf else None, "peak": FP32_MFMA_PEAK_TFLOPS,
                     "unit": "TFLOP/s", "frac": round(ib_tf / FP32_MFMA_PEAK_TFLOPS, 4) if ib_tf else None,
                     "traffic": pmc_traffic(B, D), "avg_launch_ms": round(ib_ms, 4),
                     "flop_per_launch": ib_flops, "timing": roofline_timing},
    }
    if not args.no_cpu_baseline and world == 1:
        out["cpu_baseline"] = cpu_baseline(conf, args.cpu_seconds)
    line = json.dumps(out)
    print(line, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")
    if is_dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
