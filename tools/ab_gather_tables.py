"""Interleaved in-process A/B of the two-table gather variants (tools/gather_tables_variants.hip)
on the C3 tables (user 10M x 128 + item 1M x 128, B = 65536 each), Zipf(1.05) and uniform ids,
a fresh id batch per launch (no reuse of the previous launch's rows). Build the .so on the CPU
first: hipcc --offload-arch=gfx950 -O3 -fPIC -shared tools/gather_tables_variants.hip -o
tools/_gather_tables_variants.so. Algorithmic bytes = 2 B (2 D 4 + 8)."""
import ctypes
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import bench  # noqa: E402

lib = ctypes.CDLL(os.path.join(HERE, "_gather_tables_variants.so"))
lib.gather_tables_variant.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 3 + [ctypes.c_int64] + \
    [ctypes.c_void_p] * 3 + [ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
names = ["ntl-64 (product)", "plain-64", "ntl-nts-64", "nts-64", "ntl-32", "nts-32", "ntl-128", "nts-128", "nts-16"]
D, B, R = 128, 65536, 8
dev = torch.device("cuda")
tabs = [torch.empty((n + 1, D), dtype=torch.float32, device=dev).uniform_(-0.05, 0.05) for n in (10_000_000, 1_000_000)]
outs = [torch.empty((B, D), device=dev) for _ in tabs]
rng = np.random.default_rng(1234)
nbytes = 2 * B * (2 * D * 4 + 8)
st = torch.cuda.current_stream().cuda_stream
caps = (2048, 4096, 8192, 0)
for dist in ("zipf", "uniform"):
    batches = []
    for _ in range(R):
        ids = []
        for t in tabs:
            v = t.shape[0] - 1
            x = bench.zipf_ids(rng, B, v) if dist == "zipf" else rng.integers(1, v + 1, B)
            ids.append(torch.from_numpy(x).to(dev))
        batches.append(ids)
    refs = [t[i] for t, i in zip(tabs, batches[0])]

    def run(w, cap, ids):
        return lib.gather_tables_variant(w, tabs[0].data_ptr(), ids[0].data_ptr(), outs[0].data_ptr(), B,
                                         tabs[1].data_ptr(), ids[1].data_ptr(), outs[1].data_ptr(), B, cap, st)
    for w in range(len(names)):
        for cap in caps:
            for o in outs:
                o.zero_()
            assert run(w, cap, batches[0]) == 0
            torch.cuda.synchronize()
            assert all(torch.equal(o, r) for o, r in zip(outs, refs)), (names[w], cap)
    res = {}
    combos = [(w, c) for w in range(len(names)) for c in caps]
    for rnd in range(4):
        order = rng.permutation(len(combos))
        for ci in order:
            w, cap = combos[ci]
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(R)]
            for (s, e), ids in zip(ev, batches):
                s.record()
                run(w, cap, ids)
                e.record()
            torch.cuda.synchronize()
            res.setdefault((w, cap), []).extend(s.elapsed_time(e) for s, e in ev)
    for (w, cap), ts in sorted(res.items(), key=lambda kv: np.median(kv[1])):
        ms = float(np.median(ts))
        print(f"{dist:8s} {names[w]:18s} cap={cap:5d}: median {ms*1e3:6.1f} us  min {min(ts)*1e3:6.1f} us  "
              f"{nbytes / (ms * 1e-3) / 1e9:6.0f} GB/s ({nbytes / (ms * 1e-3) / 8e12:.1%})", flush=True)
