"""A/B of the sparse Adagrad update: time + bitwise comparison between two library builds
(RECSYS_HIP_LIB_A / _B) on Zipf ids. Usage: python tools/ab_sparse.py"""
import ctypes
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda")
res = {}
for tag in ("A", "B"):
    lib = ctypes.CDLL(os.environ[f"RECSYS_HIP_LIB_{tag}"])
    for name, V, n in (("c2-items", 3706, 4096), ("c3-users", 10_000_000, 65536), ("dp8-users", 10_000_000, 524288)):
        rng = np.random.default_rng(0)
        ids = torch.from_numpy(bench.zipf_ids(rng, n, V)).to(dev)
        rows = torch.from_numpy(rng.standard_normal((n, 128)).astype(np.float32)).to(dev)
        T = torch.ones((V + 1, 128), device=dev)
        A = torch.full((V + 1, 128), 0.1, device=dev)
        it = torch.zeros((), dtype=torch.int64, device=dev)
        wsb = lib.rs_sparse_adagrad_workspace_bytes
        wsb.restype = ctypes.c_size_t
        nb = wsb(ctypes.c_int64(n), ctypes.c_int64(128), ctypes.c_int64(V + 1))
        ws = torch.empty(max(nb, 256), dtype=torch.uint8, device=dev)
        P = ctypes.c_void_p

        def step():
            rc = lib.rs_sparse_adagrad_ld_f32(P(T.data_ptr()), P(A.data_ptr()), ctypes.c_int64(V + 1),
                                              ctypes.c_int64(128), P(ids.data_ptr()), P(rows.data_ptr()),
                                              ctypes.c_int64(128), ctypes.c_int64(n), P(it.data_ptr()),
                                              ctypes.c_float(0.1), ctypes.c_float(0.96), ctypes.c_int64(1000),
                                              ctypes.c_float(1.0), ctypes.c_float(1e-7), P(ws.data_ptr()),
                                              ctypes.c_size_t(ws.numel()),
                                              P(torch.cuda.current_stream().cuda_stream))
            assert rc == 0
        step()
        torch.cuda.synchronize()
        first = (T[ids[:4096]].clone(), A[ids[:4096]].clone())
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            step()
        e.record()
        torch.cuda.synchronize()
        res[(tag, name)] = (s.elapsed_time(e) / 10, first)
for name in ("c2-items", "c3-users", "dp8-users"):
    ta, fa = res[("A", name)]
    tb, fb = res[("B", name)]
    same = torch.equal(fa[0], fb[0]) and torch.equal(fa[1], fb[1])
    print(f"{name:10s} A {ta * 1e3:8.1f} us  B {tb * 1e3:8.1f} us  bitwise-equal after 1 step: {same}")
