"""Interleaved in-process A/B of gather variants (tools/gather_variants.hip) on the C3 user
table (10M x 128 fp32). Usage: python tools/ab_gather.py  (builds tools/_gather_variants.so)"""
import ctypes
import os
import subprocess
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
so = os.path.join(HERE, "_gather_variants.so")
if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(os.path.join(HERE, "gather_variants.hip")):
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared",
                    os.path.join(HERE, "gather_variants.hip"), "-o", so], check=True)
lib = ctypes.CDLL(so)
lib.gather_variant.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                               ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
import bench  # noqa: E402

V, D = 10_000_000, 128
dev = torch.device("cuda")
table = torch.empty((V + 1, D), dtype=torch.float32, device=dev).uniform_(-0.05, 0.05)
rng = np.random.default_rng(0)
names = ["rif4-nt", "rif8-nt", "rif8-nt-ntstore", "rif8-plain", "rif16-nt", "rows8", "rows16", "q32-rif4",
         "q32-rif8", "wave-b8", "wave-b16", "wave-b32", "wr16", "wr32", "wr64"]
for n in (65536, 1 << 20, 4 << 20):
    ids = torch.from_numpy(bench.zipf_ids(rng, n, V)).to(dev)
    out = torch.empty((n, D), device=dev)
    ref = table[ids]
    res = {}
    for blocks in (256, 512, 1024, 2048, 4096):
        for w in range(len(names)):
            out.zero_()
            assert lib.gather_variant(w, table.data_ptr(), D, ids.data_ptr(), n, out.data_ptr(), blocks,
                                      torch.cuda.current_stream().cuda_stream) == 0
            torch.cuda.synchronize()
            assert torch.equal(out, ref), names[w]
    for rnd in range(5):
        for blocks in (256, 512, 1024, 2048, 4096):
            for w in range(len(names)):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(10):
                    lib.gather_variant(w, table.data_ptr(), D, ids.data_ptr(), n, out.data_ptr(), blocks,
                                       torch.cuda.current_stream().cuda_stream)
                e.record()
                torch.cuda.synchronize()
                res.setdefault((w, blocks), []).append(s.elapsed_time(e) / 10)
    for (w, blocks), ts in sorted(res.items(), key=lambda kv: np.median(kv[1]))[:8]:
        ms = float(np.median(ts))
        print(f"n={n:>8} {names[w]:16s} blocks={blocks:5d}: {ms*1e3:7.1f} us  "
              f"{n * (2 * D * 4 + 8) / (ms * 1e-3) / 1e9:6.0f} GB/s (min {min(ts)*1e3:.1f} us)")
