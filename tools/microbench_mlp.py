"""The one-launch Dense stack kernels (rs_mlp_fwd / rs_mlp_bwd_chain / rs_mlp_wgrad) at C2's tower
shapes (2 stacks, 4096 rows, widths 128-256-128-64-128): 50 launches each, HIP-event averages."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import importlib  # noqa: E402

F = importlib.import_module("recommendation-system-maang-nvidia-_amd.functional")


def main():
    dev = torch.device("cuda:0")
    M = int(os.environ.get("MB_M", "4096"))
    dims = (128, 256, 128, 64, 128)
    relus = (1, 1, 1, 0)
    L = len(relus)
    g = torch.Generator(device="cpu").manual_seed(0)
    xs = [torch.randn(M, dims[0], generator=g).to(dev) for _ in range(2)]
    Ws = [[(torch.randn(dims[l], dims[l + 1], generator=g) / dims[l] ** 0.5).to(dev) for l in range(L)]
          for _ in range(2)]
    bs = [[torch.randn(dims[l + 1], generator=g).to(dev) for l in range(L)] for _ in range(2)]
    gt = [torch.randn(M, dims[L], generator=g).to(dev) for _ in range(2)]
    ys = F.mlp_forward(xs, Ws, bs, relus, 6)
    yl = [[ys[l][s] for l in range(L)] for s in range(2)]
    gin = F.mlp_backward_chain(gt, Ws, yl, relus, 6, True)
    xl = [[xs[s]] + [ys[l][s] for l in range(L - 1)] for s in range(2)]
    gl = [[gin[l + 1][s] for l in range(L - 1)] + [gt[s]] for s in range(2)]
    ops = {
        "fwd": lambda: F.mlp_forward(xs, Ws, bs, relus, 6),
        "chain": lambda: F.mlp_backward_chain(gt, Ws, yl, relus, 6, True),
        "wgrad": lambda: F.mlp_wgrad(xl, gl, 6),
    }
    for name, fn in ops.items():
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(50):
            fn()
        b.record()
        torch.cuda.synchronize()
        print(f"{name}: {a.elapsed_time(b) / 50 * 1000:.1f} us per call (incl. launch gaps)", flush=True)


if __name__ == "__main__":
    main()
