"""The C3 tower Dense layers at B = 65536 (both towers in one grouped launch, precision 6):
forward (bias + ReLU), dX (mask epilogue) and dW + db (split-K) per layer, timed with HIP events.
Usage: python tools/microbench_towers.py [B]"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
F = importlib.import_module("recommendation-system-maang-nvidia-_amd.functional")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
dev = torch.device("cuda")
g = torch.Generator(device=dev)
g.manual_seed(0)
dims = [128, 256, 128, 64, 128]


def ev(fn, reps=20):
    """Mean time per call of fn: reps calls captured in one hipGraph and replayed between two HIP
    events (the host's per-call work outside the timing; EAGER=1: timed as eager calls)."""
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if os.environ.get("EAGER"):
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / reps * 1e3
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.stream(st):
        with torch.cuda.graph(gr, stream=st):
            for _ in range(reps):
                fn()
    torch.cuda.current_stream().wait_stream(st)
    gr.replay()
    torch.cuda.synchronize()
    s.record()
    gr.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


tot = {"fwd": 0.0, "dX": 0.0, "dW": 0.0}
for K, N in zip(dims[:-1], dims[1:]):
    xs = [torch.randn(B, K, device=dev, generator=g) for _ in range(2)]
    Ws = [torch.randn(K, N, device=dev, generator=g) / K ** 0.5 for _ in range(2)]
    bs = [torch.randn(N, device=dev, generator=g) for _ in range(2)]
    gy = [torch.randn(B, N, device=dev, generator=g) for _ in range(2)]
    tf = ev(lambda: F.gemm_group(xs, Ws, bias=bs, relu=True, precision=6))
    td = ev(lambda: F.gemm_group(gy, Ws, trans_b=True, mask=xs, precision=6))
    tw = ev(lambda: F.gemm_wgrad_bias_group(xs, gy, 6))
    mb = 2 * B * (K + N) * 4 / 1e6
    print(f"{K:4d}->{N:4d}: fwd {tf:6.1f} us ({mb / tf:5.2f} TB/s)  dX {td:6.1f} us  dW+db {tw:6.1f} us", flush=True)
    if os.environ.get("WT"):   # dX against a pre-transposed W (the forward's layout) instead of trans_b
        Wt = [w.t().contiguous() for w in Ws]
        tt = ev(lambda: F.gemm_group(gy, Wt, mask=xs, precision=6))
        tc = ev(lambda: [w.t().contiguous() for w in Ws])
        same = all(torch.equal(a, b) for a, b in zip(F.gemm_group(gy, Wt, mask=xs, precision=6),
                                                      F.gemm_group(gy, Ws, trans_b=True, mask=xs, precision=6)))
        print(f"      dX on W^T copies: {tt:6.1f} us (+ {tc:5.1f} us for the copies)  bitwise equal: {same}", flush=True)
    if os.environ.get("XG"):   # the same dW on the plane-pair GEMM: x^T image, g's dual image, split-K xgemm
        ti = ev(lambda: [F.xgemm_image(x, trans=True) for x in xs])
        tg = ev(lambda: [F.xgemm_image_dual(y, colsum=True) for y in gy])
        at = [F.xgemm_image(x, trans=True) for x in xs]
        gt = [F.xgemm_image_dual(y, colsum=True)[1] for y in gy]
        tk = ev(lambda: [F.xgemm_splitk(a, b, K, N, B) for a, b in zip(at, gt)])
        err = max((F.xgemm_splitk(a, b, K, N, B) - (x.double().t() @ y.double()).float()).abs().max().item()
                  for a, b, x, y in zip(at, gt, xs, gy))
        print(f"      xgemm dW: x^T images {ti:6.1f} us  g dual images {tg:6.1f} us  split-K {tk:6.1f} us  "
              f"sum {ti + tg + tk:6.1f} us (max err {err:.2e})", flush=True)
    tot["fwd"] += tf
    tot["dX"] += td
    tot["dW"] += tw
print("total: " + "  ".join(f"{k} {v:.1f} us" for k, v in tot.items())
      + f"  sum {sum(tot.values()):.1f} us", flush=True)
