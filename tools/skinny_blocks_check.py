"""RS_SKINNY_BLOCKS A/B check: the C3 tower forward / dX (skinny kernels) with the row blocks dealt
one per workgroup vs several per workgroup must be bitwise equal (same arithmetic per element).
Run as: RS_SKINNY_BLOCKS=<n> python tools/skinny_blocks_check.py <out.pt>; compare two outputs with
python tools/skinny_blocks_check.py --compare a.pt b.pt"""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if sys.argv[1] == "--compare":
    a, b = torch.load(sys.argv[2], weights_only=True), torch.load(sys.argv[3], weights_only=True)
    bad = [k for k in a if not torch.equal(a[k], b[k])]
    print("bitwise equal" if not bad else f"DIFFER: {bad}")
    sys.exit(1 if bad else 0)
F = importlib.import_module("recommendation-system-maang-nvidia-_amd.functional")
dev = torch.device("cuda")
g = torch.Generator(device=dev)
g.manual_seed(0)
out = {}
for B in (65536, 65536 + 77):
    for K, N in ((128, 256), (256, 128), (128, 64), (64, 128)):
        xs = [torch.randn(B, K, device=dev, generator=g) for _ in range(2)]
        Ws = [torch.randn(K, N, device=dev, generator=g) / K ** 0.5 for _ in range(2)]
        bs = [torch.randn(N, device=dev, generator=g) for _ in range(2)]
        gy = [torch.randn(B, N, device=dev, generator=g) for _ in range(2)]
        y = F.gemm_group(xs, Ws, bias=bs, relu=True, precision=6)
        dx = F.gemm_group(gy, Ws, trans_b=True, mask=xs, precision=6)
        for i in range(2):
            out[f"{B}_{K}_{N}_y{i}"] = y[i].cpu()
            out[f"{B}_{K}_{N}_dx{i}"] = dx[i].cpu()
torch.save(out, sys.argv[1])
print("saved", len(out))
