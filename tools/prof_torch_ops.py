"""Which torch (non-rs_*) kernels a bench training step launches, and from where: runs the
bench.py workload of argv[1] (c2 / c3 / c5) for 3 eager steps, then 2 under torch.profiler with
Python stacks, and prints the aten ops that reached the GPU with their calling frames."""
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
dev = torch.device("cuda", 0)
conf = dict(bench.CONFIGS[cfg])
wl = bench.setup_dcn2(conf, dev, 0, False) if cfg == "c5" else bench.setup_two_tower(conf, dev, 0, False)
for i in range(3):
    wl["train_step"](wl["batches"][i % len(wl["batches"])])
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
    for i in range(2):
        wl["train_step"](wl["batches"][i % len(wl["batches"])])
    torch.cuda.synchronize()
skip = ("aten::empty", "aten::view", "aten::as_strided", "aten::detach", "aten::reshape", "aten::t",
        "aten::contiguous", "aten::slice", "aten::select", "aten::alias", "aten::_reshape_alias", "aten::unsqueeze",
        "aten::squeeze", "aten::expand", "aten::transpose", "aten::permute", "aten::resize_", "aten::empty_like",
        "aten::empty_strided", "aten::lift_fresh", "aten::item", "aten::_local_scalar_dense")
for ev in prof.key_averages(group_by_stack_n=8):
    if not ev.key.startswith("aten::") or ev.key in skip or ev.device_time_total <= 0:
        continue
    print(f"{ev.key:32s} calls={ev.count:4d} gpu_us={ev.device_time_total:9.1f}")
    for fr in ev.stack[:8]:
        print("      ", fr)
