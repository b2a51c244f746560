"""Which ATen elementwise adds does one config-3 training step launch (autograd gradient sums, loss-term
sums)?  One step under torch.profiler (CPU op events with input shapes and Python stacks); prints each
aten::add / aten::add_ with its shapes and the innermost vst / trainer frames.   (GPU)"""
import os
import sys
from collections import Counter

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "video-style-transfer_amd")]


def main():
    import bench
    from vst import ops

    ops.use_policy("bf16x6")
    args = bench.parse()
    args.warmup, args.steps, args.prof_steps = 0, 1, 0
    step = bench.build_reconet(args, torch.device("cuda"), 0)
    step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU], record_shapes=True, with_stack=True) as prof:
        step()
        torch.cuda.synchronize()
    cnt = Counter()
    for ev in prof.events():
        if ev.name in ("aten::add", "aten::add_", "aten::sum", "aten::copy_", "aten::fill_", "aten::zero_"):
            frames = [f for f in (ev.stack or []) if "vst" in f or "train" in f or "autograd" in f][:3]
            key = (ev.name, str(ev.input_shapes[:2]), " | ".join(frames))
            cnt[key] += 1
    for (name, shp, fr), n in sorted(cnt.items(), key=lambda kv: -kv[1]):
        print(f"{n:3d} {name:12s} {shp[:70]:70s} {fr[:200]}")


if __name__ == "__main__":
    main()
