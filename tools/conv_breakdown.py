"""Per-shape time / TFLOP/s of the GEMM launches of one training step (HIP events per launch).

usage (GPU box): python tools/conv_breakdown.py [reconet|adaattn] [steps]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "video-style-transfer_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from vst import kprof  # noqa: E402


def main():
    model = sys.argv[1] if len(sys.argv) > 1 else "reconet"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    sys.argv = [sys.argv[0], "--model", model]
    args = bench.parse()
    args.batch = args.batch or (8 if model == "reconet" else 4)
    args.replay_input = True  # (one synthetic batch: the launch shapes are what is measured)
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    step = (bench.build_reconet if model == "reconet" else bench.build_adaattn)(args, dev, 0)
    step()
    torch.cuda.synchronize()
    t = kprof.KernelTimer(detail=True)
    with t:
        for _ in range(steps):
            step()
    for fam in ("conv_gemm", "wgrad", "gemm_abt"):
        rows = sorted(t.by_tag(fam).items(), key=lambda kv: -kv[1][1])
        tot = sum(v[1] for _, v in rows) / steps
        fl = sum(v[2] for _, v in rows) / steps
        print(f"== {fam}: {tot:.2f} ms/step, {fl / max(tot, 1e-9) / 1e9:.1f} TF/s")
        for tag, (n, ms, f) in rows[:25]:
            print(f"{ms / steps:7.2f} ms/step n={n // steps:3d} {f / ms / 1e9:6.1f} TF  {tag}")


if __name__ == "__main__":
    main()
