"""Why config 5's half-precision MFMA path is bf16 and not fp16: the dynamic range of the GEMM
operands of one AdaAttN train_video step.

Runs the oracle step (oracle/adaattn_ref.py, the reference's arithmetic on torch-CPU) on a B=1
synthetic triple under a TorchDispatchMode that sees every convolution / convolution_backward /
bmm / mm, and records per operand the fraction of non-zero elements outside fp16's normal range
(|x| < 6.10e-5: subnormal, 2^-14; |x| < 5.96e-8: flushed to zero; |x| > 65504: overflow).  bf16
has fp32's exponent range, so none of its operands leave it.

    python tools/fp16_range.py [--hw 64 128]   -> profiles/r02_fp16_range.json
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path[:0] = [REPO, os.path.join(REPO, "video-style-transfer_amd")]

import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

FP16_MIN_NORMAL, FP16_MIN_SUB, FP16_MAX = 2.0 ** -14, 2.0 ** -24, 65504.0
aten = torch.ops.aten
WATCH = {aten.convolution.default: "conv_fwd", aten.convolution_backward.default: "conv_bwd",
         aten.bmm.default: "bmm", aten.mm.default: "mm"}


class RangeMode(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.stats = {}

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        kind = WATCH.get(func)
        if kind is not None:
            ts = [a for a in args if isinstance(a, torch.Tensor) and a.is_floating_point()]
            if kind == "conv_bwd":
                ts = ts[:3]  # grad_output, input, weight
            for i, t in enumerate(ts):
                a = t.detach().abs().reshape(-1)
                nz = a[a > 0]
                if nz.numel() == 0:
                    continue
                s = self.stats.setdefault(f"{kind}.operand{i}", [0, 0, 0, 0, 0.0, float("inf")])
                s[0] += nz.numel()
                s[1] += int((nz < FP16_MIN_NORMAL).sum())
                s[2] += int((nz < FP16_MIN_SUB).sum())
                s[3] += int((nz > FP16_MAX).sum())
                s[4] = max(s[4], float(nz.max()))
                s[5] = min(s[5], float(nz.min()))
        return func(*args, **(kwargs or {}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hw", type=int, nargs=2, default=(64, 128))
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r02_fp16_range.json"))
    a = ap.parse_args()
    import oracle
    from oracle import adaattn_ref as A
    from oracle import shapes
    from vst.synthetic import content_style_batch

    H, W = a.hw
    P = oracle.seeded_params(shapes.stylizing_network(), 1, requires_grad=True)
    VP = oracle.seeded_params(shapes.vgg19(), 2)
    c1, c2, s = content_style_batch(99, 1, H, W)
    mode = RangeMode()
    with mode:
        L = A.adaattn_losses(P, VP, c1, c2, s)
        L["loss"].backward()
    out = {"workload": f"oracle AdaAttN train_video step, B=1, 3x{H}x{W}, seeded weights (numpy PCG64)",
           "fp16": {"min_normal": FP16_MIN_NORMAL, "min_subnormal": FP16_MIN_SUB, "max": FP16_MAX}, "operands": {}}
    for k, (n, sub, ftz, ovf, mx, mn) in sorted(mode.stats.items()):
        out["operands"][k] = {"nonzero": n, "frac_below_fp16_normal": sub / n, "frac_flushed_in_fp16": ftz / n,
                              "frac_overflow_fp16": ovf / n, "max_abs": mx, "min_abs_nonzero": mn}
        print(f"{k:20s} n={n:>10d} <normal {sub / n:.4f}  ftz {ftz / n:.4f}  overflow {ovf / n:.4f}  "
              f"max {mx:.3e} min {mn:.3e}")
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
