"""Per-layer timing of the GEMM families (conv forward, data gradient, weight gradient) on the
ReCoNet / VGG step shapes (B=8 pairs -> 16 images, 256x512) in each GEMM arithmetic mode, through
vst.ops (same packing and dispatch as the training step).  HIP events, interleaved rounds.

    python tools/gemm_modes.py [--modes f32,bf16x3] [--only res] [--reps 5]
"""
import argparse
import statistics
import sys

import torch

sys.path.insert(0, "video-style-transfer_amd")
from vst import ops  # noqa: E402

SHAPES = [  # name, N, Cin, H, W, Cout, k, stride, pad_mode, up
    ("vgg1_2", 16, 64, 256, 512, 64, 3, 1, "zero", 1),
    ("vgg2_2", 16, 128, 128, 256, 128, 3, 1, "zero", 1),
    ("vgg3_2", 16, 256, 64, 128, 256, 3, 1, "zero", 1),
    ("vgg4_2", 16, 512, 32, 64, 512, 3, 1, "zero", 1),
    ("res", 16, 192, 64, 128, 192, 3, 1, "reflect", 1),
    ("deconv1", 16, 192, 64, 128, 96, 3, 1, "reflect", 2),
    ("deconv2", 16, 96, 128, 256, 48, 3, 1, "reflect", 2),
    ("conv2", 16, 48, 256, 512, 96, 3, 2, "reflect", 1),
    ("conv3", 16, 96, 128, 256, 192, 3, 2, "reflect", 1),
    ("conv1", 16, 3, 256, 512, 48, 9, 1, "reflect", 1),
]


def make(shape, what):
    name, N, Cin, H, W, Cout, k, s, pm, up = shape
    pad = k // 2
    Ho, Wo = ops.conv_out_hw(H, W, k, s, pad, up)
    x = torch.randn(N, Cin, H, W, device="cuda")
    w = torch.randn(Cout, Cin, k, k, device="cuda") * (2.0 / (Cin * k * k)) ** 0.5
    gz = torch.randn(N, Cout, Ho, Wo, device="cuda")
    gm = ops.GM_REFLECT if pm == "reflect" else ops.GM_ZERO
    flops = 2.0 * N * Cout * Ho * Wo * Cin * k * k
    if what == "fwd":
        def fn():
            ops.gemm_role("fwd")
            return ops.conv_gemm(x, ops.packed_weight(w, False), Cout, k, Ho, Wo, gm, s, pad, up)
    elif what == "dgrad":
        def fn():
            return ops.conv_dgrad(gz, w, x.shape, k, s, pad, pm, up)
    else:
        dw = torch.empty_like(w)

        def fn():
            return ops.conv_wgrad(gz, x, w.shape, k, s, pad, pm, up, out=dw)
    return fn, flops


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="f32,bf16x3")
    ap.add_argument("--only", default=None)
    ap.add_argument("--what", default="fwd,dgrad,wgrad")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    modes = a.modes.split(",")
    cases = [(s, w) for s in SHAPES for w in a.what.split(",") if not a.only or a.only in s[0]]
    if any(s[0] == "conv1" for s, w in cases):
        cases = [(s, w) for s, w in cases if not (s[0] == "conv1" and w == "dgrad")]
    res = {(s[0], w, m): [] for s, w in cases for m in modes}
    fns = {(s[0], w): make(s, w) for s, w in cases}
    for _ in range(3):
        for m in modes:
            ops.set_gemm_mode(m, policy={})
            for s, w in cases:
                fn, fl = fns[(s[0], w)]
                fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                res[(s[0], w, m)].append(e0.elapsed_time(e1) / a.reps)
    print("case".ljust(16) + "".join(m.rjust(20) for m in modes))
    tot = {m: 0.0 for m in modes}
    for s, w in cases:
        fl = fns[(s[0], w)][1]
        line = f"{s[0]}.{w}".ljust(16)
        for m in modes:
            ms = statistics.median(res[(s[0], w, m)])
            tot[m] += ms
            line += f"{ms * 1e3:9.0f}us {fl / ms / 1e9:6.1f}TF"
        print(line, flush=True)
    print("total".ljust(16) + "".join(f"{tot[m]:17.2f}ms" for m in modes))


if __name__ == "__main__":
    main()
