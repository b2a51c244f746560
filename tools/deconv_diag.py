"""Split the per-term gradient discrepancy at one stylizer layer (GPU box): the layer's input is the
oracle's float64 activation on the rc_terms case (rounded to fp32), its upstream gradient the
oracle's exact one; HIP backward of (a) the whole conv -> IN -> ReLU block, (b) the conv data
gradient alone, (c) the InstanceNorm(+ReLU) backward alone, each vs the float64 oracle.

    python tools/deconv_diag.py [--tag b2] [--term OTL] [--layer deconv2] [--gemm f32]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "video-style-transfer_amd"), os.path.join(REPO, "tools")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle  # noqa: E402
from oracle import reconet_ref as R  # noqa: E402
from oracle import shapes  # noqa: E402

LAYERS = {"deconv1": ("res5", 3, 1, True), "deconv2": ("deconv1", 3, 1, True), "conv2": ("conv1", 3, 2, False),
          "conv3": ("conv2", 3, 2, False)}


def rel(a, e):
    a, e = a.double().cpu(), e.double().cpu()
    return float((a - e).norm() / e.norm()), float((a - e).abs().max() / e.abs().max())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="b2")
    ap.add_argument("--term", default="OTL")
    ap.add_argument("--layer", default="deconv2")
    ap.add_argument("--gemm", default="f32")
    ap.add_argument("--scope", default="stylizer", help="gemm_scope the HIP calls run in ('' = none)")
    args = ap.parse_args()
    from vst import ops

    ops.use_policy(args.gemm)
    if args.scope:
        ops._SCOPE[0] = args.scope
    d = dict(np.load(os.path.join(REPO, "tests", "golden", "rc_terms.npz")))
    seeds = d[f"{args.tag}_seeds"]
    prev, k, stride, up = LAYERS[args.layer]
    # float64 oracle: the layer input (prev block output) and the exact gradient at the layer output
    acts, grads = {}, {}
    P = {kk: v.double().requires_grad_(True) for kk, v in oracle.seeded_params(shapes.reconet(), int(seeds[0])).items()}
    VP = {kk: v.double() for kk, v in oracle.seeded_params(shapes.vgg16(), int(seeds[1])).items()}

    def keep(name, t):
        t.retain_grad()
        acts.setdefault(name, []).append(t)
        return t

    def fwd(P, x):
        x = keep("conv1", R.conv_in_relu(x, P, "conv1", 9, 1))
        x = keep("conv2", R.conv_in_relu(x, P, "conv2", 3, 2))
        x = keep("conv3", R.conv_in_relu(x, P, "conv3", 3, 2))
        for i in range(1, 6):
            x = keep(f"res{i}", R.residual_block(x, P, f"res{i}"))
        f = x
        x = keep("deconv1", R.conv_in_relu(x, P, "deconv1", 3, 1, upsample=True))
        sd1 = x
        x = keep("deconv2", R.conv_in_relu(x, P, "deconv2", 3, 1, upsample=True))
        return sd1, f, R.conv_tanh(x, P, "deconv3", 9)

    T = lambda kk: torch.from_numpy(d[f"{args.tag}_{kk}"]).double()  # noqa: E731
    L = R.reconet_losses(P, VP, T("img1").clone(), T("img2").clone(), T("flow"), T("mask"),
                         R.style_grams(VP, T("style")), forward=fwd, terms=(args.term,))
    L["loss"].backward()
    x64 = torch.cat([t.detach() for t in acts[prev]])
    gy64 = torch.cat([t.grad for t in acts[args.layer]])
    name = args.layer
    w, b = P[name + ".conv2d.weight"].detach(), P[name + ".conv2d.bias"].detach()
    gam, bet = P[name + ".instance.weight"].detach(), P[name + ".instance.bias"].detach()

    # oracle float64 pieces on the fp32-rounded input
    xr = x64.float().double().requires_grad_(True)
    z = R.conv_layer(xr, {name + ".conv2d.weight": w, name + ".conv2d.bias": b}, name, k, stride, upsample=up)
    z.retain_grad()
    y = torch.relu(R.instance_norm(z, gam, bet))
    y.backward(gy64)
    dx64, dz64 = xr.grad, z.grad
    print(f"{args.tag} {args.term} {name} ({args.gemm}, scope {args.scope!r}): x {tuple(x64.shape)} |dx| {float(dx64.norm()):.3e}")
    print(f"  relu active fraction {float((y > 0).double().mean()):.4f}; |z| near IN zero: "
          f"{int((R.instance_norm(z, gam, bet).abs() < 1e-5 * R.instance_norm(z, gam, bet).abs().max()).sum())} elems")

    dev = "cuda"
    # (a) whole block
    xg = x64.float().to(dev).requires_grad_(True)
    wg, bg, gg, beg = (t.float().to(dev).requires_grad_(True) for t in (w, b, gam, bet))
    yg = ops.conv_instance_norm(xg, wg, bg, gg, beg, stride, k // 2, "reflect", 2 if up else 1, relu=True)
    yg.backward(gy64.float().to(dev))
    print("  (a) block dx      norm/max rel err %.2e / %.2e" % rel(xg.grad, dx64))
    # (b) conv data gradient alone with the exact dz
    xg2 = x64.float().to(dev).requires_grad_(True)
    zg = ops.conv2d(xg2, wg.detach(), bg.detach(), stride=stride, pad=k // 2, pad_mode="reflect", up=2 if up else 1)
    zg.backward(dz64.float().to(dev))
    print("  (b) conv dgrad    norm/max rel err %.2e / %.2e" % rel(xg2.grad, dx64))
    print("      conv fwd z    norm/max rel err %.2e / %.2e" % rel(zg.detach(), z.detach()))
    # (c) IN + ReLU backward alone on the exact z
    zz = z.detach().float().to(dev).requires_grad_(True)
    yy = ops.instance_norm(zz, gg.detach(), beg.detach(), relu=True)
    yy.backward(gy64.float().to(dev))
    print("  (c) IN+ReLU bwd   norm/max rel err %.2e / %.2e" % rel(zz.grad, dz64))
    mask_h = (yy.detach().cpu() > 0)
    mask_e = (R.instance_norm(z.detach(), gam, bet) > 0)
    print(f"      relu mask mismatches (HIP fwd vs exact): {int((mask_h != mask_e).sum())}")


if __name__ == "__main__":
    main()
