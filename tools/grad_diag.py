"""Localise a per-term gradient discrepancy of the HIP ReCoNet step (GPU box): the gradient of the
one-term loss (tests/golden/rc_terms.npz case) w.r.t. every stylizer block's OUTPUT, HIP vs the
oracle in float64 (and the oracle in float32 beside it), norm-wise relative error per block.

    python tools/grad_diag.py [--tag b2] [--terms OTL,CL] [--gemm f32]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "video-style-transfer_amd"), os.path.join(REPO, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle  # noqa: E402
from oracle import reconet_ref as R  # noqa: E402
from oracle import shapes  # noqa: E402

BLOCKS = ("conv1", "conv2", "conv3", "res1", "res2", "res3", "res4", "res5", "deconv1", "deconv2", "deconv3")


def oracle_grads(d, tag, term, dtype):
    seeds = d[f"{tag}_seeds"]
    P = {k: v.to(dtype).requires_grad_(True) for k, v in oracle.seeded_params(shapes.reconet(), int(seeds[0])).items()}
    VP = {k: v.to(dtype) for k, v in oracle.seeded_params(shapes.vgg16(), int(seeds[1])).items()}
    acts = {b: [] for b in BLOCKS}

    def keep(name, t):
        t.retain_grad()
        acts[name].append(t)
        return t

    def fwd(P, x):
        x = keep("conv1", R.conv_in_relu(x, P, "conv1", 9, 1))
        x = keep("conv2", R.conv_in_relu(x, P, "conv2", 3, 2))
        x = keep("conv3", R.conv_in_relu(x, P, "conv3", 3, 2))
        for i in range(1, 6):
            x = keep(f"res{i}", R.residual_block(x, P, f"res{i}"))
        features = x
        x = keep("deconv1", R.conv_in_relu(x, P, "deconv1", 3, 1, upsample=True))
        sd1 = x
        x = keep("deconv2", R.conv_in_relu(x, P, "deconv2", 3, 1, upsample=True))
        return sd1, features, keep("deconv3", R.conv_tanh(x, P, "deconv3", 9))

    T = lambda k: torch.from_numpy(d[f"{tag}_{k}"]).to(dtype)  # noqa: E731
    L = R.reconet_losses(P, VP, T("img1").clone(), T("img2").clone(), T("flow"), T("mask"),
                         R.style_grams(VP, T("style")), forward=fwd, terms=(term,))
    L["loss"].backward()
    return {b: torch.cat([t.grad for t in acts[b]]).double() for b in BLOCKS}, float(L["loss"].detach())


def hip_grads(d, tag, term, nosink=False):
    from vst.reconet import network as N
    from vst.reconet.train import ReCoNetTrainer

    dev = "cuda"
    seeds = d[f"{tag}_seeds"]
    model = N.ReCoNet()
    model.load_state_dict(oracle.seeded_params(shapes.reconet(), int(seeds[0])))
    vgg = N.Vgg16()
    vgg.load_state_dict(oracle.seeded_params(shapes.vgg16(), int(seeds[1])))
    model, vgg = model.to(dev), vgg.to(dev)
    acts = {}

    def hook(name):
        def f(_m, _i, out):
            out.register_hook(lambda g, n=name: acts.__setitem__(n, g.detach().double().cpu()))
        return f

    for b in BLOCKS:
        getattr(model, b).register_forward_hook(hook(b))
    tr = ReCoNetTrainer(model, vgg, torch.from_numpy(d[f"{tag}_style"]).to(dev), terms=(term,))
    G = lambda k: torch.from_numpy(d[f"{tag}_{k}"]).to(dev)  # noqa: E731
    out = tr.losses(torch.stack([G("img1"), G("img2")]), G("flow"), G("mask"))
    tr.flat.zero_grad()
    if nosink:  # no .grad views: every weight gradient is returned to autograd instead of written in place
        for p in model.parameters():
            p.grad = None
    out["loss"].backward()
    torch.cuda.synchronize()
    return acts, float(out["loss"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="b2")
    ap.add_argument("--terms", default="OTL,CL,SL,RL,FTL")
    ap.add_argument("--gemm", default="f32")
    ap.add_argument("--nosink", action="store_true")
    args = ap.parse_args()
    from vst import ops

    ops.use_policy(args.gemm)
    d = dict(np.load(os.path.join(REPO, "tests", "golden", "rc_terms.npz")))
    for term in args.terms.split(","):
        ge, le = oracle_grads(d, args.tag, term, torch.float64)
        g32, l32 = oracle_grads(d, args.tag, term, torch.float32)
        gh, lh = hip_grads(d, args.tag, term, args.nosink)
        print(f"== {args.tag} {term} ({args.gemm}{', no sinks' if args.nosink else ''}): loss exact {le:.9e} oracle32 {l32:.9e} hip {lh:.9e}")
        for b in reversed(BLOCKS):
            e = ge[b]
            if float(e.norm()) == 0.0:
                continue
            r32 = float((g32[b] - e).norm() / e.norm())
            rh = float((gh[b] - e).norm() / e.norm()) if b in gh else float("nan")
            print(f"  d/d{b:8s} |g| {float(e.norm()):.3e}  oracle32 {r32:.2e}  hip {rh:.2e}")
        sys.stdout.flush()


if __name__ == "__main__":
    main()
