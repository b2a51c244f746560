"""Parity margin of the full ReCoNet train step (golden rc_step b1r / b2, sd_step) under GEMM
arithmetic policies: prints max(err / tolerance) of the loss terms and gradient checks of
tests/test_gpu_parity.py (<= 1 passes).  Diagnostic for choosing the default policy."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "video-style-transfer_amd")]
import oracle  # noqa: E402
from oracle import shapes  # noqa: E402
from vst import ops  # noqa: E402
from vst.reconet import network as N  # noqa: E402
from vst.reconet.train import ReCoNetTrainer  # noqa: E402

DEV = "cuda"
gold = dict(np.load(os.path.join(REPO, "tests/golden/rc_step.npz")))


def G(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def seeded(module, spec, seed):
    module.load_state_dict(dict(oracle.seeded_params(spec, seed)))
    return module


def margin(tag):
    s = gold
    seeds = s[f"{tag}_seeds"]
    model = seeded(N.ReCoNet(), shapes.reconet(), int(seeds[0])).to(DEV)
    vgg = seeded(N.Vgg16(), shapes.vgg16(), int(seeds[1])).to(DEV)
    tr = ReCoNetTrainer(model, vgg, G(s[f"{tag}_style"]))
    frames = torch.stack([G(s[f"{tag}_img1"]), G(s[f"{tag}_img2"])])
    out = tr.losses(frames, G(s[f"{tag}_flow"]), G(s[f"{tag}_mask"]))
    lm = max(abs(out[k].item() - float(s[f"{tag}_{k}"])) / (1e-3 * abs(float(s[f"{tag}_{k}"])))
             for k in ("loss", "CL", "SL", "FTL", "OTL", "RL"))
    tr.flat.zero_grad()
    out["loss"].backward()
    names = list(s[f"{tag}_names"])
    named = dict(model.named_parameters())
    gmax = max(float(s[f"{tag}_gnorm/{n}"]) for n in names)
    gm, worst = 0.0, None
    detail = []
    for n in names:
        gr = named[n].grad.detach().cpu().reshape(-1)
        gn = float(s[f"{tag}_gnorm/{n}"])
        tol = 1e-3 * gn + 1e-4 * gmax
        en = abs(float(gr.double().norm()) - gn)
        es = float(np.abs(gr[s[f"{tag}_gidx/{n}"]].numpy() - s[f"{tag}_gval/{n}"]).max())
        e = max(en, es)
        detail.append((e / tol, n, en / tol, es / tol))
        if e / tol > gm:
            gm, worst = e / tol, n
    if os.environ.get("POLICY_DETAIL"):
        for m, n, a, b in sorted(detail, reverse=True)[:4]:
            print(f"    {n:32s} margin {m:.3f} (norm {a:.3f}, samples {b:.3f})")
    return lm, gm, worst


POLICIES = {
    "f32": ("f32", {}),
    "bf16x6/wgrad-f32": ("bf16x6", {"wgrad": "f32"}),
    "bf16x6/dgrad-f32": ("bf16x6", {"dgrad": "f32"}),
    "bf16x6/stylizer-f32": ("bf16x6", {"stylizer.fwd": "f32", "stylizer.fwd_img": "f32"}),
    "bf16x6/fwd-f32": ("bf16x6", {"fwd": "f32", "fwd_img": "f32"}),
    "bf16x6/img-f32": ("bf16x6", {"fwd_img": "f32", "stylizer.fwd_img": "f32"}),
    "bf16x3": ("bf16x3", {}),
    "bf16x6": ("bf16x6", {}),
    "bf16x3/stylizer-f32": ("bf16x3", {"stylizer.fwd": "f32", "stylizer.fwd_img": "f32"}),
    "bf16x3/stylizer-bf16x6": ("bf16x3", {"stylizer.fwd": "bf16x6", "stylizer.fwd_img": "bf16x6"}),
    "parity/res-bf16x3": ("bf16x3", {"stylizer.fwd": "bf16x6", "stylizer.fwd_img": "bf16x6",
                                     "stylizer.res.fwd": "bf16x3"}),
    "parity/outer-bf16x3": ("bf16x3", {"stylizer.fwd": "bf16x3", "stylizer.fwd_img": "bf16x6",
                                       "stylizer.res.fwd": "bf16x6"}),
    "parity/img-only": ("bf16x3", {"stylizer.fwd_img": "bf16x6"}),
}
only = sys.argv[1:]
POLICIES = {k: v for k, v in POLICIES.items() if not only or k in only}
for name, (base, pol) in POLICIES.items():
    ops.set_gemm_mode(base, pol)
    for tag in ("b2", "b1r"):
        lm, gm, worst = margin(tag)
        print(f"{name:24s} {tag:4s} loss margin {lm:.3f}  grad margin {gm:.3f} ({worst})", flush=True)
