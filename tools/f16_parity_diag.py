"""Config-5 (fp16 policy) parity measurements that set the bars of tests/test_gpu_adaattn.py:

  * per-tensor gradient error relative to the tensor's OWN norm (no slack from the largest tensor),
    one train_video step at 64x128 against the reference's own fp32 step (golden aa_step) and at
    128x256 / 256x512 (B=1) against the oracle's fp32 step on the same seeded weights and triple;
  * a 5-step trajectory at 64x128 (HIP under the policy, with its dynamic loss scale, vs the oracle's
    fp32 Adam steps): per-step loss terms and the parameter displacement after 5 steps.

    python tools/f16_parity_diag.py [policy ...]      (GPU; prints one JSON object)
"""
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "video-style-transfer_amd"), os.path.join(REPO, "tests")]

import oracle  # noqa: E402
from oracle import adaattn_ref as A  # noqa: E402
from oracle import reconet_ref as R  # noqa: E402
from oracle import shapes  # noqa: E402

DEV = "cuda"


def seeded(module, spec, seed):
    P = oracle.seeded_params(spec, seed)
    with torch.no_grad():
        for n, p in module.named_parameters():
            p.copy_(P[n])
    return module.to(DEV)


def hip_models(seed_m, seed_v):
    from vst.adaattn.network import StylizingNetwork
    from vst.adaattn.vgg19 import VGG19

    return seeded(StylizingNetwork("cosine"), shapes.stylizing_network(), seed_m), seeded(VGG19(), shapes.vgg19(), seed_v)


def own_errors(grads, ref_norms, gmax):
    """{tensor: |norm - ref norm| / ref norm} for live tensors, {tensor: norm / gmax} for dead ones"""
    live, dead = {}, {}
    for n, g in grads.items():
        gn, rn = float(g.double().norm()), ref_norms[n]
        if rn < 1e-6 * gmax:
            dead[n] = gn / gmax
        else:
            live[n] = abs(gn - rn) / rn
    return live, dead


def top(d, k=6):
    return sorted(((v, n) for n, v in d.items()), reverse=True)[:k]


def step_vs_oracle(policy, B, H, W, seeds=(61, 62, 63), k=6):
    from vst import ops
    from vst.adaattn.train import AdaAttNTrainer
    from vst.synthetic import content_style_batch

    c1, c2, s = content_style_batch(seeds[2], B, H, W)
    P = oracle.seeded_params(shapes.stylizing_network(), seeds[0], requires_grad=True)
    VP = oracle.seeded_params(shapes.vgg19(), seeds[1])
    t0 = time.time()
    L = A.adaattn_losses(P, VP, c1, c2, s)
    L["loss"].backward()
    t_oracle = time.time() - t0
    ops.use_policy(policy)
    model, vgg = hip_models(seeds[0], seeds[1])
    tr = AdaAttNTrainer(model, vgg, activation="cosine")
    tr.flat.zero_grad()
    out = tr.losses(torch.stack([c1, c2, s]).to(DEV))
    unscale = tr.backward(out["loss"])
    torch.cuda.synchronize()
    grads = {n: (p.grad * unscale).detach().cpu() for n, p in model.named_parameters()}
    ref = {n: float(p.grad.double().norm()) for n, p in P.items()}
    gmax = max(ref.values())
    live, dead = own_errors(grads, ref, gmax)
    a = torch.cat([grads[n].reshape(-1).double() / (ref[n] + 1e-30) for n in P])
    b = torch.cat([P[n].grad.reshape(-1).double() / (ref[n] + 1e-30) for n in P])
    return {"size": [B, H, W], "oracle_s": round(t_oracle, 1),
            "loss_rel": {k: abs(out[k].item() - L[k].item()) / abs(L[k].item()) for k in ("loss", "loss_gs", "loss_lf", "loss_is")},
            "worst_own": top(live, k), "dead": top(dead, 3), "cosine": float(a @ b / (a.norm() * b.norm()))}


def step_vs_golden(policy):
    from vst import ops
    from vst.adaattn.train import AdaAttNTrainer

    s = dict(np.load(os.path.join(REPO, "tests", "golden", "aa_step.npz")))
    seeds = s["seeds"]
    ops.use_policy(policy)
    model, vgg = hip_models(int(seeds[0]), int(seeds[1]))
    tr = AdaAttNTrainer(model, vgg, activation="cosine")
    frames = torch.stack([torch.from_numpy(s[k]) for k in ("c1", "c2", "style")]).to(DEV)
    tr.flat.zero_grad()
    out = tr.losses(frames)
    unscale = tr.backward(out["loss"])
    torch.cuda.synchronize()
    names = [str(n) for n in s["names"]]
    named = dict(model.named_parameters())
    grads = {n: (named[n].grad * unscale).detach().cpu() for n in names}
    ref = {n: float(s[f"gnorm/{n}"]) for n in names}
    live, dead = own_errors(grads, ref, max(ref.values()))
    return {"loss_rel": {k: abs(out[k].item() - float(s[k])) / abs(float(s[k])) for k in ("loss", "loss_gs", "loss_lf", "loss_is")},
            "worst_own": top(live), "dead": top(dead, 3)}


def trajectory(policy, steps=5, B=1, H=64, W=128, seeds=(61, 62, 63)):
    from vst import ops
    from vst.adaattn.train import AdaAttNTrainer
    from vst.synthetic import content_style_batch

    c1, c2, s = content_style_batch(seeds[2], B, H, W)
    P = oracle.seeded_params(shapes.stylizing_network(), seeds[0], requires_grad=True)
    VP = oracle.seeded_params(shapes.vgg19(), seeds[1])
    P0 = {k: v.detach().clone() for k, v in P.items()}
    st, ref_losses = {}, []
    for _ in range(steps):
        L = A.adaattn_losses(P, VP, c1, c2, s)
        L["loss"].backward()
        ref_losses.append({k: L[k].item() for k in ("loss", "loss_gs", "loss_lf", "loss_is")})
        R.adam_step(P, {k: p.grad for k, p in P.items()}, st, lr=1e-4)
        for p in P.values():
            p.grad = None
    ops.use_policy(policy)
    model, vgg = hip_models(seeds[0], seeds[1])
    tr = AdaAttNTrainer(model, vgg, activation="cosine")
    frames = torch.stack([c1, c2, s]).to(DEV)
    hip_losses = []
    for _ in range(steps):
        out = tr.step(frames)
        hip_losses.append({k: out[k].item() for k in ("loss", "loss_gs", "loss_lf", "loss_is")})
    named = {n: p.detach().cpu() for n, p in model.named_parameters()}
    dh = torch.cat([(named[n] - P0[n]).reshape(-1).double() for n in P])
    dr = torch.cat([(P[n].detach() - P0[n]).reshape(-1).double() for n in P])
    per = {}
    for n in P:
        a, b = (named[n] - P0[n]).reshape(-1).double(), (P[n].detach() - P0[n]).reshape(-1).double()
        per[n] = 1.0 - float(a @ b / (a.norm() * b.norm() + 1e-30))
    return {"loss_rel_per_step": [max(abs(h[k] - r[k]) / abs(r[k]) for k in h) for h, r in zip(hip_losses, ref_losses)],
            "disp_cosine": float(dh @ dr / (dh.norm() * dr.norm())), "disp_norm_ratio": float(dh.norm() / dr.norm()),
            "worst_tensor_1_minus_cos": top(per), "skipped": tr.scaler.state_dict() if tr.scaler else None}


def main():
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    pols = sys.argv[1:] or ["f16"]
    out = {}
    for pol in pols:
        out[pol] = {"golden_64x128": step_vs_golden(pol), "oracle_128x256": step_vs_oracle(pol, 1, 128, 256),
                    "trajectory_64x128": trajectory(pol)}
        if pol == "f16":
            out[pol]["oracle_256x512"] = step_vs_oracle(pol, 1, 256, 512)
        print(json.dumps({pol: out[pol]}), flush=True)


if __name__ == "__main__":
    main()
