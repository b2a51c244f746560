"""Find the first non-finite value of an AdaAttN train_video step under a GEMM policy (GPU box):
every GEMM wrapper of vst.ops / vst.adaattn.attention is wrapped to synchronise and check its
result, and the first offender is printed with its operands' ranges, role mode and scope.

    python tools/nan_diag.py [--gemm f16] [--size 128x256]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "video-style-transfer_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gemm", default="f16")
    ap.add_argument("--size", default="128x256")
    args = ap.parse_args()
    H, W = map(int, args.size.split("x"))
    import oracle
    from oracle import shapes
    from vst import ops
    from vst.adaattn import attention
    from vst.adaattn.network import StylizingNetwork
    from vst.adaattn.train import AdaAttNTrainer
    from vst.adaattn.vgg19 import VGG19
    from vst.synthetic import content_style_batch

    ops.use_policy(args.gemm)
    seen = []

    def wrap(mod, name):
        orig = getattr(mod, name)

        def f(*a, **k):
            out = orig(*a, **k)
            torch.cuda.synchronize()
            if isinstance(out, torch.Tensor) and not seen and not bool(torch.isfinite(out).all()):
                seen.append(name)
                rng = [(tuple(t.shape), float(t.abs().max())) for t in a if isinstance(t, torch.Tensor)]
                print(f"first non-finite: {mod.__name__}.{name} mode {ops.gemm_mode_name(ops.gemm_mode())} "
                      f"scope {ops._SCOPE[0]!r}/{ops._PSCOPE[0]!r} out {tuple(out.shape)} "
                      f"nonfinite {int((~torch.isfinite(out)).sum())}; tensor args (shape, max|x|): {rng}", flush=True)
            return out

        setattr(mod, name, f)

    for n in ("conv_gemm", "conv_wgrad", "conv_wgrad_up2", "conv_wgrad_rowsplit", "conv_dgrad_padout",
              "conv_dgrad_phase2", "conv_dgrad_ring", "conv_dgrad_padout_kwu", "channel_sum"):
        wrap(ops, n)
    for n in ("gemm_abt", "bmm_at_b", "attn_gemm"):
        wrap(attention, n)
    from vst.adaattn import lossfn
    lossfn.gemm_abt = attention.gemm_abt

    model = StylizingNetwork("cosine")
    model.load_state_dict(oracle.seeded_params(shapes.stylizing_network(), 61))
    vgg = VGG19()
    vgg.load_state_dict(oracle.seeded_params(shapes.vgg19(), 62))
    model, vgg = model.cuda(), vgg.cuda()
    tr = AdaAttNTrainer(model, vgg, activation="cosine")
    c1, c2, s = content_style_batch(63, 1, H, W, device="cuda")
    tr.flat.zero_grad()
    out = tr.losses(torch.stack([c1, c2, s]))
    print("losses", {k: float(v) for k, v in out.items()}, flush=True)
    tr.backward(out["loss"])
    torch.cuda.synchronize()
    bad = [n for n, p in model.named_parameters() if not bool(torch.isfinite(p.grad).all())]
    print("non-finite parameter gradients:", len(bad), bad[:8])
    print("max |grad| x scale per module:", {n: float(p.grad.abs().max()) for n, p in list(model.named_parameters())[:6]})


if __name__ == "__main__":
    main()
