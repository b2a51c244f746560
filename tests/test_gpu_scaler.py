"""The fp16 policy's overflow guard (vst_adam_loss_scaled / vst.reconet._flat.LossScaler) on a real
MI355X.  The reference trains in fp32 and steps every batch (AA/train_video.py:121-122,
RC/train_single/train_candy.py:151-152); config 5's fp16 MFMA path must not let one overflowing
gradient write Inf / NaN into the Adam moments and the weights.  Rule (torch.cuda.amp.GradScaler's):
an Inf / NaN anywhere in the flat gradient skips the step (parameters, moments and Adam's step
count untouched) and multiplies the scale by 0.5; `growth_interval` clean steps in a row double it.
"""
import numpy as np
import pytest
import torch

from oracle import shapes

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _flat_module(seed=0):
    from vst.reconet._flat import FlatParams

    torch.manual_seed(seed)
    m = torch.nn.Sequential(torch.nn.Linear(37, 29), torch.nn.Linear(29, 5)).to(DEV)
    return m, FlatParams(m)


def _snap(flat):
    return [t.detach().clone() for t in (flat.p, flat.m, flat.v)]


def test_scaler_skips_overflow_and_backs_off():
    from vst.reconet._flat import LossScaler

    _, flat = _flat_module()
    sc = LossScaler(DEV, init_scale=1024.0, growth_interval=2)
    betas, lr, eps = (0.9, 0.999), 1e-3, 1e-8
    for bad in (float("inf"), float("-inf"), float("nan")):
        flat.g.normal_()
        flat.g[flat.numel // 3] = bad
        before = _snap(flat)
        scale0 = sc.scale()
        flat.adam_scaled(sc, lr, betas, eps)
        torch.cuda.synchronize()
        for a, b in zip(before, _snap(flat)):
            assert torch.equal(a, b), "a skipped step must leave p, m, v bitwise untouched"
        assert sc.skipped_last()
        st = sc.state_dict()
        assert st["scale"] == scale0 * 0.5 and st["step"] == 0 and st["growth_tracker"] == 0
    assert sc.state_dict()["skipped"] == 3


def test_scaler_clean_step_equals_adam_and_grows():
    """A clean step is bit-for-bit vst_adam with g * world / scale at Adam's own step count; the
    scale doubles after growth_interval clean steps."""
    from vst.reconet._flat import LossScaler

    _, flat = _flat_module(1)
    _, ref = _flat_module(1)
    sc = LossScaler(DEV, init_scale=256.0, growth_interval=2)
    betas, lr, eps, world = (0.9, 0.999), 1e-3, 1e-8, 0.5
    # a skipped step first: Adam's count must not advance
    flat.g.fill_(float("nan"))
    flat.adam_scaled(sc, lr, betas, eps, world)
    scales = []
    for k in range(1, 5):
        s = sc.scale()
        g = torch.randn(flat.numel, device=DEV) * s
        flat.g.copy_(g)
        ref.g.copy_(g)
        flat.adam_scaled(sc, lr, betas, eps, world)
        ref.adam(k, lr, betas, eps, world / s)
        torch.cuda.synchronize()
        assert not sc.skipped_last()
        for a, b in zip(_snap(flat), _snap(ref)):
            assert torch.equal(a, b), k
        scales.append(sc.scale())
    assert scales == [128.0, 256.0, 256.0, 512.0]  # backed off once, then x2 every 2 clean steps
    assert sc.state_dict()["step"] == 4


def test_scaler_state_dict_roundtrip():
    from vst.reconet._flat import LossScaler

    sc = LossScaler(DEV, init_scale=64.0, growth_interval=7)
    sd = {"scale": 8.0, "growth_tracker": 3, "step": 11, "skipped": 2, "growth_factor": 2.0,
          "backoff_factor": 0.5, "growth_interval": 5}
    sc.load_state_dict(sd)
    assert sc.state_dict() == sd


def _seeded(module, spec, seed):
    import oracle

    P = oracle.seeded_params(spec, seed)
    with torch.no_grad():
        for n, p in module.named_parameters():
            p.copy_(P[n])
    return module


@pytest.mark.parametrize("trainer", ["adaattn", "reconet"])
def test_trainer_overflow_step_skipped(trainer, monkeypatch):
    """Both trainers under the fp16 policy: an Inf injected into one gradient (after the
    all-reduce, as an overflow would arrive) skips that step and halves the scale; the next clean
    step updates the weights and Adam's step count is 1."""
    from vst import ops
    from vst.synthetic import content_style_batch

    old = ops.POLICY_NAME[0] or ops.DEFAULT_POLICY
    ops.use_policy("f16")
    try:
        if trainer == "adaattn":
            from vst.adaattn.network import StylizingNetwork
            from vst.adaattn.train import AdaAttNTrainer
            from vst.adaattn.vgg19 import VGG19

            model = _seeded(StylizingNetwork("cosine"), shapes.stylizing_network(), 61).to(DEV)
            vgg = _seeded(VGG19(), shapes.vgg19(), 62).to(DEV)
            tr = AdaAttNTrainer(model, vgg, activation="cosine")
            c1, c2, s = content_style_batch(63, 1, 64, 128)
            batch = (torch.stack([c1, c2, s]).to(DEV),)
        else:
            from vst.reconet.network import ReCoNet, Vgg16
            from vst.reconet.train import ReCoNetTrainer
            from vst.synthetic import frame_pair_batch, style_image

            model = _seeded(ReCoNet(), shapes.reconet(), 71).to(DEV)
            vgg = _seeded(Vgg16(), shapes.vgg16(), 72).to(DEV)
            img1, img2, flow, mask = frame_pair_batch(73, 1, 64, 128)
            tr = ReCoNetTrainer(model, vgg, style_image(74, 64, 128).to(DEV))
            batch = (torch.stack([img1, img2]).to(DEV), flow.to(DEV), mask.to(DEV))
        finish = tr.dp.finish
        inject = [True]

        def finish_and_poison():
            w = finish()
            if inject[0]:
                tr.flat.g[tr.flat.numel // 2] = float("inf")
            return w

        monkeypatch.setattr(tr.dp, "finish", finish_and_poison)
        p0 = tr.flat.p.clone()
        out = tr.step(*batch)
        torch.cuda.synchronize()
        assert torch.isfinite(out["loss"]).item()
        assert torch.equal(tr.flat.p, p0) and not tr.flat.m.any() and not tr.flat.v.any()
        assert tr.scaler.skipped_last() and tr.scaler.scale() == ops.loss_scale() / 2
        inject[0] = False
        # ReCoNet's loss weights (LAMBDA_F = 1e12, BETA = 2e10) put its gradients past fp16's range at
        # any scale >= 1: the scaler must keep backing off (every step skipped, nothing written)
        # until the first clean step; AdaAttN's first un-poisoned step is clean
        skipped = 0
        for _ in range(48):
            before = tr.flat.p.clone()
            tr.step(*batch)
            torch.cuda.synchronize()
            if not tr.scaler.skipped_last():
                break
            assert torch.equal(tr.flat.p, before) and not tr.flat.m.any()
            skipped += 1
        print(f"{trainer}: {skipped} overflowing steps skipped before the first clean one, "
              f"scale {tr.scaler.scale():g}")
        assert not tr.scaler.skipped_last()
        if trainer == "adaattn":
            assert skipped == 0
        st = tr.scaler.state_dict()
        assert st["step"] == 1 and st["skipped"] == skipped + 1 and tr.step_count == skipped + 2
        assert st["scale"] == ops.loss_scale() / 2 ** (skipped + 1)
        assert torch.isfinite(tr.flat.p).all() and not torch.equal(tr.flat.p, p0)
        # Adam's first step moves every parameter with a nonzero gradient by ~lr
        moved = (tr.flat.p - p0).abs()
        live = tr.flat.g != 0
        assert float(moved[live].max()) <= 1.01 * tr.lr
    finally:
        ops.use_policy(old if old in ops.POLICIES else ops.DEFAULT_POLICY)
