"""RTNSTV path (RT/network.py, RT/vgg19.py, RT/utilities.py, RT/train.py).

Golden vectors come from the reference's own code (tests/golden/gen_golden.py rtnstv):
ConvTranspose2d / Deconv / StylizingNetwork forwards and one full `train()` step (losses,
per-tensor gradient norms and samples, post-Adam heads) at B=2 32x64 and a ragged B=1 36x60.
The oracle (oracle/rtnstv_ref.py) is pinned against them on CPU; the HIP path is checked against
the same vectors on the GPU.  Tolerance: 1e-3 relative (north_star fp32 contract)."""
import numpy as np
import pytest
import torch

import oracle
from conftest import rel_err
from oracle import rtnstv_ref as RT
from oracle import shapes


def T(a):
    return torch.from_numpy(np.asarray(a))


def _deconv_params():
    return oracle.seeded_params([("deconv.weight", (6, 5, 3, 3)), ("deconv.bias", (5,)), ("norm.weight", (5,)),
                                 ("norm.bias", (5,))], 301)


def test_oracle_units_golden(golden):
    g = golden("rt_step")
    P = _deconv_params()
    x = T(g["deconv_x"])
    y = torch.nn.functional.conv_transpose2d(x, P["deconv.weight"], P["deconv.bias"], 2, 1, 1)
    assert rel_err(y, g["deconv_y"]) < 1e-5
    Q = {"d." + k: v for k, v in P.items()}
    assert rel_err(RT.deconv(x, Q, "d"), g["deconv_block_y"]) < 1e-5
    NP = oracle.seeded_params(shapes.rtnstv(), 302)
    assert rel_err(RT.stylizer_forward(NP, T(g["net_x"])), g["net_y"]) < 1e-4


def _check_step(s, tag, L, grads, params_after):
    for k in ("loss", "CL", "SL", "RL", "TL"):
        assert rel_err(float(L[k]), s[f"{tag}_{k}"]) < 1e-3, (k, float(L[k]), float(s[f"{tag}_{k}"]))
    names = list(s[f"{tag}_names"])
    gmax = max(float(s[f"{tag}_gnorm/{n}"]) for n in names)
    for n in names:
        g = grads[n].reshape(-1).double().cpu()
        gn = float(s[f"{tag}_gnorm/{n}"])
        assert abs(float(g.norm()) - gn) <= 1e-3 * gn + 1e-4 * gmax, (n, float(g.norm()), gn)
        idx = s[f"{tag}_gidx/{n}"]
        assert np.abs(g[idx].numpy() - s[f"{tag}_gval/{n}"]).max() <= 1e-3 * gn + 1e-4 * gmax, n
        if params_after is not None:
            gh = s[f"{tag}_ghead/{n}"]
            sel = np.abs(gh) > 1e-6 * gmax + 1e-2 * np.abs(gh).max()
            ph = params_after[n].reshape(-1)[:64].detach().cpu().numpy()
            assert np.abs(ph - s[f"{tag}_phead/{n}"])[sel].max(initial=0) < 1e-5, n


@pytest.mark.parametrize("tag", ["b2", "b1r"])
def test_oracle_train_step_golden(golden, tag):
    s = golden("rt_step")
    seeds = s[f"{tag}_seeds"]
    P = oracle.seeded_params(shapes.rtnstv(), int(seeds[0]), requires_grad=True)
    VP = oracle.seeded_params(shapes.vgg19_rt(), int(seeds[1]))
    grams = RT.style_grams(VP, T(s[f"{tag}_style"]))
    L = RT.rtnstv_losses(P, VP, T(s[f"{tag}_img1"]), T(s[f"{tag}_img2"]), T(s[f"{tag}_flow"]), T(s[f"{tag}_mask"]),
                         grams)
    L["loss"].backward()
    _check_step(s, tag, {k: v.item() for k, v in L.items()}, {n: p.grad for n, p in P.items()}, None)


def test_state_dict_keys_match_reference():
    from vst.rtnstv.network import StylizingNetwork
    from vst.rtnstv.vgg19 import VGG19

    for mod, spec in ((StylizingNetwork(), shapes.rtnstv()), (VGG19(), shapes.vgg19_rt())):
        assert [(k, tuple(v.shape)) for k, v in mod.state_dict().items()] == [(k, tuple(s)) for k, s in spec]


# ------------------------------------------------------------------------------------------ GPU
def _seeded(module, spec, seed):
    sd = {k: v for k, v in oracle.seeded_params(spec, seed).items()}
    module.load_state_dict(sd)
    return module


@pytest.mark.gpu
def test_conv_transpose_fwd_bwd():
    from vst import ops

    torch.manual_seed(3)
    for N, Cin, Cout, H, W in ((2, 6, 5, 7, 9), (2, 48, 32, 16, 24), (1, 32, 16, 9, 13)):
        x = torch.randn(N, Cin, H, W, requires_grad=True)
        w = (torch.randn(Cin, Cout, 3, 3) * 0.2).requires_grad_(True)
        b = torch.randn(Cout, requires_grad=True)
        y = torch.nn.functional.conv_transpose2d(x, w, b, 2, 1, 1)
        gy = torch.randn_like(y)
        y.backward(gy)
        xd, wd, bd = (t.detach().cuda().requires_grad_(True) for t in (x, w, b))
        yd = ops.conv_transpose2d(xd, wd, bd)
        yd.backward(gy.cuda())
        for a, r in ((yd, y), (xd.grad, x.grad), (wd.grad, w.grad), (bd.grad, b.grad)):
            assert rel_err(a.detach().cpu(), r.detach()) < 1e-4


@pytest.mark.gpu
def test_units_and_forward_golden(golden):
    from vst.rtnstv.network import Deconv, StylizingNetwork

    g = golden("rt_step")
    d = Deconv(6, 5, 3, 2, torch.nn.ReLU())
    d.load_state_dict(_deconv_params())
    d = d.cuda()
    with torch.no_grad():
        assert rel_err(d(T(g["deconv_x"]).cuda()).cpu(), g["deconv_block_y"]) < 1e-4
        net = _seeded(StylizingNetwork(), shapes.rtnstv(), 302).cuda()
        assert rel_err(net(T(g["net_x"]).cuda()).cpu(), g["net_y"]) < 1e-3


@pytest.mark.gpu
def test_tv_sqrt_and_tanh_image():
    from vst import ops

    torch.manual_seed(4)
    s = (torch.rand(2, 3, 11, 13) * 255)
    s[0, 0, :3, :3] = 7.0  # flat patch: the clamp(min=1e-8) branch
    s.requires_grad_(True)
    r1 = (s[:, :, :-1, 1:] - s[:, :, :-1, :-1]) ** 2
    r2 = (s[:, :, 1:, :-1] - s[:, :, :-1, :-1]) ** 2
    ref = torch.sqrt((r1 + r2).clamp(min=1e-8)).mean() * 0.5
    ref.backward()
    sd = s.detach().cuda().requires_grad_(True)
    out = ops.tv_sqrt_loss(sd, 0.5)
    out.backward()
    assert rel_err(out.item(), ref.item()) < 1e-5
    assert rel_err(sd.grad.cpu(), s.grad) < 1e-5
    v = torch.randn(2, 3, 8, 8, requires_grad=True)
    y = (torch.tanh(v) + 1) / 2 * 255
    gy = torch.randn_like(y)
    y.backward(gy)
    vd = v.detach().cuda().requires_grad_(True)
    yd = ops.tanh_image(vd)
    yd.backward(gy.cuda())
    assert rel_err(yd.detach().cpu(), y.detach()) < 1e-6 and rel_err(vd.grad.cpu(), v.grad) < 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize("tag", ["b2", "b1r"])
def test_train_step_golden(golden, tag):
    from vst.rtnstv.network import StylizingNetwork
    from vst.rtnstv.train import RTNSTVTrainer
    from vst.rtnstv.vgg19 import VGG19

    s = golden("rt_step")
    seeds = s[f"{tag}_seeds"]
    net = _seeded(StylizingNetwork(), shapes.rtnstv(), int(seeds[0])).cuda()
    vgg = _seeded(VGG19(), shapes.vgg19_rt(), int(seeds[1])).cuda()
    tr = RTNSTVTrainer(net, vgg, T(s[f"{tag}_style"]).cuda())
    frames = torch.stack([T(s[f"{tag}_img1"]), T(s[f"{tag}_img2"])]).cuda()
    tr.flat.zero_grad()
    L = tr.losses(frames, T(s[f"{tag}_flow"]).cuda(), T(s[f"{tag}_mask"]).cuda())
    L["loss"].backward()
    grads = {n: p.grad.detach().clone() for n, p in net.named_parameters()}
    tr.step_count += 1
    tr.flat.adam(tr.step_count, tr.lr, tr.betas, tr.eps)
    torch.cuda.synchronize()
    _check_step(s, tag, {k: v.item() for k, v in L.items()}, grads, dict(net.named_parameters()))
