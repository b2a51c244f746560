"""HIP path vs the oracle and the reference's golden vectors, on a real MI355X.

Tolerances (north_star: "within 1e-3 relative fp32"):
  * single ops vs the oracle (fp32 torch-CPU autograd): max|diff| <= 1e-4 * max|ref| (1e-3 for
    gradients through long reductions);
  * model forward vs golden: 1e-3 relative to the tensor's max magnitude;
  * loss terms: 1e-3 relative; gradients: per-tensor norm within 1e-3 (+1e-4 of the largest norm).
"""
import zlib

import numpy as np
import pytest
import torch
import torch.nn.functional as F

import oracle
from oracle import reconet_ref as R
from oracle import shapes

from conftest import rel_err

pytestmark = pytest.mark.gpu
DEV = "cuda"


def T(a):
    return torch.from_numpy(np.ascontiguousarray(a))


def G(a):
    return T(a).to(DEV) if isinstance(a, np.ndarray) else a.to(DEV)


def C(t):
    return t.detach().cpu()


@pytest.fixture(scope="module", autouse=True)
def _seed():
    torch.manual_seed(0)


# ----------------------------------------------------------------------------- units vs golden
def test_warp_mask_gram_norm_golden(golden):
    from vst.reconet import utilities as U

    u = golden("rc_units")
    for tag in ("img", "feat", "wide"):
        out = U.warp(G(u[f"warp_{tag}_x"]), G(u[f"warp_{tag}_flo"]))
        assert rel_err(C(out), u[f"warp_{tag}_out"]) < 1e-5, tag
    x = G(u["warp_ramp_x"])
    assert rel_err(C(U.warp(x, torch.zeros(1, 2, 4, 6, device=DEV))), u["warp_ramp_out"]) < 1e-6
    for i in range(3):
        m = U.flow_warp_mask(G(u[f"fwm{i}_f01"]), G(u[f"fwm{i}_f10"]))
        assert np.array_equal(C(m).numpy(), u[f"fwm{i}_mask"]), i
    assert rel_err(C(U.gram_matrix(G(u["gram_y"]))), u["gram_out"]) < 1e-5
    assert torch.allclose(C(U.gram_matrix(torch.ones(1, 2, 3, 3, device=DEV))), torch.full((1, 2, 2), 0.5))
    x = G(u["vggn_x"]).clone()
    out = U.vgg_normalize(x)
    assert rel_err(C(out), u["vggn_out"]) < 1e-6 and rel_err(C(x), u["vggn_x_after"]) < 1e-7


# ----------------------------------------------------------------------------- conv family vs oracle
CONV_CASES = [
    # (N, Cin, H, W, Cout, k, stride, pad_mode, up, act)
    (2, 3, 20, 28, 48, 9, 1, "reflect", 1, None),     # ReCoNet conv1 (Cin=3: kw-unfolded input)
    (1, 3, 13, 22, 48, 9, 1, "reflect", 1, None),     # conv1, width not a multiple of 4 (direct gather)
    (1, 48, 13, 22, 3, 9, 1, "reflect", 1, "tanh"),   # ConvTanh, padded width 30 (direct dgrad gather)
    (2, 48, 16, 24, 96, 3, 2, "reflect", 1, None),    # conv2 (stride 2)
    (2, 96, 10, 12, 192, 3, 2, "reflect", 1, None),   # conv3
    (1, 32, 15, 21, 64, 3, 2, "reflect", 1, None),    # stride 2, odd sizes (uneven parity phases)
    (2, 16, 3, 5, 32, 3, 2, "reflect", 1, None),      # stride 2, 3-row input (border band = all rows)
    (1, 16, 11, 13, 32, 5, 2, "reflect", 1, None),    # stride 2, k5 pad 2 (3x3 phase window)
    (2, 192, 9, 15, 192, 3, 1, "reflect", 1, None),   # residual conv, ragged
    (2, 192, 10, 32, 192, 3, 1, "reflect", 1, None),  # residual conv, 16-multiple width (halo weight gradient)
    (1, 64, 7, 48, 128, 3, 1, "zero", 1, "relu"),     # zero-pad conv over 32-channel blocks (halo weight gradient)
    (2, 192, 5, 8, 96, 3, 1, "reflect", 2, None),     # deconv1 (nearest x2 upsample)
    (1, 96, 9, 6, 48, 3, 1, "reflect", 2, None),      # deconv2
    (1, 40, 7, 33, 24, 3, 1, "reflect", 2, None),     # upsample conv, (W+1) over two k-tiles, odd H
    (2, 48, 16, 20, 3, 9, 1, "reflect", 1, "tanh"),   # deconv3 ConvTanh (Cout=3)
    (2, 3, 12, 20, 64, 3, 1, "zero", 1, "relu"),      # VGG conv1_1
    (2, 64, 8, 12, 128, 3, 1, "zero", 1, "relu"),     # VGG conv
    (1, 256, 4, 6, 512, 3, 1, "zero", 1, "relu"),     # VGG conv4_x
    # AdaAttN decoder conv7 / conv6 (64 outputs over >= 64 channels, 3x3 reflect): the weight
    # gradient as the row-split GEMM (rows (co, kh), columns (kw, ci)); ragged width: 3 x 16 + 5
    (2, 64, 6, 32, 64, 3, 1, "reflect", 1, "relu"),
    (1, 128, 5, 53, 64, 3, 1, "reflect", 1, "relu"),
    (2, 64, 8, 32, 3, 3, 1, "reflect", 1, None),      # AdaAttN decoder conv8 (dgrad: 3 source channels)
]


def _oracle_conv(x, w, b, stride, pad_mode, up, act):
    k = w.shape[-1]
    if up == 2:
        x = R.upsample_nearest2x(x)
    if pad_mode == "reflect":
        y = F.conv2d(R.reflect_pad(x, k // 2), w, b, stride=stride)
    else:
        y = F.conv2d(x, w, b, stride=stride, padding=k // 2)
    if act == "relu":
        y = torch.relu(y)
    elif act == "tanh":
        y = torch.tanh(y / 255) * 150 + 255 / 2
    return y


@pytest.fixture(params=["bf16x3", "f32", "bf16", "bf16x6", "f16"])
def gemm_mode(request):
    """Runs a test in each GEMM arithmetic mode (the `mode` argument of every GEMM entry) and
    restores the policy in force before."""
    from vst import ops

    ops.gemm_role("fwd")  # applies the environment's policy first
    old = ops.POLICY_NAME[0]
    ops.set_gemm_mode(request.param, policy={})
    yield request.param
    ops.use_policy(old)


# max|err| / max|ref| per mode: fp32 MFMA and bf16x3 (per-product error <= ~2^-16) hold the
# 1e-4 op bar; single bf16 (2^-8 per product) and fp16 (2^-11 per operand) are the reduced-precision
# paths of config 5, where ReLU decisions flip near zero, so they are held to ||err|| / ||ref||
CONV_TOL = {"f32": 1e-4, "bf16x3": 1e-4, "bf16": 5e-2, "bf16x6": 1e-4, "f16": 1e-2}
# bf16 with a ReLU: the bias gradient sums the flipped mask entries too (measured up to 5.0e-2)
BF16_RELU_GRAD_TOL = 1e-1


def _norm_err(a, b):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _mode_err(mode, a, b, relu_grad=False):
    """max-abs error for exact-ish arithmetic; a ReLU's backward under bf16 products can flip
    the mask of a pre-activation within rounding of 0 (one element of the incoming gradient
    changes), so those gradients -- and everything in bf16 -- are held to ||err|| / ||ref||."""
    if mode in ("bf16", "f16") or (relu_grad and mode != "f32"):
        return _norm_err(a, b)
    return rel_err(a, b)


@pytest.mark.parametrize("case", CONV_CASES, ids=[f"{c[1]}-{c[4]}-k{c[5]}s{c[6]}{c[7][0]}u{c[8]}{c[9] or ''}" for c in CONV_CASES])
def test_conv_fwd_bwd(case, gemm_mode):
    from vst import ops

    tol = CONV_TOL[gemm_mode]
    N, Cin, H, W, Cout, k, stride, pad_mode, up, act = case
    g = torch.Generator().manual_seed(zlib.crc32(repr(case).encode()) % 1000)  # stable across processes
    x = torch.randn(N, Cin, H, W, generator=g) * (40.0 if act == "tanh" else 1.0)
    w = torch.randn(Cout, Cin, k, k, generator=g) * (2.0 / (Cin * k * k)) ** 0.5
    b = torch.randn(Cout, generator=g) * 0.1
    xr, wr, br = (t.clone().requires_grad_(True) for t in (x, w, b))
    yr = _oracle_conv(xr, wr, br, stride, pad_mode, up, act)
    gy = torch.randn(yr.shape, generator=g)
    yr.backward(gy)

    xg, wg, bg = (G(t).requires_grad_(True) for t in (x, w, b))
    pad = k // 2
    y = ops.conv2d(xg, wg, bg, stride=stride, pad=pad, pad_mode=pad_mode, up=up, act=act)
    assert y.shape == yr.shape
    assert _mode_err(gemm_mode, C(y), yr.detach()) < tol
    y.backward(G(gy))
    rg = act == "relu"
    gtol = (1e-3 if gemm_mode == "bf16x3" else BF16_RELU_GRAD_TOL if gemm_mode in ("bf16", "f16") else tol) if rg else tol
    assert _mode_err(gemm_mode, C(xg.grad), xr.grad, rg) < gtol
    assert _mode_err(gemm_mode, C(wg.grad), wr.grad, rg) < gtol
    assert _mode_err(gemm_mode, C(bg.grad), br.grad, rg) < gtol


def test_conv_relu_frozen_weights_dgrad_mask():
    """VGG path: frozen weights, ReLU mask fused into the dgrad gather (no relu_bwd pass)."""
    from vst import ops

    g = torch.Generator().manual_seed(7)
    x = torch.randn(2, 64, 10, 14, generator=g)
    w = torch.randn(64, 64, 3, 3, generator=g) * 0.06
    b = torch.randn(64, generator=g) * 0.1
    xr = x.clone().requires_grad_(True)
    y1 = torch.relu(F.conv2d(xr, w, b, padding=1))
    y2 = torch.relu(F.conv2d(y1, w, b, padding=1))
    gy = torch.randn(y2.shape, generator=g)
    y2.backward(gy)
    xg = G(x).requires_grad_(True)
    wg, bg = G(w), G(b)
    z1 = ops.conv2d(xg, wg, bg, pad=1, act="relu")
    z2 = ops.conv2d(z1, wg, bg, pad=1, act="relu")
    z2.backward(G(gy))
    assert rel_err(C(z2), y2.detach()) < 1e-4
    assert rel_err(C(xg.grad), xr.grad) < 1e-4


@pytest.mark.parametrize("mode", ["f32", "bf16x6", "f16"])
@pytest.mark.parametrize("cmid,cout", [(32, 48), (64, 3)])
def test_reflect_conv_relu_chain_masked_dgrad(mode, cmid, cout):
    """AdaAttN decoder chain (AA/network.py:24-33, 79-99): reflect-pad conv + ReLU whose output only
    feeds the next reflect-pad conv -> the producer skips its ReLU-backward pass (premasked) and the
    consumer's data gradient applies the mask in its padded-grid epilogue and border fold (mask_dx;
    cout = 3 takes the kw-unfolded thin path).  Input and weight gradients vs fp32 torch."""
    from vst import ops

    g = torch.Generator().manual_seed(11)
    x = torch.randn(2, 16, 11, 19, generator=g)
    w1 = torch.randn(cmid, 16, 3, 3, generator=g) * 0.15
    b1 = torch.randn(cmid, generator=g) * 0.1
    w2 = torch.randn(cout, cmid, 3, 3, generator=g) * 0.1
    b2 = torch.randn(cout, generator=g) * 0.1
    ref = [t.clone().requires_grad_(True) for t in (x, w1, b1, w2, b2)]
    y1 = torch.relu(F.conv2d(R.reflect_pad(ref[0], 1), ref[1], ref[2]))
    y2 = F.conv2d(R.reflect_pad(y1, 1), ref[3], ref[4])
    gy = torch.randn(y2.shape, generator=g)
    y2.backward(gy)
    ops.gemm_role("fwd")
    old = ops.POLICY_NAME[0]
    ops.set_gemm_mode(mode, policy={})
    try:
        hip = [G(t).requires_grad_(True) for t in (x, w1, b1, w2, b2)]
        z1 = ops.conv2d(hip[0], hip[1], hip[2], pad=1, pad_mode="reflect", act="relu", premasked=True)
        z2 = ops.conv2d(z1, hip[3], hip[4], pad=1, pad_mode="reflect", mask_dx=True)
        z2.backward(G(gy))
        torch.cuda.synchronize()
    finally:
        ops.use_policy(old)
    # fp16: 2^-11 products, and the fp16 forward's ReLU decisions near 0 differ from fp32's, which moves
    # the masked gradients (the conv tests' BF16_RELU_GRAD_TOL reasoning)
    tol = 1e-2 if mode == "f16" else 1e-4
    assert _norm_err(C(z2), y2.detach()) < tol
    for a, b_, nm in zip(hip, ref, ("dx", "dw1", "db1", "dw2", "db2")):
        assert _norm_err(C(a.grad), b_.grad) < (5e-2 if mode == "f16" else tol), nm


def test_vgg_slice_fused_relu_backward():
    """run_vgg_slice: ReLU outputs consumed only by the next conv / pool get their backward mask
    from the consumer (dgrad epilogue, pool backward); the slice output keeps its own pass."""
    import torch.nn as nn

    from vst.reconet.network import run_vgg_slice

    g = torch.Generator().manual_seed(9)
    seq = nn.Sequential(nn.Conv2d(16, 32, 3, padding=1), nn.ReLU(), nn.Conv2d(32, 32, 3, padding=1), nn.ReLU(),
                        nn.MaxPool2d(2, 2), nn.Conv2d(32, 48, 3, padding=1), nn.ReLU(), nn.Conv2d(48, 48, 3, padding=1),
                        nn.ReLU())
    for prm in seq.parameters():
        prm.requires_grad_(False)
        prm.copy_(torch.randn(prm.shape, generator=g) * 0.15)
    x = torch.randn(2, 16, 12, 18, generator=g)
    xr = x.clone().requires_grad_(True)
    ref = seq(xr)
    gy = torch.randn(ref.shape, generator=g)
    ref.backward(gy)
    xg = G(x).requires_grad_(True)
    out = run_vgg_slice(seq.to(DEV), xg)
    out.backward(G(gy))
    assert rel_err(C(out), ref.detach()) < 1e-4
    assert rel_err(C(xg.grad), xr.grad) < 1e-4


@pytest.mark.parametrize("relu,res,shape", [(True, False, (2, 48, 16, 20)), (False, True, (2, 192, 9, 15)),
                                            (True, False, (1, 96, 64, 128)),
                                            # the one-pass LDS backward (8192 < HW <= 32768, HW % 4 == 0):
                                            # recomputed ReLU mask, mask from y (residual), partial last column
                                            (True, False, (2, 8, 128, 256)), (True, True, (2, 6, 96, 200)),
                                            (False, False, (1, 5, 100, 120)),
                                            # the two-pass kernels: HW > 32768, and HW % 4 != 0
                                            (True, False, (1, 4, 256, 260)), (True, False, (1, 3, 101, 103))])
def test_instance_norm(relu, res, shape):
    from vst import ops

    g = torch.Generator().manual_seed(3)
    x = torch.randn(shape, generator=g) * 3 + 1.5
    w = 1 + 0.1 * torch.randn(shape[1], generator=g)
    b = 0.1 * torch.randn(shape[1], generator=g)
    r = torch.randn(shape, generator=g)
    xr, wr, br, rr = (t.clone().requires_grad_(True) for t in (x, w, b, r))
    yr = R.instance_norm(xr, wr, br)
    if relu:
        yr = torch.relu(yr)
    if res:
        yr = yr + rr
    gy = torch.randn(shape, generator=g)
    yr.backward(gy)
    xg, wg, bg, rg = (G(t).requires_grad_(True) for t in (x, w, b, r))
    y = ops.instance_norm(xg, wg, bg, relu=relu, res=rg if res else None)
    y.backward(G(gy))
    assert rel_err(C(y), yr.detach()) < 1e-5
    assert rel_err(C(xg.grad), xr.grad) < 1e-4
    assert rel_err(C(wg.grad), wr.grad) < 1e-4
    assert rel_err(C(bg.grad), br.grad) < 1e-4
    if res:
        assert rel_err(C(rg.grad), rr.grad) < 1e-6


def test_pool_warp_gram_losses_bwd():
    from vst import ops

    g = torch.Generator().manual_seed(11)
    # maxpool (odd size drops the trailing row/col)
    x = torch.randn(2, 8, 9, 15, generator=g)
    xr = x.clone().requires_grad_(True)
    yr = R.maxpool2x2(xr)
    gy = torch.randn(yr.shape, generator=g)
    yr.backward(gy)
    xg = G(x).requires_grad_(True)
    y = ops.maxpool2x2(xg)
    y.backward(G(gy))
    assert torch.equal(C(y), yr.detach()) and rel_err(C(xg.grad), xr.grad) < 1e-6
    # warp backward (gather form)
    x = torch.randn(2, 5, 12, 20, generator=g)
    flo = torch.rand(2, 2, 12, 20, generator=g) * 8 - 4
    xr = x.clone().requires_grad_(True)
    yr = R.warp(xr, flo)
    gy = torch.randn(yr.shape, generator=g)
    yr.backward(gy)
    xg = G(x).requires_grad_(True)
    y = ops.warp(xg, G(flo))
    y.backward(G(gy))
    assert rel_err(C(y), yr.detach()) < 1e-5 and rel_err(C(xg.grad), xr.grad) < 1e-5
    # gram + broadcast style MSE backward
    f = torch.randn(3, 64, 7, 9, generator=g)
    gs = torch.randn(1, 64, 64, generator=g) * 0.1
    fr = f.clone().requires_grad_(True)
    lr_ = F.mse_loss(R.gram_matrix(fr), gs.expand(3, -1, -1)) * 7.0
    lr_.backward()
    fg = G(f).requires_grad_(True)
    lg = ops.mse(ops.gram_matrix(fg), G(gs), 7.0)
    lg.backward()
    assert rel_err(C(lg), lr_.detach()) < 1e-5 and rel_err(C(fg.grad), fr.grad) < 1e-4
    # TV
    s = torch.randn(2, 3, 10, 13, generator=g)
    sr = s.clone().requires_grad_(True)
    tr = 0.5 * torch.sum((sr[:, :, :-1, 1:] - sr[:, :, :-1, :-1]) ** 2 + (sr[:, :, 1:, :-1] - sr[:, :, :-1, :-1]) ** 2)
    tr.backward()
    sg = G(s).requires_grad_(True)
    tg = ops.tv_loss(sg, 0.5)
    tg.backward()
    assert rel_err(C(tg), tr.detach()) < 1e-5 and rel_err(C(sg.grad), sr.grad) < 1e-5


@pytest.mark.parametrize("flow", ["random", "converging"])
def test_warp_bwd_gather(flow):
    """Gather-form warp backward vs the oracle's autograd, with more channels than one channel
    group and (converging) flows that overflow the per-source tap lists (atomic excess pass)."""
    from vst import ops

    g = torch.Generator().manual_seed(21)
    B, Cc, H, W = 2, 19, 10, 24
    x = torch.randn(B, Cc, H, W, generator=g)
    if flow == "random":
        flo = torch.rand(B, 2, H, W, generator=g) * 6 - 3
    else:  # every pixel of a row samples near column 5 / row 4: dozens of taps per source pixel
        xs = torch.arange(W, dtype=torch.float32).view(1, 1, W).expand(B, H, W)
        ys = torch.arange(H, dtype=torch.float32).view(1, H, 1).expand(B, H, W)
        flo = torch.stack([5.3 - xs, 4.6 - ys], 1) + torch.rand(B, 2, H, W, generator=g) * 0.2
    xr = x.clone().requires_grad_(True)
    yr = R.warp(xr, flo)
    gy = torch.randn(yr.shape, generator=g)
    yr.backward(gy)
    xg = G(x).requires_grad_(True)
    y = ops.warp(xg, G(flo))
    y.backward(G(gy))
    assert rel_err(C(xg.grad), xr.grad) < 1e-5


# ----------------------------------------------------------------------------- models vs golden
def _seeded(module, spec, seed):
    params = oracle.seeded_params(spec, seed)
    sd = module.state_dict()
    assert sorted(sd) == sorted(params), "state_dict keys differ from the reference"
    module.load_state_dict({k: v for k, v in params.items()})
    return module


def test_state_dict_keys_match_reference():
    from vst.reconet import network as N

    for cls, spec in ((N.ReCoNet, shapes.reconet()), (N.ReCoNetSD1, shapes.reconet_sd1()),
                      (N.ReCoNetSD2, shapes.reconet_sd2()), (N.Vgg16, shapes.vgg16())):
        sd = cls().state_dict()
        assert [(k, tuple(v.shape)) for k, v in sd.items()] == [(k, tuple(s)) for k, s in spec], cls.__name__


def test_reconet_vgg16_forward_golden(golden):
    from vst.reconet import network as N

    f = golden("rc_fwd")
    m = _seeded(N.ReCoNet(), shapes.reconet(), 1).to(DEV)
    with torch.no_grad():
        for tag in ("a", "ragged"):
            sd1, feat, out = m(G(f[f"reconet_{tag}_x"]))
            assert rel_err(C(sd1), f[f"reconet_{tag}_sd1"]) < 1e-3
            assert rel_err(C(feat), f[f"reconet_{tag}_features"]) < 1e-3
            assert rel_err(C(out), f[f"reconet_{tag}_out"]) < 1e-3
        v = _seeded(N.Vgg16(), shapes.vgg16(), 4).to(DEV)
        outs = v(G(f["vgg16_x"]))
        for name in outs._fields:
            assert rel_err(C(getattr(outs, name)), f["vgg16_" + name]) < 1e-3, name


def test_sd_checkpoints_forward_golden(golden):
    from vst.reconet import network as N

    f = golden("rc_fwd")
    ck = golden("rc_sd_ckpt")
    for cls in (N.ReCoNetSD1, N.ReCoNetSD2):
        net = cls()
        net.load_state_dict({k.split("/", 1)[1]: T(v) for k, v in ck.items() if k.startswith(cls.__name__ + "/")})
        net = net.to(DEV)
        with torch.no_grad():
            outs = net(G(f["sd_x"]))
        for i, o in enumerate(outs):
            assert rel_err(C(o), f[f"{cls.__name__}_out{i}"]) < 1e-3, (cls.__name__, i)


@pytest.mark.parametrize("tag", ["b2", "b1r"])
def test_train_step_golden(golden, tag, step_policy):
    """One full train_candy step (losses, gradients, Adam update) vs the reference's own train()."""
    from vst.reconet import network as N
    from vst.reconet.train import ReCoNetTrainer

    s = golden("rc_step")
    seeds = s[f"{tag}_seeds"]
    model = _seeded(N.ReCoNet(), shapes.reconet(), int(seeds[0])).to(DEV)
    vgg = _seeded(N.Vgg16(), shapes.vgg16(), int(seeds[1])).to(DEV)
    tr = ReCoNetTrainer(model, vgg, G(s[f"{tag}_style"]))
    frames = torch.stack([G(s[f"{tag}_img1"]), G(s[f"{tag}_img2"])])
    out = tr.losses(frames, G(s[f"{tag}_flow"]), G(s[f"{tag}_mask"]))
    for k in ("loss", "CL", "SL", "FTL", "OTL", "RL"):
        assert rel_err(out[k].item(), s[f"{tag}_{k}"]) < 1e-3, k
    tr.flat.zero_grad()
    out["loss"].backward()
    names = list(s[f"{tag}_names"])
    named = dict(model.named_parameters())
    gmax = max(float(s[f"{tag}_gnorm/{n}"]) for n in names)
    for n in names:
        gr = C(named[n].grad).reshape(-1)
        gn = float(s[f"{tag}_gnorm/{n}"])
        assert abs(float(gr.double().norm()) - gn) <= 1e-3 * gn + 1e-4 * gmax, n
        idx = s[f"{tag}_gidx/{n}"]
        assert np.abs(gr[idx].numpy() - s[f"{tag}_gval/{n}"]).max() <= 1e-3 * gn + 1e-4 * gmax, n
    tr.step_count = 0
    tr.flat.adam(1, tr.lr, tr.betas, tr.eps)
    for n in names:
        gh = s[f"{tag}_ghead/{n}"]
        sel = np.abs(gh) > 1e-6 * gmax + 1e-2 * np.abs(gh).max()
        got = C(named[n]).reshape(-1)[:64].numpy()
        assert np.abs(got - s[f"{tag}_phead/{n}"])[sel].max(initial=0) < 1e-5, n


@pytest.mark.parametrize("term", ["FTL", "OTL", "CL", "SL", "RL"])
@pytest.mark.parametrize("tag", ["b2", "b1r"])
def test_train_step_per_term_golden(golden, tag, term, step_policy):
    """Each train_candy loss term ALONE through the HIP trainer (`terms=(term,)`) vs the reference's
    own train() with the other four weight constants zeroed and vs the float64 gradient of the same
    term (tests/golden/rc_terms.npz).  At the seeded init FTL is >99.99 % of every stylizer gradient
    of the full step, so this is the check that pins the OTL, content, Gram-style and TV backward.
    Bar (conftest.term_grad_margins): term value 1e-4 relative; every gradient tensor's norm and 256
    sampled elements within TERM_REL = 2e-3 of that tensor's OWN exact norm (or 4x the reference's own
    fp32 error, where that is larger -- the ConvTanh bias under OTL / TV); tensors whose exact gradient
    is zero (conv biases feeding InstanceNorm; the decoder under FTL) below 1e-5 of the largest norm.
    (Why 2e-3 and not fp32 rounding: conftest.TERM_REL; the decision-independent 2e-5 check of every
    block's backward under each term is test_stylizer_block_chain_per_term.)"""
    import conftest
    from vst.reconet import network as N
    from vst.reconet.train import ReCoNetTrainer

    d = golden("rc_terms")
    seeds = d[f"{tag}_seeds"]
    model = _seeded(N.ReCoNet(), shapes.reconet(), int(seeds[0])).to(DEV)
    vgg = _seeded(N.Vgg16(), shapes.vgg16(), int(seeds[1])).to(DEV)
    tr = ReCoNetTrainer(model, vgg, G(d[f"{tag}_style"]), terms=(term,))
    frames = torch.stack([G(d[f"{tag}_img1"]), G(d[f"{tag}_img2"])])
    out = tr.losses(frames, G(d[f"{tag}_flow"]), G(d[f"{tag}_mask"]))
    p = f"{tag}_{term}_"
    assert rel_err(out["loss"].item(), d[p + "term"]) < 1e-4, (out["loss"].item(), float(d[p + "term"]))
    tr.flat.zero_grad()
    out["loss"].backward()
    grads = {n: C(v.grad if v.grad is not None else torch.zeros_like(v)).numpy()
             for n, v in model.named_parameters()}
    m = conftest.term_grad_margins(d, p, grads)
    worst = sorted(m, key=m.get)[-3:]
    print(f"per-term {tag} {term} {step_policy}: worst margins", {n: round(m[n], 3) for n in worst})
    assert m[worst[-1]] <= 1.0, (worst[-1], m[worst[-1]])


# Block chain: every stylizer block's backward, driven by each loss term's own EXACT gradient signal.
# The float64 oracle runs the one-term step (rc_terms case) and records each block's input and the
# exact gradient at its output; the HIP block then gets that input (rounded to fp32) and that
# gradient, and its input gradient and parameter gradients are compared with the float64 backward of
# the same block on the same rounded input.  Unlike the whole-step check, an fp32 ReLU / InstanceNorm
# decision that flips far upstream cannot move these numbers, so the bar is near fp32 rounding.
BLOCK_TOL = 2e-5
BLOCKS = (("conv1", 9, 1, False), ("conv2", 3, 2, False), ("conv3", 3, 2, False), ("res1",), ("res2",), ("res3",),
          ("res4",), ("res5",), ("deconv1", 3, 1, True), ("deconv2", 3, 1, True), ("deconv3", 9))


def _oracle_block(P, name, spec, x):
    if name.startswith("res"):
        return R.residual_block(x, P, name)
    if name == "deconv3":
        return R.conv_tanh(x, P, name, 9)
    _, k, s, up = spec
    return R.conv_in_relu(x, P, name, k, s, upsample=up)


def _exact_block_io(d, tag, term):
    """float64 one-term step: {block: (input, gradient at output)}."""
    seeds = d[f"{tag}_seeds"]
    P = {k: v.double().requires_grad_(True) for k, v in oracle.seeded_params(shapes.reconet(), int(seeds[0])).items()}
    VP = {k: v.double() for k, v in oracle.seeded_params(shapes.vgg16(), int(seeds[1])).items()}
    io = {b[0]: ([], []) for b in BLOCKS}

    def fwd(P_, x):
        outs = {}
        for spec in BLOCKS:
            io[spec[0]][0].append(x.detach())
            y = _oracle_block(P_, spec[0], spec, x)
            y.retain_grad()
            io[spec[0]][1].append(y)
            outs[spec[0]] = y
            x = y
        # vgg_normalize_ divides the styled output in place: hand it a copy
        return outs["deconv1"], outs["res5"], outs["deconv3"] * 1.0

    T = lambda k: torch.from_numpy(d[f"{tag}_{k}"]).double()  # noqa: E731
    L = R.reconet_losses(P, VP, T("img1").clone(), T("img2").clone(), T("flow"), T("mask"),
                         R.style_grams(VP, T("style")), forward=fwd, terms=(term,))
    L["loss"].backward()
    return P, {b: (torch.cat(xs), torch.cat([y.grad if y.grad is not None else torch.zeros_like(y) for y in ys]))
               for b, (xs, ys) in io.items()}


@pytest.mark.parametrize("term", ["FTL", "OTL", "CL", "SL", "RL"])
@pytest.mark.parametrize("tag", ["b2", "b1r"])
def test_stylizer_block_chain_per_term(golden, tag, term, step_policy):
    """Each ReCoNet block (conv1..3, res1..5, deconv1..3) backward on HIP under each loss term's exact
    gradient signal: input gradient and every parameter gradient within BLOCK_TOL (norm-wise, of the
    tensor's own float64 norm; conv biases feeding InstanceNorm, whose exact gradient is 0, below
    BLOCK_TOL of the block's largest parameter-gradient norm; the ConvTanh bias gradient, a plain sum
    over every pixel with heavy cancellation under OTL / TV, additionally gets the fp32 summation bound
    64 ulp x the sum of magnitudes -- the reference's own fp32 value sits 2.5e-4..6e-4 from exact
    there).  Parameter gradients go through the in-place .grad sinks as in the trainer."""
    from vst import ops
    from vst.reconet import network as N

    d = golden("rc_terms")
    P64, io = _exact_block_io(d, tag, term)
    model = _seeded(N.ReCoNet(), shapes.reconet(), int(d[f"{tag}_seeds"][0])).to(DEV)
    worst = (0.0, None)
    for spec in BLOCKS:
        name = spec[0]
        x64, gy64 = io[name]
        if float(gy64.norm()) == 0.0:
            continue  # the term does not reach this block (FTL: the decoder)
        need_dx = name != "conv1"
        xr = x64.float().double().requires_grad_(need_dx)
        Pb = {k: v.detach().clone().requires_grad_(True) for k, v in P64.items() if k.startswith(name + ".")}
        if name == "deconv3":  # ConvTanh: keep the pre-tanh gradient, whose plain sum is the bias gradient
            z = R.conv_layer(xr, Pb, name, 9, 1)
            z.retain_grad()
            (torch.tanh(z / 255) * 150 + 255 / 2).backward(gy64)
            # fp32 summation bound of a sum with cancellation: 64 ulp of the sum of magnitudes
            bias_l1 = 64 * 2.0 ** -24 * float(z.grad.abs().sum(dim=(0, 2, 3)).norm())
        else:
            _oracle_block(Pb, name, spec, xr).backward(gy64)
            bias_l1 = 0.0
        mod = getattr(model, name)
        for p in mod.parameters():
            p.grad = torch.zeros_like(p)
        xg = G(xr.detach().float()).requires_grad_(need_dx)
        with ops.gemm_scope("stylizer"):
            yg = mod(xg)
        yg.backward(G(gy64.float()))
        errs = {}
        if need_dx:
            errs["dx"] = _norm_err(C(xg.grad), xr.grad)
        named = dict(mod.named_parameters())
        pmax = max(float(v.grad.norm()) for v in Pb.values())
        for k, v in Pb.items():
            got = C(named[k[len(name) + 1:]].grad).double()
            e = float(v.grad.norm())
            if e < 1e-6 * pmax:
                errs[k] = float(got.norm()) / pmax
            elif k.endswith("conv2d.bias") and bias_l1:
                errs[k] = float((got - v.grad).norm()) / (e + bias_l1 / BLOCK_TOL)
            else:
                errs[k] = float((got - v.grad).norm()) / e
        k = max(errs, key=errs.get)
        if errs[k] > worst[0]:
            worst = (errs[k], f"{name}:{k}")
        assert errs[k] <= BLOCK_TOL, (name, k, errs[k])
    print(f"block chain {tag} {term} {step_policy}: worst {worst[0]:.2e} ({worst[1]})")


CLONE_SCRIPTS = {"coco": ("train_coco2014", 1), "cocor": ("train_coco2014", 1), "noftl": ("train_Flow_noFTL", 1),
                 "multi": ("train_Flow", 4)}


@pytest.mark.parametrize("tag", sorted(CLONE_SCRIPTS))
def test_clone_train_step_golden(golden, tag, step_policy):
    """The reference's loop-body clones on HIP vs their own train(): train_coco2014 (BASELINE config 2:
    single images, content + style only), train_Flow_noFTL (no FTL) and train_multiple/train_Flow
    (input_frame_num = 4, 12-channel conv1, VGG on the last frame's channels).  Losses 1e-3
    relative; every gradient tensor's norm and 256 sampled elements within 1e-3 of its norm
    (+1e-4 of the largest); the post-Adam parameter heads 1e-5."""
    from vst.reconet import network as N
    from vst.reconet.train import ReCoNetTrainer

    s = golden("rc_clones")
    script, nfr = CLONE_SCRIPTS[tag]
    seeds = s[f"{tag}_seeds"]
    model = _seeded(N.ReCoNet(nfr), shapes.reconet(nfr), int(seeds[0])).to(DEV)
    vgg = _seeded(N.Vgg16(), shapes.vgg16(), int(seeds[1])).to(DEV)
    tr = ReCoNetTrainer.for_script(script, model, vgg, G(s[f"{tag}_style"]))
    terms = sorted(s[f"{tag}_terms"])
    assert sorted(tr.terms) == terms
    if tr.single:
        out = tr.losses(G(s[f"{tag}_img"]))
    else:
        frames = torch.stack([G(s[f"{tag}_img1"]), G(s[f"{tag}_img2"])])
        out = tr.losses(frames, G(s[f"{tag}_flow"]), G(s[f"{tag}_mask"]))
    for k in ["loss"] + terms:
        assert rel_err(out[k].item(), s[f"{tag}_{k}"]) < 1e-3, k
    tr.flat.zero_grad()
    out["loss"].backward()
    names = list(s[f"{tag}_names"])
    named = dict(model.named_parameters())
    gmax = max(float(s[f"{tag}_gnorm/{n}"]) for n in names)
    for n in names:
        gr = C(named[n].grad).reshape(-1)
        gn = float(s[f"{tag}_gnorm/{n}"])
        assert abs(float(gr.double().norm()) - gn) <= 1e-3 * gn + 1e-4 * gmax, n
        idx = s[f"{tag}_gidx/{n}"]
        assert np.abs(gr[idx].numpy() - s[f"{tag}_gval/{n}"]).max() <= 1e-3 * gn + 1e-4 * gmax, n
    tr.flat.adam(1, tr.lr, tr.betas, tr.eps)
    for n in names:
        gh = s[f"{tag}_ghead/{n}"]
        sel = np.abs(gh) > 1e-6 * gmax + 1e-2 * np.abs(gh).max()
        got = C(named[n]).reshape(-1)[:64].numpy()
        assert np.abs(got - s[f"{tag}_phead/{n}"])[sel].max(initial=0) < 1e-5, n


def test_sd2_distillation_step_golden(golden):
    """One train_Flow_SD2 step (student ReCoNetSD2, teacher ReCoNetSD1) vs the reference's own train()."""
    from vst.reconet import network as N
    from vst.reconet.train import SD_LOSS_WEIGHTS, ReCoNetTrainer

    s = golden("sd_step")
    seeds = s["sd2_seeds"]
    teacher = _seeded(N.ReCoNetSD1(), shapes.reconet_sd1(), int(seeds[0]))
    student = _seeded(N.ReCoNetSD2(), shapes.reconet_sd2(), int(seeds[1]))
    student.load_state_dict(teacher.state_dict(), strict=False)  # train_Flow_SD2.py:45
    teacher, student = teacher.to(DEV).eval(), student.to(DEV)
    vgg = _seeded(N.Vgg16(), shapes.vgg16(), int(seeds[2])).to(DEV)
    tr = ReCoNetTrainer(student, vgg, G(s["sd2_style"]), weights=SD_LOSS_WEIGHTS, teacher=teacher, sd_index=(0, 0))
    frames = torch.stack([G(s["sd2_img1"]), G(s["sd2_img2"])])
    tr.flat.zero_grad()
    out = tr.losses(frames, G(s["sd2_flow"]), G(s["sd2_mask"]))
    for k in ("loss", "CL", "SL", "FTL", "OTL", "RL", "SDL"):
        assert rel_err(out[k].item(), s[f"sd2_{k}"]) < 1e-3, k
    out["loss"].backward()
    names = list(s["sd2_names"])
    named = dict(student.named_parameters())
    gmax = max(float(s[f"sd2_gnorm/{n}"]) for n in names)
    for n in names:
        gr = C(named[n].grad).reshape(-1)
        gn = float(s[f"sd2_gnorm/{n}"])
        assert abs(float(gr.double().norm()) - gn) <= 1e-3 * gn + 1e-4 * gmax, n
        idx = s[f"sd2_gidx/{n}"]
        assert np.abs(gr[idx].numpy() - s[f"sd2_gval/{n}"]).max() <= 1e-3 * gn + 1e-4 * gmax, n


def test_fit_loop_sync_free_log(tmp_path):
    """vst.reconet.loop.fit over a FramePairLoader-shaped batch stream with StepLog: the JSONL
    means equal the per-step loss terms the trainer returned (read back only at the end), and the
    epoch checkpoint has the reference's state_dict keys."""
    import json

    from vst.reconet import network as N
    from vst.reconet.loop import StepLog, fit
    from vst.reconet.train import ReCoNetTrainer
    from vst.synthetic import frame_pair_batch, style_image

    model = _seeded(N.ReCoNet(), shapes.reconet(), 1).to(DEV)
    vgg = _seeded(N.Vgg16(), shapes.vgg16(), 2).to(DEV)
    tr = ReCoNetTrainer(model, vgg, G(style_image(3, 32, 64)))
    batches = [tuple(G(t) for t in frame_pair_batch(40 + i, 1, 32, 64, mask_fn=R.flow_warp_mask)) for i in range(3)]
    outs = []
    step = tr.step
    tr.step = lambda *a: outs.append(step(*a)) or outs[-1]
    log = StepLog(str(tmp_path / "log.jsonl"), every=2, units_per_step=1)
    fit(tr, batches, epochs=1, log=log, checkpoint=str(tmp_path / "ckpt_{epoch}.pth"))
    recs = [json.loads(line) for line in open(tmp_path / "log.jsonl")]
    assert [r["steps"] for r in recs] == [2, 1]
    for k in ("loss", "FTL", "OTL", "CL", "SL", "RL"):
        vals = [float(o[k]) for o in outs]
        assert abs(recs[0][k] - (vals[0] + vals[1]) / 2) <= 1e-6 * abs(recs[0][k]), k
        assert abs(recs[1][k] - vals[2]) <= 1e-6 * abs(recs[1][k]), k
    sd = torch.load(tmp_path / "ckpt_1.pth", weights_only=True)
    assert sorted(sd) == sorted(n for n, _ in shapes.reconet())
