"""CPU restatement of the reference RTNSTV training path.  TEST INFRASTRUCTURE ONLY.

Plain torch-CPU fp32 ops written from RT/network.py, RT/vgg19.py, RT/utilities.py and
RT/train.py (not imported from them), pinned against golden vectors produced by running the
reference's own train() (`tests/golden/gen_golden.py rtnstv` -> tests/golden/rt_step.npz).
Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s cpu_baseline leg may import it.
"""
import torch
import torch.nn.functional as F

from .reconet_ref import (IMAGENET_MEAN, IMAGENET_STD, instance_norm, reflect_pad, vgg_forward,  # noqa: F401
                          warp)

LOSS_WEIGHTS = dict(ALPHA=1e7, BETA=5e7, GAMMA=5e-1, LAMBDA=1e6)  # RT/train.py:28-31
# torchvision VGG19 features[0:23] split at relu1_2 / relu2_2 / relu3_2 / relu4_2 (RT/vgg19.py:18-32)
VGG19_RT_PLAN = [
    [(1, 0), (1, 2)],
    ["M", (2, 5), (2, 7)],
    ["M", (3, 10), (3, 12)],
    [(4, 14), (4, 16), "M", (4, 19), (4, 21)],
]


def conv(x, P, name, k, stride, act=None):
    """Conv (RT/network.py:10-26): reflect pad k//2 -> conv -> IN(affine) -> act."""
    y = F.conv2d(reflect_pad(x, k // 2), P[name + ".conv.weight"], P[name + ".conv.bias"], stride=stride)
    y = instance_norm(y, P[name + ".norm.weight"], P[name + ".norm.bias"])
    return act(y) if act is not None else y


def deconv(x, P, name, act=torch.relu):
    """Deconv (RT/network.py:49-62): ConvTranspose2d(k3, s2, p1, op1) -> IN -> act."""
    y = F.conv_transpose2d(x, P[name + ".deconv.weight"], P[name + ".deconv.bias"], stride=2, padding=1,
                           output_padding=1)
    y = instance_norm(y, P[name + ".norm.weight"], P[name + ".norm.bias"])
    return act(y) if act is not None else y


def stylizer_forward(P, x):
    """StylizingNetwork.forward (RT/network.py:80-94)."""
    x = conv(x, P, "conv1", 3, 1, torch.relu)
    x = conv(x, P, "conv2", 3, 2, torch.relu)
    x = conv(x, P, "conv3", 3, 2, torch.relu)
    for i in range(1, 6):
        x = conv(conv(x, P, f"res{i}.conv1", 3, 1, torch.relu), P, f"res{i}.conv2", 3, 1) + x
    x = deconv(x, P, "deconv1")
    x = deconv(x, P, "deconv2")
    x = conv(x, P, "conv4", 3, 1, torch.tanh)
    return (x + 1) / 2 * 255


def vgg_normalize(x):
    """RT/utilities.py:163-169 (out of place)."""
    mean = torch.tensor(IMAGENET_MEAN, dtype=x.dtype).view(-1, 1, 1)
    std = torch.tensor(IMAGENET_STD, dtype=x.dtype).view(-1, 1, 1)
    return (x / 255.0 - mean) / std


def vgg19(VP, x):
    return vgg_forward(VP, vgg_normalize(x), VGG19_RT_PLAN)


def gram_matrix(y):
    """RT/utilities.py:155-160: F F^T / (H W)."""
    b, c, h, w = y.shape
    f = y.reshape(b, c, h * w)
    return f.bmm(f.transpose(1, 2)) / (h * w)


def style_grams(VP, style):
    with torch.no_grad():
        return [gram_matrix(f) for f in vgg19(VP, style)]


def spatial_loss(content, styled, grams, VP, w=LOSS_WEIGHTS):
    """RT/train.py:36-61."""
    cf = vgg19(VP, content)[3]
    sf = vgg19(VP, styled)
    cl = F.mse_loss(cf, sf[3]) * w["ALPHA"]
    sl = 0
    for gs, f in zip(grams, sf):
        g = gram_matrix(f)
        sl = sl + F.mse_loss(g, gs.expand(g.shape[0], -1, -1))
    reg1 = (styled[:, :, :-1, 1:] - styled[:, :, :-1, :-1]) ** 2
    reg2 = (styled[:, :, 1:, :-1] - styled[:, :, :-1, :-1]) ** 2
    rl = torch.sqrt((reg1 + reg2).clamp(min=1e-8)).mean() * w["GAMMA"]
    return cl, sl * w["BETA"], rl


def rtnstv_losses(P, VP, img1, img2, flow, mask, grams, w=LOSS_WEIGHTS):
    """One RT/train.py step's loss terms (:117-139): dict(loss, CL, SL, RL, TL)."""
    s1 = stylizer_forward(P, img1)
    s2 = stylizer_forward(P, img2)
    c1, st1, r1 = spatial_loss(img1, s1, grams, VP, w)
    c2, st2, r2 = spatial_loss(img2, s2, grams, VP, w)
    m = mask.unsqueeze(1).expand(-1, s2.shape[1], -1, -1)
    tl = (m * (s2 - warp(s1, flow)) ** 2).sum() / (m.sum() + 1e-8) * w["LAMBDA"]
    out = {"CL": c1 + c2, "SL": st1 + st2, "RL": r1 + r2, "TL": tl}
    out["loss"] = out["CL"] + out["SL"] + out["RL"] + out["TL"]
    return out
