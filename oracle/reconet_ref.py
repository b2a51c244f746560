"""CPU restatement of the reference ReCoNet training path.  TEST INFRASTRUCTURE ONLY.

This is the oracle the HIP path is checked against: plain torch-CPU fp32 ops, written from
the reference's semantics (not imported from it), pinned against golden vectors produced by
running the reference itself (`tests/golden/gen_golden.py` -> tests/golden/rc_*.npz).
Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s cpu_baseline leg may import it;
the product path (`video-style-transfer_amd/vst`) never does.

Parameters travel as plain dicts keyed exactly like the reference's state_dicts
(`conv1.conv2d.weight`, `res1.in1.bias`, `slice1.0.weight`, ...).
Gradients come from torch autograd over this restatement.
"""
import numpy as np
import torch
import torch.nn.functional as F

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


# ------------------------------------------------------------------ elementary ops
def reflect_index(n, p):
    """Indices of ReflectionPad (no edge repeat) for a length-n axis padded by p each side."""
    i = np.arange(-p, n + p)
    i = np.abs(i)
    i = np.where(i > n - 1, 2 * (n - 1) - i, i)
    return torch.from_numpy(i.astype(np.int64))


def reflect_pad(x, p):
    """`torch.nn.ReflectionPad2d(p)` (RC/network.py:68-69,73)."""
    if p == 0:
        return x
    H, W = x.shape[-2:]
    return x.index_select(-2, reflect_index(H, p)).index_select(-1, reflect_index(W, p))


def upsample_nearest2x(x):
    """`F.interpolate(x, scale_factor=2)` default mode 'nearest' (RC/network.py:117)."""
    return x.repeat_interleave(2, dim=-2).repeat_interleave(2, dim=-1)


def instance_norm(x, w, b, eps=1e-5):
    """`nn.InstanceNorm2d(C, affine=True)`: biased variance, eps 1e-5, no running stats."""
    mu = x.mean(dim=(2, 3), keepdim=True)
    var = ((x - mu) ** 2).mean(dim=(2, 3), keepdim=True)
    return (x - mu) / torch.sqrt(var + eps) * w.view(1, -1, 1, 1) + b.view(1, -1, 1, 1)


def conv_layer(x, P, name, k, stride, upsample=False):
    """ConvLayer / UpsampleConvLayer (RC/network.py:63-75, 101-120): [up x2] -> reflect -> conv."""
    if upsample:
        x = upsample_nearest2x(x)
    x = reflect_pad(x, k // 2)
    return F.conv2d(x, P[name + ".conv2d.weight"], P[name + ".conv2d.bias"], stride=stride)


def conv_in_relu(x, P, name, k, stride, upsample=False):
    """ConvInstRelu / UpsampleConvInstRelu (RC/network.py:88-98, 123-133)."""
    y = conv_layer(x, P, name, k, stride, upsample)
    return torch.relu(instance_norm(y, P[name + ".instance.weight"], P[name + ".instance.bias"]))


def conv_tanh(x, P, name, k):
    """ConvTanh (RC/network.py:78-85): tanh(y / 255) * 150 + 255 / 2."""
    return torch.tanh(conv_layer(x, P, name, k, 1) / 255) * 150 + 255 / 2


def residual_block(x, P, name):
    """ResidualBlock (RC/network.py:136-150): IN2(conv2(relu(IN1(conv1 x)))) + x (no final relu)."""
    h = conv_layer(x, P, name + ".conv1", 3, 1)
    h = torch.relu(instance_norm(h, P[name + ".in1.weight"], P[name + ".in1.bias"]))
    h = conv_layer(h, P, name + ".conv2", 3, 1)
    return instance_norm(h, P[name + ".in2.weight"], P[name + ".in2.bias"]) + x


# ------------------------------------------------------------------ models
def reconet_forward(P, x):
    """ReCoNet.forward (RC/network.py:153-190) -> (sd1, features, out)."""
    x = conv_in_relu(x, P, "conv1", 9, 1)
    x = conv_in_relu(x, P, "conv2", 3, 2)
    x = conv_in_relu(x, P, "conv3", 3, 2)
    for i in range(1, 6):
        x = residual_block(x, P, f"res{i}")
    features = x
    x = conv_in_relu(x, P, "deconv1", 3, 1, upsample=True)
    sd1 = x
    x = conv_in_relu(x, P, "deconv2", 3, 1, upsample=True)
    return sd1, features, conv_tanh(x, P, "deconv3", 9)


def reconet_sd1_forward(P, x):
    """ReCoNetSD1.forward (RC/network.py:193-237) -> (sd2, sd, features, out)."""
    x = conv_in_relu(x, P, "conv1", 9, 1)
    x = conv_in_relu(x, P, "conv2", 3, 2)
    x = conv_in_relu(x, P, "conv3_sd", 3, 2)
    sd2 = x
    for i in range(1, 6):
        x = residual_block(x, P, f"res{i}_sd")
    features = x
    x = conv_in_relu(x, P, "deconv1_sd", 3, 1, upsample=True)
    sd = x
    x = conv_in_relu(x, P, "deconv2", 3, 1, upsample=True)
    return sd2, sd, features, conv_tanh(x, P, "deconv3", 9)


def reconet_sd2_forward(P, x):
    """ReCoNetSD2.forward (RC/network.py:240-279) -> (sd, features, out)."""
    x = conv_in_relu(x, P, "conv1_sd2", 9, 1)
    x = conv_in_relu(x, P, "conv2_sd2", 3, 2)
    x = conv_in_relu(x, P, "conv3_sd2", 3, 2)
    sd = x
    for i in range(1, 6):
        x = residual_block(x, P, f"res{i}_sd")
    features = x
    x = conv_in_relu(x, P, "deconv1_sd2", 3, 1, upsample=True)
    x = conv_in_relu(x, P, "deconv2_sd2", 3, 1, upsample=True)
    return sd, features, conv_tanh(x, P, "deconv3_sd2", 9)


# torchvision VGG16 features[0:23] split at relu1_2/2_2/3_3/4_3 (RC/network.py:9-40):
# (slice, torchvision index) per conv, "M" = MaxPool2d(2, 2)
VGG16_PLAN = [
    [(1, 0), (1, 2)],
    ["M", (2, 5), (2, 7)],
    ["M", (3, 10), (3, 12), (3, 14)],
    ["M", (4, 17), (4, 19), (4, 21)],
]
# torchvision VGG19 features[0:30] split at relu1_1..relu5_1 (AA/vgg19.py:19-37)
VGG19_PLAN = [
    [(1, 0)],
    [(2, 2), "M", (2, 5)],
    [(3, 7), "M", (3, 10)],
    [(4, 12), (4, 14), (4, 16), "M", (4, 19)],
    [(5, 21), (5, 23), (5, 25), "M", (5, 28)],
]


def maxpool2x2(x):
    """`nn.MaxPool2d(2, 2)` (floor mode: a trailing odd row/column is dropped)."""
    B, C, H, W = x.shape
    x = x[:, :, : H // 2 * 2, : W // 2 * 2]
    return x.reshape(B, C, H // 2, 2, W // 2, 2).amax(dim=(3, 5))


def vgg_forward(P, x, plan):
    """Frozen VGG slices: conv3x3 pad 1 (zeros) + bias + ReLU, MaxPool; returns per-slice outputs."""
    outs = []
    for sl in plan:
        for op in sl:
            if op == "M":
                x = maxpool2x2(x)
            else:
                s, i = op
                x = torch.relu(F.conv2d(x, P[f"slice{s}.{i}.weight"], P[f"slice{s}.{i}.bias"], padding=1))
        outs.append(x)
    return outs


# ------------------------------------------------------------------ utilities (RC/utilities.py)
def vgg_normalize_(x):
    """RC/utilities.py:101-106: x.div_(255) IN PLACE, then returns (x - mean) / std."""
    mean = torch.tensor(IMAGENET_MEAN, dtype=x.dtype).view(-1, 1, 1)
    std = torch.tensor(IMAGENET_STD, dtype=x.dtype).view(-1, 1, 1)
    x = x.div_(255.0)
    return (x - mean) / std


def gram_matrix(y):
    """RC/utilities.py:93-98: F F^T / (C H W)."""
    b, c, h, w = y.shape
    f = y.reshape(b, c, h * w)
    return f.bmm(f.transpose(1, 2)) / (c * h * w)


def _sample_coords(flo, H, W):
    """Source pixel coords of `warp`: grid normalised by (W-1) then grid_sample(align_corners=False)
    un-normalises by W, so x_src = ((2 (x+u) / (W-1) - 1) + 1) * W / 2 - 0.5 (same fp32 op order)."""
    xx = torch.arange(W, dtype=torch.float32).view(1, 1, W)
    yy = torch.arange(H, dtype=torch.float32).view(1, H, 1)
    gx = 2.0 * (xx + flo[:, 0]) / max(W - 1, 1) - 1.0
    gy = 2.0 * (yy + flo[:, 1]) / max(H - 1, 1) - 1.0
    return ((gx + 1) * W - 1) / 2, ((gy + 1) * H - 1) / 2


def bilinear_zeros(x, sx, sy):
    """Bilinear gather with zero padding outside [0,W-1]x[0,H-1] (grid_sample 'zeros')."""
    B, C, H, W = x.shape
    x0 = torch.floor(sx)
    y0 = torch.floor(sy)
    wx1 = sx - x0
    wy1 = sy - y0
    out = torch.zeros_like(x)
    flat = x.reshape(B, C, H * W)
    for dy, wy in ((0, 1 - wy1), (1, wy1)):
        for dx, wx in ((0, 1 - wx1), (1, wx1)):
            xi = (x0 + dx).long()
            yi = (y0 + dy).long()
            valid = (xi >= 0) & (xi < W) & (yi >= 0) & (yi < H)
            idx = (yi.clamp(0, H - 1) * W + xi.clamp(0, W - 1)).reshape(B, 1, H * W).expand(B, C, H * W)
            v = flat.gather(2, idx).reshape(B, C, H, W)
            out = out + v * (wx * wy * valid).unsqueeze(1)
    return out


def warp(x, flo):
    """RC/utilities.py:39-57 (bilinear, zeros padding, align_corners=False, /(W-1) grid)."""
    B, C, H, W = x.shape
    sx, sy = _sample_coords(flo, H, W)
    return bilinear_zeros(x, sx, sy)


def flow_warp_mask(flo01, flo10, threshold=2):
    """RC/utilities.py:60-90: forward-backward consistency mask (2,H,W),(2,H,W) -> (H,W) 0/1."""
    _, H, W = flo01.shape
    grid = torch.stack(torch.meshgrid(torch.arange(W, dtype=torch.float32), torch.arange(H, dtype=torch.float32), indexing="xy"))
    sx, sy = _sample_coords(flo10.unsqueeze(0), H, W)
    fw = bilinear_zeros((grid + flo01).unsqueeze(0), sx, sy)[0]
    err = (fw - grid).abs().sum(0)
    return (err < threshold).float()


def resize_bilinear(x, size):
    """`F.interpolate(x, size, mode='bilinear')` with align_corners=False (source = (d+0.5)s-0.5,
    clamped at 0; upper neighbour clamped to n-1)."""
    B, C, H, W = x.shape
    Ho, Wo = size

    def axis(n_in, n_out):
        s = n_in / n_out
        src = ((torch.arange(n_out, dtype=torch.float32) + 0.5) * s - 0.5).clamp(min=0)
        i0 = src.floor().long().clamp(max=n_in - 1)
        i1 = (i0 + 1).clamp(max=n_in - 1)
        l1 = src - i0.float()
        return i0, i1, 1 - l1, l1

    y0, y1, wy0, wy1 = axis(H, Ho)
    x0, x1, wx0, wx1 = axis(W, Wo)
    r0 = x.index_select(2, y0)
    r1 = x.index_select(2, y1)
    top = r0.index_select(3, x0) * wx0 + r0.index_select(3, x1) * wx1
    bot = r1.index_select(3, x0) * wx0 + r1.index_select(3, x1) * wx1
    return top * wy0.view(-1, 1) + bot * wy1.view(-1, 1)


# ------------------------------------------------------------------ training step
LOSS_WEIGHTS = dict(ALPHA=1e5, BETA=2e10, GAMMA=1e-2, LAMBDA_F=1e12, LAMBDA_O=1e7)


def style_grams(VP, style):
    """train_candy.py:55-56: grams of Vgg16(vgg_normalize(style))."""
    return [gram_matrix(f) for f in vgg_forward(VP, vgg_normalize_(style.clone()), VGG16_PLAN)]


ALL_TERMS = ("FTL", "OTL", "CL", "SL", "RL")


def reconet_losses(P, VP, img1, img2, flow, mask, grams, w=LOSS_WEIGHTS, temporal=True, forward=None, teacher=None,
                   terms=None):
    """Loss terms of one `train_candy` step (RC/train_single/train_candy.py:77-148), or of the
    distillation trainers (RC/train_single/train_Flow_SD{1,2}.py:80-160) with
    `forward` = the student's forward and `teacher` = (TP, teacher_forward, t_idx, s_idx): the
    symmetric distillation term SDL = 0.01*BETA*(mse(t1, s1) + mse(t2, s2)) is computed and
    reported but, as in the reference, not added to the total.
    `terms`: the loss terms summed into `loss` (default all; CL SL RL with temporal=False) -- the
    reference's clones: train_Flow_noFTL.py:125 (OTL CL SL RL), train_multiple/train_Flow.py (all,
    12-channel frames, `index` = the last frame's channels).
    Returns dict(loss, CL, SL, FTL, OTL, RL[, SDL]) as 0-d tensors (autograd-connected to P)."""
    if terms is None:
        terms = ALL_TERMS if temporal else ("CL", "SL", "RL")
    forward = reconet_forward if forward is None else forward
    o1 = forward(P, img1)
    o2 = forward(P, img2)
    fmap1, s1 = o1[-2], o1[-1]
    fmap2, s2 = o2[-2], o2[-1]
    s1 = vgg_normalize_(s1)
    s2 = vgg_normalize_(s2)
    idx = list(range(img1.shape[1] - 3, img1.shape[1]))  # the last frame's channels (`index`)
    i1 = vgg_normalize_(img1[:, idx])
    i2 = vgg_normalize_(img2[:, idx])
    sf1 = vgg_forward(VP, s1, VGG16_PLAN)
    sf2 = vgg_forward(VP, s2, VGG16_PLAN)
    cf1 = vgg_forward(VP, i1, VGG16_PLAN)
    cf2 = vgg_forward(VP, i2, VGG16_PLAN)
    out = {}
    if "FTL" in terms:
        Hf, Wf = fmap1.shape[2:]
        ff = resize_bilinear(flow, (Hf, Wf))
        ff = torch.stack([ff[:, 0] * (float(Wf) / flow.shape[3]), ff[:, 1] * (float(Hf) / flow.shape[2])], 1)
        wf = warp(fmap1, ff)
        fm = (resize_bilinear(mask.unsqueeze(1), (Hf, Wf)) > 0).float().expand(-1, fmap1.shape[1], -1, -1)
        out["FTL"] = torch.sum(fm * (fmap2 - wf) ** 2) * (1 / int(fm.count_nonzero())) * w["LAMBDA_F"]
    if "OTL" in terms:
        ot = s2 - warp(s1, flow)
        it = i2 - warp(i1, flow)
        it = (0.2126 * it[:, 0] + 0.7152 * it[:, 1] + 0.0722 * it[:, 2]).unsqueeze(1).expand(-1, 3, -1, -1)
        m3 = mask.unsqueeze(1).expand(-1, 3, -1, -1)
        out["OTL"] = torch.sum(m3 * (ot - it) ** 2) * (1 / int(m3.count_nonzero())) * w["LAMBDA_O"]
    out["CL"] = (F.mse_loss(sf1[2], cf1[2]) + F.mse_loss(sf2[2], cf2[2])) * w["ALPHA"]
    sl = 0
    for i, gs in enumerate(grams):
        g1 = gram_matrix(sf1[i])
        g2 = gram_matrix(sf2[i])
        sl = sl + F.mse_loss(g1, gs.expand_as(g1)) + F.mse_loss(g2, gs.expand_as(g2))
    out["SL"] = sl * w["BETA"]
    reg = ((s1[:, :, :-1, 1:] - s1[:, :, :-1, :-1]) ** 2 + (s1[:, :, 1:, :-1] - s1[:, :, :-1, :-1]) ** 2
           + (s2[:, :, :-1, 1:] - s2[:, :, :-1, :-1]) ** 2 + (s2[:, :, 1:, :-1] - s2[:, :, :-1, :-1]) ** 2)
    out["RL"] = w["GAMMA"] * torch.sum(reg)
    if "RL" not in terms:
        del out["RL"]
    out["loss"] = sum(out[k] for k in ALL_TERMS if k in terms)
    if teacher is not None:
        TP, tfwd, ti, si = teacher
        with torch.no_grad():
            t1, t2 = tfwd(TP, img1)[ti], tfwd(TP, img2)[ti]
        out["SDL"] = (F.mse_loss(t1, o1[si]) + F.mse_loss(t2, o2[si])) * (0.01 * w["BETA"])
    return out


def reconet_single_losses(P, VP, img, grams, w=LOSS_WEIGHTS, forward=None):
    """Loss terms of one `train_coco2014` step (RC/train_single/train_coco2014.py:65-86): single
    images, content (relu3_3 MSE x ALPHA) + Gram style (x BETA), no temporal terms, no TV.
    Returns dict(loss, CL, SL)."""
    forward = reconet_forward if forward is None else forward
    s = vgg_normalize_(forward(P, img)[-1])                      # :65, :68
    i = vgg_normalize_(img.clone())                               # :69 (in place on the batch)
    sf = vgg_forward(VP, s, VGG16_PLAN)
    cf = vgg_forward(VP, i, VGG16_PLAN)
    out = {"CL": F.mse_loss(sf[2], cf[2]) * w["ALPHA"]}          # :74-76
    sl = 0
    for k, gs in enumerate(grams):                                # :79-83
        g = gram_matrix(sf[k])
        sl = sl + F.mse_loss(g, gs.expand_as(g))
    out["SL"] = sl * w["BETA"]
    out["loss"] = out["CL"] + out["SL"]                           # :86
    return out


def adam_step(params, grads, state, lr=1e-3, b1=0.9, b2=0.999, eps=1e-8):
    """torch.optim.Adam defaults (no weight decay, no amsgrad): one step, in place."""
    state["t"] = state.get("t", 0) + 1
    t = state["t"]
    for k, p in params.items():
        g = grads[k]
        m = state.setdefault("m_" + k, torch.zeros_like(p))
        v = state.setdefault("v_" + k, torch.zeros_like(p))
        m.mul_(b1).add_(g, alpha=1 - b1)
        v.mul_(b2).addcmul_(g, g, value=1 - b2)
        denom = (v.sqrt() / np.sqrt(1 - b2 ** t)).add_(eps)
        p.data.addcdiv_(m, denom, value=-lr / (1 - b1 ** t))


# ------------------------------------------------------------------ inference (RC/utilities.py:108-235)
def cvframe_to_tensor(frame):
    """RC/utilities.py:118-123 for a 360x640 BGR uint8 frame: BGR2RGB, ToTensor, mul(255)."""
    rgb = torch.from_numpy(np.ascontiguousarray(frame[..., ::-1]))
    return rgb.permute(2, 0, 1).contiguous().float().div(255).mul(255)


def _styled_windows(forward, P, frames, n, first_frame):
    if first_frame is None or first_frame < n:
        first_frame = n
    frames = list(frames)[first_frame - n:]
    imgs = [cvframe_to_tensor(f) for f in frames]
    with torch.no_grad():
        for t in range(n - 1, len(imgs)):
            x = torch.cat(imgs[t - n + 1:t + 1], 0).unsqueeze(0)
            yield imgs[t].unsqueeze(0), forward(P, x)[-1].clamp(0, 255)


def inference(forward, P, frames, n, first_frame=None):
    """Inference.__iter__ (RC/utilities.py:209-235): HxWx3 uint8 BGR stylised frames."""
    return [np.ascontiguousarray(y[0].permute(1, 2, 0).numpy()[..., ::-1]).astype(np.uint8)
            for _, y in _styled_windows(forward, P, frames, n, first_frame)]


def calculate_mse(forward, P, frames, n):
    """calculate_mse (RC/utilities.py:126-176)."""
    loss, count, prev = 0, 0, None
    for x, y in _styled_windows(forward, P, frames, n, None):
        if prev is not None:
            loss += F.mse_loss(x - prev[0], y - prev[1]).item()
            count += 1
        prev = (x, y)
    return loss / count
