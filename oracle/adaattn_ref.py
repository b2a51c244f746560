"""CPU restatement of the reference AdaAttN video-training path.  TEST INFRASTRUCTURE ONLY
(see oracle/__init__.py).  Pinned by tests/golden/aa_*.npz produced from the reference itself.

Follows AA/vgg19.py:43-63, AA/utilities.py:79-109, AA/network.py:11-251, AA/lossfn.py:5-53,
AA/train_video.py:78-118, AA/train_image.py:69-106.  Parameters are dicts keyed like the reference
state_dicts.
"""
import torch
import torch.nn.functional as F

from . import reconet_ref as R
from .shapes import ADAATTN_LEVELS, DECODER

FEATS = ("relu1_1", "relu2_1", "relu3_1", "relu4_1", "relu5_1")


def vgg_normalize(x, dtype=torch.float32):
    """AA/utilities.py:79-85 (out of place): (x/255 - mean)/std (dtype: float64 only for the exact
    reference values the conditioning-aware tolerances are built from)."""
    mean = torch.tensor(R.IMAGENET_MEAN, dtype=dtype).view(-1, 1, 1)
    std = torch.tensor(R.IMAGENET_STD, dtype=dtype).view(-1, 1, 1)
    return (x.to(dtype) / 255.0 - mean) / std


def vgg19(VP, x, dtype=torch.float32):
    """AA/vgg19.py:43-63 -> dict relu1_1..relu5_1."""
    return dict(zip(FEATS, R.vgg_forward(VP, vgg_normalize(x, dtype), R.VGG19_PLAN)))


def feature_down_sample(feat, last):
    """AA/utilities.py:98-109: bilinear (align_corners=False) resize of levels < last, concat."""
    size = feat[last].shape[-2:]
    return torch.cat([R.resize_bilinear(feat[i], size) for i in range(last)] + [feat[last]], dim=1)


def instance_norm(x, eps=1e-5):
    """nn.InstanceNorm2d(C, affine=False)."""
    mu = x.mean(dim=(2, 3), keepdim=True)
    var = ((x - mu) ** 2).mean(dim=(2, 3), keepdim=True)
    return (x - mu) / torch.sqrt(var + eps)


def cosine_attention(q, k):
    """AA/network.py:115-125: q (b, N, d), k (b, d, M): s = qk/(|q||k|) + 1, a = s / sum_j s."""
    qn = torch.sqrt((q * q).sum(-1, keepdim=True))
    kn = torch.sqrt((k * k).sum(1, keepdim=True))
    s = torch.bmm(q, k) / torch.bmm(qn, kn) + 1
    return s / s.sum(dim=-1, keepdim=True)


def softmax_attention(q, k):
    """AA/network.py:100-106: softmax(q k) over the style positions."""
    return torch.softmax(torch.bmm(q, k), dim=-1)


def adaattn(P, prefix, c_x, s_x, c_1x, s_1x, activation="cosine"):
    """AA/network.py:191-220 (prefix=None -> AdaAttnNoConv, AA/network.py:142-171)."""
    Q, K, V = instance_norm(c_1x), instance_norm(s_1x), s_x
    if prefix is not None:
        Q = F.conv2d(Q, P[prefix + ".f.weight"], P[prefix + ".f.bias"])
        K = F.conv2d(K, P[prefix + ".g.weight"], P[prefix + ".g.bias"])
        V = F.conv2d(V, P[prefix + ".h.weight"], P[prefix + ".h.bias"])
    b, _, h, w = Q.shape
    Qt = Q.reshape(b, -1, h * w).permute(0, 2, 1)
    b, _, hs, ws = K.shape
    Km = K.reshape(b, -1, hs * ws)
    Vt = V.reshape(b, -1, hs * ws).permute(0, 2, 1)
    A = cosine_attention(Qt, Km) if activation == "cosine" else softmax_attention(Qt, Km)
    M = torch.bmm(A, Vt)
    S = torch.sqrt((torch.bmm(A, Vt ** 2) - M ** 2).clamp(min=1e-6))
    b, _, h, w = c_x.shape
    M = M.reshape(b, h, w, -1).permute(0, 3, 1, 2)
    S = S.reshape(b, h, w, -1).permute(0, 3, 1, 2)
    return S * instance_norm(c_x) + M


def attention_moments(Q, K, V, activation="cosine"):
    """The two moments AdaAttN reads from its attention (AA/network.py:205-213), materialised as the
    reference computes them: A = activation(Q^T K) (b, Nc, Ns), M = A V^T, S = sqrt(clamp(A (V^2)^T
    - M^2, 1e-6)).  Q (b, d, h, w), K (b, d, hs, ws), V (b, dv, hs, ws); returns M, S as (b, dv, h, w)."""
    b, d, h, w = Q.shape
    Qt = Q.reshape(b, d, h * w).permute(0, 2, 1)
    Km = K.reshape(b, d, -1)
    Vt = V.reshape(b, V.shape[1], -1).permute(0, 2, 1)
    A = cosine_attention(Qt, Km) if activation == "cosine" else softmax_attention(Qt, Km)
    M = torch.bmm(A, Vt)
    S = torch.sqrt((torch.bmm(A, Vt ** 2) - M ** 2).clamp(min=1e-6))
    return (M.reshape(b, h, w, -1).permute(0, 3, 1, 2), S.reshape(b, h, w, -1).permute(0, 3, 1, 2))


def cosine_moments_exact(Q, K, V):
    """EXACT evaluator of `attention_moments(..., "cosine")` for sizes whose Nc x Ns matrix is too
    large for the CPU (config 5 level 3: 32768^2 per image): the same quantity re-associated, in
    float64.  With q^ = q/|q|, k^ = k/|k|, A_ij = (q^_i.k^_j + 1) / sum_j (q^_i.k^_j + 1), so
      [M; E2]_i = (G^T q^_i + sum_j u_j) / (q^_i . sum_j k^_j + Ns),  G = K^ U^T,  U = [V; V^2],
    an identity of real arithmetic (not an approximation); in float64 its rounding is ~1e-13, far
    below any fp32 path's error, so it is the yardstick both the reference's fp32 form and the HIP
    path are measured against.  Checked against the materialised form in float64 by
    tests/test_oracle_golden.py::test_cosine_moments_exact."""
    b, d, h, w = Q.shape
    dv = V.shape[1]
    q = Q.double().reshape(b, d, -1)
    k = K.double().reshape(b, d, -1)
    v = V.double().reshape(b, dv, -1)
    qh = q / torch.sqrt((q * q).sum(1, keepdim=True))
    kh = k / torch.sqrt((k * k).sum(1, keepdim=True))
    U = torch.cat([v, v * v], 1)                                  # (b, 2dv, Ns)
    G = torch.bmm(kh, U.transpose(1, 2))                          # (b, d, 2dv)
    num = torch.bmm(G.transpose(1, 2), qh) + U.sum(2, keepdim=True)  # (b, 2dv, Nc)
    den = (qh * kh.sum(2, keepdim=True)).sum(1, keepdim=True) + k.shape[2]  # (b, 1, Nc)
    mom = num / den
    M, E2 = mom[:, :dv], mom[:, dv:]
    S = torch.sqrt((E2 - M * M).clamp(min=1e-6))
    return M.reshape(b, dv, h, w), S.reshape(b, dv, h, w)


def upsample2(x):
    """F.interpolate(scale_factor=2, mode='bilinear', align_corners=False)."""
    return R.resize_bilinear(x, (2 * x.shape[2], 2 * x.shape[3]))


def decoder(P, x5, x4, x3):
    """AA/network.py:79-99."""
    def conv(x, name):
        relu = dict((n, r) for n, _, _, r in DECODER)[name]
        key = f"decoder.{name}.conv.conv" if relu else f"decoder.{name}.conv"
        y = F.conv2d(R.reflect_pad(x, 1), P[key + ".weight"], P[key + ".bias"])
        return torch.relu(y) if relu else y

    x = upsample2(x5) + x4
    x = conv(x, "conv1")
    x = upsample2(conv(x, "conv2"))
    x = torch.cat([x, x3], dim=1)
    for n in ("conv3.0", "conv3.1", "conv3.2"):
        x = conv(x, n)
    x = upsample2(conv(x, "conv4"))
    x = upsample2(conv(conv(x, "conv5"), "conv6"))
    return conv(conv(x, "conv7"), "conv8")


def stylize(P, fc, fs, activation="cosine"):
    """StylizingNetwork.forward (AA/network.py:237-251)."""
    lc, ls = list(fc.values()), list(fs.values())
    outs = []
    for i in range(3):
        idx = i + 2
        outs.append(adaattn(P, f"adaattn.{i}", lc[idx], ls[idx], feature_down_sample(lc, idx), feature_down_sample(ls, idx),
                            activation))
    return decoder(P, outs[2], outs[1], outs[0])


def global_stylized_loss(fcs, fs):
    """AA/lossfn.py:5-17 (MSE of channel means + MSE of unbiased channel stds)."""
    return F.mse_loss(fcs.mean(dim=(2, 3)), fs.mean(dim=(2, 3))) + F.mse_loss(fcs.std(dim=(2, 3)), fs.std(dim=(2, 3)))


def cosine_distance(fu, fv):
    """AA/lossfn.py:25-38: 1 - (Fu Fv^T) / (|fu| |fv|^T + 1e-6), (b, c, c)."""
    b, c = fu.shape[:2]
    u = fu.reshape(b, c, -1)
    v = fv.reshape(b, c, -1)
    un = torch.sqrt((u * u).sum(-1, keepdim=True))
    vn = torch.sqrt((v * v).sum(-1, keepdim=True))
    return 1 - torch.bmm(u, v.transpose(1, 2)) / (torch.bmm(un, vn.transpose(1, 2)) + 1e-6)


def image_similarity_loss(fc1, fc2, fcs1, fcs2):
    """AA/lossfn.py:41-53: column-normalised cosine distances, L1 summed over the batch / (h w)."""
    n = fc1.shape[2] * fc1.shape[3]
    d1 = cosine_distance(fc1, fc2)
    d2 = cosine_distance(fcs1, fcs2)
    d1 = d1 / d1.sum(dim=1, keepdim=True)
    d2 = d2 / d2.sum(dim=1, keepdim=True)
    return torch.abs(d1 - d2).sum() / n


WEIGHTS = dict(LAMBDA_G=10.0, LAMBDA_L=3.0, LAMBDA_IS=100.0)


def adaattn_losses(P, VP, c1, c2, s, w=WEIGHTS):
    """Loss terms of one train_video step (AA/train_video.py:78-118)."""
    fc1, fc2, fs = vgg19(VP, c1), vgg19(VP, c2), vgg19(VP, s)
    fc1 = {k: v.detach() for k, v in fc1.items()}
    fc2 = {k: v.detach() for k, v in fc2.items()}
    fs = {k: v.detach() for k, v in fs.items()}
    cs1, cs2 = stylize(P, fc1, fs), stylize(P, fc2, fs)
    fcs1, fcs2 = vgg19(VP, cs1), vgg19(VP, cs2)
    gs = sum(global_stylized_loss(fcs1[k], fs[k]) for k in FEATS[1:]) * w["LAMBDA_G"]
    l1, ls = list(fc1.values()), list(fs.values())
    lf = 0
    for i in range(3):
        idx = i + 2
        t = adaattn(None, None, l1[idx], ls[idx], feature_down_sample(l1, idx), feature_down_sample(ls, idx))
        lf = lf + F.mse_loss(fcs1[FEATS[idx]], t)
    lf = lf * w["LAMBDA_L"]
    isl = sum(image_similarity_loss(fc1[k], fc2[k], fcs1[k], fcs2[k]) for k in FEATS[1:4]) * w["LAMBDA_IS"]
    return {"loss": gs + lf + isl, "loss_gs": gs, "loss_lf": lf, "loss_is": isl}


IMAGE_WEIGHTS = dict(LAMBDA_G=10.0, LAMBDA_L=3.0)  # AA/train_image.py:20-21


def adaattn_image_losses(P, VP, c, s, w=IMAGE_WEIGHTS, activation="softmax", dtype=torch.float32):
    """Loss terms of one train_image step (AA/train_image.py:69-106): single content images, softmax
    attention (ACTIAVTION = "softmax", :22), global-stylized + local-feature losses, no IS term.
    dtype=float64 (with float64 P / VP) gives the exact values of the same step."""
    fc = {k: v.detach() for k, v in vgg19(VP, c, dtype).items()}
    fs = {k: v.detach() for k, v in vgg19(VP, s, dtype).items()}
    fcs = vgg19(VP, stylize(P, fc, fs, activation), dtype)
    gs = sum(global_stylized_loss(fcs[k], fs[k]) for k in FEATS[1:]) * w["LAMBDA_G"]
    lc, ls = list(fc.values()), list(fs.values())
    lf = 0
    for i in range(3):
        idx = i + 2
        t = adaattn(None, None, lc[idx], ls[idx], feature_down_sample(lc, idx), feature_down_sample(ls, idx), activation)
        lf = lf + F.mse_loss(fcs[FEATS[idx]], t)
    lf = lf * w["LAMBDA_L"]
    return {"loss": gs + lf, "loss_gs": gs, "loss_lf": lf}
