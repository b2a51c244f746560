"""Drop-in for AA/lossfn.py on HIP kernels.

`loss_fn` arguments are accepted for signature parity; an `nn.MSELoss(reduction="mean")` (what
both reference trainers pass) is executed by the library's MSE kernel, any other callable is
applied to the kernel-computed statistics as given.
"""
import torch
from torch.autograd import Function
from torch import nn

from .. import ops
from .._lib import VstError, lib, ptr, stream
from .attention import gemm_abt


def _empty(shape, like):
    return torch.empty(shape, device=like.device, dtype=torch.float32)


class PlaneMeanStdFn(Function):
    """(x.mean(dim=(2, 3)), x.std(dim=(2, 3))) — unbiased std, fp64 accumulation."""

    @staticmethod
    def forward(ctx, x):
        x = ops._check(x, "mean/std input", 4)
        N, C, H, W = x.shape
        mean, std = _empty((N, C), x), _empty((N, C), x)
        lib.vst_plane_meanstd(ptr(x), ptr(mean), ptr(std), N * C, H * W, stream())
        ctx.save_for_backward(x, mean, std)
        return mean, std

    @staticmethod
    def backward(ctx, gmean, gstd):
        x, mean, std = ctx.saved_tensors
        N, C, H, W = x.shape
        gx = _empty(x.shape, x)
        lib.vst_plane_meanstd_bwd(ptr(x), ptr(mean), ptr(std), ptr(None if gmean is None else gmean.contiguous()),
                                  ptr(None if gstd is None else gstd.contiguous()), ptr(gx), N * C, H * W, stream())
        return gx


def plane_mean_std(x):
    return PlaneMeanStdFn.apply(x)


def _apply_loss(loss_fn, a, b, weight=1.0):
    if loss_fn is None or (isinstance(loss_fn, nn.MSELoss) and loss_fn.reduction == "mean"):
        return ops.mse(a, b, weight)
    out = loss_fn(a, b)
    return out if weight == 1.0 else out * weight


def global_stylized_loss(fcs, fs, loss_fn=None, weight=1.0):
    """AA/lossfn.py:5-17: loss_fn(mean_cs, mean_s) + loss_fn(std_cs, std_s) over (H, W)."""
    mcs, scs = plane_mean_std(fcs)
    with torch.no_grad():
        ms, ss = plane_mean_std(fs)
    return ops.sum_scalars(_apply_loss(loss_fn, mcs, ms, weight), _apply_loss(loss_fn, scs, ss, weight))


def local_feature_loss(fcs, adaattn, loss_fn=None, weight=1.0):
    """AA/lossfn.py:20-22."""
    return _apply_loss(loss_fn, fcs, adaattn, weight)


def _flat(x):
    N, C, H, W = x.shape
    return ops._check(x, "cosine-distance input", 4).view(N, C, H * W)


def plane_norm(x):
    N, C, P = x.shape
    out = _empty((N, C), x)
    lib.vst_plane_norm(ptr(x), ptr(out), N * C, P, stream())
    return out


def cosine_distance(fu, fv):
    """AA/lossfn.py:25-38 (forward): 1 - Fu Fv^T / (|fu| |fv|^T + 1e-6), (b, c, c)."""
    u, v = _flat(fu), _flat(fv)
    if u.shape != v.shape:
        raise VstError("cosine_distance: shape mismatch")
    N, C, _ = u.shape
    G = gemm_abt(u, v, role="loss_fwd")
    un, vn = plane_norm(u), plane_norm(v)
    D = _empty((N, C, C), u)
    lib.vst_cosdist(ptr(G), ptr(un), ptr(vn), ptr(D), N, C, stream())
    return D


class ImageSimilarityFn(Function):
    """weight * image_similarity_loss (AA/lossfn.py:41-53); gradient w.r.t. fcs1, fcs2 (the
    content-side features fc1, fc2 are VGG outputs of data and carry none)."""

    @staticmethod
    def forward(ctx, fc1, fc2, fcs1, fcs2, weight):
        c1, c2, s1, s2 = (_flat(t) for t in (fc1, fc2, fcs1, fcs2))
        if not (c1.shape == c2.shape == s1.shape == s2.shape):
            raise VstError("image_similarity_loss: all four feature maps must share a shape")
        N, C, P = c1.shape
        Gc, Gs = gemm_abt(c1, c2, role="loss_fwd"), gemm_abt(s1, s2, role="loss_fwd")
        unc, vnc, uns, vns = plane_norm(c1), plane_norm(c2), plane_norm(s1), plane_norm(s2)
        colc, cols = _empty((N, C), c1), _empty((N, C), c1)
        partial = _empty((N * C,), c1)
        lib.vst_simloss(ptr(Gc), ptr(unc), ptr(vnc), ptr(Gs), ptr(uns), ptr(vns), ptr(colc), ptr(cols), ptr(partial),
                        N, C, P, stream())
        st = _empty((3,), c1)
        ws = _empty((ops.LOSS_WS,), c1)
        lib.vst_sum_scaled(ptr(partial), N * C, float(weight), ptr(ws), ptr(st), stream())
        ctx.weight = float(weight)
        ctx.save_for_backward(Gc, unc, vnc, Gs, uns, vns, colc, cols, s1, s2)
        ctx.shape = fcs1.shape
        return st[0]

    @staticmethod
    def backward(ctx, g):
        Gc, unc, vnc, Gs, uns, vns, colc, cols, s1, s2 = ctx.saved_tensors
        N, C, P = s1.shape
        dG = _empty((N, C, C), s1)
        dun = _empty((N, C), s1)
        dvn = _empty((N, C), s1)
        lib.vst_simloss_bwd(ptr(Gc), ptr(unc), ptr(vnc), ptr(Gs), ptr(uns), ptr(vns), ptr(colc), ptr(cols),
                            ptr(g.contiguous()), ctx.weight, ptr(dG), ptr(dun), ptr(dvn), N, C, P, stream())
        from .attention import bmm_at_b

        d1 = d2 = None
        if ctx.needs_input_grad[2]:
            # d s1[i] = sum_j dG[i][j] s2[j]  -> A op [k=j][m=i] = dG[i][j] (transpose)
            d1 = bmm_at_b(dG, C, C, True, s2, P, role="loss_dgrad")
            lib.vst_plane_norm_grad(ptr(d1), ptr(dun), ptr(uns), ptr(s1), N * C, P, stream())
            d1 = d1.view(ctx.shape)
        if ctx.needs_input_grad[3]:
            # d s2[j] = sum_i dG[i][j] s1[i]  -> A op [k=i][m=j] = dG[i][j]
            d2 = bmm_at_b(dG, C, C, False, s1, P, role="loss_dgrad")
            lib.vst_plane_norm_grad(ptr(d2), ptr(dvn), ptr(vns), ptr(s2), N * C, P, stream())
            d2 = d2.view(ctx.shape)
        if ctx.needs_input_grad[0] or ctx.needs_input_grad[1]:
            raise VstError("image_similarity_loss: gradient w.r.t. the content features is not on the reference path")
        return None, None, d1, d2, None


def image_similarity_loss(fc1, fc2, fcs1, fcs2, weight=1.0):
    """AA/lossfn.py:41-53 (times `weight`, folded into the reduction kernel)."""
    return ImageSimilarityFn.apply(fc1, fc2, fcs1, fcs2, weight)
