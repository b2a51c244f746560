"""Drop-in for the AdaAttN path's helpers in AA/utilities.py on HIP kernels."""
import torch

from .. import ops
from .._lib import VstError
from ..reconet.utilities import flow_warp_mask, warp  # noqa: F401  (AA/utilities.py:112-163, same arithmetic)


def vgg_normalize(batch):
    """AA/utilities.py:79-85 (out of place): (batch/255 - mean)/std, differentiable."""
    return ops.VggNormalizeFn.apply(batch.float() if batch.dtype != torch.float32 else batch)


class _FeatureDownSample(torch.autograd.Function):
    @staticmethod
    def forward(ctx, last_feat_idx, *feat):
        size = feat[last_feat_idx].shape[-2:]
        N = feat[0].shape[0]
        chans = [f.shape[1] for f in feat[: last_feat_idx + 1]]
        out = torch.empty((N, sum(chans)) + tuple(size), device=feat[0].device, dtype=torch.float32)
        off = 0
        for i in range(last_feat_idx):
            ops.resize_bilinear(feat[i], size, out=out[:, off:off + chans[i]])
            off += chans[i]
        ops.copy_into(ops._check(feat[last_feat_idx], "feature"), out[:, off:])
        ctx.meta = (last_feat_idx, [f.shape for f in feat[: last_feat_idx + 1]], chans, len(feat))
        return out

    @staticmethod
    def backward(ctx, g):
        last, shapes, chans, nfeat = ctx.meta
        g = g.contiguous()
        grads, off = [], 0
        for i in range(last + 1):
            gi = None
            if ctx.needs_input_grad[1 + i]:
                sl = g[:, off:off + chans[i]]
                gi = (ops.resize_bilinear_bwd(sl, shapes[i]) if i < last
                      else ops.copy_into(sl, torch.empty(shapes[i], device=g.device, dtype=torch.float32)))
            grads.append(gi)
            off += chans[i]
        return (None, *grads, *([None] * (nfeat - last - 1)))


def feature_down_sample(feat, last_feat_idx):
    """AA/utilities.py:98-109: bilinear (align_corners=False) resize of feat[0:last] to
    feat[last]'s size, concatenated with feat[last] along channels — written in place into one
    buffer (no per-level temporaries, no torch.cat)."""
    feat = list(feat)
    if not 0 < last_feat_idx < len(feat):
        raise VstError(f"feature_down_sample: index {last_feat_idx} out of range")
    return _FeatureDownSample.apply(last_feat_idx, *feat)
