"""Drop-in MI355X implementation of the hot-path helpers of RC/utilities.py.

Same names and argument meaning as the reference; every one runs a HIP kernel (vst.ops).
"""
from .. import ops


def warp(x, flo, padding_mode="zeros"):
    """RC/utilities.py:39-57: bilinear grid_sample of x at (grid + flo), zeros padding,
    align_corners=False with the grid normalised by (W-1) (zero flow is not the identity)."""
    if padding_mode != "zeros":
        raise ValueError("only padding_mode='zeros' is on the reference path")
    return ops.warp(x, flo)


def flow_warp_mask(flo01, flo10, padding_mode="zeros", threshold=2):
    """RC/utilities.py:60-90 (and AA/utilities.py:133-163 with `threshold`): (2,H,W) flows ->
    (H,W) float 0/1 forward-backward consistency mask.  Also accepts batched (B,2,H,W)."""
    if padding_mode != "zeros":
        raise ValueError("only padding_mode='zeros' is on the reference path")
    return ops.flow_warp_mask(flo01, flo10, threshold)


def gram_matrix(y):
    """RC/utilities.py:93-98: F F^T / (C H W), F = y.view(b, c, h*w)."""
    return ops.gram_matrix(y)


def vgg_normalize(batch):
    """RC/utilities.py:101-106: divides `batch` by 255 IN PLACE, returns (batch - mean) / std."""
    _, out = ops.VggNormalizeInplaceFn.apply(batch)
    return out
