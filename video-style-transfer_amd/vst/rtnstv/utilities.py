"""Drop-in MI355X implementation of the hot-path helpers of RT/utilities.py."""
from .. import ops
from ..reconet.utilities import flow_warp_mask  # noqa: F401  (RT/utilities.py:80-110, same arithmetic)


def warp(x, flo, padding_mode="zeros"):
    """RT/utilities.py:59-77 (grid normalised by max(W - 1, 1): the same as RC's for W, H > 1)."""
    if padding_mode != "zeros":
        raise ValueError("only padding_mode='zeros' is on the reference path")
    if x.shape[2] < 2 or x.shape[3] < 2:
        raise ValueError("warp: frames must be at least 2x2")
    return ops.warp(x, flo)


def gram_matrix(y):
    """RT/utilities.py:155-160: F F^T / (H W) (not C H W as in ReCoNet / AdaAttN)."""
    return ops.gram_matrix(y, per_hw=True)


def vgg_normalize(batch):
    """RT/utilities.py:163-169: (batch / 255 - mean) / std, out of place."""
    return ops.VggNormalizeFn.apply(batch.float())
