"""Drop-in for AA/vgg19.py:8-63 (frozen VGG19 encoder, relu1_1..relu5_1) on HIP kernels.

Same slice layout and state_dict keys (`slice1.0.weight` ... `slice5.28.bias`).  `weights`: path
to a local torchvision vgg19 state dict (the reference downloads IMAGENET1K_V1; there is no
network here), otherwise torchvision's default initialisation.
"""
import os

import torch
import torch.nn as nn

from .. import ops
from ..reconet.network import _load_torchvision_features, run_vgg_slice, vgg_features
from .utilities import vgg_normalize

# torchvision VGG19 "E" features[0:30]
_VGG19_CFG = [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512]
_SLICES = ((0, 2), (2, 7), (7, 12), (12, 21), (21, 30))
FEATURES = ("relu1_1", "relu2_1", "relu3_1", "relu4_1", "relu5_1")
# VST_FEATURE_SPLIT=0: slice boundaries through autograd's sum + a separate ReLU backward (A/B only)
_SPLIT = os.environ.get("VST_FEATURE_SPLIT", "1") != "0"


class VGG19(nn.Module):
    def __init__(self, weights=None):
        super().__init__()
        feats = vgg_features(_VGG19_CFG, 30)
        _load_torchvision_features(feats, weights)
        for s, (a, b) in enumerate(_SLICES, 1):
            seq = nn.Sequential()
            for x in range(a, b):
                seq.add_module(str(x), feats[x])
            setattr(self, f"slice{s}", seq)
        for param in self.parameters():
            param.requires_grad = False

    def forward(self, x):
        x = vgg_normalize(x)
        out = {}
        for s, name in enumerate(FEATURES, 1):
            last = s == len(FEATURES)
            with ops.gemm_scope(f"s{s}"):  # (policy keys may name a slice: "<scope>.s<k>.<role>")
                if _SPLIT and not last and torch.is_grad_enabled() and x.requires_grad:
                    # slice boundary with a gradient: the feature's two consumers (losses, next slice)
                    # meet in FeatureSplitFn's fused backward, so the producing conv runs premasked
                    x = run_vgg_slice(getattr(self, f"slice{s}"), x, premasked_out=True)
                    out[name], x = ops.feature_split(x)
                else:
                    x = run_vgg_slice(getattr(self, f"slice{s}"), x)
                    out[name] = x
        return out
