"""Drop-in for RT/vgg19.py:8-58: frozen VGG19 features[0:23] split at relu1_2 / relu2_2 / relu3_2 /
relu4_2 (state_dict keys `slice1.0.weight` ... `slice4.21.bias`), on HIP kernels.  `weights`:
path to a local torchvision vgg19 state dict (the reference downloads IMAGENET1K_V1; there is no
network here), otherwise torchvision's default initialisation."""
import torch.nn as nn

from ..reconet.network import _load_torchvision_features, run_vgg_slice, vgg_features
from .utilities import vgg_normalize

_VGG19_CFG = [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512]
_SLICES = ((0, 4), (4, 9), (9, 14), (14, 23))
FEATURES = ("relu1_2", "relu2_2", "relu3_2", "relu4_2")


class VGG19(nn.Module):
    def __init__(self, weights=None):
        super().__init__()
        feats = vgg_features(_VGG19_CFG, 23)
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
            x = run_vgg_slice(getattr(self, f"slice{s}"), x)
            out[name] = x
        return out
