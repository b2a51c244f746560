"""Architecture-only VGG feature stacks (torchvision cfg "D" = VGG16, "E" = VGG19).

Layer order matches torchvision's `features` Sequential: Conv3x3(pad 1) -> ReLU(inplace)
per number, MaxPool2d(2, 2) per "M".  The `weights=` argument is accepted and ignored
(no network); the golden generator loads seeded weights afterwards.
"""
import torch.nn as nn

_CFG = {
    "D": [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"],
    "E": [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512, 512, 512, "M"],
}


class _VGG(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        layers = []
        cin = 3
        for v in _CFG[cfg]:
            if v == "M":
                layers.append(nn.MaxPool2d(kernel_size=2, stride=2))
            else:
                layers.append(nn.Conv2d(cin, v, kernel_size=3, padding=1))
                layers.append(nn.ReLU(inplace=True))
                cin = v
        self.features = nn.Sequential(*layers)


def vgg16(weights=None, **_):
    return _VGG("D")


def vgg19(weights=None, **_):
    return _VGG("E")
