"""Minimal `torchvision.transforms` objects the reference constructs at import time."""
import numpy as np
import torch


class Compose:
    def __init__(self, ts):
        self.ts = ts

    def __call__(self, x):
        for t in self.ts:
            x = t(x)
        return x


class Lambda:
    def __init__(self, f):
        self.f = f

    def __call__(self, x):
        return self.f(x)


class ToTensor:
    def __call__(self, x):
        a = np.asarray(x)
        if a.ndim == 2:
            a = a[:, :, None]
        t = torch.from_numpy(np.ascontiguousarray(a.transpose(2, 0, 1)))
        return t.float().div(255) if a.dtype == np.uint8 else t.float()


class ToPILImage:
    def __call__(self, x):
        raise NotImplementedError("stub")


class GaussianBlur:
    def __init__(self, *a, **k):
        pass

    def __call__(self, x):
        raise NotImplementedError("stub")


class Resize(GaussianBlur):
    pass


class RandomCrop(GaussianBlur):
    pass


class CenterCrop(GaussianBlur):
    pass


class Normalize(GaussianBlur):
    pass
