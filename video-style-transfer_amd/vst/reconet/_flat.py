"""Flat parameter / gradient / Adam-state buffers for a module.

Every parameter becomes a view into one contiguous fp32 buffer and its `.grad` a view into a
second one, so autograd accumulates straight into the flat gradient (AccumulateGrad adds in
place into an existing .grad), the DDP all-reduce is ONE RCCL call and Adam is ONE kernel
(`vst_adam`) over the whole model (62 tensors / 3,763,011 floats for ReCoNet).
"""
import torch
from torch.autograd.graph import increment_version

from .._lib import lib, ptr, stream


class FlatParams:
    def __init__(self, module):
        params = [p for p in module.parameters() if p.requires_grad]
        n = sum(p.numel() for p in params)
        dev = params[0].device
        self.p = torch.empty(n, device=dev, dtype=torch.float32)
        self.g = torch.zeros(n, device=dev, dtype=torch.float32)
        self.m = torch.zeros(n, device=dev, dtype=torch.float32)
        self.v = torch.zeros(n, device=dev, dtype=torch.float32)
        off = 0
        with torch.no_grad():
            for prm in params:
                k = prm.numel()
                self.p[off:off + k].copy_(prm.reshape(-1))
                prm.data = self.p[off:off + k].view_as(prm)
                prm.grad = self.g[off:off + k].view_as(prm)
                off += k
        self.params = params
        self.numel = n

    def zero_grad(self):
        self.g.zero_()
        for prm, (off, k) in zip(self.params, self._spans()):
            if prm.grad is None or prm.grad.data_ptr() != self.g[off:off + k].data_ptr():
                prm.grad = self.g[off:off + k].view_as(prm)

    def _spans(self):
        off = 0
        for prm in self.params:
            yield off, prm.numel()
            off += prm.numel()

    def adam(self, step, lr, betas, eps, gscale=1.0):
        lib.vst_adam(ptr(self.p), ptr(self.g), ptr(self.m), ptr(self.v), self.numel, float(lr), float(betas[0]),
                     float(betas[1]), float(eps), int(step), float(gscale), stream())
        # the kernel updated every parameter in place: bump the version counter the parameter views
        # share with the flat buffer, so a graph saved before this step refuses to run backward
        increment_version(self.p)
