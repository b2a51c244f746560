"""Drop-in MI355X implementation of RT/network.py (RTNSTV StylizingNetwork).

Same class names, constructor arguments and state_dict keys as the reference
(`conv1.conv.weight`, `conv1.norm.bias`, `res1.conv2.conv.weight`, `deconv1.deconv.weight`, ...).
`nn.Conv2d` / `nn.ConvTranspose2d` / `nn.InstanceNorm2d` are parameter containers only; the
forward and backward run libvst_hip.so kernels through `vst.ops`:
  * Conv (RT/network.py:10-26): reflect pad folded into the conv gather, conv bias + InstanceNorm
    (+ ReLU) as in ReCoNet's ConvInstRelu; a Tanh activation is its own kernel;
  * Res (RT/network.py:29-46): the residual add is fused into the second InstanceNorm;
  * Deconv (RT/network.py:49-62): ConvTranspose2d(k, s, p=1, op=1) as the transposed implicit GEMM
    (vst.ops.ConvTranspose2dFn) + InstanceNorm + ReLU;
  * StylizingNetwork's output `(tanh(x) + 1) / 2 * 255` (RT/network.py:93) is one kernel.
"""
import numpy as np
import torch
import torch.nn as nn

from .. import ops
from .._lib import VstError


def _act_kind(activation):
    if activation is None:
        return None
    if isinstance(activation, nn.ReLU):
        return "relu"
    if isinstance(activation, nn.Tanh):
        return "tanh"
    raise VstError(f"activation {type(activation).__name__} is not on the reference path (ReLU, Tanh, None)")


class Conv(nn.Module):
    """RT/network.py:10-26: ReflectionPad2d(k // 2) -> Conv2d(k, stride) -> InstanceNorm2d(affine) -> act."""

    def __init__(self, in_channels, out_channels, kernel_size, stride, activation=None):
        super().__init__()
        self.pad_size = int(np.floor(kernel_size / 2))
        self.pad = nn.ReflectionPad2d(self.pad_size)
        self.conv = nn.Conv2d(in_channels, out_channels, kernel_size, stride)
        self.norm = nn.InstanceNorm2d(out_channels, affine=True)
        self.activation = activation
        self._kind = _act_kind(activation)

    def _normed(self, x, relu=False, res=None):
        return ops.conv_instance_norm(x, self.conv.weight, self.conv.bias, self.norm.weight, self.norm.bias,
                                      stride=self.conv.stride[0], pad=self.pad_size, pad_mode="reflect", relu=relu,
                                      res=res, eps=self.norm.eps)

    def forward(self, x, image_out=False):
        """image_out: fuse StylizingNetwork's `(x + 1) / 2 * 255` into the Tanh kernel."""
        if self._kind == "tanh":
            return ops.tanh_image(self._normed(x), image=image_out)
        return self._normed(x, relu=self._kind == "relu")


class Res(nn.Module):
    """RT/network.py:29-46: conv2(conv1(x)) + x (residual zero-padded on channels if narrower)."""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.conv1 = Conv(in_channels, out_channels, 3, 1, nn.ReLU())
        self.conv2 = Conv(out_channels, out_channels, 3, 1, None)

    def forward(self, x):
        residual = x
        h = self.conv1(x)
        cout = self.conv2.conv.out_channels
        if residual.shape[1] != cout:
            pad = residual.new_zeros((residual.shape[0], cout - residual.shape[1]) + tuple(residual.shape[2:]))
            residual = torch.cat([residual, pad], 1)
        if self.conv2._kind is not None:
            raise VstError("Res: conv2 has no activation in the reference")
        return self.conv2._normed(h, res=residual)


class Deconv(nn.Module):
    """RT/network.py:49-62: ConvTranspose2d(k, stride, padding=1, output_padding=1) -> IN -> act."""

    def __init__(self, in_channels, out_channels, kernel_size, stride, activation=None):
        super().__init__()
        self.deconv = nn.ConvTranspose2d(in_channels, out_channels, kernel_size, stride, padding=1, output_padding=1)
        self.norm = nn.InstanceNorm2d(out_channels, affine=True)
        self.activation = activation
        self._kind = _act_kind(activation)

    def forward(self, x):
        d = self.deconv
        y = ops.conv_transpose_instance_norm(x, d.weight, d.bias, self.norm.weight, self.norm.bias, stride=d.stride[0],
                                             pad=d.padding[0], out_pad=d.output_padding[0],
                                             relu=self._kind == "relu", eps=self.norm.eps)
        if self._kind == "tanh":
            y = ops.tanh_image(y, image=False)
        return y


class StylizingNetwork(nn.Module):
    """RT/network.py:65-94."""

    def __init__(self):
        super().__init__()
        self.conv1 = Conv(3, 16, 3, 1, nn.ReLU())
        self.conv2 = Conv(16, 32, 3, 2, nn.ReLU())
        self.conv3 = Conv(32, 48, 3, 2, nn.ReLU())
        self.res1 = Res(48, 48)
        self.res2 = Res(48, 48)
        self.res3 = Res(48, 48)
        self.res4 = Res(48, 48)
        self.res5 = Res(48, 48)
        self.deconv1 = Deconv(48, 32, 3, 2, nn.ReLU())
        self.deconv2 = Deconv(32, 16, 3, 2, nn.ReLU())
        self.conv4 = Conv(16, 3, 3, 1, nn.Tanh())

    def forward(self, x):
        with ops.gemm_scope("stylizer"):
            x = self.conv1(x)
            x = self.conv2(x)
            x = self.conv3(x)
            x = self.res1(x)
            x = self.res2(x)
            x = self.res3(x)
            x = self.res4(x)
            x = self.res5(x)
            x = self.deconv1(x)
            x = self.deconv2(x)
            return self.conv4(x, image_out=True)
