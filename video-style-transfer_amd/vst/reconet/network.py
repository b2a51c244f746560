"""Drop-in MI355X implementation of RC/network.py (ReCoNet stylizer, SD1/SD2 students, Vgg16).

Same class names, constructor arguments, forward return types and state_dict keys as the
reference, so reference checkpoints load unchanged (`conv1.conv2d.weight`, `res1.in1.bias`,
`slice4.21.weight`, ...).  `nn.Conv2d` / `nn.InstanceNorm2d` are kept only as parameter
containers (and for their default initialisation); every forward and backward runs the HIP
kernels of libvst_hip.so through `vst.ops`:
  * reflection pad / nearest x2 upsample are folded into the conv's gather (never materialised),
  * InstanceNorm + ReLU (+ the residual add) is one kernel,
  * ConvTanh's `tanh(y/255)*150 + 255/2` is the conv epilogue,
  * VGG Conv+bias+ReLU is one kernel, MaxPool is its own kernel.
"""
from collections import namedtuple

import numpy as np
import torch
import torch.nn as nn

from .. import ops

VggOutputs = namedtuple("VggOutputs", ["relu1_2", "relu2_2", "relu3_3", "relu4_3"])

# torchvision VGG16 "D" features[0:23]
_VGG16_CFG = [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512]


def vgg_features(cfg, n_layers):
    """torchvision-layout `features` Sequential (Conv3x3 pad 1 / ReLU(inplace) / MaxPool2d(2,2))."""
    layers, cin = [], 3
    for v in cfg:
        if v == "M":
            layers.append(nn.MaxPool2d(kernel_size=2, stride=2))
        else:
            layers += [nn.Conv2d(cin, v, kernel_size=3, padding=1), nn.ReLU(inplace=True)]
            cin = v
    return layers[:n_layers]


def run_vgg_slice(seq, x, skip_pool=False, premasked_out=False):
    """Forward of one VGG slice on HIP kernels: Conv2d followed by ReLU -> fused conv+bias+relu.
    A ReLU output consumed only by the next module of the slice (a conv or a max-pool) never sees
    a separate ReLU-backward pass: the consumer's backward applies the mask (dgrad epilogue /
    pool backward) and the producer is marked premasked.  Slice outputs (loss features) keep it,
    unless premasked_out (the output goes through ops.feature_pool, whose backward masks);
    skip_pool: the slice's leading MaxPool2d already ran in ops.feature_pool."""
    mods = list(seq.children())
    if skip_pool:
        if not isinstance(mods[0], nn.MaxPool2d):
            raise RuntimeError("slice boundary without a leading MaxPool2d")
        mods = mods[1:]
    i = 0
    fuse_next = False  # the previous conv's ReLU output is consumed only by mods[i]
    while i < len(mods):
        m = mods[i]
        if isinstance(m, nn.Conv2d):
            relu = i + 1 < len(mods) and isinstance(mods[i + 1], nn.ReLU)
            nxt = mods[i + 2] if relu and i + 2 < len(mods) else None
            internal = relu and (isinstance(nxt, (nn.Conv2d, nn.MaxPool2d)) or (nxt is None and premasked_out))
            x = ops.conv2d(x, m.weight, m.bias, stride=m.stride[0], pad=m.padding[0], pad_mode="zero",
                           act="relu" if relu else None, mask_dx=fuse_next, premasked=internal)
            fuse_next = internal
            i += 2 if relu else 1
        elif isinstance(m, nn.MaxPool2d):
            x = ops.maxpool2x2(x, relu_mask=fuse_next)
            fuse_next = False
            i += 1
        elif isinstance(m, nn.ReLU):
            raise RuntimeError("standalone ReLU outside a conv+relu pair is not on the VGG path")
        else:
            raise RuntimeError(f"unsupported VGG layer {m}")
    return x


def _load_torchvision_features(layers, weights):
    """Optional pretrained weights from a local torchvision-format state dict (no download)."""
    if weights is None:
        return
    sd = torch.load(weights, map_location="cpu", weights_only=True)
    for idx, m in enumerate(layers):
        if isinstance(m, nn.Conv2d):
            m.weight.data.copy_(sd[f"features.{idx}.weight"])
            m.bias.data.copy_(sd[f"features.{idx}.bias"])


class Vgg16(nn.Module):
    """RC/network.py:9-40.  `weights`: path to a local torchvision vgg16 state dict; the reference
    downloads IMAGENET1K_V1 (no network here), otherwise torchvision's default init."""

    def __init__(self, device="cpu", weights=None):
        super().__init__()
        feats = vgg_features(_VGG16_CFG, 23)
        _load_torchvision_features(feats, weights)
        self.slice1 = nn.Sequential()
        self.slice2 = nn.Sequential()
        self.slice3 = nn.Sequential()
        self.slice4 = nn.Sequential()
        for x in range(4):
            self.slice1.add_module(str(x), feats[x].to(device))
        for x in range(4, 9):
            self.slice2.add_module(str(x), feats[x].to(device))
        for x in range(9, 16):
            self.slice3.add_module(str(x), feats[x].to(device))
        for x in range(16, 23):
            self.slice4.add_module(str(x), feats[x].to(device))
        for p in self.parameters():
            p.requires_grad = False

    def forward(self, X):
        return VggOutputs(*self.features_upto(X, 4))

    def features_upto(self, X, n):
        """relu1_2 .. the n-th slice output only (the trainer's content pass needs relu3_3 alone,
        so its slice-4 convolutions are skipped; the outputs computed are identical).
        Slice outputs that feed the next slice are loss features AND that slice's pool input:
        pool, gradient sum and ReLU backward fuse at each boundary (ops.feature_pool)."""
        slices = (self.slice1, self.slice2, self.slice3, self.slice4)[:n]
        outs, x = [], X
        for i, sl in enumerate(slices):
            last = i == len(slices) - 1
            h = run_vgg_slice(sl, x, skip_pool=i > 0, premasked_out=not last)
            if not last:
                h, x = ops.feature_pool(h)
            outs.append(h)
        return outs


class SelectiveLoadModule(torch.nn.Module):
    """RC/network.py:46-60 (name-filtered load_state_dict)."""

    def forward(self, x):
        return x

    def load_state_dict(self, state_dict):
        own_state = self.state_dict()
        for name, param in state_dict.items():
            if name in own_state:
                own_state[name].copy_(param)


class ConvLayer(nn.Module):
    """RC/network.py:63-75: ReflectionPad2d(k//2) -> Conv2d (pad folded into the gather)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride, bias=True):
        super().__init__()
        self.reflection_padding = int(np.floor(kernel_size / 2))
        self.reflection_pad = nn.ReflectionPad2d(self.reflection_padding)  # kept for module parity
        self.conv2d = nn.Conv2d(in_channels, out_channels, kernel_size, stride=stride, bias=bias)

    def _conv(self, x, act=None, up=1):
        return ops.conv2d(x, self.conv2d.weight, self.conv2d.bias, stride=self.conv2d.stride[0],
                          pad=self.reflection_padding, pad_mode="reflect", up=up, act=act)

    def forward(self, x):
        return self._conv(x)


class ConvTanh(ConvLayer):
    """RC/network.py:78-85: tanh(conv/255) * 150 + 255/2 as the conv epilogue."""

    def __init__(self, in_channels, out_channels, kernel_size, stride):
        super().__init__(in_channels, out_channels, kernel_size, stride)
        self.tanh = nn.Tanh()

    def forward(self, x):
        return self._conv(x, act="tanh")


class ConvInstRelu(ConvLayer):
    """RC/network.py:88-98."""

    def __init__(self, in_channels, out_channels, kernel_size, stride):
        super().__init__(in_channels, out_channels, kernel_size, stride)
        self.instance = nn.InstanceNorm2d(out_channels, affine=True)
        self.relu = nn.ReLU()

    def forward(self, x):
        c = self.conv2d
        return ops.conv_instance_norm(x, c.weight, c.bias, self.instance.weight, self.instance.bias, c.stride[0],
                                      self.reflection_padding, "reflect", 1, relu=True, eps=self.instance.eps)


class UpsampleConvLayer(nn.Module):
    """RC/network.py:101-120: nearest x`upsample` -> reflect pad -> conv, all in the conv gather."""

    def __init__(self, in_channels, out_channels, kernel_size, stride, upsample=None):
        super().__init__()
        self.upsample = upsample
        self.reflection_padding = int(np.floor(kernel_size / 2))
        self.reflection_pad = nn.ReflectionPad2d(self.reflection_padding)
        self.conv2d = nn.Conv2d(in_channels, out_channels, kernel_size, stride)
        if upsample not in (None, 1, 2):
            raise ValueError("only nearest x2 upsampling is on the reference path")

    def _conv(self, x):
        return ops.conv2d(x, self.conv2d.weight, self.conv2d.bias, stride=self.conv2d.stride[0],
                          pad=self.reflection_padding, pad_mode="reflect", up=self.upsample or 1)

    def forward(self, x):
        return self._conv(x)


class UpsampleConvInstRelu(UpsampleConvLayer):
    """RC/network.py:123-133."""

    def __init__(self, in_channels, out_channels, kernel_size, stride, upsample=None):
        super().__init__(in_channels, out_channels, kernel_size, stride, upsample)
        self.instance = nn.InstanceNorm2d(out_channels, affine=True)
        self.relu = nn.ReLU()

    def forward(self, x):
        c = self.conv2d
        return ops.conv_instance_norm(x, c.weight, c.bias, self.instance.weight, self.instance.bias, c.stride[0],
                                      self.reflection_padding, "reflect", self.upsample or 1, relu=True,
                                      eps=self.instance.eps)


class ResidualBlock(nn.Module):
    """RC/network.py:136-150: IN2(conv2(relu(IN1(conv1 x)))) + x, the add fused into IN2."""

    def __init__(self, in_channels, out_channels, kernel_size=3, stride=1):
        super().__init__()
        self.conv1 = ConvLayer(in_channels, out_channels, kernel_size, stride)
        self.in1 = nn.InstanceNorm2d(out_channels, affine=True)
        self.conv2 = ConvLayer(out_channels, out_channels, kernel_size, stride)
        self.in2 = nn.InstanceNorm2d(out_channels, affine=True)
        self.relu = nn.ReLU()

    def forward(self, x):
        c1, c2 = self.conv1.conv2d, self.conv2.conv2d
        p1, p2 = self.conv1.reflection_padding, self.conv2.reflection_padding
        # x feeds conv1 and the skip: their gradients meet in one vst_sum4 pass (ops.fork)
        xc, xs = ops.fork(x, 2)
        with ops.gemm_scope("res"):
            out = ops.conv_instance_norm(xc, c1.weight, c1.bias, self.in1.weight, self.in1.bias, c1.stride[0], p1,
                                         relu=True, eps=self.in1.eps)
            return ops.conv_instance_norm(out, c2.weight, c2.bias, self.in2.weight, self.in2.bias, c2.stride[0], p2,
                                          relu=False, res=xs, eps=self.in2.eps)


class ReCoNet(nn.Module):
    """RC/network.py:153-190 -> (sd1, features, out)."""

    def __init__(self, input_frame_num=1):
        super().__init__()
        self.conv1 = ConvInstRelu(3 * input_frame_num, 48, kernel_size=9, stride=1)
        self.conv2 = ConvInstRelu(48, 96, kernel_size=3, stride=2)
        self.conv3 = ConvInstRelu(96, 192, kernel_size=3, stride=2)
        self.res1 = ResidualBlock(192, 192)
        self.res2 = ResidualBlock(192, 192)
        self.res3 = ResidualBlock(192, 192)
        self.res4 = ResidualBlock(192, 192)
        self.res5 = ResidualBlock(192, 192)
        self.deconv1 = UpsampleConvInstRelu(192, 96, kernel_size=3, stride=1, upsample=2)
        self.deconv2 = UpsampleConvInstRelu(96, 48, kernel_size=3, stride=1, upsample=2)
        self.deconv3 = ConvTanh(48, 3, kernel_size=9, stride=1)

    def forward(self, x):
        with ops.gemm_scope("stylizer"):
            return self._forward(x)

    def _forward(self, x):
        x = self.conv1(x)
        x = self.conv2(x)
        x = self.conv3(x)
        x = self.res1(x)
        x = self.res2(x)
        x = self.res3(x)
        x = self.res4(x)
        x = self.res5(x)
        x, features = ops.fork(x, 2)  # read by deconv1 and by the caller's feature temporal loss
        x = self.deconv1(x)
        sd1 = x
        x = self.deconv2(x)
        x = self.deconv3(x)
        return (sd1, features, x)


class ReCoNetSD1(nn.Module):
    """RC/network.py:193-237 -> (sd2, sd, features, out)."""

    def __init__(self, input_frame_num=1):
        super().__init__()
        self.conv1 = ConvInstRelu(3 * input_frame_num, 32, kernel_size=9, stride=1)
        self.conv2 = ConvInstRelu(32, 64, kernel_size=3, stride=2)
        self.conv3_sd = ConvInstRelu(64, 64, kernel_size=3, stride=2)
        self.res1_sd = ResidualBlock(64, 64)
        self.res2_sd = ResidualBlock(64, 64)
        self.res3_sd = ResidualBlock(64, 64)
        self.res4_sd = ResidualBlock(64, 64)
        self.res5_sd = ResidualBlock(64, 64)
        self.deconv1_sd = UpsampleConvInstRelu(64, 64, kernel_size=3, stride=1, upsample=2)
        self.deconv2 = UpsampleConvInstRelu(64, 32, kernel_size=3, stride=1, upsample=2)
        self.deconv3 = ConvTanh(32, 3, kernel_size=9, stride=1)

    def forward(self, x):
        with ops.gemm_scope("stylizer"):
            return self._forward(x)

    def _forward(self, x):
        x = self.conv1(x)
        x = self.conv2(x)
        x = self.conv3_sd(x)
        sd2 = x
        x = self.res1_sd(x)
        x = self.res2_sd(x)
        x = self.res3_sd(x)
        x = self.res4_sd(x)
        x = self.res5_sd(x)
        x, features = ops.fork(x, 2)
        x = self.deconv1_sd(x)
        sd = x
        x = self.deconv2(x)
        x = self.deconv3(x)
        return (sd2, sd, features, x)


class ReCoNetSD2(nn.Module):
    """RC/network.py:240-279 -> (sd, features, out)."""

    def __init__(self, input_frame_num=1):
        super().__init__()
        self.conv1_sd2 = ConvInstRelu(3 * input_frame_num, 16, kernel_size=9, stride=1)
        self.conv2_sd2 = ConvInstRelu(16, 32, kernel_size=3, stride=2)
        self.conv3_sd2 = ConvInstRelu(32, 64, kernel_size=3, stride=2)
        self.res1_sd = ResidualBlock(64, 64)
        self.res2_sd = ResidualBlock(64, 64)
        self.res3_sd = ResidualBlock(64, 64)
        self.res4_sd = ResidualBlock(64, 64)
        self.res5_sd = ResidualBlock(64, 64)
        self.deconv1_sd2 = UpsampleConvInstRelu(64, 32, kernel_size=3, stride=1, upsample=2)
        self.deconv2_sd2 = UpsampleConvInstRelu(32, 16, kernel_size=3, stride=1, upsample=2)
        self.deconv3_sd2 = ConvTanh(16, 3, kernel_size=9, stride=1)

    def forward(self, x):
        with ops.gemm_scope("stylizer"):
            return self._forward(x)

    def _forward(self, x):
        x = self.conv1_sd2(x)
        x = self.conv2_sd2(x)
        x = self.conv3_sd2(x)
        sd = x
        x = self.res1_sd(x)
        x = self.res2_sd(x)
        x = self.res3_sd(x)
        x = self.res4_sd(x)
        x = self.res5_sd(x)
        x, features = ops.fork(x, 2)
        x = self.deconv1_sd2(x)
        x = self.deconv2_sd2(x)
        x = self.deconv3_sd2(x)
        return (sd, features, x)
