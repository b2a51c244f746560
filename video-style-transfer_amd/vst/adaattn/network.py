"""Drop-in MI355X implementation of AA/network.py (AdaAttN stylizing network).

Same class names, constructor arguments and state_dict keys as the reference
(`adaattn.0.f.weight`, `decoder.conv3.1.conv.conv.bias`, `decoder.conv8.conv.weight`, ...), so
reference checkpoints load unchanged.  `nn.Conv2d` modules are parameter containers; every
forward and backward runs libvst_hip.so kernels through `vst.ops` / `vst.adaattn.attention`:
  * reflection pad is folded into the conv gather, conv + bias + ReLU is one kernel,
  * the decoder's `interpolate(x5) + x4` and `cat([interpolate(x), x3])` write one buffer,
  * the 1x1 f/g/h convs are MFMA GEMMs; the cosine attention never forms the Nc x Ns matrix (its
    two moments are an exact re-association over the style positions) and the softmax attention
    forms it in blocks of query rows (see attention.py).
"""
import numpy as np
import torch
import torch.nn as nn

from .. import ops
from .attention import COSINE, SOFTMAX, adaattn, instance_norm_plain
from .utilities import feature_down_sample


class Conv(nn.Module):
    """AA/network.py:11-21: ReflectionPad2d(k//2) + Conv2d."""

    def __init__(self, in_channels, out_channels, kernel_size, stride):
        super().__init__()
        pad = int(np.floor(kernel_size / 2))
        self.pad = nn.ReflectionPad2d(pad)
        self.conv = nn.Conv2d(in_channels, out_channels, kernel_size, stride)

    def run(self, x, act=None, mask_dx=False, premasked=False):
        c = self.conv
        return ops.conv2d(x, c.weight, c.bias, stride=c.stride[0], pad=self.pad.padding[0], pad_mode="reflect", act=act,
                          mask_dx=mask_dx, premasked=premasked)

    def forward(self, x):
        return self.run(x)


class ConvReLU(nn.Module):
    """AA/network.py:24-33."""

    def __init__(self, in_channels, out_channels, kernel_size, stride):
        super().__init__()
        self.conv = Conv(in_channels, out_channels, kernel_size, stride)
        self.relu = nn.ReLU()

    def run(self, x, act="relu", mask_dx=False, premasked=False):
        return self.conv.run(x, act=act, mask_dx=mask_dx, premasked=premasked)

    def forward(self, x):
        return self.conv.run(x, act="relu")


class ConvTanh(nn.Module):
    """AA/network.py:36-46: (tanh(conv(x)) + 1) / 2 * 255 (defined, not used by StylizingNetwork):
    the conv kernel, then the tanh-image kernel (forward and backward on the device)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride):
        super().__init__()
        self.conv = Conv(in_channels, out_channels, kernel_size, stride)
        self.tanh = nn.Tanh()

    def forward(self, x):
        return ops.tanh_image(self.conv.run(x), image=True)


class ConvReluInterpolate(nn.Module):
    """AA/network.py:49-60."""

    def __init__(self, in_channels, out_channels, kernel_size, stride, scale_factor):
        super().__init__()
        self.conv = Conv(in_channels, out_channels, kernel_size, stride)
        self.relu = nn.ReLU()
        self.scale_factor = scale_factor

    def forward(self, x):
        y = self.conv.run(x, act="relu")
        if self.scale_factor == 2:
            return ops.upsample2x(y)
        # F.interpolate(scale_factor=s, bilinear, align_corners=False): output floor(H s) x floor(W s),
        # output pixel i reads source (i + 0.5) / s - 0.5 -- any s, whole-number output or not
        return ops.interpolate_scale(y, self.scale_factor)


class Decoder(nn.Module):
    """AA/network.py:63-99."""

    def __init__(self):
        super().__init__()
        self.conv1 = ConvReLU(512, 512, kernel_size=3, stride=1)
        self.conv2 = ConvReLU(512, 256, kernel_size=3, stride=1)
        self.conv3 = nn.Sequential(
            ConvReLU(512, 256, kernel_size=3, stride=1),
            ConvReLU(256, 256, kernel_size=3, stride=1),
            ConvReLU(256, 256, kernel_size=3, stride=1),
        )
        self.conv4 = ConvReLU(256, 128, kernel_size=3, stride=1)
        self.conv5 = ConvReLU(128, 128, kernel_size=3, stride=1)
        self.conv6 = ConvReLU(128, 64, kernel_size=3, stride=1)
        self.conv7 = ConvReLU(64, 64, kernel_size=3, stride=1)
        self.conv8 = Conv(64, 3, kernel_size=3, stride=1)

    def forward(self, x5, x4, x3):
        with ops.gemm_scope("stylizer"), ops.gemm_scope("dec"):  # channel-blocked K order (ops.gemm_role)
            return self._forward(x5, x4, x3)

    def _forward(self, x5, x4, x3):
        # a ConvReLU whose output only feeds the next conv leaves its ReLU backward to that conv's
        # data gradient (premasked -> mask_dx: the mask is applied in the dgrad epilogue and border
        # fold); one whose output feeds an upsample leaves it to the upsample's adjoint (relu_mask)
        def run(m, x, mask_dx=False, premasked=False):
            return m.run(x, act="relu" if isinstance(m, ConvReLU) else None, mask_dx=mask_dx, premasked=premasked)

        x = ops.upsample2x(x5, addend=x4)
        x = run(self.conv1, x, premasked=True)
        x = ops.upsample_cat(run(self.conv2, x, mask_dx=True, premasked=True), x3, relu_mask=True)
        x = run(self.conv3[0], x, premasked=True)
        x = run(self.conv3[1], x, mask_dx=True, premasked=True)
        x = run(self.conv3[2], x, mask_dx=True, premasked=True)
        x = ops.upsample2x(run(self.conv4, x, mask_dx=True, premasked=True), relu_mask=True)
        x = run(self.conv5, x, premasked=True)
        x = ops.upsample2x(run(self.conv6, x, mask_dx=True, premasked=True), relu_mask=True)
        x = run(self.conv7, x, premasked=True)
        return run(self.conv8, x, mask_dx=True)


class Softmax(nn.Module):
    """AA/network.py:102-108 (marker module: the attention kernels read `kind`)."""

    kind = SOFTMAX

    def __init__(self):
        super().__init__()
        self.softmax = nn.Softmax(dim=-1)


class CosineSimilarity(nn.Module):
    """AA/network.py:111-125 (marker module)."""

    kind = COSINE


def _activation(name):
    if name == "softmax":
        return Softmax()
    if name == "cosine":
        return CosineSimilarity()
    raise ValueError(f"Unknown activation function: {name}")


class AdaAttnNoConv(nn.Module):
    """AA/network.py:128-171: attention on instance-normalised features, no projections."""

    def __init__(self, v_dim, qk_dim, activation="softmax"):
        super().__init__()
        self.norm_q = nn.InstanceNorm2d(qk_dim, affine=False)
        self.norm_k = nn.InstanceNorm2d(qk_dim, affine=False)
        self.norm_v = nn.InstanceNorm2d(v_dim, affine=False)
        self.activation = _activation(activation)

    def forward(self, c_x, s_x, c_1x, s_1x):
        Q = instance_norm_plain(c_1x)
        K = instance_norm_plain(s_1x)
        return adaattn(Q, K, s_x.contiguous(), instance_norm_plain(c_x), self.activation.kind)


class AdaAttN(nn.Module):
    """AA/network.py:174-220: Q = f(IN(c_1x)), K = g(IN(s_1x)), V = h(s_x)."""

    def __init__(self, v_dim, qk_dim, activation="softmax"):
        super().__init__()
        self.f = nn.Conv2d(qk_dim, qk_dim, 1)
        self.g = nn.Conv2d(qk_dim, qk_dim, 1)
        self.h = nn.Conv2d(v_dim, v_dim, 1)
        self.norm_q = nn.InstanceNorm2d(qk_dim, affine=False)
        self.norm_k = nn.InstanceNorm2d(qk_dim, affine=False)
        self.norm_v = nn.InstanceNorm2d(v_dim, affine=False)
        self.activation = _activation(activation)

    def forward(self, c_x, s_x, c_1x, s_1x):
        with ops.gemm_scope("stylizer"):
            return self._forward(c_x, s_x, c_1x, s_1x)

    def _forward(self, c_x, s_x, c_1x, s_1x):
        with ops.gemm_scope("attn"):  # policy key "stylizer.attn.<role>" (fp16 policy: bf16x3 here)
            Q = ops.conv2d(instance_norm_plain(c_1x), self.f.weight, self.f.bias)
            K = ops.conv2d(instance_norm_plain(s_1x), self.g.weight, self.g.bias)
            V = ops.conv2d(s_x, self.h.weight, self.h.bias)
        return adaattn(Q, K, V, instance_norm_plain(c_x), self.activation.kind)


class StylizingNetwork(nn.Module):
    """AA/network.py:223-251."""

    def __init__(self, activation="softmax"):
        super().__init__()
        self.adaattn = nn.ModuleList([
            AdaAttN(256, 64 + 128 + 256, activation=activation),
            AdaAttN(512, 64 + 128 + 256 + 512, activation=activation),
            AdaAttN(512, 64 + 128 + 256 + 512 + 512, activation=activation),
        ])
        self.decoder = Decoder()

    def forward(self, fc, fs, down=None):
        """down (optional, not in the reference's signature): ({idx: feature_down_sample(fc, idx)},
        {idx: feature_down_sample(fs, idx)}) for idx 2..4, already formed by the caller (the
        trainers form them once per step for the model and the AdaAttnNoConv loss targets)."""
        with ops.gemm_scope("stylizer"):
            return self._forward(fc, fs, down)

    def _forward(self, fc, fs, down=None):
        fc = list(fc.values())
        fs = list(fs.values())
        outs = []
        for i in range(3):
            idx = i + 2
            c_1x = feature_down_sample(fc, idx) if down is None else down[0][idx]
            s_1x = feature_down_sample(fs, idx) if down is None else down[1][idx]
            outs.append(self.adaattn[i](fc[idx], fs[idx], c_1x, s_1x))
        return self.decoder(outs[2], outs[1], outs[0])
