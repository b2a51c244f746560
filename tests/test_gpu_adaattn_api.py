"""The public AA/network.py blocks that StylizingNetwork does not use, against the reference's own
definitions restated in torch fp64 (AA/network.py:36-46 ConvTanh, :49-60 ConvReluInterpolate):
forward and input / parameter gradients on the HIP path."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref_conv(x, w, b):
    return F.conv2d(F.pad(x, (1, 1, 1, 1), mode="reflect"), w, b)


def _check(mod, ref_fn, x, tol):
    xd = x.to(DEV).requires_grad_(True)
    y = mod(xd)
    g = torch.randn(y.shape, generator=torch.Generator().manual_seed(5)).to(DEV)
    y.backward(g)
    w = mod.conv.conv.weight.detach().double().cpu().requires_grad_(True)
    b = mod.conv.conv.bias.detach().double().cpu().requires_grad_(True)
    xr = x.double().requires_grad_(True)
    yr = ref_fn(xr, w, b)
    yr.backward(g.double().cpu())
    assert y.shape == yr.shape
    rel = lambda a, r: float((a.detach().double().cpu() - r).abs().max() / r.abs().max())  # noqa: E731
    assert rel(y, yr.detach()) < tol
    assert rel(xd.grad, xr.grad) < tol
    assert rel(mod.conv.conv.weight.grad, w.grad) < tol
    assert rel(mod.conv.conv.bias.grad, b.grad) < tol


def test_conv_tanh_forward_backward():
    from vst.adaattn.network import ConvTanh

    torch.manual_seed(0)
    m = ConvTanh(64, 3, 3, 1).to(DEV)
    with torch.no_grad():
        m.conv.conv.weight.mul_(0.5)
    x = torch.randn(2, 64, 20, 36) * 2
    _check(m, lambda x, w, b: (torch.tanh(_ref_conv(x, w, b)) + 1) / 2 * 255, x, 1e-4)


@pytest.mark.parametrize("scale", [2, 0.5, 4])
def test_conv_relu_interpolate_scales(scale):
    from vst.adaattn.network import ConvReluInterpolate

    torch.manual_seed(1)
    m = ConvReluInterpolate(32, 48, 3, 1, scale).to(DEV)
    x = torch.randn(2, 32, 16, 24)
    _check(m, lambda x, w, b: F.interpolate(F.relu(_ref_conv(x, w, b)), scale_factor=scale, mode="bilinear",
                                            align_corners=False), x, 1e-4)


@pytest.mark.parametrize("scale", [1.5, 0.7, 3.3, 0.25])
def test_conv_relu_interpolate_inexact_sizes(scale):
    """Scale factors whose output is not H*s x W*s exactly (7 x 9 maps): output floor(H s) x floor(W s),
    source coordinate (d + 0.5) / s - 0.5 -- F.interpolate's own mapping, forward and backward."""
    from vst.adaattn.network import ConvReluInterpolate

    torch.manual_seed(2)
    m = ConvReluInterpolate(16, 16, 3, 1, scale).to(DEV)
    x = torch.randn(2, 16, 7, 9)
    _check(m, lambda x, w, b: F.interpolate(F.relu(_ref_conv(x, w, b)), scale_factor=scale, mode="bilinear",
                                            align_corners=False), x, 1e-4)
