"""The halo weight gradient (csrc/wgrad_halo.hip) of 3x3 stride-1 pad-1 convolutions -- ResidualBlock
(RC/network.py:136-150) and the AdaAttN decoder convs (AA/network.py:9-33) -- against the row-tiled
kernel (VST_GEMM_PERTAP in the call's mode: the same products, another fp32 summation order) and
float64.  Shapes cover the step's layer widths (192 residual, 64 / 128 / 256 decoder), ragged heights,
several row chunks and strips, both borders, accumulate, and the three split-product modes."""
import pytest
import torch

from vst._lib import lib

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF16, BF16X6, F16, PERTAP = 2, 3, 4, 32
TOL = {BF16X6: 5e-6, F16: 3e-3, BF16: 2e-2}  # max |err| / max |dW| vs float64


def _rand(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(DEV)


def _wgrad(dy, x, Cout, gmode, mode, out=None):
    N, Cin, H, W = x.shape
    nf = lib.vst_conv_wgrad_workspace(N, Cin, H, W, Cout, H, W, 3, 3, gmode, 1, 1, 1, mode)
    assert nf > 0
    ws = torch.empty(nf, device=DEV)
    acc = out is not None
    dw = torch.full((Cout, Cin, 3, 3), float("nan"), device=DEV) if out is None else out
    lib.vst_conv_wgrad(dy.data_ptr(), x.data_ptr(), dw.data_ptr(), ws.data_ptr(), nf, N, Cin, H, W, Cout, H, W, 3, 3,
                       gmode, 1, 1, 1, int(acc), mode, torch.cuda.current_stream().cuda_stream)
    return dw


def _ref(dy, x, gmode):
    x64 = x.double()
    xp = torch.nn.functional.pad(x64, (1, 1, 1, 1), mode="reflect" if gmode == 0 else "constant")
    return torch.nn.grad.conv2d_weight(xp, (dy.shape[1], x.shape[1], 3, 3), dy.double())


# (N, Cin, H, W, Cout): residual 192 (ragged rows, several strips), decoder widths, tall (row chunks)
# (the single-product modes walk 32-column strips on 64-row tiles and 64-column strips on 128-row ones:
# other widths fall back to the row-tiled kernel)
SHAPES = [(2, 192, 20, 48, 192), (2, 192, 20, 48, 64), (1, 64, 9, 32, 64), (2, 128, 16, 64, 128), (1, 256, 8, 16, 256),
          (1, 32, 70, 16, 64), (3, 96, 13, 32, 192), (2, 64, 11, 96, 64), (1, 128, 7, 128, 64), (1, 64, 6, 192, 256),
          (2, 32, 5, 128, 128)]


@pytest.mark.parametrize("mode", [BF16X6, F16, BF16])
@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("gmode", [0, 1])
def test_halo_wgrad_vs_rowtiled_and_fp64(mode, shape, gmode):
    N, Cin, H, W, Cout = shape
    x = _rand(N, Cin, H, W, seed=1, scale=2.0)
    dy = _rand(N, Cout, H, W, seed=2, scale=0.5)
    halo = _wgrad(dy, x, Cout, gmode, mode)
    rowt = _wgrad(dy, x, Cout, gmode, mode | PERTAP)
    torch.cuda.synchronize()
    assert torch.isfinite(halo).all()
    ref = _ref(dy, x, gmode)
    scale = float(ref.abs().max())
    err = float((halo.double() - ref).abs().max()) / scale
    err_rt = float((rowt.double() - ref).abs().max()) / scale
    assert err < TOL[mode], (err, err_rt)
    # the two kernels form the same products: they agree to the mode's product rounding
    assert float((halo - rowt).abs().max()) / scale < 2 * TOL[mode]


def test_halo_wgrad_accumulate_and_deterministic():
    N, Cin, H, W, Cout = 2, 192, 12, 32, 192
    x = _rand(N, Cin, H, W, seed=3)
    dy = _rand(N, Cout, H, W, seed=4)
    base = _rand(Cout, Cin, 3, 3, seed=5)
    a = _wgrad(dy, x, Cout, 0, BF16X6, out=base.clone())
    b = _wgrad(dy, x, Cout, 0, BF16X6)
    c = _wgrad(dy, x, Cout, 0, BF16X6)
    torch.cuda.synchronize()
    assert torch.equal(b, c)  # fixed slab order: bitwise reproducible
    assert float((a - (b + base)).abs().max()) <= 1e-6 * float(a.abs().max())


def test_halo_wgrad_workspace_query():
    """The workspace query plans exactly what the launch uses; shapes outside the halo kernel's
    domain (odd width, stride 2, fp32 mode) keep the row-tiled kernel's size."""
    q = lib.vst_conv_wgrad_workspace
    assert q(16, 192, 64, 128, 192, 64, 128, 3, 3, 0, 1, 1, 1, F16) > 0
    assert q(16, 192, 64, 128, 192, 64, 128, 3, 3, 0, 1, 1, 1, F16) != q(16, 192, 64, 128, 192, 64, 128, 3, 3, 0, 1,
                                                                        1, 1, F16 | PERTAP)
    # (the kernel choice is the caller's: vst.ops keeps ReCoNet's bf16x6 192-row layers on the
    # row-tiled kernel by passing VST_GEMM_PERTAP)
    assert q(16, 192, 64, 128, 192, 64, 128, 3, 3, 0, 1, 1, 1, BF16X6) != q(16, 192, 64, 128, 192, 64, 128, 3, 3, 0, 1,
                                                                           1, 1, BF16X6 | PERTAP)
    assert q(2, 192, 9, 15, 192, 9, 15, 3, 3, 0, 1, 1, 1, BF16X6) == lib.vst_wgrad_workspace(2, 192, 1728, 135)
    assert q(2, 192, 8, 16, 192, 8, 16, 3, 3, 0, 1, 1, 1, 0) == lib.vst_wgrad_workspace(2, 192, 1728, 128)


def test_halo_wgrad_undersized_workspace_runs_rowtiled():
    """vst_conv_wgrad takes the workspace's size: a caller that sizes it by the row-tiled
    kernel's rule (vst_wgrad_workspace) below the halo slabs gets the row-tiled kernel -- bitwise the
    VST_GEMM_PERTAP result -- instead of an out-of-bounds slab write; below both sizes the call is
    refused."""
    from vst._lib import VstError

    # (a shape whose halo slabs outgrow the row-tiled workspace: few channel blocks, many strips)
    N, Cin, H, W, Cout = 1, 32, 128, 256, 32
    x = _rand(N, Cin, H, W, seed=6)
    dy = _rand(N, Cout, H, W, seed=7)
    st = torch.cuda.current_stream().cuda_stream
    for mode in (BF16X6, F16):
        halo_nf = lib.vst_conv_wgrad_workspace(N, Cin, H, W, Cout, H, W, 3, 3, 0, 1, 1, 1, mode)
        rt_nf = lib.vst_wgrad_workspace(N, Cout, 9 * Cin, H * W)
        assert halo_nf > rt_nf > 0, (halo_nf, rt_nf)
        ws = torch.empty(rt_nf, device=DEV)
        dw = torch.full((Cout, Cin, 3, 3), float("nan"), device=DEV)
        lib.vst_conv_wgrad(dy.data_ptr(), x.data_ptr(), dw.data_ptr(), ws.data_ptr(), rt_nf, N, Cin, H, W, Cout, H, W,
                           3, 3, 0, 1, 1, 1, 0, mode, st)
        ref = _wgrad(dy, x, Cout, 0, mode | PERTAP)
        torch.cuda.synchronize()
        assert torch.equal(dw, ref)
        with pytest.raises(VstError):
            lib.vst_conv_wgrad(dy.data_ptr(), x.data_ptr(), dw.data_ptr(), ws.data_ptr(), rt_nf - 1, N, Cin, H, W,
                               Cout, H, W, 3, 3, 0, 1, 1, 1, 0, mode, st)


# (N, Cin, H, W, Cout): the AdaAttN decoder's last conv (64 -> 3), one-quad-per-lane widths with several
# row lanes per block (W 12, 32), two column blocks (W 1040), 1 / 2 / 4 output channels, ragged rows
THIN_SHAPES = [(2, 64, 16, 32, 3), (1, 8, 9, 12, 3), (1, 16, 7, 1040, 3), (1, 4, 5, 8, 1), (2, 12, 37, 16, 4),
               (3, 64, 10, 64, 2), (1, 64, 130, 256, 3)]


@pytest.mark.parametrize("shape", THIN_SHAPES)
@pytest.mark.parametrize("gmode", [0, 1])
@pytest.mark.parametrize("mode", [BF16X6, F16])
def test_thin_wgrad_vs_fp64(shape, gmode, mode):
    """Cout <= 4 (AA/network.py:99, the decoder's last conv): vst_conv_wgrad runs the fp32 VALU kernel
    whatever the mode's MFMA arithmetic -- within fp32 summation error of float64, and against the
    row-tiled GEMM (VST_GEMM_PERTAP) to that GEMM's own product rounding."""
    N, Cin, H, W, Cout = shape
    x = _rand(N, Cin, H, W, seed=11, scale=2.0)
    dy = _rand(N, Cout, H, W, seed=12, scale=0.5)
    thin = _wgrad(dy, x, Cout, gmode, mode)
    rowt = _wgrad(dy, x, Cout, gmode, mode | PERTAP)
    torch.cuda.synchronize()
    ref = _ref(dy, x, gmode)
    scale = float(ref.abs().max())
    err = float((thin.double() - ref).abs().max()) / scale
    assert err < 2e-6, err
    assert float((rowt.double() - ref).abs().max()) / scale < TOL[mode]


def test_thin_wgrad_accumulate_deterministic_and_workspace():
    N, Cin, H, W, Cout = 2, 64, 24, 64, 3
    x = _rand(N, Cin, H, W, seed=13)
    dy = _rand(N, Cout, H, W, seed=14)
    base = _rand(Cout, Cin, 3, 3, seed=15)
    a = _wgrad(dy, x, Cout, 0, F16, out=base.clone())
    b = _wgrad(dy, x, Cout, 0, F16)
    c = _wgrad(dy, x, Cout, 0, BF16X6)
    torch.cuda.synchronize()
    assert torch.equal(b, c)  # fp32 VALU: the mode does not enter
    assert torch.equal(a, b + base)  # the reduce adds the slab sum onto dw in one rounding
    q = lib.vst_conv_wgrad_workspace
    assert q(N, Cin, H, W, Cout, H, W, 3, 3, 0, 1, 1, 1, F16) != q(N, Cin, H, W, Cout, H, W, 3, 3, 0, 1, 1, 1, F16 | PERTAP)


@pytest.mark.parametrize("shape", THIN_SHAPES)
@pytest.mark.parametrize("reflect", [True, False])
@pytest.mark.parametrize("masked", [True, False])
def test_thin_dgrad_vs_fp64(shape, reflect, masked):
    """Cout <= 4 data gradient (the AdaAttN decoder's last conv under its fused ReLU mask,
    AA/network.py:99): vst_conv_dgrad_thin -- interior on the VALU, the reflect ring folded by
    vst_fold_border -- against float64 autograd of the padded conv, masked by x > 0."""
    from vst._lib import lib as L

    N, Cin, H, W, Cout = shape
    x = _rand(N, Cin, H, W, seed=21)
    w = _rand(Cout, Cin, 3, 3, seed=22, scale=0.1)
    dy = _rand(N, Cout, H, W, seed=23)
    dx = torch.full_like(x, float("nan"))
    border = torch.full((N, Cin, H + 2, W + 2), float("nan"), device=DEV) if reflect else None
    st = torch.cuda.current_stream().cuda_stream
    assert L.vst_conv_dgrad_thin(dy.data_ptr(), w.data_ptr(), x.data_ptr() if masked else None, dx.data_ptr(),
                                 border.data_ptr() if reflect else None, N, Cout, Cin, H, W, int(reflect), st) == 0
    torch.cuda.synchronize()
    xd = torch.zeros(N, Cin, H, W, dtype=torch.float64, device=DEV, requires_grad=True)
    xp = torch.nn.functional.pad(xd, (1, 1, 1, 1), mode="reflect" if reflect else "constant")
    torch.nn.functional.conv2d(xp, w.double()).backward(dy.double())
    ref = xd.grad * (x > 0).double() if masked else xd.grad
    err = float((dx.double() - ref).abs().max()) / float(ref.abs().max())
    assert err < 2e-6, err
