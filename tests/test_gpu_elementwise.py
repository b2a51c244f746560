"""Vector / row-grid forms of the pooling, resize and attention elementwise kernels, on a real MI355X.

The library picks them when the shapes and alignments allow (W % 4 == 0 and 16-byte aligned planes
for the 2x2 max-pool, a plane count that fits the grid for resize / outer_axpy / column-norm
adjoint / copy_planes, n % 4 == 0 for the ReLU backward) and falls back to the flat per-element
kernels otherwise; both forms are checked here against the torch fp32 CPU reference of the same op
(MaxPool2d routes a window's gradient to its first maximum in scan order; F.interpolate bilinear,
align_corners=False, AA/network.py:59 / AA/utilities.py:98-109).  Pooling and copies are bit-exact;
resize within 1e-6 relative.
"""
import pytest
import torch
import torch.nn.functional as F

from conftest import rel_err

pytestmark = pytest.mark.gpu
DEV = "cuda"


def G(t):
    return t.to(DEV)


def C(t):
    return t.detach().cpu()


# (N, C, H, W): odd H (trailing row), W % 4 == 0 (vector form); W % 4 != 0 (flat form)
POOL_SHAPES = [(2, 8, 9, 16), (3, 4, 8, 32), (1, 5, 12, 20), (2, 3, 9, 15), (2, 4, 8, 10)]


@pytest.mark.parametrize("shape", POOL_SHAPES)
def test_maxpool_fwd_bwd(shape):
    from vst import ops

    g = torch.Generator().manual_seed(3)
    x = torch.randn(shape, generator=g)
    x[0, 0, 0, 1] = float("nan")  # NaN wins its window (forward value and routed gradient)
    xr = x.clone().requires_grad_(True)
    yr = F.max_pool2d(xr, 2, 2)
    gy = torch.randn(yr.shape, generator=g)
    yr.backward(gy)
    xg = G(x).requires_grad_(True)
    y = ops.maxpool2x2(xg)
    y.backward(G(gy))
    assert torch.equal(C(y).isnan(), yr.detach().isnan())
    assert torch.equal(torch.nan_to_num(C(y)), torch.nan_to_num(yr.detach()))
    assert torch.equal(C(xg.grad), xr.grad)


@pytest.mark.parametrize("shape", POOL_SHAPES)
def test_maxpool_relu_mask_and_feature_pool(shape):
    """pool backward with the producer's ReLU mask folded in, and the slice-boundary form
    relu_mask(pool_bwd(g_pool) + g_feature)."""
    from vst import ops

    g = torch.Generator().manual_seed(5)
    h = torch.relu(torch.randn(shape, generator=g))
    gp = torch.randn(shape[:2] + (shape[2] // 2, shape[3] // 2), generator=g)
    gf = torch.randn(shape, generator=g)
    hr = h.clone().requires_grad_(True)
    F.max_pool2d(hr, 2, 2).backward(gp)
    ref_pool = hr.grad * (h > 0)
    ref_feat = (hr.grad + gf) * (h > 0)

    hg = G(h).requires_grad_(True)
    ops.maxpool2x2(hg, relu_mask=True).backward(G(gp))
    assert torch.equal(C(hg.grad), ref_pool)

    hg = G(h).requires_grad_(True)
    f, p = ops.feature_pool(hg)
    torch.autograd.backward([f, p], [G(gf), G(gp)])
    assert torch.equal(C(hg.grad), ref_feat)

    hg = G(h).requires_grad_(True)  # only the feature gradient (g_pool is None)
    f, p = ops.feature_pool(hg)
    f.backward(G(gf))
    assert torch.equal(C(hg.grad), gf * (h > 0))


@pytest.mark.parametrize("src,dst", [((2, 16, 17, 30), (9, 12)), ((3, 8, 64, 128), (16, 32)), ((2, 4, 8, 16), (16, 32))])
def test_resize_bilinear(src, dst):
    from vst import ops

    g = torch.Generator().manual_seed(7)
    x = torch.randn(src, generator=g)
    ref = F.interpolate(x, size=dst, mode="bilinear", align_corners=False)
    out = ops.resize_bilinear(G(x), dst)
    assert rel_err(C(out), ref) < 1e-6
    # per-channel scale into a channel slice of a larger buffer (concat target)
    sc = torch.rand(src[1], generator=g)
    buf = torch.zeros((src[0], src[1] + 3) + dst, device=DEV)
    ops.resize_bilinear(G(x), dst, chscale=G(sc), out=buf[:, 3:])
    assert rel_err(C(buf[:, 3:]), ref * sc.view(1, -1, 1, 1)) < 1e-6
    assert not C(buf[:, :3]).any()
    # + addend (dense output)
    add = torch.randn((src[0], src[1]) + dst, generator=g)
    out = ops.resize_bilinear(G(x), dst, addend=G(add))
    assert rel_err(C(out), ref + add) < 1e-6


def _offset_view(t, k):
    """a copy of t whose data starts k floats into a fresh buffer (misaligned for k = 1)."""
    buf = torch.zeros(t.numel() + 4, device=t.device)
    v = buf[k:k + t.numel()].view(t.shape)
    v.copy_(t)
    return v


@pytest.mark.parametrize("shape", [(2, 5, 7, 10), (1, 3, 1, 2), (2, 16, 9, 130), (1, 4, 33, 64)])
def test_resize_up2_bitwise(shape):
    """The exact x2 upsample kernel (aligned operands, Ho = 2H, Wo = 2W: eight outputs per thread from
    registers) against the per-element kernel (the same call on a misaligned input): bitwise, with
    chscale / binarize / addend / a channel-slice output; and F.interpolate within 1e-6."""
    from vst import ops

    g = torch.Generator().manual_seed(11)
    N, Cc, H, W = shape
    x = torch.randn(shape, generator=g)
    dst = (2 * H, 2 * W)
    ref = F.interpolate(x, size=dst, mode="bilinear", align_corners=False)
    xa, xm = _offset_view(G(x), 0), _offset_view(G(x), 1)
    a = ops.resize_bilinear(xa, dst)
    assert rel_err(C(a), ref) < 1e-6
    assert torch.equal(a, ops.resize_bilinear(xm, dst))
    sc = G(torch.rand(Cc, generator=g) - 0.3)
    add = G(torch.randn((N, Cc) + dst, generator=g))
    for kw in ({"chscale": sc}, {"binarize": True}, {"addend": add}, {"chscale": sc, "addend": add}):
        assert torch.equal(ops.resize_bilinear(xa, dst, **kw), ops.resize_bilinear(xm, dst, **kw)), kw
    bufa = torch.full((N, Cc + 4) + dst, float("nan"), device=DEV)
    bufm = bufa.clone()
    ops.resize_bilinear(xa, dst, chscale=sc, out=bufa[:, 4:])
    ops.resize_bilinear(xm, dst, chscale=sc, out=bufm[:, 4:])
    assert torch.equal(bufa[:, 4:], bufm[:, 4:])
    assert torch.isnan(bufa[:, :4]).all()


@pytest.mark.parametrize("n", [4096 * 3, 4097])
def test_relu_bwd(n):
    from vst import ops

    g = torch.Generator().manual_seed(9)
    gy, y = torch.randn(n, generator=g), torch.relu(torch.randn(n, generator=g))
    out = ops.relu_bwd(G(gy).view(1, 1, 1, n), G(y).view(1, 1, 1, n))
    assert torch.equal(C(out).view(-1), gy * (y > 0))


@pytest.mark.parametrize("N,M,P", [(2, 24, 300), (3, 5, 1024), (1, 7, 1)])
def test_outer_axpy_and_normalize_bwd(N, M, P):
    from vst import _lib
    from vst.adaattn import attention as A

    g = torch.Generator().manual_seed(13)
    x = torch.randn(N, M, P, generator=g)
    u = torch.randn(N, M, generator=g)
    v = torch.randn(N, P, generator=g)
    w = torch.rand(N, P, generator=g) + 0.5
    ref = (x + 0.75 * u[:, :, None] * v[:, None, :]) * w[:, None, :]
    out = torch.empty(N, M, P, device=DEV)
    _lib.lib.vst_outer_axpy(*(t.data_ptr() for t in (G(x), G(u), G(v), G(w))), 0.75, out.data_ptr(), N, M, P,
                            torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert rel_err(C(out), ref) < 1e-6
    # column-normalisation adjoint: (dxh - xh * t) * s with t = sum_c xh dxh
    xh, dxh = G(x), G(torch.randn(N, M, P, generator=g))
    s = G(w)
    got = A._normalize_bwd(xh, dxh, s)
    t = (C(xh) * C(dxh)).sum(1, keepdim=True)
    assert rel_err(C(got), (C(dxh) - C(xh) * t) * w[:, None, :]) < 1e-5


def test_copy_planes():
    from vst import ops

    g = torch.Generator().manual_seed(17)
    src = torch.randn(3, 4, 8, 16, generator=g)
    buf = torch.zeros(3, 9, 8, 16, device=DEV)
    ops.copy_into(G(src), buf[:, 2:6])  # vector form: strides and offsets multiples of 4 floats
    assert torch.equal(C(buf[:, 2:6]), src) and not C(buf[:, :2]).any() and not C(buf[:, 6:]).any()
    src = torch.randn(3, 1, 5, 3, generator=g)  # 15 floats per image: flat form
    buf = torch.zeros(3, 2, 5, 3, device=DEV)
    ops.copy_into(G(src), buf[:, 1:])
    assert torch.equal(C(buf[:, 1:]), src) and not C(buf[:, :1]).any()


@pytest.mark.parametrize("n", [4096 * 3, 4097])
def test_relu_bwd_add_and_feature_split(n):
    """VGG19 slice boundary: relu_mask(g_feature + g_next) in one pass (AA/vgg19.py:39-63)."""
    from vst import ops

    g = torch.Generator().manual_seed(19)
    h = torch.relu(torch.randn(1, 1, 1, n, generator=g))
    g1, g2 = torch.randn(h.shape, generator=g), torch.randn(h.shape, generator=g)
    hg = G(h).requires_grad_(True)
    f, x = ops.feature_split(hg)
    torch.autograd.backward([f, x], [G(g1), G(g2)])
    assert torch.equal(C(hg.grad), (g1 + g2) * (h > 0))
    hg = G(h).requires_grad_(True)  # one consumer only
    f, x = ops.feature_split(hg)
    (x * G(g2)).sum().backward()
    assert torch.equal(C(hg.grad), g2 * (h > 0))


@pytest.mark.parametrize("N,C,P", [(2, 6, 4096), (3, 5, 1030), (1, 3, 7)])
def test_plane_and_channel_reductions(N, C, P):
    """plane_dot / channel_dot (AdaAttN linear attention, AA/network.py:121-124) and channel_sum
    (conv bias gradient): plane_dot / channel_sum take their float4 forms when P % 4 == 0 and the
    scalar forms otherwise; channel_dot is scalar."""
    from vst import ops
    from vst.adaattn import attention as A

    g = torch.Generator().manual_seed(23)
    x, y = torch.randn(N, C, P, generator=g), torch.randn(N, C, P, generator=g)
    w, v = torch.randn(N, P, generator=g), torch.randn(N, C, generator=g)
    xd, yd = x.double(), y.double()
    assert rel_err(C_(A.plane_dot(G(x))), xd.sum(2)) < 1e-6
    assert rel_err(C_(A.plane_dot(G(x), G(w))), (xd * w.double()[:, None]).sum(2)) < 1e-6
    assert rel_err(C_(A.channel_dot(G(x), y=G(y))), (xd * yd).sum(1)) < 1e-6
    assert rel_err(C_(A.channel_dot(G(x), v=G(v))), (xd * v.double()[:, :, None]).sum(1)) < 1e-6
    assert rel_err(C_(ops.channel_sum(G(x).view(N, C, 1, P))), xd.sum((0, 2))) < 1e-6


def C_(t):
    return t.detach().cpu().double()


@pytest.mark.parametrize("mode", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("transpose", [0, 1])
def test_pack_matrix_row_form_matches_flat_form(mode, transpose):
    """vst_pack_matrix (the attention GEMMs' packed A operand): the one-thread-per-(k-tile, row) form
    (16-byte aligned output) and the per-element form (taken for a misaligned output) write the same
    bytes, in every GEMM mode, for both operand orientations and a ragged M x K."""
    from vst import _lib

    B, M, K, Mpad, Kpad = 3, 45, 70, 64, 80
    g = torch.Generator().manual_seed(29)
    x = G(torch.randn(B, M * K, generator=g))
    words = B * Mpad * Kpad * (3 if mode == 3 else 2) // 2
    st = torch.cuda.current_stream().cuda_stream
    a = torch.full((words,), 7.0, device=DEV)
    b = torch.full((words + 1,), 7.0, device=DEV)
    _lib.lib.vst_pack_matrix(x.data_ptr(), a.data_ptr(), B, M, K, transpose, Mpad, Kpad, M * K, mode, st)
    _lib.lib.vst_pack_matrix(x.data_ptr(), b.data_ptr() + 4, B, M, K, transpose, Mpad, Kpad, M * K, mode, st)
    torch.cuda.synchronize()
    assert torch.equal(C(a).view(torch.int32), C(b[1:]).view(torch.int32))


def _buf(t, misalign):
    """t on the device, 16-byte aligned (vector kernels) or offset by one float (flat fallback)"""
    if not misalign:
        return G(t.contiguous())
    b = torch.empty(t.numel() + 1, device=DEV)
    v = b[1:].view(t.shape)
    v.copy_(G(t))
    return v


def _st():
    return torch.cuda.current_stream().cuda_stream


@pytest.mark.parametrize("misalign", [False, True])
def test_adaattn_elementwise_vec_and_flat(misalign):
    """square_concat, adaattn_out, adaattn_out_bwd_scaled, plane_norm (AA/network.py:205-220): the
    division-free float4 forms (aligned) and the flat forms (misaligned) against torch fp32."""
    from vst._lib import lib

    g = torch.Generator().manual_seed(11)
    N, dv, P = 3, 8, 36
    per = dv * P
    V = torch.randn(N, per, generator=g)
    M = torch.randn(N, per, generator=g)
    E2 = M * M + torch.rand(N, per, generator=g) * 2 - 0.2  # some variances below the 1e-6 clamp
    MV = torch.cat([M, E2], 1)
    cn = torch.randn(N, per, generator=g)
    dout = torch.randn(N, per, generator=g)
    w = torch.rand(N, P, generator=g) + 0.5
    Vd, MVd, cnd, doutd, wd = (_buf(t, misalign) for t in (V, MV, cn, dout, w))
    VV2, out, dMV = (_buf(torch.zeros(s), misalign) for s in ((N, 2 * per), (N, per), (N, 2 * per)))
    lib.vst_square_concat(Vd.data_ptr(), VV2.data_ptr(), N, per, _st())
    lib.vst_adaattn_out(MVd.data_ptr(), cnd.data_ptr(), out.data_ptr(), N, per, _st())
    lib.vst_adaattn_out_bwd_scaled(doutd.data_ptr(), MVd.data_ptr(), cnd.data_ptr(), wd.data_ptr(), dMV.data_ptr(), N,
                                   per, P, _st())
    xs = torch.randn(5, 64 * 20, generator=g)
    xsd, nrm = _buf(xs, misalign), _buf(torch.zeros(5), misalign)
    lib.vst_plane_norm(xsd.data_ptr(), nrm.data_ptr(), 5, 64 * 20, _st())
    torch.cuda.synchronize()
    assert torch.equal(C(VV2), torch.cat([V, V * V], 1))
    var = E2 - M * M
    assert rel_err(C(out).numpy(), (torch.sqrt(torch.clamp(var, min=1e-6)) * cn + M).numpy()) < 1e-6
    dvar = torch.where(var >= 1e-6, dout * cn * 0.5 / torch.sqrt(var.clamp_min(1e-30)), torch.zeros_like(var))
    s = w.repeat(1, dv)
    ref = torch.cat([(dout - 2 * M * dvar) * s, dvar * s], 1)
    assert rel_err(C(dMV).numpy(), ref.numpy()) < 1e-5
    assert rel_err(C(nrm).numpy(), xs.double().norm(dim=1).float().numpy()) < 1e-6


@pytest.mark.parametrize("shape,B,halves", [((4, 3, 8, 16), 2, (1, 1)), ((4, 5, 7, 9), 2, (3, 1)),
                                            ((2, 6, 4, 4), 0, (1, 1)), ((6, 2, 5, 8), 3, (2, 0))])
@pytest.mark.parametrize("n", [0, 1, 2, 5])
def test_fork_gradient_sums(shape, B, halves, n):
    """ops.fork (ForkFn): every consumer's gradient arrives separately and vst_sum4 adds them per batch
    half (the residual skip, feature map, stylised frame and loss-feature sums of the two training
    steps) -- against the gradient autograd's own additions give for the same consumers (torch fp32,
    CPU), 1e-6 relative; vst_sum4 covers 1..4 addends per pass, n = 5 chains two passes."""
    from vst import ops

    if n == 0 and not B:
        pytest.skip("no consumers")
    g = torch.Generator().manual_seed(n + 10 * B)
    x = torch.randn(*shape, generator=g)
    h1, h2 = halves if B else (0, 0)
    ws = [torch.randn(*shape, generator=g) for _ in range(n)]
    w1 = [torch.randn(B, *shape[1:], generator=g) for _ in range(h1)]
    w2 = [torch.randn(shape[0] - B, *shape[1:], generator=g) for _ in range(h2)]
    xd = G(x).requires_grad_(True)
    outs = ops.fork(xd, n, B, halves)
    assert len(outs) == n + h1 + h2
    terms = [(o * G(w)).sum() for o, w in zip(outs, ws + w1 + w2)]
    torch.stack(terms).sum().backward()
    xr = x.clone().requires_grad_(True)
    ref = [(xr * w).sum() for w in ws] + [(xr[:B] * w).sum() for w in w1] + [(xr[B:] * w).sum() for w in w2]
    torch.stack(ref).sum().backward()
    assert rel_err(C(xd.grad), xr.grad) < 1e-6


def test_sum_scalars_and_backward_seed():
    """ops.sum_scalars (SumScalarsFn): the loss-term sums of both trainers in vst_sum4 passes; the
    gradient reaches every term unchanged.  ops.backward_seed: the cached 0-d 1.0 the trainers seed
    backward with."""
    from vst import ops

    g = torch.Generator().manual_seed(3)
    xs = [G(torch.randn(5, generator=g)).requires_grad_(True) for _ in range(7)]
    terms = [(x * x).sum() for x in xs]
    for k in (1, 2, 4, 5, 7):
        tot = ops.sum_scalars(*terms[:k])
        ref = sum(float(t.detach()) for t in terms[:k])
        assert abs(float(tot) - ref) <= 1e-6 * abs(ref)
    for x in xs:
        x.grad = None
    tot = ops.sum_scalars(*terms)
    seed = ops.backward_seed(tot)
    assert seed.shape == () and float(seed) == 1.0
    tot.backward(seed)
    for x in xs:
        assert torch.equal(C(x.grad), C(2 * x.detach()))
    assert float(ops.backward_seed(tot)) == 1.0  # backward left the cached seed unchanged
