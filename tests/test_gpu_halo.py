"""The halo-tiled 3x3 conv kernel (csrc/conv_halo_kernel.h) against the per-tap kernel and fp64.

Every 3x3 stride-1 conv / data gradient in the channel-blocked K order (VST_GEMM_KBLOCK) runs on the
halo kernel; VST_GEMM_PERTAP forces the per-tap kernel for the same call.  Both sum the same k-tiles
in the same order with the same MFMA sequence, so their outputs must be BITWISE equal -- for every
border rule (reflect / zero forward, transposed data gradient with and without the gathered ReLU
mask, the padded-grid data gradient with its border side buffer), epilogue and ragged tile edge.
The shapes are the training paths' 3x3 layers at reduced size (VGG16 / VGG19 64..512 channels,
ReCoNet residual 192, AdaAttN decoder 256 / 128 / 64) plus ragged grids.  These small grids would be
split over the channel blocks (split-K: fewer than 512 blocks); the bitwise comparisons keep the
halo launch unsplit (VST_GEMM_NOSPLIT), and the split results are held to the unsplit ones within
fp32 summation-order rounding and to fp64.

The 2x2 form of the same kernel (KS = 2) runs the phase-stacked GEMMs: the stride-2 data gradient
(four parity phases of the padded grid, EPI_PHASE2, ReCoNet conv2 / conv3, RC/network.py:161-162) and
the nearest-x2 upsample forward (edge-clamped source grid, UpsampleConvLayer RC/network.py:114-120);
those are held bitwise to the per-tap kernel and to fp64 the same way."""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from vst._lib import lib

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF16X3, BF16, BF16X6, F16 = 1, 2, 3, 4
KBLOCK, PERTAP, NOSPLIT = 16, 32, 64
GM_REFLECT, GM_ZERO, GM_TRANSPOSED = 0, 1, 2
EPI_BIAS, EPI_RELU, EPI_MASK, EPI_ACCUM, EPI_PADOUT = 1, 2, 8, 16, 128


# output error vs fp64 (max-norm relative) by product precision
TOL = {BF16X6: 5e-6, BF16X3: 1e-4, F16: 2e-3, BF16: 2e-2}


def _dims(M, K):
    mp, kp = ctypes.c_int(), ctypes.c_int()
    assert lib.vst_conv_pack_dims(M, K, ctypes.byref(mp), ctypes.byref(kp)) == 0
    return mp.value, kp.value


def _pack(w, mode, transposed=False):
    Cout, Cin, KH, KW = w.shape
    M = Cin if transposed else Cout
    Mpad, Kpad = _dims(M, KH * KW * (Cout if transposed else Cin))
    n = Mpad * Kpad * 3 // 2 if (mode & 7) == BF16X6 else Mpad * Kpad
    p = torch.empty(n, device=DEV)
    lib.vst_pack_weight(w.data_ptr(), p.data_ptr(), Cout, Cin, KH, KW, int(transposed), 0, Mpad, Kpad, mode,
                        torch.cuda.current_stream().cuda_stream)
    return p


def _ws_bytes(N, Cs, M, Ho, Wo, gmode, pad, epi, mode):
    return lib.vst_conv_splitk_workspace(N, Cs, M, Ho, Wo, 3, 3, gmode, 1, pad, pad, 1, epi, 0, mode)


def _conv(src, wp, M, Ho, Wo, gmode, pad, mode, epi=0, bias=None, mask=None, gmask=None, out=None, ws=True,
          stream=None):
    """ws: supply the split-K workspace the library asks for (caller-owned, from torch's allocator)."""
    N, Cs, Hs, Ws = src.shape
    if out is None:
        out = torch.full((N, M, Ho, Wo), float("nan"), device=DEV)
    P = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    nb = _ws_bytes(N, Cs, M, Ho, Wo, gmode, pad, epi, mode) if ws else 0
    wsb = torch.empty((nb + 3) // 4, device=DEV) if nb else None
    st = stream if stream is not None else torch.cuda.current_stream()
    lib.vst_conv_gemm_padx(src.data_ptr(), wp.data_ptr(), P(bias), P(mask), out.data_ptr(), N, Cs, Hs, Ws, M, 9 * Cs,
                           Ho, Wo, 3, 3, gmode, 1, pad, pad, 1, epi, 0, None, P(gmask), P(wsb), nb, mode,
                           st.cuda_stream)
    if wsb is not None:
        wsb.record_stream(st)
    return out


def _rand(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(DEV)


MODES = [BF16X6, F16, BF16, BF16X3]
# (N, Cin, H, W, Cout): VGG layers, ReCoNet residual, AdaAttN decoder, ragged tiles
SHAPES = [(2, 64, 37, 70, 64), (1, 128, 16, 64, 128), (2, 192, 20, 36, 192), (1, 256, 9, 40, 256),
          (1, 64, 12, 33, 512), (1, 32, 7, 31, 256), (2, 16, 5, 3, 64), (1, 256, 8, 16, 128)]


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("pad_mode", ["reflect", "zero"])
def test_halo_forward_bitwise(mode, shape, pad_mode):
    N, Cin, H, W, Cout = shape
    if pad_mode == "reflect" and min(H, W) < 2:
        pytest.skip("reflect pad needs 2 pixels")
    x = _rand(N, Cin, H, W, seed=1, scale=3.0)
    w = _rand(Cout, Cin, 3, 3, seed=2, scale=0.05)
    b = _rand(Cout, seed=3)
    m = mode | KBLOCK
    wp = _pack(w, m)
    gm = GM_REFLECT if pad_mode == "reflect" else GM_ZERO
    epi = EPI_BIAS | (EPI_RELU if pad_mode == "zero" else 0)
    halo = _conv(x, wp, Cout, H, W, gm, 1, m | NOSPLIT, epi, bias=b)
    ref = _conv(x, wp, Cout, H, W, gm, 1, m | PERTAP, epi, bias=b)
    torch.cuda.synchronize()
    assert torch.equal(halo, ref), float((halo - ref).abs().max())
    # and the conv itself, against fp64
    xp = F.pad(x.double(), (1, 1, 1, 1), mode="reflect" if pad_mode == "reflect" else "constant")
    y = F.conv2d(xp, w.double(), b.double())
    if pad_mode == "zero":
        y = y.clamp_min(0)
    err = float((halo.double() - y).abs().max() / y.abs().max())
    assert err < TOL[mode], err


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("shape", SHAPES[:5])
@pytest.mark.parametrize("masked", [False, True])
def test_halo_dgrad_bitwise(mode, shape, masked):
    """Zero-pad data gradient (VGG): dX = transposed gather over dY, with the ReLU mask of the
    layer's output gathered onto dY (gmask) and the input-side mask in the epilogue (EPI_MASK)."""
    N, Cin, H, W, Cout = shape
    dy = _rand(N, Cout, H, W, seed=4)
    w = _rand(Cout, Cin, 3, 3, seed=5, scale=0.05)
    m = mode | KBLOCK
    wp = _pack(w, m, transposed=True)
    gmask = _rand(N, Cout, H, W, seed=6) if masked else None
    dmask = _rand(N, Cin, H, W, seed=7) if masked else None
    epi = EPI_MASK if masked else 0
    halo = _conv(dy, wp, Cin, H, W, GM_TRANSPOSED, 1, m | NOSPLIT, epi, mask=dmask, gmask=gmask)
    ref = _conv(dy, wp, Cin, H, W, GM_TRANSPOSED, 1, m | PERTAP, epi, mask=dmask, gmask=gmask)
    torch.cuda.synchronize()
    assert torch.equal(halo, ref), float((halo - ref).abs().max())
    g = dy.double() * (gmask > 0).double() if masked else dy.double()
    dx = torch.nn.grad.conv2d_input((N, Cin, H, W), w.double(), g, padding=1)
    if masked:
        dx = dx * (dmask > 0).double()
    err = float((halo.double() - dx).abs().max() / dx.abs().max())
    assert err < TOL[mode], err


@pytest.mark.parametrize("mode", [BF16X6, F16])
@pytest.mark.parametrize("shape", [(2, 192, 20, 36, 192), (1, 64, 11, 45, 64), (1, 128, 6, 9, 128)])
def test_halo_padout_dgrad_bitwise(mode, shape):
    """ReCoNet ResidualBlock data gradient (reflect pad 1): the transposed GEMM over the padded grid,
    interior straight into dx, border into the side buffer (EPI_PADOUT), then vst_fold_border."""
    N, Cin, H, W, Cout = shape
    dy = _rand(N, Cout, H, W, seed=8)
    w = _rand(Cout, Cin, 3, 3, seed=9, scale=0.05)
    m = mode | KBLOCK
    wp = _pack(w, m, transposed=True)
    st = torch.cuda.current_stream().cuda_stream
    res = []
    for mm in (m | NOSPLIT, m | PERTAP, m):
        dx = torch.full((N, Cin, H, W), float("nan"), device=DEV)
        border = torch.zeros(N, Cin, H + 2, W + 2, device=DEV)
        nb = lib.vst_conv_splitk_workspace(N, Cout, Cin, H + 2, W + 2, 3, 3, GM_TRANSPOSED, 1, 0, 0, 1, EPI_PADOUT, 0, mm)
        ws = torch.empty((nb + 3) // 4, device=DEV) if nb else None
        lib.vst_conv_dgrad_padout(dy.data_ptr(), wp.data_ptr(), None, dx.data_ptr(), border.data_ptr(), N, Cout, H, W,
                                  Cin, H, W, 3, 1, None if ws is None else ws.data_ptr(), nb, mm, st)
        lib.vst_fold_border(border.data_ptr(), None, dx.data_ptr(), N * Cin, H, W, 1, st)
        res.append(dx)
    torch.cuda.synchronize()
    assert torch.equal(res[0], res[1]), float((res[0] - res[1]).abs().max())
    assert float((res[2] - res[0]).abs().max() / res[0].abs().max()) < 1e-5  # split-K (bf16x6): summation order
    x = torch.zeros(N, Cin, H, W, dtype=torch.float64, device=DEV, requires_grad=True)
    y = F.conv2d(F.pad(x, (1, 1, 1, 1), mode="reflect"), w.double())
    y.backward(dy.double())
    err = float((res[0].double() - x.grad).abs().max() / x.grad.abs().max())
    assert err < (5e-6 if mode == BF16X6 else 2e-3), err


def test_halo_accumulate_and_fallbacks():
    """EPI_ACCUM adds into the output; Cout = 3 / 96 (pack Mpad not a multiple of the halo block)
    stay on the per-tap kernel and still compute the conv."""
    x = _rand(1, 64, 10, 40, seed=10)
    w = _rand(64, 64, 3, 3, seed=11, scale=0.05)
    m = BF16X6 | KBLOCK
    wp = _pack(w, m)
    base = _rand(1, 64, 10, 40, seed=12)
    a = _conv(x, wp, 64, 10, 40, GM_ZERO, 1, m | NOSPLIT, EPI_ACCUM, out=base.clone())
    b = _conv(x, wp, 64, 10, 40, GM_ZERO, 1, m | PERTAP, EPI_ACCUM, out=base.clone())
    assert torch.equal(a, b)
    for cout in (3, 96):
        w2 = _rand(cout, 64, 3, 3, seed=13, scale=0.05)
        y = _conv(x, _pack(w2, m), cout, 10, 40, GM_REFLECT, 1, m)
        ref = F.conv2d(F.pad(x.double(), (1, 1, 1, 1), mode="reflect"), w2.double())
        assert float((y.double() - ref).abs().max() / ref.abs().max()) < 2e-6


@pytest.mark.parametrize("mode", [BF16X6, BF16, F16])
@pytest.mark.parametrize("shape", [(4, 192, 64, 128, 192), (2, 192, 20, 36, 192), (1, 128, 16, 64, 128),
                                   (1, 256, 8, 16, 128)])
@pytest.mark.parametrize("epi", ["bias_relu", "mask", "accum"])
def test_halo_split_k(mode, shape, epi):
    """Split-K (the grid under 512 blocks; ReCoNet's residual layer at a quarter batch first): the
    slices' sums added in order then the epilogue, against the unsplit launch (same k-tiles, other
    fp32 summation order) and fp64."""
    N, Cin, H, W, Cout = shape
    x = _rand(N, Cin, H, W, seed=21, scale=3.0)
    w = _rand(Cout, Cin, 3, 3, seed=22, scale=0.05)
    b = _rand(Cout, seed=23)
    mask = _rand(N, Cout, H, W, seed=24)
    base = _rand(N, Cout, H, W, seed=25)
    m = mode | KBLOCK
    wp = _pack(w, m)
    e = {"bias_relu": EPI_BIAS | EPI_RELU, "mask": EPI_MASK, "accum": EPI_ACCUM}[epi]
    kw = dict(bias=b) if epi == "bias_relu" else dict(mask=mask) if epi == "mask" else {}
    # every shape here under-fills the chip: the split is planned (the library asks for workspace)
    nb = _ws_bytes(N, Cin, Cout, H, W, GM_REFLECT, 1, e, m)
    assert nb > 0, nb
    assert _ws_bytes(N, Cin, Cout, H, W, GM_REFLECT, 1, e, m | NOSPLIT) == 0
    outs = [_conv(x, wp, Cout, H, W, GM_REFLECT, 1, mm, e, out=base.clone() if epi == "accum" else None, ws=w_, **kw)
            for mm, w_ in ((m, True), (m | NOSPLIT, True), (m, False))]
    torch.cuda.synchronize()
    split, whole, nows = outs
    # no workspace given: the same launch runs unsplit, bitwise the NOSPLIT result
    assert torch.equal(nows, whole)
    assert not torch.isnan(split).any()
    y = F.conv2d(F.pad(x.double(), (1, 1, 1, 1), mode="reflect"), w.double())
    if epi == "bias_relu":
        y = (y + b.double().view(1, -1, 1, 1)).clamp_min(0)
    elif epi == "mask":
        y = y * (mask > 0).double()
    else:
        y = y + base.double()
    scale = float(y.abs().max())
    assert float((split - whole).abs().max()) / scale < 1e-5  # fp32 summation order over K = 9 Cin
    err = float((split.double() - y).abs().max()) / scale
    assert err < TOL[mode], err


@pytest.mark.parametrize("threads", [False, True])
def test_split_k_two_streams(threads):
    """Split-K launches on two streams at once (issued from one or two host threads), each with its
    own caller-owned workspace: every result equals its stream's own unsplit (NOSPLIT) launch up to fp32
    summation order, and repeated launches are bitwise reproducible (no shared library scratch)."""
    import threading

    shapes = [(2, 192, 20, 36, 192), (1, 256, 8, 16, 128)]
    m = BF16X6 | KBLOCK
    jobs = []
    for i, (N, Cin, H, W, Cout) in enumerate(shapes):
        x = _rand(N, Cin, H, W, seed=40 + i, scale=3.0)
        w = _rand(Cout, Cin, 3, 3, seed=50 + i, scale=0.05)
        assert _ws_bytes(N, Cin, Cout, H, W, GM_REFLECT, 1, 0, m) > 0
        jobs.append((x, _pack(w, m), Cout, H, W))
    streams = [torch.cuda.Stream() for _ in jobs]
    torch.cuda.synchronize()
    ref = [_conv(x, wp, C, H, W, GM_REFLECT, 1, m | NOSPLIT) for x, wp, C, H, W in jobs]
    reps = 20
    outs = [[None] * reps for _ in jobs]

    def issue(i):
        x, wp, C, H, W = jobs[i]
        with torch.cuda.stream(streams[i]):
            for r in range(reps):
                outs[i][r] = _conv(x, wp, C, H, W, GM_REFLECT, 1, m, stream=streams[i])

    if threads:
        ts = [threading.Thread(target=issue, args=(i,)) for i in range(len(jobs))]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
    else:
        for i in range(len(jobs)):
            issue(i)
    torch.cuda.synchronize()
    for i in range(len(jobs)):
        scale = float(ref[i].abs().max())
        assert float((outs[i][0] - ref[i]).abs().max()) / scale < 1e-5
        for r in range(1, reps):
            assert torch.equal(outs[i][r], outs[i][0])


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("shape", [(2, 48, 30, 62, 96), (1, 96, 16, 34, 192), (1, 32, 9, 13, 64), (2, 64, 7, 40, 32)])
def test_halo2_stride2_dgrad_bitwise(mode, shape):
    """Stride-2 reflect-pad 3x3 conv input gradient (vst_conv_dgrad_s2): rows ci*4 + phase over the
    phase grid, 2x2 transposed taps, interior into dx and border into the side buffer, then folded."""
    N, Cin, H, W, Cout = shape
    KS, pad = 3, 1
    Ho, Wo = (H + 2 * pad - KS) // 2 + 1, (W + 2 * pad - KS) // 2 + 1
    dy = _rand(N, Cout, Ho, Wo, seed=60)
    w = _rand(Cout, Cin, KS, KS, seed=61, scale=0.05)
    st = torch.cuda.current_stream().cuda_stream
    res = []
    for mm in (mode | KBLOCK, mode | KBLOCK | PERTAP):
        Mpad, Kpad = _dims(4 * Cin, 4 * Cout)
        wp = torch.empty(Mpad * Kpad * 3 // 2 if mode == BF16X6 else Mpad * Kpad, device=DEV)
        assert lib.vst_pack_weight_phase2(w.data_ptr(), wp.data_ptr(), Cout, Cin, KS, Mpad, Kpad, mm, st) == 0
        dx = torch.full((N, Cin, H, W), float("nan"), device=DEV)
        border = torch.zeros(N, Cin, H + 2 * pad, W + 2 * pad, device=DEV)
        assert lib.vst_conv_dgrad_s2(dy.data_ptr(), wp.data_ptr(), None, dx.data_ptr(), border.data_ptr(), N, Cout, Ho,
                                     Wo, Cin, H, W, KS, pad, mm, st) == 0
        lib.vst_fold_border(border.data_ptr(), None, dx.data_ptr(), N * Cin, H, W, pad, st)
        res.append(dx)
    torch.cuda.synchronize()
    assert torch.equal(res[0], res[1]), float((res[0] - res[1]).abs().max())
    x = torch.zeros(N, Cin, H, W, dtype=torch.float64, device=DEV, requires_grad=True)
    F.conv2d(F.pad(x, (pad,) * 4, mode="reflect"), w.double(), stride=2).backward(dy.double())
    err = float((res[0].double() - x.grad).abs().max() / x.grad.abs().max())
    assert err < TOL[mode], err


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("shape", [(2, 192, 12, 20, 96), (1, 96, 15, 33, 48), (1, 64, 5, 9, 64), (2, 32, 8, 31, 32)])
def test_halo2_up2_forward_bitwise(mode, shape):
    """Nearest-x2 upsample -> reflect pad 1 -> 3x3 conv + bias (vst_conv_up2_fwd): the phase-stacked
    2x2 GEMM over the (H+1) x (W+1) edge-clamped source grid, four phase rows per channel scattered."""
    N, Cin, H, W, Cout = shape
    x = _rand(N, Cin, H, W, seed=62, scale=3.0)
    w = _rand(Cout, Cin, 3, 3, seed=63, scale=0.05)
    b = _rand(Cout, seed=64)
    st = torch.cuda.current_stream().cuda_stream
    w2 = torch.empty(4 * Cout, Cin, 2, 2, device=DEV)
    assert lib.vst_up2_phase_weights(w.data_ptr(), w2.data_ptr(), Cout, Cin, st) == 0
    res = []
    for mm in (mode | KBLOCK, mode | KBLOCK | PERTAP):
        wp = _pack(w2, mm)
        out = torch.full((N, Cout, 2 * H, 2 * W), float("nan"), device=DEV)
        assert lib.vst_conv_up2_fwd(x.data_ptr(), wp.data_ptr(), b.data_ptr(), out.data_ptr(), N, Cin, H, W, Cout, mm,
                                    st) == 0
        res.append(out)
    torch.cuda.synchronize()
    assert torch.equal(res[0], res[1]), float((res[0] - res[1]).abs().max())
    xu = F.interpolate(x.double(), scale_factor=2, mode="nearest")
    y = F.conv2d(F.pad(xu, (1, 1, 1, 1), mode="reflect"), w.double(), b.double())
    err = float((res[0].double() - y).abs().max() / y.abs().max())
    assert err < TOL[mode], err


def _pack_kwu(w, mode, transposed):
    Cout, Cin, K, _ = w.shape
    C = Cout if transposed else Cin
    Cu = (C * K + 15) // 16 * 16
    M = Cin if transposed else Cout
    Mpad, Kpad = _dims(M, K * Cu)
    p = torch.empty(Mpad * Kpad * 3 // 2 if (mode & 7) == BF16X6 else Mpad * Kpad, device=DEV)
    assert lib.vst_pack_weight_kwu(w.data_ptr(), p.data_ptr(), Cout, Cin, K, Cu, int(transposed), Mpad, Kpad, mode,
                                   torch.cuda.current_stream().cuda_stream) == 0
    return p, Cu


def _unfold(x, K, off, sgn, Wout, reflect, Cu):
    N, C, H, W = x.shape
    out = torch.full((N, Cu, H, Wout), float("nan"), device=DEV)
    assert lib.vst_unfold_kw(x.data_ptr(), out.data_ptr(), N, C, H, W, Wout, K, Cu, sgn, off, int(reflect),
                             torch.cuda.current_stream().cuda_stream) == 0
    return out


def _unfold_ref(x, K, off, sgn, Wout, reflect, Cu):
    """out[n][c*K + kw][y][v] = x[n][c][y][v + sgn*kw + off]: single reflection or zero outside; channels
    >= C*K zero (the vst_unfold_kw contract, include/vst_hip.h)."""
    N, C, H, W = x.shape
    out = torch.zeros((N, Cu, H, Wout), device=x.device)
    v = torch.arange(Wout, device=x.device)
    for c in range(C):
        for kw in range(K):
            xs = v + sgn * kw + off
            if reflect:
                xs = xs.abs()
                xs = torch.where(xs >= W, 2 * W - 2 - xs, xs)
            ok = (xs >= 0) & (xs < W)
            out[:, c * K + kw, :, ok] = x[:, c, :, xs[ok]]
    return out


@pytest.mark.parametrize("case", [
    (2, 3, 7, 64, 64, 9, 32, -4, 1, True),     # ReCoNet conv1's forward unfold (27 -> 32: a zero group)
    (2, 3, 5, 30, 40, 9, 32, 0, -1, False),    # ConvTanh's padded-grid data gradient (rows rounded to 4)
    (1, 5, 3, 13, 16, 3, 16, -1, 1, True),     # K = 3, 15 -> 16
    (1, 2, 4, 9, 12, 9, 32, -4, 1, True),      # Cu spans two zero groups (18 -> 32)
    (3, 3, 2, 700, 704, 9, 27, -4, 1, False),  # exact fit, a row wider than one block
])
def test_unfold_kw_exact(case):
    """vst_unfold_kw (one thread writes the K unfolded rows of a source row segment) against a torch
    gather: a copy, so bitwise; NaN-filled output proves every element, zero channels included, is
    written."""
    N, C, H, W, Wout, K, Cu, off, sgn, reflect = case
    x = _rand(N, C, H, W, seed=73)
    got = _unfold(x, K, off, sgn, Wout, reflect, Cu)
    torch.cuda.synchronize()
    assert torch.equal(got, _unfold_ref(x, K, off, sgn, Wout, reflect, Cu))


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("shape", [(2, 3, 40, 64, 48), (1, 3, 17, 96, 32), (1, 3, 33, 32, 64)])
def test_halo91_kwu_forward_bitwise(mode, shape):
    """9x9 reflect-pad conv of a 3-channel frame (ReCoNet conv1, RC/network.py:158) as a 9 x 1 conv over
    the kw-unfolded input (vst_unfold_kw: 27 -> 32 channels): the halo kernel's 9 x 1 form against the
    per-tap kernel (bitwise) and float64."""
    N, Cin, H, W, Cout = shape
    K, pad = 9, 4
    x = _rand(N, Cin, H, W, seed=70, scale=50.0)
    w = _rand(Cout, Cin, K, K, seed=71, scale=0.02)
    b = _rand(Cout, seed=72)
    st = torch.cuda.current_stream().cuda_stream
    res = []
    for mm in (mode | KBLOCK, mode | KBLOCK | PERTAP):
        wp, Cu = _pack_kwu(w, mm, False)
        xu = _unfold(x, K, -pad, 1, W, True, Cu)
        out = torch.full((N, Cout, H, W), float("nan"), device=DEV)
        assert lib.vst_conv_gemm_padx(xu.data_ptr(), wp.data_ptr(), b.data_ptr(), None, out.data_ptr(), N, Cu, H, W,
                                      Cout, K * Cu, H, W, K, 1, GM_REFLECT, 1, pad, 0, 1, EPI_BIAS, 0, None, None, None,
                                      0, mm, st) == 0
        res.append(out)
    torch.cuda.synchronize()
    assert torch.equal(res[0], res[1]), float((res[0] - res[1]).abs().max())
    y = F.conv2d(F.pad(x.double(), (pad,) * 4, mode="reflect"), w.double(), b.double())
    err = float((res[0].double() - y).abs().max() / y.abs().max())
    assert err < TOL[mode], err


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("shape", [(2, 48, 24, 64, 3, 9), (1, 32, 13, 32, 3, 9), (1, 48, 11, 62, 3, 9),
                                   (2, 64, 12, 32, 3, 3), (1, 64, 9, 30, 3, 3)])
def test_halo91_kwu_padout_dgrad_bitwise(mode, shape):
    """ConvTanh's data gradient (48 -> 3 channels, 9x9 reflect pad 4, RC/network.py:78-85) and the
    AdaAttN decoder's last conv's (64 -> 3, 3x3 reflect pad 1, AA/network.py:99): the output gradient
    kw-unfolded over the padded width (rows rounded up to 4 wide: 62 + 8 -> 72, 32 + 2 -> 36), a K x 1
    transposed GEMM over the padded grid (interior into dx, border into the side buffer, EPI_PADOUT),
    then vst_fold_border -- halo vs per-tap bitwise, and float64."""
    N, Cin, H, W, Cout, K = shape
    pad = K // 2
    dy = _rand(N, Cout, H, W, seed=73)
    w = _rand(Cout, Cin, K, K, seed=74, scale=0.02)
    st = torch.cuda.current_stream().cuda_stream
    res = []
    for mm in (mode | KBLOCK, mode | KBLOCK | PERTAP):
        wp, Cu = _pack_kwu(w, mm, True)
        dyu = _unfold(dy, K, 0, -1, (W + 2 * pad + 3) // 4 * 4, False, Cu)
        dx = torch.full((N, Cin, H, W), float("nan"), device=DEV)
        border = torch.zeros(N, Cin, H + 2 * pad, W + 2 * pad, device=DEV)
        assert lib.vst_conv_dgrad_padout_kwu(dyu.data_ptr(), wp.data_ptr(), None, dx.data_ptr(), border.data_ptr(), N,
                                             Cu, H, Cin, H, W, K, pad, mm, st) == 0
        assert lib.vst_fold_border(border.data_ptr(), None, dx.data_ptr(), N * Cin, H, W, pad, st) == 0
        res.append(dx)
    torch.cuda.synchronize()
    assert torch.equal(res[0], res[1]), float((res[0] - res[1]).abs().max())
    x = torch.zeros(N, Cin, H, W, dtype=torch.float64, device=DEV, requires_grad=True)
    F.conv2d(F.pad(x, (pad,) * 4, mode="reflect"), w.double()).backward(dy.double())
    err = float((res[0].double() - x.grad).abs().max() / x.grad.abs().max())
    assert err < TOL[mode], err


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("shape", [(2, 48, 24, 64, 3), (1, 32, 13, 40, 3), (1, 16, 37, 96, 3)])
def test_halo19_rowsplit_forward_bitwise(mode, shape):
    """ConvTanh's forward (48 -> 3 channels, 9x9 reflect pad 4, RC/network.py:78-85) as the row-split
    GEMM: rows (co, kh) = 27 of a 32-row pack, a 1 x 9 conv over the reflect-padded rows (output
    (H + 8) x W).  The halo kernel's 1 x 9 form (32-row block, 16 output rows per tile, ragged rows and
    columns) against the per-tap kernel (bitwise, unsplit) and float64 (F.conv2d over the padded frame
    with the (co, kh) rows as output channels)."""
    N, Cin, H, W, Cout = shape
    K, pad = 9, 4
    x = _rand(N, Cin, H, W, seed=80, scale=3.0)
    w = _rand(Cout, Cin, K, K, seed=81, scale=0.02)
    st = torch.cuda.current_stream().cuda_stream
    M, Hq = Cout * K, H + K - 1
    Mpad, Kpad = _dims(M, K * Cin)
    res = []
    for mm in (mode | KBLOCK | NOSPLIT, mode | KBLOCK | PERTAP, mode | KBLOCK):
        n = Mpad * Kpad * 3 // 2 if (mm & 7) == BF16X6 else Mpad * Kpad
        wp = torch.empty(n, device=DEV)
        assert lib.vst_pack_weight(w.data_ptr(), wp.data_ptr(), Cout, Cin, K, K, 0, 1, Mpad, Kpad, mm, st) == 0
        nb = lib.vst_conv_splitk_workspace(N, Cin, M, Hq, W, 1, K, GM_REFLECT, 1, pad, pad, 1, 0, 0, mm)
        wsb = torch.empty((nb + 3) // 4, device=DEV) if nb else None
        out = torch.full((N, M, Hq, W), float("nan"), device=DEV)
        assert lib.vst_conv_gemm_padx(x.data_ptr(), wp.data_ptr(), None, None, out.data_ptr(), N, Cin, H, W, M, K * Cin,
                                      Hq, W, 1, K, GM_REFLECT, 1, pad, pad, 1, 0, 0, None, None,
                                      None if wsb is None else wsb.data_ptr(), nb, mm, st) == 0
        res.append(out)
    torch.cuda.synchronize()
    assert torch.equal(res[0], res[1]), float((res[0] - res[1]).abs().max())
    w2 = w.double().permute(0, 2, 1, 3).reshape(M, Cin, 1, K)  # row (co, kh), taps (0, kw)
    y = F.conv2d(F.pad(x.double(), (pad,) * 4, mode="reflect"), w2)
    for r in (res[0], res[2]):  # unsplit and (where the grid is small) split-K
        err = float((r.double() - y).abs().max() / y.abs().max())
        assert err < TOL[mode], err
