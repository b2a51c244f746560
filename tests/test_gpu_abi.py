"""The C ABI is stateless and re-entrant: GEMM arithmetic is a per-call
argument, so two precisions can be in flight at once on two streams, issued from two host threads,
each with its own packed operand, and both results stay correct."""
import ctypes
import threading

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from vst._lib import lib

pytestmark = pytest.mark.gpu
DEV = "cuda"
F32, BF16X3, BF16, BF16X6 = 0, 1, 2, 3
GM_ZERO = 1


def _dims(M, K):
    mp, kp = ctypes.c_int(), ctypes.c_int()
    assert lib.vst_conv_pack_dims(M, K, ctypes.byref(mp), ctypes.byref(kp)) == 0
    return mp.value, kp.value


def _pack(w, mode, st):
    Cout, Cin, KH, KW = w.shape
    Mpad, Kpad = _dims(Cout, KH * KW * Cin)
    n = Mpad * Kpad * 3 // 2 if mode == BF16X6 else Mpad * Kpad
    p = torch.empty(n, device=DEV)
    lib.vst_pack_weight(w.data_ptr(), p.data_ptr(), Cout, Cin, KH, KW, 0, 0, Mpad, Kpad, mode, st.cuda_stream)
    return p


def _conv(x, wp, out, Cout, mode, st):
    N, Cin, H, W = x.shape
    lib.vst_conv_gemm(x.data_ptr(), wp.data_ptr(), None, None, out.data_ptr(), N, Cin, H, W, Cout, 9 * Cin, H, W, 3, 3,
                      GM_ZERO, 1, 1, 1, 0, 0, None, None, None, 0, mode, st.cuda_stream)


def _err(y, ref):
    return float((y.cpu() - ref).abs().max() / ref.abs().max())


@pytest.mark.parametrize("threads", [False, True])
def test_two_precisions_interleaved_on_two_streams(threads):
    g = torch.Generator().manual_seed(3)
    N, Cin, Cout, H, W = 2, 64, 64, 40, 56
    x = torch.randn(N, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) * 0.05
    ref = F.conv2d(x.double(), w.double(), padding=1).float()
    xd, wd = x.to(DEV), w.to(DEV)
    modes = (F32, BF16, BF16X6, BF16X3)
    streams = [torch.cuda.Stream() for _ in modes]
    packs = [_pack(wd, m, s) for m, s in zip(modes, streams)]
    outs = [torch.full((N, Cout, H, W), float("nan"), device=DEV) for _ in modes]
    torch.cuda.synchronize()
    reps = 25

    def issue(i):
        for _ in range(reps):
            _conv(xd, packs[i], outs[i], Cout, modes[i], streams[i])

    if threads:
        ts = [threading.Thread(target=issue, args=(i,)) for i in range(len(modes))]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
    else:
        for _ in range(reps):  # host calls alternate modes launch by launch
            for i in range(len(modes)):
                _conv(xd, packs[i], outs[i], Cout, modes[i], streams[i])
    torch.cuda.synchronize()
    e = dict(zip(modes, (_err(o, ref) for o in outs)))
    assert e[F32] < 2e-6, e          # exact products, fp32 accumulation
    assert e[BF16X6] < 2e-6, e       # fp32-class split products
    assert e[BF16X3] < 2e-5, e       # ~2^-16 per product
    assert 1e-4 < e[BF16] < 2e-2, e  # single bf16 products: visibly coarser, still the same conv
    # each stream's result is its own mode's: no cross-talk through library state
    assert not torch.equal(outs[0], outs[1])


def test_pack_is_bound_to_its_mode():
    """A packed operand carries its mode's layout: the same weights packed in two modes differ in
    size (bf16x6 blocks are 1.5x) and in content."""
    w = torch.randn(64, 64, 3, 3, device=DEV) * 0.05
    st = torch.cuda.current_stream()
    a, b, c = _pack(w, F32, st), _pack(w, BF16X3, st), _pack(w, BF16X6, st)
    torch.cuda.synchronize()
    assert a.numel() == b.numel() and c.numel() == a.numel() * 3 // 2
    assert not torch.equal(a, b)
    assert np.isfinite(a.cpu().numpy()).all()
