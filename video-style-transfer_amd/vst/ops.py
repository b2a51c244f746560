"""Autograd operators over libvst_hip.so.  Every forward AND backward runs a HIP kernel of the
library on the current stream; there is no PyTorch-compute or CPU fallback (torch only allocates
device memory).  Reference call sites each operator replaces are cited per class.
"""
import contextlib
import ctypes
import os
import threading
import weakref

import numpy as np
import torch
from torch.autograd import Function

from . import kprof
from ._lib import VstError, lib, ptr, ptr_rows, stream

GM_REFLECT, GM_ZERO, GM_TRANSPOSED = 0, 1, 2
EPI_BIAS, EPI_RELU, EPI_TANH, EPI_MASK, EPI_ACCUM = 1, 2, 4, 8, 16
LOSS_WS = 2048


def _empty(shape, like):
    return torch.empty(shape, device=like.device, dtype=torch.float32)


def _zeros(shape, like):
    return torch.zeros(shape, device=like.device, dtype=torch.float32)


def _check(t, name, ndim=None):
    if not t.is_cuda or t.dtype != torch.float32:
        raise VstError(f"{name}: expected a float32 HIP tensor, got {t.dtype} on {t.device}")
    if ndim is not None and t.dim() != ndim:
        raise VstError(f"{name}: expected {ndim}-D, got shape {tuple(t.shape)}")
    return t.contiguous()


GEMM_MODES = {"f32": 0, "bf16x3": 1, "bf16": 2, "bf16x6": 3, "f16": 4}
KBLOCK = 16  # VST_GEMM_KBLOCK: channel-blocked K order flag of a conv pack + GEMM call pair
PERTAP = 32  # VST_GEMM_PERTAP: the per-tap conv / row-tiled weight-gradient kernel for this call
# where the channel-blocked K order applies (VST_KBLOCK): "res" (default) the loss networks, the
# ReCoNet stylizer's residual blocks and the AdaAttN decoder (scope "stylizer.dec": no InstanceNorm
# there, and its 3x3 convs then run on the halo-tiled kernel); "1" nowhere inside a stylizer; "2"
# everywhere (diagnostic: fails the ragged golden step, tools/policy_check.py); "0" off
_KB = os.environ.get("VST_KBLOCK", "res")
KBLOCK_ON = _KB != "0"
KBLOCK_STYLIZER = _KB == "2"
KBLOCK_RES = _KB in ("2", "res")
KBLOCK_UP2 = KBLOCK_ON and os.environ.get("VST_KBLOCK_UP2", "1") != "0"  # A/B: the up2 phase forward blocked
# the kw-unfolded 9x9 forward (ReCoNet conv1) in the channel-blocked order, i.e. on the halo kernel's 9 x 1
# form: off -- like the stylizer's other forwards (above), the blocked order moves the ragged golden
# step's conv1 InstanceNorm-weight gradient past its bar under bf16x6 (margin 1.05); its data gradient
# (ConvTanh's, in the backward) takes the 9 x 1 halo form
KBLOCK_KWU = KBLOCK_ON and os.environ.get("VST_KBLOCK_KWU", "0") != "0"
# The C ABI is stateless: every GEMM / pack entry takes its arithmetic mode as an argument.  This
# module chooses that argument per call from a named policy (base mode + per-role overrides,
# optionally per model scope); _CUR holds the mode chosen by the latest gemm_role() call, which
# the pack and GEMM calls that follow it pass to the library.
class _ThreadSlot(threading.local):
    """One value per host thread, indexed like the one-element lists it replaces (slot[0])."""

    def __init__(self, value=None):
        self.value = value

    def __getitem__(self, _i):
        return self.value

    def __setitem__(self, _i, v):
        self.value = v


_BASE_MODE = [None]  # base mode of the selected policy (process-wide)
# mode of the GEMM being set up (gemm_role) and the model scope: per host thread, so two threads
# issuing ops (trainers on separate streams, autograd's device thread) never pack under one mode and
# launch under another
_CUR = _ThreadSlot()
# per-role overrides of the base mode; roles: "fwd" (forward products), "fwd_img" (Cin = 3),
# "dgrad" (data gradients, Gram backward), "wgrad" (weight gradients, Gram), "attn_cosine" /
# "attn_softmax" (AdaAttN attention products, fwd + bwd), "loss_fwd" / "loss_dgrad" (the AdaAttN
# cosine-distance products of the image-similarity loss)
GEMM_POLICY = {}
DEFAULT_POLICY = "f32"


def _mode_id(mode):
    m = GEMM_MODES.get(mode, mode)
    if m not in GEMM_MODES.values():
        raise VstError(f"unknown GEMM mode {mode!r} (one of {sorted(GEMM_MODES)})")
    return int(m)


# Named policies (base mode, per-role overrides).
#   "f32" (default): exact fp32 MFMA products everywhere.
#   "bf16x6": every GEMM (conv fwd / dgrad / wgrad, Gram, attention) on three-way split bf16
#     products, per-product error ~2^-24 (fp32-class) at 2.7x the fp32 MFMA rate; the softmax
#     attention (exp of raw dot products) stays exact fp32.
#   "parity": bf16x3 split MFMA (~2^-16 per product) for every GEMM except the stylizer forwards,
#     which run bf16x6: their outputs feed InstanceNorm, whose mean subtraction and ReLU decisions
#     amplify a 5e-6 relative product error into 1e-3 of a gradient element's tensor norm
#     (tools/policy_check.py: all stylizer forwards bf16x3 -> 1.07 of the gradient tolerance on the
#     ragged golden step; none -> 0.002); the softmax attention stays exact fp32.
#   "bf16x3": every GEMM split in two (fails the ragged golden step's gradient tolerance, 1.07).
#   "bf16": single bf16 products (~2^-8): a reduced-precision option for BASELINE config 5.
#   "f16": single fp16 products (~2^-11 per operand) with a dynamic loss scale starting at
#     LOSS_SCALE: the fp16 MFMA path BASELINE config 5 names.
POLICIES = {
    "f32": ("f32", {}),
    "bf16x6": ("bf16x6", {"attn_softmax": "f32"}),
    "parity": ("bf16x3", {"stylizer.fwd": "bf16x6", "stylizer.fwd_img": "bf16x6", "attn_softmax": "f32"}),
    "bf16x3": ("bf16x3", {}),
    "bf16": ("bf16", {}),
    # inside the AdaAttN modules (the 1x1 f / g / h projections and the linear-form cosine
    # attention, whose intermediates G = K^ [V; V^2]^T sum over every style position) and in the
    # image-similarity loss (the C x C cosine-distance matrix gradient) the 2^12-scaled gradients
    # leave fp16's range (tools/nan_diag.py): those products stay on bf16x3 (fp32 exponent range,
    # ~2^-16; a small share of the step's FLOPs).  So does the loss network's forward over the
    # stylised frames (scope "lossnet"): its ReLU / max-pool decisions and the feature differences the
    # losses take route the whole backward, and in fp16 they made the attention-parameter gradients
    # noise-dominated -- a 2^-20 nudge of the input moved them by up to 9 % (tools/f16_sensitivity.py,
    # DESIGN.md section 4.4)
    "f16": ("f16", {"stylizer.attn.fwd": "bf16x3", "stylizer.attn.dgrad": "bf16x3", "stylizer.attn.wgrad": "bf16x3",
                    "attn_cosine": "bf16x3", "attn_softmax": "f32", "loss_fwd": "bf16x3", "loss_dgrad": "bf16x3",
                    "lossnet.fwd": "bf16x3", "lossnet.fwd_img": "bf16x3"}),
}
# Initial loss scale of a policy: the trainers run backward from loss * scale and Adam unscales
# (fp16: the dynamic scaler starts here, vst/reconet/_flat.py LossScaler).
# fp16 operands must lie in [6.1e-5, 65504] to keep their 11-bit significand: the step's
# backward GEMM operands (gradients) reach at most ~0.85 and go down to ~1e-11
# (profiles/r02_fp16_range.json), so 2^12 lifts all but the smallest into the normal range while
# leaving 16x headroom below the fp16 maximum; forward operands (|x| <= ~3.5e3) are not scaled.
LOSS_SCALE = {"f16": 2.0 ** 12}


def loss_scale():
    """The initial loss scale of the selected policy (1.0 unless the policy computes in fp16)."""
    _ensure_policy()
    return LOSS_SCALE.get(POLICY_NAME[0], 1.0)


def _ensure_policy():
    if POLICY_NAME[0] is None:
        use_policy(os.environ.get("VST_GEMM_POLICY", DEFAULT_POLICY))


def base_gemm_mode():
    """Base GEMM mode of the selected policy (0 f32, 1 bf16x3, 2 bf16, 3 bf16x6)."""
    _ensure_policy()
    return _BASE_MODE[0]


def gemm_mode():
    """The mode passed to the library by the pack / GEMM calls being issued (set by gemm_role)."""
    _ensure_policy()
    return _BASE_MODE[0] if _CUR[0] is None else _CUR[0]


def gemm_mode_name(mode=None):
    mode = base_gemm_mode() if mode is None else mode
    return {v: k for k, v in GEMM_MODES.items()}[mode & ~KBLOCK]


def use_policy(name):
    """Select a named policy (POLICIES); returns (base mode, overrides)."""
    if name not in POLICIES:
        raise VstError(f"unknown GEMM policy {name!r} (one of {sorted(POLICIES)})")
    base, pol = POLICIES[name]
    set_gemm_mode(base, pol)
    POLICY_NAME[0] = name
    return POLICIES[name]


POLICY_NAME = [None]


def set_gemm_mode(mode, policy=None):
    """mode: 0..3 or "f32"/"bf16x3"/"bf16"/"bf16x6"; policy: {role: mode} overrides (replaces GEMM_POLICY)."""
    POLICY_NAME[0] = "custom"
    _BASE_MODE[0] = _CUR[0] = _mode_id(mode)
    if policy is not None:
        GEMM_POLICY.clear()
        GEMM_POLICY.update({r: _mode_id(m) for r, m in policy.items()})


def policy_modes():
    """Names of every mode the selected policy can launch (for labelling results)."""
    _ensure_policy()
    return sorted({gemm_mode_name(m) for m in [_BASE_MODE[0], *GEMM_POLICY.values()]})


_SCOPE = _ThreadSlot()
_PSCOPE = _ThreadSlot()  # forward scope re-entered by a backward (policy_scope)


@contextlib.contextmanager
def gemm_scope(name):
    """Name the model part whose GEMMs run inside; scopes nest ("stylizer" then "res" ->
    "stylizer.res") and policy keys "<scope>.<role>" match the innermost scope first, then each
    enclosing one, then "<role>"."""
    old = _SCOPE[0]
    # re-entering the innermost scope (a module that names itself, called from a parent of the same
    # name: AdaAttN / Decoder inside StylizingNetwork) leaves it as is, so "stylizer.attn" stays the
    # key its policy entries name
    _SCOPE[0] = name if old is None else old if old.rpartition(".")[2] == name else f"{old}.{name}"
    try:
        yield
    finally:
        _SCOPE[0] = old


@contextlib.contextmanager
def policy_scope(name):
    """Backward passes run after their forward's gemm_scope has closed (and on autograd's thread):
    a Function that recorded its forward scope re-enters it here, for the POLICY lookup of its
    backward GEMMs only (the channel-blocked K-order choice keeps using the live scope)."""
    old = _PSCOPE[0]
    _PSCOPE[0] = name
    try:
        yield
    finally:
        _PSCOPE[0] = old


def gemm_role(role):
    """Choose the mode for a GEMM of `role` (call before packing its A operand); the first call
    applies the VST_GEMM_POLICY environment variable (default "f32")."""
    m = role_mode(role)
    _CUR[0] = m
    return m


def role_mode(role):
    """The mode gemm_role(role) would choose here, without making it the current one."""
    _ensure_policy()
    m = None
    sc = _PSCOPE[0] if _PSCOPE[0] is not None else _SCOPE[0]
    while sc is not None and m is None:
        m = GEMM_POLICY.get(f"{sc}.{role}")
        sc = sc.rpartition(".")[0] or None
    if m is None:
        m = GEMM_POLICY.get(role, _BASE_MODE[0])
    # channel-blocked K order (VST_GEMM_KBLOCK): consecutive k-tiles revisit the same 16 source
    # channels over all taps, so the gathered rows come from L2 instead of the Infinity Cache.  The
    # stylizer's forward keeps the tap-major order outside its residual blocks: there the blocked
    # order moves the ragged golden step's IN-parameter gradients past the bar under bf16x6
    # (margin 2.7; residual blocks alone: 0.000 -- tools/policy_check.py, VST_KBLOCK=2 / res)
    sc = _SCOPE[0]
    in_stylizer = sc is not None and sc.split(".")[0] == "stylizer"
    if KBLOCK_ON and (KBLOCK_STYLIZER or not in_stylizer or
                      (KBLOCK_RES and (sc.startswith("stylizer.res") or "dec" in sc.split(".")))):
        m |= KBLOCK
    return m


UP2_FWD = os.environ.get("VST_UP2_FWD", "1") != "0"  # A/B: phase-stacked nearest-x2 forward
CIN3_DIRECT = os.environ.get("VST_CIN3_DIRECT", "1") != "0"  # A/B: direct VALU kernel for 3-channel 3x3 convs
_IN_YMASK = os.environ.get("VST_IN_YMASK", "0") != "0"  # A/B: InstanceNorm backward reads the ReLU mask from y


def pack_floats(Mpad, Kpad):
    """Floats of one packed A operand in the current mode (bf16x6 blocks are 96 B, others 64 B)."""
    return Kpad * Mpad * 3 // 2 if (gemm_mode() & ~KBLOCK) == 3 else Kpad * Mpad


def pack_dims(M, K):
    mp, kp = ctypes.c_int(), ctypes.c_int()
    lib.vst_conv_pack_dims(M, K, ctypes.byref(mp), ctypes.byref(kp))
    return mp.value, kp.value


# frozen (requires_grad=False) weights: packs cached per weight OBJECT (weak keys, so a freed
# tensor's entry dies with it and a new tensor at a recycled address never hits a stale pack),
# validated against the tensor's version counter (in-place updates / load_state_dict re-pack).
_PACK_CACHE = {}  # id(w) -> (weakref(w), {key: (pack, event after the pack, stream it was packed on)})


def _cache_entry(w):
    hit = _PACK_CACHE.get(id(w))
    if hit is not None and hit[0]() is w:
        return hit[1]
    return {}


def packed_weight(w, transposed, split_kh=False, kwu=False):
    """Tap-major A[k][m] pack of a conv weight (split_kh: rows (co, kh), k = (kw, ci); kwu: over a
    kw-unfolded source, k = kh*Cu + c*K + kw)."""
    key = (w._version, w.data_ptr(), tuple(w.shape), bool(transposed), bool(split_kh), bool(kwu), gemm_mode())
    if not w.requires_grad:
        hit = _cache_entry(w).get(key)
        if hit is not None:
            out, done, made_on = hit
            if done is not None and made_on != stream():
                # packed on another stream (the side stream's content pass shares the loss net's
                # packs): wait for the pack, and keep the buffer from reuse until this stream is done
                cur = torch.cuda.current_stream(out.device)
                cur.wait_event(done)
                out.record_stream(cur)
            return out
    Cout, Cin, KH, KW = w.shape
    if kwu:
        Cu = kwu_channels(Cout if transposed else Cin, KW)
        M, K = (Cin if transposed else Cout), KH * Cu
    elif split_kh:
        M, K = Cout * KH, KW * Cin
    else:
        M, K = (Cin, KH * KW * Cout) if transposed else (Cout, KH * KW * Cin)
    Mpad, Kpad = pack_dims(M, K)
    out = _empty((pack_floats(Mpad, Kpad),), w)
    inject_delay("pack")
    if kwu:
        lib.vst_pack_weight_kwu(ptr(w), ptr(out), Cout, Cin, KW, Cu, int(transposed), Mpad, Kpad, gemm_mode(), stream())
    else:
        lib.vst_pack_weight(ptr(w), ptr(out), Cout, Cin, KH, KW, int(transposed), int(split_kh), Mpad, Kpad, gemm_mode(),
                            stream())
    if not w.requires_grad:
        entry = {k: v for k, v in _cache_entry(w).items() if k[0] == key[0] and k[1] == key[1]}
        done = None
        if out.is_cuda:
            done = torch.cuda.Event()
            done.record(torch.cuda.current_stream(out.device))
        entry[key] = (out, done, stream() if out.is_cuda else None)
        wid = id(w)
        _PACK_CACHE[wid] = (weakref.ref(w, lambda _r, wid=wid: _PACK_CACHE.pop(wid, None)), entry)
    return out


def kwu_channels(C, ks):
    """channels of the kw-unfolded tensor: C*ks rounded up to the 16-channel k-tile"""
    return (C * ks + 15) // 16 * 16


def kwu_ok(C, ks, stride, up, Wout):
    """Thin tensors (3-channel images, the ConvTanh output gradient) under a KxK stride-1 kernel:
    unfold along kw (C*K <= 32 channels) so the GEMM runs on the 16-channel k-tile path."""
    return C % 16 != 0 and ks > 1 and C * ks <= 32 and stride == 1 and up == 1 and Wout % 4 == 0


def _round4(n):
    return (n + 3) // 4 * 4


def unfold_kw(x, ks, off, sgn, Wout, reflect):
    """out[n][c*ks + kw][y][v] = x[n][c][y][v + sgn*kw + off] (reflect or zero outside)."""
    N, C, H, W = x.shape
    Cu = kwu_channels(C, ks)
    out = _empty((N, Cu, H, Wout), x)
    lib.vst_unfold_kw(ptr(x), ptr(out), N, C, H, W, Wout, ks, Cu, sgn, off, int(reflect), stream())
    return out


def conv_out_hw(H, W, ks, stride, pad, up):
    return (H * up + 2 * pad - ks) // stride + 1, (W * up + 2 * pad - ks) // stride + 1


def conv_gemm(src, wpack, M, ks, Ho, Wo, gmode, stride, pad, up, epi=0, bias=None, out=None, aux=None, gmask=None,
              a_batch_stride=0, mask=None, algo_flops=None, kh=None, pad_x=None):
    """ks: kernel width; kh: kernel height (defaults to ks); pad_x: column padding (defaults to pad)."""
    N, Cs, Hs, Ws = src.shape
    kh = ks if kh is None else kh
    if out is None:
        out = _empty((N, M, Ho, Wo), src)
    pad_x = pad if pad_x is None else pad_x
    mode = gemm_mode()
    ws, nws = splitk_workspace(src, N, Cs, M, Ho, Wo, kh, ks, gmode, stride, pad, pad_x, up, epi, a_batch_stride, mode)
    tok = kprof.begin(algo_flops if algo_flops is not None else 2.0 * N * M * Ho * Wo * Cs * ks * kh,
                      4.0 * (src.numel() + wpack.numel() + out.numel()),
                      (N, Cs, Hs, Ws, M, Ho, Wo, kh, ks, gmode, stride, pad, up), mode)
    lib.vst_conv_gemm_padx(ptr(src), ptr(wpack), ptr(bias), ptr(mask), ptr(out), N, Cs, Hs, Ws, M, kh * ks * Cs, Ho,
                           Wo, kh, ks, gmode, stride, pad, pad_x, up, epi, a_batch_stride, ptr(aux), ptr(gmask), ptr(ws),
                           nws, mode, stream())
    kprof.end(tok)
    return out


SPLITK = os.environ.get("VST_SPLITK", "1") != "0"  # A/B: no workspace -> every launch runs unsplit
_SPLITK_WS = {}  # launch geometry -> split-K workspace bytes (vst_conv_splitk_workspace; host arithmetic)
EPI_PADOUT = 128


def splitk_workspace(like, *geom):
    """(workspace tensor or None, bytes) for a conv GEMM launch of geometry `geom`
    (vst_conv_splitk_workspace's arguments): the split-K scratch comes from PyTorch's caching
    allocator on the current stream, so the library never allocates (include/vst_hip.h)."""
    if not SPLITK:
        return None, 0
    nb = _SPLITK_WS.get(geom)
    if nb is None:
        nb = _SPLITK_WS[geom] = int(lib.vst_conv_splitk_workspace(*geom))
    if nb <= 0:
        return None, 0
    return _empty(((nb + 3) // 4,), like), nb


def conv_dgrad(gz, w, x_shape, ks, stride, pad, pad_mode, up, gmask=None, dmask=None):
    """Input gradient of (upsample x`up` -> pad -> conv(stride)) given the conv-output grad gz;
    dmask: multiply the result by (dmask > 0) in the GEMM epilogue (zero-pad path, and the
    stride-1 reflect-pad padded-grid path with its border fold)."""
    gemm_role("dgrad")
    N, Cin, H, W = x_shape
    Cout = w.shape[0]
    Ho, Wo = gz.shape[2:]
    flops = 2.0 * N * Cout * Ho * Wo * Cin * ks * ks
    if (pad_mode == "zero" and up == 1 and stride == 1 and dmask is None and gmask is None and Cin % 16 != 0
            and Cin * ks * ks <= 32 and (H, W) == tuple(gz.shape[2:])):
        # few input channels (VGG conv1_1): tap-split 1x1 GEMM (rows (c, kh, kw)) + shift-sum
        P = conv_gemm(gz, packed_weight(w.view(Cout, Cin * ks * ks, 1, 1), transposed=True), Cin * ks * ks, 1, H, W,
                      GM_ZERO, 1, 0, 1, algo_flops=flops)
        dx = _empty(x_shape, gz)
        lib.vst_tapsum(ptr(P), ptr(dx), N, Cin, H, W, ks, pad, 0, stream())
        return dx
    if thin_dgrad_ok(Cout, Cin, ks, stride, pad, up, W) and gmask is None:
        return conv_dgrad_thin(gz, w, x_shape, pad_mode == "reflect", dmask)
    if pad_mode == "zero" and up == 1:
        return conv_gemm(gz, packed_weight(w, transposed=True), Cin, ks, H, W, GM_TRANSPOSED, stride, pad, 1,
                         gmask=gmask, algo_flops=flops, epi=EPI_MASK if dmask is not None else 0,
                         mask=dmask.contiguous() if dmask is not None else None)
    padout = pad_mode == "reflect" and stride == 1 and up == 1 and gmask is None and 0 < pad < min(H, W)
    if dmask is not None and not padout:
        raise VstError("dgrad: fused ReLU mask only on the zero-pad and stride-1 reflect-pad paths")
    if pad_mode != "reflect":
        raise VstError("dgrad: zero padding with upsampling is not on the reference path")
    if stride == 2 and up == 1:
        return conv_dgrad_phase2(gz, w, x_shape, ks, pad, gmask, flops)
    if padout:
        dm = dmask.contiguous() if dmask is not None else None
        if kwu_ok(Cout, ks, stride, up, _round4(W + 2 * pad)) and w.shape[2] == ks:
            return conv_dgrad_padout_kwu(gz, w, x_shape, ks, pad, flops, dm)
        return conv_dgrad_padout(gz, w, x_shape, ks, pad, flops, dm)
    if stride == 1 and gmask is None and ks % 2 == 1 and ks > 1 and pad == ks // 2 and min(H, W) * up > ks + 1:
        return conv_dgrad_ring(gz, w, x_shape, ks, up, flops)
    Hp, Wp = H * up + 2 * pad, W * up + 2 * pad
    dpad = conv_gemm(gz, packed_weight(w, transposed=True), Cin, ks, Hp, Wp, GM_TRANSPOSED, stride, 0, 1, gmask=gmask,
                     algo_flops=flops)
    dx = _empty(x_shape, gz)
    lib.vst_fold_reflect(ptr(dpad), ptr(dx), N * Cin, H, W, pad, up, 0, stream())
    return dx


THIN_DGRAD = os.environ.get("VST_THIN_DGRAD", "1") != "0"  # A/B: Cout <= 4 3x3 data gradients on the VALU kernel


def thin_dgrad_ok(Cout, Cin, ks, stride, pad, up, W):
    return THIN_DGRAD and Cout <= 4 and ks == 3 and stride == 1 and pad == 1 and up == 1 and Cin % 2 == 0 \
        and W % 4 == 0 and W >= 8


def conv_dgrad_thin(gz, w, x_shape, reflect, dmask=None):
    """Data gradient of a 3x3 stride-1 pad-1 conv with <= 4 output channels (the AdaAttN decoder's last
    conv, AA/network.py:99) on vst_conv_dgrad_thin: exact fp32 VALU, the fused ReLU mask applied."""
    N, Cin, H, W = x_shape
    Cout = w.shape[0]
    dx = _empty(x_shape, gz)
    border = _empty((N, Cin, H + 2, W + 2), gz) if reflect else None
    dm = dmask.contiguous() if dmask is not None else None
    tok = kprof.begin(2.0 * N * Cout * H * W * Cin * 9, 4.0 * (gz.numel() + 2 * dx.numel()),
                      ("thin_dgrad", N, Cout, Cin, H, W), gemm_mode())
    lib.vst_conv_dgrad_thin(ptr(gz), ptr(w.contiguous()), ptr(dm), ptr(dx), ptr(border), N, Cout, Cin, H, W,
                            int(reflect), stream())
    kprof.end(tok, family="thin")  # (a VALU kernel: outside the MFMA families' rooflines)
    return dx


def conv_dgrad_padout(gz, w, x_shape, ks, pad, flops, dmask=None):
    """Stride-1 reflect-pad conv input gradient: the transposed GEMM over the padded grid writes
    its interior straight into dx and its border into a side buffer, folded into dx's border band."""
    N, Cin, H, W = x_shape
    Cout, Ho, Wo = w.shape[0], gz.shape[2], gz.shape[3]
    wp = packed_weight(w, transposed=True)
    dx = _empty(x_shape, gz)
    border = _empty((N, Cin, H + 2 * pad, W + 2 * pad), gz)
    mode = gemm_mode()
    ws, nws = splitk_workspace(gz, N, Cout, Cin, H + 2 * pad, W + 2 * pad, ks, ks, GM_TRANSPOSED, 1, 0, 0, 1,
                               EPI_PADOUT | (EPI_MASK if dmask is not None else 0), 0, mode)
    tok = kprof.begin(flops, 4.0 * (gz.numel() + wp.numel() + dx.numel()),
                      (N, Cout, Ho, Wo, Cin, H + 2 * pad, W + 2 * pad, ks, ks, GM_TRANSPOSED, 1, 0, 1), mode)
    lib.vst_conv_dgrad_padout(ptr(gz), ptr(wp), ptr(dmask), ptr(dx), ptr(border), N, Cout, Ho, Wo, Cin, H, W, ks, pad,
                              ptr(ws), nws, mode, stream())
    kprof.end(tok)
    lib.vst_fold_border(ptr(border), ptr(dmask), ptr(dx), N * Cin, H, W, pad, stream())
    return dx


HALO91 = os.environ.get("VST_HALO91", "1") != "0"  # A/B: ConvTanh's data gradient on the 9 x 1 halo form


def conv_dgrad_padout_kwu(gz, w, x_shape, ks, pad, flops, dmask=None):
    """conv_dgrad_padout for a thin output gradient (ConvTanh 48->3): dy is kw-unfolded first,
    dyu[co*K + kw][y][v] = dy[co][y][v - kw] over the padded width, so the transposed GEMM is a
    Kx1 gather over 16-multiple channels."""
    N, Cin, H, W = x_shape
    Ho = gz.shape[2]
    dyu = unfold_kw(gz, ks, 0, -1, _round4(W + 2 * pad), reflect=False)
    wp = packed_weight(w, True, kwu=True)
    dx = _empty(x_shape, gz)
    border = _empty((N, Cin, H + 2 * pad, W + 2 * pad), gz)
    tok = kprof.begin(flops, 4.0 * (gz.numel() + wp.numel() + dx.numel()),
                      (N, dyu.shape[1], Ho, W + 2 * pad, Cin, H + 2 * pad, W + 2 * pad, 1, ks, GM_TRANSPOSED, 1, 0, 1),
                      gemm_mode())
    lib.vst_conv_dgrad_padout_kwu(ptr(dyu), ptr(wp), ptr(dmask), ptr(dx), ptr(border), N, dyu.shape[1], Ho, Cin, H, W,
                                  ks, pad, gemm_mode() | (0 if HALO91 else PERTAP), stream())
    kprof.end(tok)
    lib.vst_fold_border(ptr(border), ptr(dmask), ptr(dx), N * Cin, H, W, pad, stream())
    return dx


def conv_dgrad_ring(gz, w, x_shape, ks, up, flops):
    """Stride-1 reflect-pad (optionally nearest-x2-upsampled) conv input gradient on the unpadded
    grid: core GEMM + the padded grid's border ring folded into dx's border band."""
    N, Cin, H, W = x_shape
    Cout = w.shape[0]
    p = ks // 2
    w = w.contiguous()
    if up == 1:
        dx = conv_gemm(gz, packed_weight(w, transposed=True), Cin, ks, H, W, GM_TRANSPOSED, 1, p, 1, algo_flops=flops)
    else:
        Mpad, Kpad = pack_dims(Cin, (ks + 1) * (ks + 1) * Cout)
        wp = _empty((pack_floats(Mpad, Kpad),), w)
        lib.vst_pack_weight_upsum(ptr(w), ptr(wp), Cout, Cin, ks, Mpad, Kpad, gemm_mode(), stream())
        dx = conv_gemm(gz, wp, Cin, ks + 1, H, W, GM_ZERO, 2, ks - 1 - p, 1, algo_flops=flops)
    Hv, Wv = H * up, W * up
    ring = _empty((N * Cin * lib.vst_dgrad_ring_size(Hv, Wv, ks, Cout),), gz)
    lib.vst_dgrad_ring(ptr(gz), ptr(w), ptr(ring), N, Cout, Cin, ks, Hv, Wv, stream())
    lib.vst_fold_ring(ptr(ring), ptr(dx), N * Cin, H, W, ks, up, Cout, stream())
    return dx


def conv_dgrad_phase2(gz, w, x_shape, ks, pad, gmask=None, flops=None):
    """Stride-2 reflect-pad conv input gradient: one transposed GEMM over the 4 parity phases of
    the padded grid (rows ci*4 + phase), interior written straight into dx, border folded after."""
    N, Cin, H, W = x_shape
    Cout, Ho, Wo = w.shape[0], gz.shape[2], gz.shape[3]
    k2 = (ks + 1) // 2
    Mpad, Kpad = pack_dims(4 * Cin, k2 * k2 * Cout)
    wp = _empty((pack_floats(Mpad, Kpad),), w)
    lib.vst_pack_weight_phase2(ptr(w.contiguous()), ptr(wp), Cout, Cin, ks, Mpad, Kpad, gemm_mode(), stream())
    dx = _empty(x_shape, gz)
    border = _empty((N, Cin, H + 2 * pad, W + 2 * pad), gz)
    Hc, Wc = (H + 2 * pad + 1) // 2, (W + 2 * pad + 1) // 2
    tok = kprof.begin(flops if flops is not None else 2.0 * N * Cout * Ho * Wo * Cin * ks * ks,
                      4.0 * (gz.numel() + wp.numel() + dx.numel()),
                      (N, Cout, Ho, Wo, 4 * Cin, Hc, Wc, k2, k2, GM_TRANSPOSED, 1, 0, 1), gemm_mode())
    lib.vst_conv_dgrad_s2(ptr(gz), ptr(wp), ptr(gmask), ptr(dx), ptr(border), N, Cout, Ho, Wo, Cin, H, W, ks, pad,
                          gemm_mode(), stream())
    kprof.end(tok)
    lib.vst_fold_border(ptr(border), None, ptr(dx), N * Cin, H, W, pad, stream())
    return dx


_WGRAD_UP2 = os.environ.get("VST_WGRAD_UP2", "1") != "0"  # A/B switch for the phase-stacked up2 path


# ReCoNet's bf16x6 residual weight gradients (192 rows) stay on the row-tiled kernel: the halo weight
# gradient is a little faster in isolation (32-column strips: 0.578 vs 0.619 ms, tools/wgrad_bench.py)
# but, on the side stream beside the data-gradient GEMMs, overlaps them worse (its blocks hold up to
# 115 KB of LDS): config 3 45.00 / 45.02 ms per step with it vs 44.75 / 44.76 (one box,
# tools/gpu_r05_k3.sh; the 16-column form: 45.97 vs 44.80).
# Everywhere else the halo form wins (AdaAttN decoder shapes 0.69-0.75 of the row-tiled time under
# bf16x6, 0.46-0.65 under fp16).
WGRAD_HALO_RES = os.environ.get("VST_WGRAD_HALO_RES", "0") != "0"  # A/B


def conv_wgrad(gz, x, w_shape, ks, stride, pad, pad_mode, up, out=None):
    gemm_role("wgrad")
    N, Cin, H, W = x.shape
    Cout = w_shape[0]
    Ho, Wo = gz.shape[2:]
    if _WGRAD_UP2 and up == 2 and ks == 3 and stride == 1 and pad == 1 and pad_mode == "reflect":
        return conv_wgrad_up2(gz, x, w_shape, out)
    gm = GM_REFLECT if pad_mode == "reflect" else GM_ZERO
    mode = gemm_mode()
    if not WGRAD_HALO_RES and (mode & 7) == GEMM_MODES["bf16x6"] and Cout % 192 == 0 and Cout % 128 != 0:
        mode |= PERTAP
    if not THIN_WGRAD and Cout <= 4:
        mode |= PERTAP  # (the A/B switch: the row-tiled GEMM instead of the VALU kernel)
    nws = lib.vst_conv_wgrad_workspace(N, Cin, H, W, Cout, Ho, Wo, ks, ks, gm, stride, pad, up, mode)
    ws = _empty((nws,), x)
    acc = out is not None
    dw = _empty(w_shape, x) if out is None else out
    tok = kprof.begin(2.0 * N * Cout * Ho * Wo * Cin * ks * ks, 4.0 * (gz.numel() + x.numel() + dw.numel()),
                      ("wgrad", N, Cin, H, W, Cout, Ho, Wo, ks, stride, pad, up), mode)
    lib.vst_conv_wgrad(ptr(gz), ptr(x), ptr(dw), ptr(ws), nws, N, Cin, H, W, Cout, Ho, Wo, ks, ks, gm, stride, pad,
                       up, int(acc), mode, stream())
    kprof.end(tok, family="thin" if pad == 1 and thin_wgrad_ok(Cout, Cin, ks, stride, up, W) else "wgrad")
    return dw


def conv_wgrad_up2(gz, x, w_shape, out=None):
    """Weight gradient of UpsampleConvLayer (nearest x2, reflect pad 1, k3; RC/network.py:114-120)
    as the phase-stacked source-grid GEMM (vst_conv_wgrad_up2)."""
    N, Cin, H, W = x.shape
    Cout = w_shape[0]
    ws = _empty((lib.vst_conv_wgrad_up2_workspace(N, Cin, H, W, Cout),), x)
    acc = out is not None
    dw = _empty(w_shape, x) if out is None else out
    tok = kprof.begin(2.0 * N * Cout * 4 * H * W * Cin * 9, 4.0 * (gz.numel() + x.numel() + dw.numel()),
                      ("wgrad_up2", N, Cin, H, W, Cout), gemm_mode())
    lib.vst_conv_wgrad_up2(ptr(gz), ptr(x), ptr(dw), ptr(ws), N, Cin, H, W, Cout, int(acc), gemm_mode(), stream())
    kprof.end(tok, family="wgrad")
    return dw


def rowsplit_ok(Cout, ks, stride, pad_mode, up):
    """Tiny-Cout stride-1 reflect convs (ConvTanh 48->3 k9) run as row-split GEMMs."""
    return Cout * ks <= 32 and ks > 1 and stride == 1 and pad_mode == "reflect" and up == 1


RS_WGRAD = os.environ.get("VST_RSW", "1") != "0"
THIN_WGRAD = os.environ.get("VST_THIN_WGRAD", "1") != "0"  # A/B: Cout <= 4 3x3 weight gradients on the VALU kernel


def thin_wgrad_ok(Cout, Cin, ks, stride, up, W):
    """vst_conv_wgrad's own choice (csrc/wgrad_gemm.hip thin_wgrad_ok) for pad-1 convs"""
    return THIN_WGRAD and Cout <= 4 and ks == 3 and stride == 1 and up == 1 and Cin % 4 == 0 and W % 4 == 0 and W >= 8


def rowsplit_wgrad_ok(Cout, Cin, ks, stride, pad_mode, up, W):
    """Weight gradients that run as row-split GEMMs: the tiny-Cout convs above, and 64-output
    3x3 stride-1 reflect convs over >= 64 channels (the AdaAttN decoder's conv6 / conv7,
    AA/network.py:93-96).  Rows (co, kh) read dY[co][y - kh], columns (kw, ci) read x[ci][y][x + kw]:
    M = 3 Cout and J = 3 Cin instead of M = Cout and J = 9 Cin, so each dY tile feeds 3x the rows and
    is re-read for 3x fewer column tiles (64 x 576 -> 192 x 192 for 64 -> 64)."""
    if thin_wgrad_ok(Cout, Cin, ks, stride, up, W):
        return False  # vst_conv_wgrad's fp32 VALU kernel (the AdaAttN decoder's last conv, 64 -> 3)
    if rowsplit_ok(Cout, ks, stride, pad_mode, up):
        return True
    if not (RS_WGRAD and Cout <= 64 and Cin >= 64 and ks == 3 and stride == 1 and pad_mode == "reflect" and up == 1
            and W % 16 == 0):
        return False
    # the halo weight gradient (vst_conv_wgrad: 32-channel multiples, split-product modes) beats the
    # row-split GEMM on these shapes (fp16 decoder conv6 1.12 vs 1.41 ms, conv7 3.6 vs 4.5 ms at config 5,
    # tools/wgrad_bench.py); the row-split form stays for the f32 / bf16x3 modes and the widths the halo
    # kernel does not take (csrc/wgrad_halo.hip wgrad_halo_ok: its 64-row blocks walk 32-column strips
    # in every split-product mode, so W % 32 == 0)
    return not (Cin % 32 == 0 and W % 32 == 0 and (role_mode("wgrad") & 7) in (
        GEMM_MODES["bf16x6"], GEMM_MODES["bf16"], GEMM_MODES["f16"]))


KBLOCK_RS = KBLOCK_ON and os.environ.get("VST_KBLOCK_RS", "1") != "0"  # A/B: the row-split forward blocked


def conv_fwd_rowsplit(x, w, b, epi, aux):
    N, Cin, H, W = x.shape
    Cout, _, K, _ = w.shape
    Hq = H + K - 1
    # the 1 x K GEMM in the channel-blocked K order: the halo kernel's 1 x 9 form (the source rows
    # staged once per 16-channel block for the nine column taps)
    if KBLOCK_RS and Cin % 16 == 0:
        _CUR[0] |= KBLOCK
    P = conv_gemm(x, packed_weight(w, False, split_kh=True), Cout * K, K, Hq, W, GM_REFLECT, 1, K // 2, 1, kh=1,
                  algo_flops=2.0 * N * Cout * H * W * Cin * K * K)
    out = _empty((N, Cout, H, W), x)
    lib.vst_rowsplit_reduce(ptr(P), ptr(b), ptr(out), ptr(aux), N, Cout, K, H, W, epi, stream())
    return out


def conv_wgrad_rowsplit(gz, x, w_shape, out=None):
    gemm_role("wgrad")
    N, Cin, H, W = x.shape
    Cout, _, K, _ = w_shape
    ws = _empty((lib.vst_wgrad_workspace(N, Cout * K, K * Cin, (H + K - 1) * W),), x)
    acc = out is not None
    dw = _empty(w_shape, x) if out is None else out
    lib.vst_conv_wgrad_rowsplit(ptr(gz), ptr(x), ptr(dw), ptr(ws), N, Cin, H, W, Cout, K, int(acc), gemm_mode(), stream())
    return dw


def channel_sum(x, out=None):
    N, C = x.shape[:2]
    HW = x[0, 0].numel()
    acc = out is not None
    out = _empty((C,), x) if out is None else out
    part = _empty((N * C,), x)
    lib.vst_channel_sum(ptr(x), ptr(out), ptr(part), N, C, HW, int(acc), stream())
    return out


def grad_sink(p):
    """The .grad buffer of a leaf parameter that kernels can accumulate into directly (and the
    Function then returns None for it, skipping autograd's AccumulateGrad add); None otherwise.
    FlatParams pre-creates these views into the flat gradient buffer."""
    if p is None or not p.requires_grad or p.grad_fn is not None:
        return None
    g = p.grad
    if g is None or g.dtype != torch.float32 or not g.is_contiguous() or g.shape != p.shape or not g.is_cuda:
        return None
    return g


WGRAD_SIDE = os.environ.get("VST_WGRAD_SIDE", "1") != "0"  # A/B: weight gradients on a second stream
_SIDE = {}
_SIDE_SINKS = set()  # data_ptr of the gradients accumulated on a side stream since the last join
FIRST_INLINE = os.environ.get("VST_FIRST_INLINE", "1") != "0"  # A/B: no-data-gradient layers' wgrad in line


def _side_stream(dev):
    s = _SIDE.get(dev)
    if s is None:
        s = _SIDE[dev] = torch.cuda.Stream(device=dev)
    return s


def join_side_streams():
    """The current stream waits for every weight gradient queued on the side streams (called at the
    end of each backward pass and by the data-parallel bucket launch before it reads the flat
    gradient)."""
    for dev, s in _SIDE.items():
        torch.cuda.current_stream(dev).wait_stream(s)
    _SIDE_SINKS.clear()


def wgrad_into_sink(compute, sink, *used, overlap=True):
    """Run `compute()` -- a weight-gradient GEMM accumulating into the leaf gradient `sink` -- on a
    second HIP stream of the device.  A layer's weight gradient is read only by the optimizer, its
    data gradient by the next layer back, so the wgrad GEMMs (latency-bound, about a third
    MFMA-busy: profiles/r04_mfma_busy_*.json) run beside the MFMA-bound data-gradient GEMMs of the
    layers before them instead of in series.  Ordering: the side stream first waits for the current
    stream (the inputs `used` and the zeroed sink are ready), `used` are recorded on it so the
    caching allocator keeps them until it is done, and a final callback of the backward pass makes
    the caller's stream wait for it (so `.grad` and the optimizer see the finished gradients).
    Gradients returned to autograd (no sink) stay on the current stream, and so does the weight
    gradient of a layer with no data gradient (`overlap=False`: the network's first conv), which then
    runs beside the previous layer's weight gradient still on the side stream."""
    if not (WGRAD_SIDE and sink is not None and sink.is_cuda):
        return compute()
    if FIRST_INLINE and not overlap and sink.data_ptr() not in _SIDE_SINKS:  # (else: keep the sink's writes in order)
        return compute()
    _SIDE_SINKS.add(sink.data_ptr())
    dev = sink.device
    side = _side_stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        inject_delay("wgrad_side")
        compute()
    for t in used:
        t.record_stream(side)
    torch.autograd.Variable._execution_engine.queue_callback(join_side_streams)
    return sink


CONTENT_SIDE = os.environ.get("VST_CONTENT_SIDE", "1") != "0"  # A/B: input-only targets on the side stream


class _SideBranch:
    """`with side_branch(*inputs) as side:` runs its body (no-grad work that depends on `inputs`
    only) on the device's side stream, beside what the current stream does next; `side.produced(*t)`
    names the tensors the body made (their memory is then recorded on the current stream, which
    reads and frees them), `side.join()` makes the current stream wait for the body before it reads
    them.  On CPU tensors (or with VST_CONTENT_SIDE=0) the body runs in line."""

    def __init__(self, inputs):
        ts = [t for t in inputs if isinstance(t, torch.Tensor)]
        self.on = CONTENT_SIDE and bool(ts) and ts[0].is_cuda
        self.inputs, self.ctx, self.made = ts, None, []
        if self.on:
            dev = ts[0].device
            self.main, self.side = torch.cuda.current_stream(dev), _side_stream(dev)

    def __enter__(self):
        if self.on:
            self.side.wait_stream(self.main)
            for t in self.inputs:
                t.record_stream(self.side)
            self.ctx = torch.cuda.stream(self.side)
            self.ctx.__enter__()
            inject_delay("side_branch")
        return self

    def __exit__(self, *exc):
        if self.ctx is not None:
            self.ctx.__exit__(*exc)
            self.ctx = None
        return False

    def produced(self, *ts):
        self.made = [t for t in ts if isinstance(t, torch.Tensor)]

    def join(self):
        if self.on:
            self.main.wait_stream(self.side)
            for t in self.made:
                t.record_stream(self.main)


def side_branch(*inputs):
    return _SideBranch(inputs)


_CONST_FILL = {}  # id(constant) -> (event after its fill, streams ordered after that event)


def persistent(t):
    """A lazily created constant kept in a module-level cache (read afterwards from either stream):
    an event is recorded after its fill on the creating stream; `constant(t)` makes any other
    stream wait for that event the first time it reads t (no host synchronisation)."""
    if t.is_cuda:
        cur = torch.cuda.current_stream(t.device)
        ev = torch.cuda.Event()
        ev.record(cur)
        _CONST_FILL[id(t)] = (ev, {cur})
    return t


def persistent_full(like, *fills):
    """persistent() constants [n] filled with `value` for each (n, value) in `fills`, all covered by
    one event recorded after the last fill."""
    ts = [torch.empty(n, device=like.device, dtype=torch.float32) for n, _ in fills]
    inject_delay("persistent")
    for t, (_, v) in zip(ts, fills):
        if t.is_cuda:
            lib.vst_fill(ptr(t), t.numel(), float(v), stream())
        else:
            t.fill_(v)
    if like.is_cuda:
        cur = torch.cuda.current_stream(like.device)
        ev = torch.cuda.Event()
        ev.record(cur)
        for t in ts:
            _CONST_FILL[id(t)] = (ev, {cur})
    return ts


# Test hooks (tests/test_gpu_streams.py): {placement: iterations} -> vst_test_delay(iterations) is
# enqueued on the current stream at that cross-stream hand-off ("side_branch": head of the input-only
# side branch; "wgrad_side": head of each side-stream weight gradient; "pack": before each weight pack
# kernel; "persistent": before the fill of each lazily created constant).  Empty in normal runs.
TEST_DELAY = {}


def inject_delay(place):
    it = TEST_DELAY.get(place)
    if it:
        lib.vst_test_delay(int(it), stream())


def constant(t):
    """Hand out a `persistent` constant on the current stream: a stream other than the one that
    filled it first waits on the fill's event (once per stream).  Cached constants are never freed,
    so their ids stay unique."""
    e = _CONST_FILL.get(id(t))
    if e is not None:
        cur = torch.cuda.current_stream(t.device)
        if cur not in e[1]:
            cur.wait_event(e[0])
            e[1].add(cur)
    return t


class Conv2dFn(Function):
    """[nearest x`up` upsample] -> (reflect|zero) pad -> Conv2d(ks, stride) [+bias] [-> ReLU | ReCoNet tanh].
    Replaces RC/network.py:72-75 (ConvLayer), 114-120 (UpsampleConvLayer), 83-85 (ConvTanh) and the
    torchvision VGG Conv2d+ReLU pairs (RC/network.py:17-24, AA/vgg19.py:19-37)."""

    @staticmethod
    def forward(ctx, x, w, b, stride, pad, pad_mode, up, act, bias_const=None, mask_dx=False, premasked=False):
        """bias_const: a bias added in the epilogue whose gradient another Function produces
        (conv -> InstanceNorm: the norm's backward already sums the conv-output gradient).
        mask_dx: x is a ReLU output consumed only by this conv -> the data gradient is written
        masked by x > 0 (the ReLU backward of the producer, fused into this dgrad's epilogue);
        premasked: this conv's ReLU output is consumed only by such a masking consumer, so the
        incoming gradient is already masked and the separate ReLU-backward pass is skipped."""
        x = _check(x, "conv input", 4)
        w = w.contiguous()
        N, Cin, H, W = x.shape
        Cout, _, ks, _ = w.shape
        Ho, Wo = conv_out_hw(H, W, ks, stride, pad, up)
        if bias_const is not None:
            b = bias_const
        epi = (EPI_BIAS if b is not None else 0) | (EPI_RELU if act == "relu" else 0) | (EPI_TANH if act == "tanh" else 0)
        aux = _empty((N, Cout, Ho, Wo), x) if act == "tanh" else None
        bias = b.contiguous() if b is not None else None
        # image-space inputs (3 channels: ReCoNet conv1 on raw [0, 255] frames, VGG conv1_1) have a
        # large common offset that the following InstanceNorm subtracts again: their products
        # need fp32 relative precision (role "fwd_img")
        gemm_role("fwd_img" if Cin == 3 else "fwd")
        if rowsplit_ok(Cout, ks, stride, pad_mode, up) and pad == ks // 2:
            out = conv_fwd_rowsplit(x, w, bias, epi, aux)
        elif CIN3_DIRECT and Cin == 3 and ks == 3 and stride == 1 and up == 1 and pad == 1 and act in (None, "relu") \
                and H > 1 and W > 1:
            # VGG conv1_1: 27 MACs per output, bound by the output write -> direct fp32 VALU kernel
            out = _empty((N, Cout, Ho, Wo), x)
            lib.vst_conv_cin3_k3(ptr(x), ptr(w), ptr(bias), ptr(out), N, H, W, Cout, int(pad_mode == "reflect"),
                                 int(act == "relu"), stream())
        elif UP2_FWD and up == 2 and ks == 3 and stride == 1 and pad == 1 and pad_mode == "reflect" and act is None:
            # UpsampleConvLayer: phase-stacked 2x2 GEMM on the source grid (tap-summed weights), in
            # the channel-blocked K order (the halo-tiled kernel's 2x2 form)
            if KBLOCK_UP2:
                _CUR[0] |= KBLOCK
            w2 = _empty((4 * Cout, Cin, 2, 2), w)
            lib.vst_up2_phase_weights(ptr(w), ptr(w2), Cout, Cin, stream())
            out = _empty((N, Cout, Ho, Wo), x)
            wp = packed_weight(w2, False)
            tok = kprof.begin(2.0 * N * Cout * Ho * Wo * Cin * ks * ks, 4.0 * (x.numel() + wp.numel() + out.numel()),
                              (N, Cin, H, W, 4 * Cout, H + 1, W + 1, 2, 2, 3, 1, 1, 1), gemm_mode())
            lib.vst_conv_up2_fwd(ptr(x), ptr(wp), ptr(bias), ptr(out), N, Cin, H, W, Cout, gemm_mode(), stream())
            kprof.end(tok)
        elif kwu_ok(Cin, ks, stride, up, W) and 0 < pad < min(H, W) and Ho == H and Wo == W:
            # thin input (3-channel frames): kw-unfold, then a Kx1 conv on the 16-channel k-tile path, in
            # the channel-blocked K order (the halo-tiled kernel's 9 x 1 form)
            if KBLOCK_KWU:
                _CUR[0] |= KBLOCK
            xu = unfold_kw(x, ks, -pad, 1, W, pad_mode == "reflect")
            out = conv_gemm(xu, packed_weight(w, False, kwu=True), Cout, 1, Ho, Wo,
                            GM_REFLECT if pad_mode == "reflect" else GM_ZERO, 1, pad, 1, epi=epi, bias=bias, aux=aux,
                            kh=ks, pad_x=0, algo_flops=2.0 * N * Cout * Ho * Wo * Cin * ks * ks)
            # (the weight gradient stays on x: over the unfolded input its columns pad 243 -> 384,
            # measured 1.7x slower)
        else:
            out = conv_gemm(x, packed_weight(w, False), Cout, ks, Ho, Wo, GM_REFLECT if pad_mode == "reflect" else GM_ZERO,
                            stride, pad, up, epi=epi, bias=bias, aux=aux)
        ctx.geom = (ks, stride, pad, pad_mode, up, act)
        ctx.scope = _SCOPE[0]
        ctx.relu_flags = (bool(mask_dx), bool(premasked))
        ctx.has_bias = b is not None and bias_const is None
        ctx.params = (w, b)  # leaves: weight gradients go straight into their .grad when possible
        ctx.save_for_backward(x, w, out if act == "relu" else None, aux)
        return out

    @staticmethod
    def backward(ctx, gy):
        with policy_scope(ctx.scope):
            return Conv2dFn._backward(ctx, gy)

    @staticmethod
    def _backward(ctx, gy):
        x, w, y, t = ctx.saved_tensors
        ks, stride, pad, pad_mode, up, act = ctx.geom
        gy = gy.contiguous()
        gz, gmask = gy, None
        if act == "tanh":
            gz = _empty(gy.shape, gy)
            lib.vst_tanh_out_bwd(ptr(gy), ptr(t), ptr(gz), gy.numel(), gy[0, 0].numel(), 0, stream())
        elif act == "relu" and not ctx.relu_flags[1]:
            # a separate masking pass (3 HBM streams) measured cheaper than gathering the mask
            # inside the dgrad GEMM (one extra load per gathered element, 9x per output)
            gz = _empty(gy.shape, gy)
            lib.vst_relu_bwd(ptr(gy), ptr(y), ptr(gz), gy.numel(), stream())
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = conv_dgrad(gz, w, x.shape, ks, stride, pad, pad_mode, up, gmask=gmask,
                            dmask=x if ctx.relu_flags[0] else None)
        if ctx.needs_input_grad[1]:
            sink = grad_sink(ctx.params[0])
            if rowsplit_wgrad_ok(w.shape[0], w.shape[1], ks, stride, pad_mode, up, x.shape[3]) and pad == ks // 2:
                dw = wgrad_into_sink(lambda: conv_wgrad_rowsplit(gz, x, w.shape, out=sink), sink, gz, x,
                                     overlap=ctx.needs_input_grad[0])
            else:
                dw = wgrad_into_sink(lambda: conv_wgrad(gz, x, w.shape, ks, stride, pad, pad_mode, up, out=sink),
                                     sink, gz, x, overlap=ctx.needs_input_grad[0])
            dw = None if sink is not None else dw
        if ctx.has_bias and ctx.needs_input_grad[2]:
            sink = grad_sink(ctx.params[1])
            db = channel_sum(gz, out=sink)
            db = None if sink is not None else db
        return dx, dw, db, None, None, None, None, None, None, None, None


def conv2d(x, w, b=None, stride=1, pad=0, pad_mode="zero", up=1, act=None, mask_dx=False, premasked=False):
    return Conv2dFn.apply(x, w, b, stride, pad, pad_mode, up, act, None, mask_dx, premasked)


class InstanceNormFn(Function):
    """InstanceNorm2d(C, affine=True) [-> ReLU] [+ residual] (RC/network.py:91-97, 126-132, 140-150)."""

    @staticmethod
    def forward(ctx, x, w, b, res, relu, eps, conv_bias=None):
        """conv_bias: bias of the conv producing x (added in that conv's epilogue); its gradient,
        sum of dx over (n, h, w), falls out of this backward's per-plane partials."""
        x = _check(x, "instance_norm input", 4)
        N, C, H, W = x.shape
        y = _empty(x.shape, x)
        stats = _empty((N * C * 2,), x)
        res_c = res.contiguous() if res is not None else None
        lib.vst_instnorm_fwd(ptr(x), ptr(w.contiguous()), ptr(b.contiguous()), ptr(res_c), ptr(y), ptr(stats), N, C,
                             H * W, float(eps), int(relu), stream())
        ctx.relu = relu
        ctx.has_res = res is not None
        ctx.params = (w, b, conv_bias)
        # the backward recomputes the ReLU mask from x and b; y > 0 is the mask only without a
        # residual added after the ReLU (y = relu(.) + res)
        keep_y = relu and _IN_YMASK and res is None
        # b is saved (not read live from ctx.params) so an in-place update of it before this
        # backward -- the recomputed ReLU mask depends on it -- trips autograd's version check
        # (FlatParams.adam bumps the flat buffer's version after its kernel)
        ctx.save_for_backward(x, y if keep_y else None, stats, w, b)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, y, stats, w, b = ctx.saved_tensors
        gy = gy.contiguous()
        N, C, H, W = x.shape
        gx = _empty(x.shape, x)
        sw, sb = grad_sink(ctx.params[0]), grad_sink(ctx.params[1])
        need_c = ctx.params[2] is not None and ctx.needs_input_grad[6]
        sc = grad_sink(ctx.params[2]) if need_c else None
        direct = sw is not None and sb is not None and (not need_c or sc is not None)
        gw = sw if direct else _empty((C,), x)
        gb = sb if direct else _empty((C,), x)
        gc = (sc if direct else _empty((C,), x)) if need_c else None
        part = _empty((N * C * 3,), x)
        lib.vst_instnorm_bwd(ptr(gy), ptr(x), ptr(y), ptr(b.contiguous()), ptr(stats), ptr(w.contiguous()),
                             ptr(gx), ptr(gw), ptr(gb), ptr(gc), ptr(part), N, C, H * W, int(ctx.relu), int(direct),
                             stream())
        gres = gy if ctx.has_res else None
        if direct:
            gw = gb = gc = None
        return gx, gw, gb, gres, None, None, gc


def instance_norm(x, w, b, relu=False, res=None, eps=1e-5):
    return InstanceNormFn.apply(x, w, b, res, relu, eps)


def conv_instance_norm(x, w, b, gamma, beta, stride=1, pad=0, pad_mode="reflect", up=1, relu=False, res=None,
                       eps=1e-5):
    """conv [+bias] -> InstanceNorm(affine) [-> ReLU] [+ res] (ConvInstRelu, UpsampleConvInstRelu,
    ResidualBlock halves).  The conv bias gradient comes out of the norm's backward partials, so
    no separate channel-sum pass re-reads the gradient."""
    if b is None:
        return instance_norm(conv2d(x, w, None, stride, pad, pad_mode, up), gamma, beta, relu, res, eps)
    y = Conv2dFn.apply(x, w, None, stride, pad, pad_mode, up, None, b.detach())
    return InstanceNormFn.apply(y, gamma, beta, res, relu, eps, b)


class MaxPool2x2Fn(Function):
    """nn.MaxPool2d(2, 2) of the VGG feature stacks."""

    @staticmethod
    def forward(ctx, x, relu_mask=False):
        x = _check(x, "maxpool input", 4)
        N, C, H, W = x.shape
        y = _empty((N, C, H // 2, W // 2), x)
        lib.vst_maxpool2x2_fwd(ptr(x), ptr(y), N * C, H, W, stream())
        ctx.relu_mask = relu_mask
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, gy):
        (x,) = ctx.saved_tensors
        N, C, H, W = x.shape
        gx = _empty(x.shape, x)
        lib.vst_maxpool2x2_bwd(ptr(x), ptr(gy.contiguous()), ptr(gx), N * C, H, W, int(ctx.relu_mask), stream())
        return gx, None


def maxpool2x2(x, relu_mask=False):
    """relu_mask: x is a ReLU output consumed only by this pool; the ReLU backward is folded into
    the pool's backward (the producing conv is then built with premasked=True)."""
    return MaxPool2x2Fn.apply(x, relu_mask)


class FeaturePoolFn(Function):
    """A VGG slice output h (a ReLU output) that is both a loss feature and the next slice's
    MaxPool2d(2, 2) input (RC/network.py:33-40 slice boundaries): returns (h, maxpool(h)); the
    backward is relu_mask(pool_bwd(g_pool) + g_feature) in one pass, replacing autograd's sum of
    the two gradients, the pool backward and the producer's ReLU backward (the producing conv is
    then built premasked)."""

    @staticmethod
    def forward(ctx, h):
        h = _check(h, "feature", 4)
        N, C, H, W = h.shape
        p = _empty((N, C, H // 2, W // 2), h)
        lib.vst_maxpool2x2_fwd(ptr(h), ptr(p), N * C, H, W, stream())
        ctx.save_for_backward(h)
        ctx.set_materialize_grads(False)
        return h.view_as(h), p

    @staticmethod
    def backward(ctx, g_feat, g_pool):
        (h,) = ctx.saved_tensors
        N, C, H, W = h.shape
        gx = _empty(h.shape, h)
        lib.vst_maxpool2x2_bwd_add(ptr(h), ptr(g_pool.contiguous() if g_pool is not None else None),
                                   ptr(g_feat.contiguous() if g_feat is not None else None), ptr(gx), N * C, H, W, 1,
                                   stream())
        return gx


def feature_pool(h):
    """(h, maxpool2x2(h)) with the fused slice-boundary backward of FeaturePoolFn."""
    return FeaturePoolFn.apply(h)


class FeatureSplitFn(Function):
    """A VGG slice output h (a ReLU output) that is both a loss feature and the next slice's conv
    input (AA/vgg19.py:39-63: relu1_1 .. relu4_1 feed slice2 .. slice5 and the losses): returns two
    views of h; the backward is relu_mask(g_feature + g_next) in one pass (vst_relu_bwd_add),
    replacing autograd's sum of the two gradients and the producer's ReLU backward (the producing
    conv is then built premasked)."""

    @staticmethod
    def forward(ctx, h):
        h = _check(h, "feature", 4)
        ctx.save_for_backward(h)
        ctx.set_materialize_grads(False)
        return h.view_as(h), h.view_as(h)

    @staticmethod
    def backward(ctx, g_feat, g_next):
        (h,) = ctx.saved_tensors
        gs = [g.contiguous() for g in (g_feat, g_next) if g is not None]
        if not gs:
            return None
        gx = _empty(h.shape, h)
        lib.vst_relu_bwd_add(ptr(gs[0]), ptr(gs[1]) if len(gs) > 1 else None, ptr(h), ptr(gx), h.numel(), stream())
        return gx


def feature_split(h):
    """(h, h) with the fused slice-boundary backward of FeatureSplitFn."""
    return FeatureSplitFn.apply(h)


class WarpFn(Function):
    """utilities.warp (RC/utilities.py:39-57); gradient w.r.t. x only (flow is data)."""

    @staticmethod
    def forward(ctx, x, flo):
        x = _check(x, "warp input", 4)
        flo = _check(flo, "flow", 4)
        B, C, H, W = x.shape
        if flo.shape != (B, 2, H, W):
            raise VstError(f"warp: flow shape {tuple(flo.shape)} does not match {(B, 2, H, W)}")
        out = _empty(x.shape, x)
        lib.vst_warp_fwd(ptr(x), ptr(flo), ptr(out), B, C, H, W, stream())
        ctx.save_for_backward(flo)
        ctx.shape = x.shape
        return out

    @staticmethod
    def backward(ctx, gout):
        (flo,) = ctx.saved_tensors
        B, C, H, W = ctx.shape
        gx = _empty(ctx.shape, flo)
        ws = _empty(((lib.vst_warp_bwd_workspace(B, H, W) + 3) // 4,), flo)
        lib.vst_warp_bwd_gather(ptr(gout.contiguous()), ptr(flo), ptr(gx), ptr(ws), B, C, H, W, 0, stream())
        return gx, None


def warp(x, flo):
    return WarpFn.apply(x, flo)


class GramFn(Function):
    """gram_matrix (RC/utilities.py:93-98): F F^T / (C H W) per sample, MFMA split-K."""

    @staticmethod
    def forward(ctx, y, per_hw=False):
        """per_hw: divide by H*W only (RT/utilities.py:155-160) instead of C*H*W."""
        y = _check(y, "gram input", 4)
        N, C, H, W = y.shape
        g = _empty((N, C, C), y)
        ws = _empty((lib.vst_wgrad_workspace(N, C, C, H * W),), y)
        gemm_role("fwd")
        ctx.scale = 1.0 / (H * W) if per_hw else 1.0 / (C * H * W)
        lib.vst_gram(ptr(y), ptr(g), ptr(ws), N, C, H * W, ctx.scale, gemm_mode(), stream())
        ctx.save_for_backward(y)
        return g

    @staticmethod
    def backward(ctx, gg):
        (y,) = ctx.saved_tensors
        N, C, H, W = y.shape
        gemm_role("dgrad")  # before sizing S: the pack layout (and size) is the dgrad role's mode
        Mpad, Kpad = pack_dims(C, C)
        S = _empty((N * pack_floats(Mpad, Kpad),), y)
        lib.vst_symmetrize(ptr(gg.contiguous()), ptr(S), N, C, Kpad, Mpad, ctx.scale, gemm_mode(), stream())
        dy = conv_gemm(y.view(N, C, 1, H * W), S, C, 1, 1, H * W, GM_ZERO, 1, 0, 1, a_batch_stride=pack_floats(Mpad, Kpad))
        return dy.view(N, C, H, W), None


def gram_matrix(y, per_hw=False):
    return GramFn.apply(y, per_hw)


class VggNormalizeFn(Function):
    """vgg_normalize's arithmetic (x/255 - mean)/std, out of place (AA/utilities.py:79-85 form)."""

    @staticmethod
    def forward(ctx, x):
        x = _check(x, "vgg_normalize input", 4)
        N, C, H, W = x.shape
        if C != 3:
            raise VstError("vgg_normalize expects 3 channels")
        out = _empty(x.shape, x)
        lib.vst_vgg_normalize(ptr(x), ptr(out), N, H * W, 0, stream())
        return out

    @staticmethod
    def backward(ctx, g):
        N, C, H, W = g.shape
        gx = _empty(g.shape, g)
        lib.vst_vgg_normalize_bwd(ptr(g.contiguous()), None, ptr(gx), N, H * W, stream())
        return gx


class VggNormalizeInplaceFn(Function):
    """RC/utilities.py:101-106: `batch.div_(255)` mutates the argument, then returns (batch-mean)/std.
    Returns (mutated x, normalized); the caller keeps the second."""

    @staticmethod
    def forward(ctx, x):
        if not x.is_contiguous():
            raise VstError("vgg_normalize (in place) needs a contiguous tensor")
        _check(x, "vgg_normalize input", 4)
        N, C, H, W = x.shape
        out = _empty(x.shape, x)
        lib.vst_vgg_normalize(ptr(x), ptr(out), N, H * W, 1, stream())
        ctx.mark_dirty(x)
        return x, out

    @staticmethod
    def backward(ctx, gscaled, gout):
        N, C, H, W = gout.shape
        gx = _empty(gout.shape, gout)
        gs = gscaled.contiguous() if gscaled is not None else None
        lib.vst_vgg_normalize_bwd(ptr(gout.contiguous()), ptr(gs), ptr(gx), N, H * W, stream())
        return gx


# ------------------------------------------------------------------ losses (0-d outputs)
class MSEFn(Function):
    """weight * mean((a - b)^2); b may be one sample broadcast over a's batch (gram_s.expand)."""

    @staticmethod
    def forward(ctx, a, b, weight):
        a = _check(a, "mse a")
        b = _check(b, "mse b")
        n, nb = a.numel(), b.numel()
        if n % nb:
            raise VstError("mse: b must broadcast over a's leading dim")
        ws = _empty((LOSS_WS,), a)
        st = _empty((3,), a)
        lib.vst_mse_fwd(ptr(a), ptr(b), n, nb, float(weight), ptr(ws), ptr(st), stream())
        ctx.save_for_backward(a, b, st)
        return st[0]

    @staticmethod
    def backward(ctx, g):
        a, b, st = ctx.saved_tensors
        ga = _empty(a.shape, a) if ctx.needs_input_grad[0] else None
        gb = _empty(b.shape, b) if ctx.needs_input_grad[1] and a.numel() == b.numel() else None
        if ctx.needs_input_grad[1] and gb is None:
            raise VstError("mse: gradient for a broadcast target is not supported")
        lib.vst_mse_bwd(ptr(a), ptr(b), a.numel(), b.numel(), ptr(g.contiguous()), ptr(st), ptr(ga), ptr(gb), stream())
        return ga, gb, None


def mse(a, b, weight=1.0):
    return MSEFn.apply(a, b, weight)


def sum_into(out, parts):
    """out = sum of `parts` (same-shape contiguous tensors; None skipped; zeros when none) with
    vst_sum4, four addends per pass, left to right."""
    parts = [p.contiguous() for p in parts if p is not None]
    n = out.numel()
    if not parts:
        lib.vst_fill(ptr(out), n, 0.0, stream())
        return out
    src = parts[:4]
    lib.vst_sum4(*[ptr(p) for p in src + [None] * (4 - len(src))], ptr(out), n, stream())
    for i in range(4, len(parts), 3):
        src = parts[i:i + 3]
        lib.vst_sum4(ptr(out), *[ptr(p) for p in src + [None] * (3 - len(src))], ptr(out), n, stream())
    return out


class ForkFn(Function):
    """A tensor read by several ops (the gradient sums of RC/network.py:136-150's residual skip, the
    ReCoNet feature map read by deconv1 and the feature temporal loss, the stylised frame read by the
    VGG pass, the output temporal loss and TV, train_candy.py:91-145; the AdaAttN loss features read
    by two or three loss terms, AA/train_video.py:103-118): `n` aliases of x plus, with B > 0,
    `h1` aliases of its batch half x[:B] and `h2` of x[B:] -- each a separate autograd output, so
    backward receives every consumer's gradient on its own and sums them in one vst_sum4 pass per
    batch half.  Autograd would add them two at a time with ATen kernels, and each slice's backward
    would zero-fill and copy a full-size tensor."""

    @staticmethod
    def forward(ctx, x, n, B, h1, h2):
        ctx.n, ctx.B, ctx.h, ctx.shape = n, B, (h1, h2), x.shape
        outs = [x.view_as(x) for _ in range(n)]
        if B:
            outs += [x[:B].view_as(x[:B]) for _ in range(h1)] + [x[B:].view_as(x[B:]) for _ in range(h2)]
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gs):
        n, B, (h1, h2) = ctx.n, ctx.B, ctx.h
        full = gs[:n]
        like = next(g for g in gs if g is not None)
        gx = _empty(ctx.shape, like)
        if not B:
            sum_into(gx, full)
        else:
            parts = (gs[n:n + h1], gs[n + h1:n + h1 + h2])
            for h, sl in enumerate((slice(0, B), slice(B, ctx.shape[0]))):
                sum_into(gx[sl], [None if g is None else g[sl] for g in full] + list(parts[h]))
        return gx, None, None, None, None


FORK = os.environ.get("VST_FORK", "1") != "0"  # A/B: autograd's own gradient sums and scalar adds


def fork(x, n, B=0, halves=(1, 1)):
    """(x as `n` separate autograd outputs [, halves[0] x x[:B], halves[1] x x[B:]]) -- see ForkFn;
    plain views when no gradient is recorded (and for host tensors: the CPU data-parallel tests run
    the module structure over oracle layers, and autograd sums there)."""
    h1, h2 = halves if B else (0, 0)
    if not (FORK and torch.is_grad_enabled() and x.requires_grad and x.is_cuda):
        return tuple([x] * n + [x[:B]] * h1 + [x[B:]] * h2)
    return ForkFn.apply(x, n, B, h1, h2)


class SumScalarsFn(Function):
    """Sum of 0-d loss terms (train_candy.py:148, the style term's layer sum :132-138, AA/train_video.py
    :118) in vst_sum4 passes instead of one ATen add per term; backward hands the incoming gradient to
    every term."""

    @staticmethod
    def forward(ctx, *ts):
        ctx.k = len(ts)
        out = _empty((), ts[0])
        return sum_into(out, list(ts))

    @staticmethod
    def backward(ctx, g):
        return (g,) * ctx.k


def sum_scalars(*ts):
    ts = [t for t in ts if t is not None]
    if not FORK:
        return sum(ts[1:], ts[0])
    return ts[0] if len(ts) == 1 else SumScalarsFn.apply(*ts)


_SEED = {}


def backward_seed(like):
    """A cached 0-d 1.0 on like's device: the seed of loss.backward() without the fill kernel
    torch.ones_like would launch every step (persistent: created once, read by autograd only)."""
    t = _SEED.get(like.device)
    if t is None:
        t = _SEED[like.device] = persistent_full(like, (1, 1.0))[0]
    return constant(t).view(())


class MaskedTemporalFn(Function):
    """mode 0: FTL (train_candy.py:97-106); mode 1: OTL (train_candy.py:109-123).  The reference's
    nnz = torch.nonzero(mask).shape[0] is counted on device (no host sync)."""

    @staticmethod
    def forward(ctx, mode, a, b, c, d, mask, weight):
        a, b = _check(a, "a", 4), _check(b, "b", 4)
        mask = _check(mask, "mask")
        N, C, H, W = a.shape
        c = c.contiguous() if c is not None else None
        d = d.contiguous() if d is not None else None
        ws = _empty((LOSS_WS,), a)
        st = _empty((3,), a)
        lib.vst_masked_sqdiff_fwd(mode, ptr(a), ptr(b), ptr(c), ptr(d), ptr(mask), N, C, H * W, float(weight), ptr(ws),
                                  ptr(st), stream())
        ctx.mode = mode
        ctx.save_for_backward(a, b, c, d, mask, st)
        return st[0]

    @staticmethod
    def backward(ctx, g):
        a, b, c, d, mask, st = ctx.saved_tensors
        N, C, H, W = a.shape
        ga = _empty(a.shape, a) if ctx.needs_input_grad[1] else None
        gb = _empty(b.shape, b) if ctx.needs_input_grad[2] else None
        if ga is not None or gb is not None:
            lib.vst_masked_sqdiff_bwd(ctx.mode, ptr(a), ptr(b), ptr(c), ptr(d), ptr(mask), N, C, H * W,
                                      ptr(g.contiguous()), ptr(st), ptr(ga), ptr(gb), stream())
        return None, ga, gb, None, None, None, None


def feature_temporal_loss(f2, warped_f1, feature_mask, weight):
    return MaskedTemporalFn.apply(0, f2, warped_f1, None, None, feature_mask, weight)


def output_temporal_loss(s2, warped_s1, i2, warped_i1, mask, weight):
    return MaskedTemporalFn.apply(1, s2, warped_s1, i2, warped_i1, mask, weight)


class TVFn(Function):
    """weight * sum(dx^2 + dy^2) over [:, :, :-1, :-1] (train_candy.py:141-145)."""

    @staticmethod
    def forward(ctx, s, weight):
        s = _check(s, "tv input", 4)
        N, C, H, W = s.shape
        ws = _empty((LOSS_WS,), s)
        st = _empty((3,), s)
        lib.vst_tv_fwd(ptr(s), N * C, H, W, float(weight), ptr(ws), ptr(st), stream())
        ctx.save_for_backward(s, st)
        return st[0]

    @staticmethod
    def backward(ctx, g):
        s, st = ctx.saved_tensors
        N, C, H, W = s.shape
        gs = _empty(s.shape, s)
        lib.vst_tv_bwd(ptr(s), N * C, H, W, ptr(g.contiguous()), ptr(st), ptr(gs), stream())
        return gs, None


def tv_loss(s, weight):
    return TVFn.apply(s, weight)


# ------------------------------------------------------------------ resize / concat
def resize_bilinear(x, size, chscale=None, binarize=False, out=None, addend=None, scale=None):
    """F.interpolate(x, size, mode='bilinear', align_corners=False) [* chscale[c]] [> 0] [+ addend].
    `out` may be a per-sample-contiguous slice of a larger buffer (channel concat).  `scale` = (sy, sx):
    explicit coordinate scales (input pixels per output pixel; F.interpolate(scale_factor=s) uses 1/s)."""
    x = _check(x, "resize input", 4)
    N, C, H, W = x.shape
    Ho, Wo = size
    if out is None:
        out = _empty((N, C, Ho, Wo), x)
    if tuple(out.shape) != (N, C, Ho, Wo):
        raise VstError(f"resize: out shape {tuple(out.shape)} != {(N, C, Ho, Wo)}")
    optr, obs = ptr_rows(out)
    if addend is not None:
        addend = _check(addend, "resize addend", 4)
        if tuple(addend.shape) != (N, C, Ho, Wo) or obs != C * Ho * Wo:
            raise VstError("resize: addend must match a dense output")
    if scale is None:
        lib.vst_resize_bilinear(ptr(x), optr, N * C, C, H, W, Ho, Wo, ptr(chscale), int(binarize),
                                obs if obs != C * Ho * Wo else 0, ptr(addend), stream())
    else:
        lib.vst_resize_bilinear_scaled(ptr(x), optr, N * C, C, H, W, Ho, Wo, float(scale[0]), float(scale[1]),
                                       ptr(chscale), int(binarize), obs if obs != C * Ho * Wo else 0, ptr(addend),
                                       stream())
    return out


class ResizeFn(Function):
    """F.interpolate(x, size, mode='bilinear', align_corners=False) with its adjoint (gather form)."""

    @staticmethod
    def forward(ctx, x, size, scale=None):
        ctx.x_shape = x.shape
        ctx.scale = scale
        return resize_bilinear(x.contiguous(), size, scale=scale)

    @staticmethod
    def backward(ctx, g):
        return resize_bilinear_bwd(g.contiguous(), ctx.x_shape, ctx.scale), None, None


def resize(x, size, scale=None):
    """Differentiable bilinear resize (align_corners=False) to `size` = (Ho, Wo); `scale` = (sy, sx)
    coordinate scales when they are not H / Ho, W / Wo (see resize_bilinear)."""
    return ResizeFn.apply(x, tuple(int(v) for v in size), scale)


def interpolate_scale(x, s):
    """F.interpolate(x, scale_factor=s, mode='bilinear', align_corners=False) for any s > 0
    (AA/network.py:57-59): output floor(H s) x floor(W s), source coordinate (d + 0.5) / s - 0.5 with
    1 / s rounded to fp32 as ATen's area_pixel_compute_scale does."""
    N, C, H, W = x.shape
    s = float(s)
    Ho, Wo = int(np.floor(H * s)), int(np.floor(W * s))
    if Ho < 1 or Wo < 1:
        raise VstError(f"interpolate: scale_factor {s} on a {H}x{W} map gives an empty output")
    inv = float(np.float32(1.0 / s))
    return resize(x, (Ho, Wo), scale=(inv, inv))


def resize_bilinear_bwd(gout, x_shape, scale=None):
    """Adjoint of resize_bilinear w.r.t. x; gout may be a per-sample-contiguous slice."""
    N, C, H, W = x_shape
    Ho, Wo = gout.shape[2:]
    gptr, gbs = ptr_rows(gout)
    gx = _empty(x_shape, gout)
    if scale is None:
        lib.vst_resize_bilinear_bwd(gptr, ptr(gx), N * C, C, H, W, Ho, Wo, gbs if gbs != C * Ho * Wo else 0, stream())
    else:
        lib.vst_resize_bilinear_scaled_bwd(gptr, ptr(gx), N * C, C, H, W, Ho, Wo, float(scale[0]), float(scale[1]),
                                           gbs if gbs != C * Ho * Wo else 0, stream())
    return gx


def upsample2x_bwd(gout, x, relu_mask=False):
    """Adjoint of the x2 upsample w.r.t. its input x (fixed-stencil kernel), times (x > 0) when x is
    a ReLU output whose backward is fused here (relu_mask)."""
    N, C, H, W = x.shape
    gptr, gbs = ptr_rows(gout)
    if relu_mask and (W % 2 or (gptr | x.data_ptr()) % 16):  # the stencil kernel's float4 / float2 access
        return relu_bwd(upsample2x_bwd(gout, x), x)
    gx = _empty(x.shape, gout)
    lib.vst_upsample2x_bwd(gptr, ptr(x) if relu_mask else None, ptr(gx), N * C, C, H, W,
                           gbs if gbs != C * 4 * H * W else 0, stream())
    return gx


def relu_bwd(gy, y):
    """gy * (y > 0) (ATen threshold_backward on a ReLU result)."""
    gz = _empty(gy.shape, gy)
    lib.vst_relu_bwd(ptr(gy), ptr(y), ptr(gz), gy.numel(), stream())
    return gz


def copy_into(src, dst):
    """dst[n] = src[n] for per-sample-contiguous src/dst (slices of concat buffers)."""
    if tuple(src.shape) != tuple(dst.shape):
        raise VstError(f"copy: shape {tuple(src.shape)} != {tuple(dst.shape)}")
    sp, sbs = ptr_rows(src)
    dp, dbs = ptr_rows(dst)
    lib.vst_copy_planes(sp, sbs, dp, dbs, src.shape[0], src[0].numel(), stream())
    return dst


class Upsample2xFn(Function):
    """F.interpolate(x, scale_factor=2, mode='bilinear', align_corners=False) [+ addend]
    (AA/network.py:59, 80; the decoder's `self.upsample(x5) + x4`).  relu_mask: x is the output of
    a ConvReLU whose ReLU backward this op applies (the producer then runs with premasked=True)."""

    @staticmethod
    def forward(ctx, x, addend, relu_mask):
        x = _check(x, "upsample input", 4)
        N, C, H, W = x.shape
        ctx.has_add = addend is not None
        ctx.relu_mask = bool(relu_mask)
        ctx.save_for_backward(x)
        return resize_bilinear(x, (2 * H, 2 * W), addend=addend)

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        x, = ctx.saved_tensors
        gx = upsample2x_bwd(g, x, ctx.relu_mask) if ctx.needs_input_grad[0] else None
        return gx, (g if ctx.has_add and ctx.needs_input_grad[1] else None), None


def upsample2x(x, addend=None, relu_mask=False):
    return Upsample2xFn.apply(x, addend, relu_mask)


class UpsampleCatFn(Function):
    """torch.cat([upsample2x(x), y], dim=1) written straight into one buffer (AA/network.py:85-87)."""

    @staticmethod
    def forward(ctx, x, y, relu_mask):
        x = _check(x, "upsample-cat x", 4)
        y = _check(y, "upsample-cat y", 4)
        N, C1, H, W = x.shape
        C2 = y.shape[1]
        if tuple(y.shape) != (N, C2, 2 * H, 2 * W):
            raise VstError("upsample-cat: skip tensor shape mismatch")
        out = _empty((N, C1 + C2, 2 * H, 2 * W), x)
        resize_bilinear(x, (2 * H, 2 * W), out=out[:, :C1])
        copy_into(y, out[:, C1:])
        ctx.C1 = C1
        ctx.relu_mask = bool(relu_mask)
        ctx.save_for_backward(x)
        return out

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        x, = ctx.saved_tensors
        C1 = ctx.C1
        gx = upsample2x_bwd(g[:, :C1], x, ctx.relu_mask) if ctx.needs_input_grad[0] else None
        gy = None
        if ctx.needs_input_grad[1]:
            gs = g[:, C1:]
            gy = copy_into(gs, _empty(gs.shape, g))
        return gx, gy, None


def upsample_cat(x, y, relu_mask=False):
    """cat([upsample2x(x), y]); relu_mask as in upsample2x."""
    return UpsampleCatFn.apply(x, y, relu_mask)


def flow_warp_mask(flo01, flo10, threshold=2.0):
    """(B,2,H,W) x2 -> (B,H,W) 0/1, or (2,H,W) -> (H,W) like RC/utilities.py:60-90."""
    single = flo01.dim() == 3
    f01 = _check(flo01.unsqueeze(0) if single else flo01, "flo01", 4)
    f10 = _check(flo10.unsqueeze(0) if single else flo10, "flo10", 4)
    B, _, H, W = f01.shape
    mask = _empty((B, H, W), f01)
    lib.vst_flow_warp_mask(ptr(f01), ptr(f10), ptr(mask), B, H, W, float(threshold), stream())
    return mask[0] if single else mask


# ---------------------------------------------------------------- video frames (inference path)
def _ptr_u8(t, name):
    if not t.is_cuda or t.dtype != torch.uint8 or not t.is_contiguous():
        raise VstError(f"{name}: need a contiguous uint8 HIP (cuda) tensor; there is no CPU path")
    return t.data_ptr()


def frames_to_tensor(frames, bgr=True, out=None):
    """RC/utilities.py:108-123 (tensor half of cvframe_to_tensor) on N frames at once:
    (N,H,W,3) uint8 cv2 frames -> (N,3,H,W) fp32 RGB in [0,255] (ToTensor then mul(255))."""
    if frames.dim() != 4 or frames.shape[-1] != 3:
        raise VstError(f"frames must be (N,H,W,3) uint8, got {tuple(frames.shape)}")
    N, H, W, _ = frames.shape
    out = torch.empty((N, 3, H, W), dtype=torch.float32, device=frames.device) if out is None else out
    lib.vst_frames_to_tensor(_ptr_u8(frames, "frames"), ptr(out), N, H, W, int(bgr), stream())
    return out


def tensor_to_frames(y, bgr=True, clamped=None, frames=None):
    """RC/utilities.py:213-219 on N frames at once: (N,3,H,W) fp32 -> clamp(0,255) -> (N,H,W,3)
    uint8 (cv2 BGR order, truncating astype).  `clamped` optionally receives the clamped fp32."""
    y = _check(y, "y", 4)
    N, C, H, W = y.shape
    if C != 3:
        raise VstError(f"stylised frames must have 3 channels, got {C}")
    if frames is None:
        frames = torch.empty((N, H, W, 3), dtype=torch.uint8, device=y.device)
    lib.vst_tensor_to_frames(ptr(y), ptr(clamped), _ptr_u8(frames, "frames"), N, H, W, int(bgr), stream())
    return frames


FRAME_MSE_WS_BYTES = 16384  # VST_FRAME_MSE_WS_BYTES (include/vst_hip.h)


def frame_diff_mse(x0, x1, y0, y1, out):
    """RC/utilities.py:151-161: out[0] = MSELoss(mean)(x1 - x0, y1 - y0), on the device."""
    for t, n in ((x0, "x0"), (x1, "x1"), (y0, "y0"), (y1, "y1")):
        _check(t, n)
        if t.shape != x0.shape:
            raise VstError(f"{n}: shape {tuple(t.shape)} != {tuple(x0.shape)}")
    # per-call workspace from the caching allocator (stream-ordered reuse; no scratch shared by streams)
    ws = torch.empty(FRAME_MSE_WS_BYTES // 4, dtype=torch.float32, device=x0.device)
    lib.vst_frame_diff_mse(ptr(x0), ptr(x1), ptr(y0), ptr(y1), x0.numel(), ptr(ws), ptr(out), stream())
    return out


# ---------------------------------------------------------------- RTNSTV (RT/network.py, RT/train.py)
class ConvTranspose2dFn(Function):
    """nn.ConvTranspose2d(Cin, Cout, k, stride, padding, output_padding) (RT/network.py:50-52) as the
    data gradient of the zero-padded strided conv it transposes: forward = transposed implicit GEMM
    (the conv dgrad kernel), input grad = that conv's forward GEMM, weight grad = its wgrad GEMM
    with the roles of input and output-gradient swapped.  bias_const as in Conv2dFn (the following
    InstanceNorm's backward produces the bias gradient)."""

    @staticmethod
    def forward(ctx, x, w, b, stride, pad, out_pad, bias_const=None):
        x = _check(x, "conv_transpose input", 4)
        w = w.contiguous()
        N, Cin, H, W = x.shape
        if w.shape[0] != Cin or w.shape[2] != w.shape[3]:
            raise VstError(f"conv_transpose: weight {tuple(w.shape)} does not match input channels {Cin}")
        Cout, ks = w.shape[1], w.shape[2]
        Ho = (H - 1) * stride - 2 * pad + ks + out_pad
        Wo = (W - 1) * stride - 2 * pad + ks + out_pad
        if conv_out_hw(Ho, Wo, ks, stride, pad, 1) != (H, W):
            raise VstError("conv_transpose: output size is not the transposed conv's input size")
        if bias_const is not None:
            b = bias_const
        gemm_role("fwd")
        flops = 2.0 * N * Cin * H * W * Cout * ks * ks
        out = conv_gemm(x, packed_weight(w, transposed=True), Cout, ks, Ho, Wo, GM_TRANSPOSED, stride, pad, 1,
                        epi=EPI_BIAS if b is not None else 0, bias=b.contiguous() if b is not None else None,
                        algo_flops=flops)
        ctx.geom = (ks, stride, pad)
        ctx.has_bias = b is not None and bias_const is None
        ctx.params = (w, b)
        ctx.save_for_backward(x, w)
        return out

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        ks, stride, pad = ctx.geom
        gy = gy.contiguous()
        N, Cin, H, W = x.shape
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            gemm_role("dgrad")
            dx = conv_gemm(gy, packed_weight(w, False), Cin, ks, H, W, GM_ZERO, stride, pad, 1)
        if ctx.needs_input_grad[1]:
            sink = grad_sink(ctx.params[0])
            dw = wgrad_into_sink(lambda: conv_wgrad(x, gy, w.shape, ks, stride, pad, "zero", 1, out=sink), sink, x, gy)
            dw = None if sink is not None else dw
        if ctx.has_bias and ctx.needs_input_grad[2]:
            sink = grad_sink(ctx.params[1])
            db = channel_sum(gy, out=sink)
            db = None if sink is not None else db
        return dx, dw, db, None, None, None, None


def conv_transpose2d(x, w, b=None, stride=2, pad=1, out_pad=1):
    return ConvTranspose2dFn.apply(x, w, b, stride, pad, out_pad)


def conv_transpose_instance_norm(x, w, b, gamma, beta, stride=2, pad=1, out_pad=1, relu=False, eps=1e-5):
    """ConvTranspose2d [+bias] -> InstanceNorm(affine) [-> ReLU] (RT/network.py:55-60)."""
    if b is None:
        return instance_norm(conv_transpose2d(x, w, None, stride, pad, out_pad), gamma, beta, relu, None, eps)
    y = ConvTranspose2dFn.apply(x, w, None, stride, pad, out_pad, b.detach())
    return InstanceNormFn.apply(y, gamma, beta, None, relu, eps, b)


class TanhImageFn(Function):
    """(tanh(v) + 1) / 2 * 255 (RT/network.py:93 after conv4's Tanh), or plain tanh (image=False)."""

    @staticmethod
    def forward(ctx, v, image=True):
        v = _check(v, "tanh_image input")
        y, t = _empty(v.shape, v), _empty(v.shape, v)
        lib.vst_tanh_image_fwd(ptr(v), ptr(y), ptr(t), v.numel(), int(image), stream())
        ctx.image = bool(image)
        ctx.save_for_backward(t)
        return y

    @staticmethod
    def backward(ctx, gy):
        (t,) = ctx.saved_tensors
        gv = _empty(t.shape, t)
        lib.vst_tanh_image_bwd(ptr(gy.contiguous()), ptr(t), ptr(gv), t.numel(), int(ctx.image), stream())
        return gv, None


def tanh_image(v, image=True):
    return TanhImageFn.apply(v, image)


class TVSqrtFn(Function):
    """weight * mean(sqrt(clamp(dx^2 + dy^2, 1e-8))) over [:, :, :-1, :-1] (RT/train.py:57-61)."""

    @staticmethod
    def forward(ctx, s, weight):
        s = _check(s, "tv input", 4)
        N, C, H, W = s.shape
        ws = _empty((LOSS_WS,), s)
        st = _empty((3,), s)
        lib.vst_tv_sqrt_fwd(ptr(s), N * C, H, W, float(weight), ptr(ws), ptr(st), stream())
        ctx.save_for_backward(s, st)
        return st[0]

    @staticmethod
    def backward(ctx, g):
        s, st = ctx.saved_tensors
        N, C, H, W = s.shape
        gs = _empty(s.shape, s)
        lib.vst_tv_sqrt_bwd(ptr(s), N * C, H, W, ptr(g.contiguous()), ptr(st), ptr(gs), stream())
        return gs, None


def tv_sqrt_loss(s, weight):
    return TVSqrtFn.apply(s, weight)


# ---------------------------------------------------- flow-dataset frame-pair preparation
def _ptr_typed(t, dtype, name):
    if not t.is_cuda or t.dtype != dtype or not t.is_contiguous():
        raise VstError(f"{name}: need a contiguous {dtype} HIP (cuda) tensor; there is no CPU path")
    return t.data_ptr()


def pil_bilinear_coeffs(in_size, out_size):
    """Host-side Pillow BILINEAR tables for one axis (vst_pil_bilinear_coeffs):
    (bounds (out, 2) int32, kk (out, ksize) int32)."""
    import numpy as np

    ksize = 3
    while True:
        bounds = np.zeros((out_size, 2), np.int32)
        kk = np.zeros((out_size, ksize), np.int32)
        need = lib.load().vst_pil_bilinear_coeffs(
            in_size, out_size, bounds.ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
            kk.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), ksize)
        if need == 0:
            return bounds, kk
        if need < 0:
            raise VstError(f"vst_pil_bilinear_coeffs({in_size}, {out_size}) failed (rc={need})")
        ksize = need


_PIL_TABLES = {}


def _pil_tables(in_size, out_size, device):
    key = (in_size, out_size, str(device))
    t = _PIL_TABLES.get(key)
    if t is None:
        b, k = pil_bilinear_coeffs(in_size, out_size)
        bd = torch.from_numpy(b).to(device)
        t = (bd, persistent(torch.from_numpy(k).to(device)), k.shape[1])
        _PIL_TABLES[key] = t
    constant(t[1])  # (the loader's background thread stages on its own stream)
    return t


def _pil_resize(src, size, out, mode):
    N, Hs, Ws, C = src.shape
    Wo, Ho = size
    hb, hk, hks = _pil_tables(Ws, Wo, src.device)
    vb, vk, vks = _pil_tables(Hs, Ho, src.device)
    ip = lambda t: _ptr_typed(t, torch.int32, "pil table")  # noqa: E731
    lib.vst_pil_resize_u8(_ptr_u8(src, "images"), ptr(out), N, Hs, Ws, C, Ho, Wo, ip(hb), ip(hk), hks, ip(vb),
                          ip(vk), vks, mode, stream())
    return out


def pil_resize_to_tensor255(images, size, out=None):
    """`toTensor255(Image.fromarray(img).resize(size, Image.BILINEAR))` (RC/datasets.py:116-118) for
    N images at once: (N, Hs, Ws, C) uint8 -> (N, C, H, W) fp32, size = (W, H) as PIL takes it.
    Bit-exact with Pillow's 8-bit resampler."""
    if images.dim() != 4:
        raise VstError(f"images must be (N,H,W,C) uint8, got {tuple(images.shape)}")
    N, _, _, C = images.shape
    Wo, Ho = size
    out = torch.empty((N, C, Ho, Wo), dtype=torch.float32, device=images.device) if out is None else out
    if tuple(out.shape) != (N, C, Ho, Wo):
        raise VstError(f"pil resize: out shape {tuple(out.shape)} != {(N, C, Ho, Wo)}")
    return _pil_resize(images, size, out, 0)


def apply_motion_mask(mask, motion):
    """mask *= 1 - (toTensor(motion.resize(size, BILINEAR)) != 0) (RC/datasets.py:138-144), in place:
    mask (N, H, W) fp32 0/1, motion (N, Hs, Ws) uint8 boundary images."""
    if motion.dim() != 3 or mask.dim() != 3 or motion.shape[0] != mask.shape[0]:
        raise VstError("motion mask: need mask (N,H,W) fp32 and motion (N,Hs,Ws) uint8")
    N, Ho, Wo = mask.shape
    _pil_resize(motion.unsqueeze(-1), (Wo, Ho), mask, 1)
    return mask


def flow_prep(raw, big_endian, size, out=None):
    """RC/datasets.py:121-136 for N flows: raw = (N, Hs, Ws, Cr) int32 tensor holding the PFM
    payload bits in file order (bottom-up rows, `big_endian` byte order) -> (N, 2, H, W) fp32 =
    flipud, [:-1], bilinear resize to size = (W, H), then the reference's per-channel rescale
    (x by H/Hs, y by W/Ws -- the factors RC/datasets.py:133-136 apply)."""
    if raw.dim() != 4 or raw.shape[-1] < 2:
        raise VstError(f"raw flows must be (N,H,W,C>=2), got {tuple(raw.shape)}")
    N, Hs, Ws, Cr = raw.shape
    Wo, Ho = size
    out = torch.empty((N, 2, Ho, Wo), dtype=torch.float32, device=raw.device) if out is None else out
    # the reference multiplies a float32 tensor by a Python float: the factor rounds to fp32
    sx, sy = Ho / Hs, Wo / Ws
    lib.vst_flow_prep(_ptr_typed(raw, torch.int32, "raw flows"), ptr(out), N, Hs, Ws, Cr, int(bool(big_endian)), Ho,
                      Wo, sx, sy, stream())
    return out
