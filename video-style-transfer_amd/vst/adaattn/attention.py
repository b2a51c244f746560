"""AdaAttN attention on HIP kernels (AA/network.py:102-220).

Layout per image n (all fp32, HBM-resident, contiguous):
  Q [d][Nc], K [d][Ns], V [dv][Ns]  (channel-major feature planes, Nc = h*w, Ns = hs*ws)
  S [Nc][Ns] raw Q^T K, A [Nc][Ns] attention rows, VV2 [2dv][Ns] = [V; V^2], MV [2dv][Nc] = [M; E2]
The reference forms Q^T, V^T by permute and runs torch.bmm; here every product reads the
channel-major planes directly:
  S   = Q^T K        conv_gemm 1x1 "conv", per-image packed A = pack(Q)      (MFMA)
  MV  = VV2 A^T      gemm_abt (split-K MFMA)
backward:
  dA   = dMV^T VV2   conv_gemm, A = pack(dMV)
  dVV2 = dMV A       conv_gemm, A = pack(dMV^T)
  dQ   = K dS^T      gemm_abt,  then + dqn/qn * Q   (cosine norms)
  dK   = Q dS        conv_gemm, A = pack(Q^T),    then + dkn/kn * K

Cosine activation (the train_video path): S is never stored.  rowsum_i = (Q_i . kbar)/qn_i + Ns
with kbar = sum_j K_j/kn_j, so A = S c_i ks_j + e_i (c = 1/(rowsum qn), e = 1/rowsum, ks = 1/kn)
is the S GEMM's epilogue; in the backward r_i = sum_j dA_ij A_ij = sum_v dMV_vi MV_vi, so
dS = (dA - r_i) c_i ks_j is the dA GEMM's epilogue, and the norm gradients have closed forms:
dqn_i = -(e_i/qn_i)(r_i Ns - sum_v dMV_vi vsum_v),  dkn_j = -ks_j^2 sum_c K_cj (Y_cj - qt_c) with
Y = Z^T [V;V^2], Z = (c . dMV) Q^T, qt = Q (c r).  Every N^2 pass is a GEMM; the rest is O(d N).
"""
import torch
from torch.autograd import Function

from .. import ops
from .._lib import VstError, lib, ptr, stream

COSINE, SOFTMAX = "cosine", "softmax"


def _empty(shape, like):
    return torch.empty(shape, device=like.device, dtype=torch.float32)


def packed_matrix(x, M, K, transpose, role="attn"):
    """Per-image packed GEMM A operand from x[n] = X[K][M] (transpose=False) or X[M][K]."""
    ops.gemm_role(role)
    N = x.shape[0]
    Mpad, Kpad = ops.pack_dims(M, K)
    per = ops.pack_floats(Mpad, Kpad)
    ap = _empty((N * per,), x)
    lib.vst_pack_matrix(ptr(x), ptr(ap), N, M, K, int(transpose), Mpad, Kpad, M * K, ops.gemm_mode(), stream())
    return ap, per


def bmm_at_b(x, M, K, transpose, b, P, out=None, role="attn", accumulate=False):
    """out[n] = Aop[n]^T-as-packed @ b[n]:  out[n][m][p] = sum_k Aop[n][k][m] b[n][k][p], where
    Aop[n][k][m] = x[n][k][m] (transpose=False) or x[n][m][k] (transpose=True); accumulate: out +=."""
    N = b.shape[0]
    ap, abs_ = packed_matrix(x, M, K, transpose, role)
    o = ops.conv_gemm(b.view(N, K, 1, P), ap, M, 1, 1, P, ops.GM_ZERO, 1, 0, 1, a_batch_stride=abs_,
                      out=None if out is None else out.view(N, M, 1, P), epi=ops.EPI_ACCUM if accumulate else 0)
    return o.view(N, M, P)


def copy_cols(src, c0, C, dst=None, d0=0):
    """Column block [.., c0:c0+C] of src [N][R][P] into dst [N][R][Pd] at column d0 (a new dense
    [N][R][C] when dst is None): N*R rows of C floats through the plane-copy kernel."""
    N, R, P = src.shape
    if dst is None:
        dst = _empty((N, R, C), src)
    Pd = dst.shape[2]
    if not (src.is_contiguous() and dst.is_contiguous() and dst.shape[:2] == (N, R) and c0 + C <= P and d0 + C <= Pd):
        raise VstError("copy_cols: shapes")
    lib.vst_copy_planes(ptr(src) + 4 * c0, P, ptr(dst) + 4 * d0, Pd, N * R, C, stream())
    return dst


def gemm_abt(a, b, scale=1.0, role="attn"):
    """out[n][m][j] = scale * sum_r a[n][m][r] b[n][j][r]."""
    ops.gemm_role(role)
    N, M, R = a.shape
    J = b.shape[1]
    if b.shape[0] != N or b.shape[2] != R:
        raise VstError(f"gemm_abt: {tuple(a.shape)} x {tuple(b.shape)}^T")
    out = _empty((N, M, J), a)
    ws = _empty((lib.vst_wgrad_workspace(N, M, J, R),), a)
    from .. import kprof

    tok = kprof.begin(2.0 * N * M * J * R, 4.0 * (a.numel() + b.numel() + out.numel()), ("abt", N, M, J, R), ops.gemm_mode())
    lib.vst_gemm_abt(ptr(a), ptr(b), ptr(out), ptr(ws), N, M, J, R, float(scale), ops.gemm_mode(), stream())
    kprof.end(tok, family="gemm_abt")
    return out


def _vec(shape, like):
    return torch.empty(shape, device=like.device, dtype=torch.float32)


_ONES = {}


def _ones(n, like):
    """A cached all-ones vector (the unit row / column scale of attn_gemm's affine epilogue)."""
    key = (like.device, n)
    v = _ONES.get(key)
    if v is None:
        v = _ONES[key] = ops.persistent_full(like, (n, 1.0))[0]
    return ops.constant(v)


def attn_gemm(x, M, K, b, P, rb, cg, ra=None, rd=None, role="attn", transpose=False):
    """out[n][m][p] = (sum_k Aop[n][k][m] b[n][k][p] + ra[n][m]) * rb[n][m] * cg[n][p] + rd[n][m] with
    Aop as in bmm_at_b (x[n] = X[K][M], or X[M][K] when transpose); rb / cg None = 1."""
    N = b.shape[0]
    rb = _ones(N * M, b) if rb is None else rb
    cg = _ones(N * P, b) if cg is None else cg
    ap, abs_ = packed_matrix(x, M, K, transpose, role)
    out = _empty((N, M, P), b)
    from .. import kprof

    tok = kprof.begin(2.0 * N * M * P * K, 4.0 * (b.numel() + ap.numel() + out.numel()), ("attn", N, M, K, P), ops.gemm_mode())
    lib.vst_attn_gemm(ptr(b), ptr(ap), ptr(out), N, K, P, M, abs_, ptr(ra), ptr(rb), ptr(rd), ptr(cg), ops.gemm_mode(), stream())
    kprof.end(tok)
    return out


def plane_dot(x, w=None):
    N, C, P = x.shape
    out = _vec((N, C), x)
    lib.vst_plane_dot(ptr(x), ptr(w), ptr(out), N, C, P, stream())
    return out


def channel_dot(x, v=None, y=None):
    N, C, P = x.shape
    out = _vec((N, P), x)
    lib.vst_channel_dot(ptr(x), ptr(v), ptr(y), ptr(out), N, C, P, stream())
    return out


def channel_norm(x):
    """||x[n][:][p]||_2 over channels -> [N][P] (LA.vector_norm, AA/network.py:121-122)."""
    N, C, P = x.shape
    out = _empty((N, P), x)
    lib.vst_channel_norm(ptr(x), ptr(out), N, C, P, stream())
    return out


def attention_rows(S, activation, qn=None, kn=None):
    N, Nc, Ns = S.shape
    A = _empty(S.shape, S)
    if activation == COSINE:
        rowsum = _empty((N, Nc), S)
        lib.vst_cos_attn_rows(ptr(S), ptr(qn), ptr(kn), ptr(A), ptr(rowsum), N, Nc, Ns, stream())
        return A, rowsum
    if activation == SOFTMAX:
        lib.vst_softmax_rows(ptr(S), ptr(A), N * Nc, Ns, stream())
        return A, None
    raise ValueError(f"Unknown activation function: {activation}")


# Softmax attention (the image trainer's activation, AA/network.py:102-108, 191-220) has no linear
# form: A = softmax_rows(Q^T K) must be formed.  It is formed in blocks of query rows (columns of
# Q): each block's S / A ([N][rows][Ns]) is computed, used and dropped, so HBM holds
# O(rows * Ns) per image instead of O(Nc * Ns) (config-5 size, relu3_1: 4 GB -> <= the block budget
# per image).  A row's softmax sees its whole key row, so every element is computed exactly as in
# the full-matrix form; the backward recomputes a block's S and A instead of storing them
# (flash-attention's trade: one extra Q^T K GEMM), and accumulates dK and dV over the blocks.
SOFTMAX_BLOCK_BYTES = 256 << 20  # S (or A, dS) bytes per block over the whole batch


def _softmax_rows_per_block(N, Nc, Ns, budget=None):
    budget = SOFTMAX_BLOCK_BYTES if budget is None else budget
    rows = max(1, budget // (4 * N * Ns))
    if rows >= Nc:
        return Nc
    return max(32, rows // 32 * 32)


class AdaAttnFn(Function):
    """out = sqrt(clamp(A V^2 - (A V)^2, 1e-6)) * cn + A V  with A = activation(Q^T K)
    (AA/network.py:191-220 after the 1x1 convs).  Gradients for Q, K, V.  Softmax: query-row blocks
    (see above); cosine with a materialised A (kept for tests; the product path uses
    LinearCosineAttnFn)."""

    @staticmethod
    def forward(ctx, Q, K, V, cn, activation, block_rows=None):
        N, d, h, w = Q.shape
        _, _, hs, ws = K.shape
        dv = V.shape[1]
        Nc, Ns = h * w, hs * ws
        if K.shape[:2] != (N, d) or V.shape != (N, dv, hs, ws) or cn.shape != (N, dv, h, w):
            raise VstError(f"adaattn: Q{tuple(Q.shape)} K{tuple(K.shape)} V{tuple(V.shape)} c{tuple(cn.shape)}")
        Q, K, V, cn = (ops._check(t, "adaattn operand", 4) for t in (Q, K, V, cn))
        Qm, Km = Q.view(N, d, Nc), K.view(N, d, Ns)
        role = "attn_" + activation
        qn = kn = S = rowsum = None
        VV2 = _empty((N, 2 * dv, Ns), V)
        lib.vst_square_concat(ptr(V), ptr(VV2), N, dv * Ns, stream())
        if activation == COSINE:
            qn, kn = channel_norm(Qm), channel_norm(Km)
            ks = _vec((N, Ns), Q)
            lib.vst_reciprocal(ptr(kn), ptr(ks), N * Ns, stream())
            qkbar = channel_dot(Qm, v=plane_dot(Km, ks))
            c, e = _vec((N, Nc), Q), _vec((N, Nc), Q)
            lib.vst_attn_fwd_rows(ptr(qkbar), ptr(qn), ptr(c), ptr(e), N * Nc, Ns, stream())
            A = attn_gemm(Qm, Nc, d, Km, Ns, rb=c, cg=ks, rd=e, role=role)  # [N][Nc][Ns], S never stored
            rowsum = (ks, c, e)
            MV = gemm_abt(VV2, A, role=role)  # [N][2dv][Nc]
            C = Nc
        elif activation == SOFTMAX:
            C = _softmax_rows_per_block(N, Nc, Ns) if block_rows is None else min(int(block_rows), Nc)
            A = None
            if C == Nc:
                S = bmm_at_b(Qm, Nc, d, False, Km, Ns, role=role)  # [N][Nc][Ns]
                A, _ = attention_rows(S, activation)
                del S
                MV = gemm_abt(VV2, A, role=role)
            else:
                MV = _empty((N, 2 * dv, Nc), V)
                for c0 in range(0, Nc, C):
                    Cb = min(C, Nc - c0)
                    Ab = _softmax_block(Qm, Km, c0, Cb, role)
                    copy_cols(gemm_abt(VV2, Ab, role=role), 0, Cb, dst=MV, d0=c0)
        else:
            raise ValueError(f"Unknown activation function: {activation}")
        out = _empty((N, dv, h, w), V)
        lib.vst_adaattn_out(ptr(MV), ptr(cn), ptr(out), N, dv * Nc, stream())
        ctx.activation = activation
        ctx.dims = (N, d, dv, Nc, Ns, C)
        if any(ctx.needs_input_grad[:3]):
            extra = rowsum if rowsum is not None else (None, None, None)
            ctx.save_for_backward(Q, K, V, cn, qn, kn, A, VV2, MV, *extra)
        return out

    @staticmethod
    def backward(ctx, dout):
        Q, K, V, cn, qn, kn, A, VV2, MV, ks, c, e = ctx.saved_tensors
        N, d, dv, Nc, Ns, C = ctx.dims
        role = "attn_" + ctx.activation
        if ctx.needs_input_grad[3]:
            raise VstError("adaattn: gradient w.r.t. the content features (norm_v(c_x)) is not on the reference path")
        dout = dout.contiguous()
        dMV = _empty(MV.shape, MV)
        lib.vst_adaattn_out_bwd(ptr(dout), ptr(MV), ptr(cn), ptr(dMV), N, dv * Nc, stream())
        Qm, Km = Q.view(N, d, Nc), K.view(N, d, Ns)
        gq, gk, gv = ctx.needs_input_grad[:3]
        if ctx.activation == SOFTMAX:
            dQm = _empty((N, d, Nc), Q) if gq else None
            dKm = _empty((N, d, Ns), K) if gk else None
            dVV2 = _empty((N, 2 * dv, Ns), V) if gv else None
            for c0 in range(0, Nc, C):
                Cb = min(C, Nc - c0)
                full = Cb == Nc
                Ab = A if full and A is not None else _softmax_block(Qm, Km, c0, Cb, role)  # recomputed
                dMVb = dMV if full else copy_cols(dMV, c0, Cb)
                Qb = Qm if full else copy_cols(Qm, c0, Cb)
                if gv:
                    bmm_at_b(dMVb, 2 * dv, Cb, True, Ab, Ns, out=dVV2, role=role, accumulate=c0 > 0)
                if gq or gk:
                    dS = bmm_at_b(dMVb, Cb, 2 * dv, False, VV2, Ns, role=role)  # dA  [N][Cb][Ns]
                    lib.vst_softmax_rows_bwd(ptr(dS), ptr(Ab), ptr(dS), N * Cb, Ns, stream())
                    if gq:
                        dQb = gemm_abt(Km, dS, role=role)  # [N][d][Cb]
                        if full:
                            dQm = dQb
                        else:
                            copy_cols(dQb, 0, Cb, dst=dQm, d0=c0)
                    if gk:
                        bmm_at_b(Qb, d, Cb, True, dS, Ns, out=dKm, role=role, accumulate=c0 > 0)  # [N][d][Ns]
            dV = None
            if gv:
                dV = _empty(V.shape, V)
                lib.vst_square_concat_bwd(ptr(dVV2), ptr(V), ptr(dV), N, dv * Ns, stream())
            return (dQm.view(Q.shape) if gq else None, dKm.view(K.shape) if gk else None, dV, None, None, None)
        dQ = dK = dV = None
        if gv:
            dVV2 = bmm_at_b(dMV, 2 * dv, Nc, True, A, Ns, role=role)  # [N][2dv][Ns]
            dV = _empty(V.shape, V)
            lib.vst_square_concat_bwd(ptr(dVV2), ptr(V), ptr(dV), N, dv * Ns, stream())
            del dVV2
        if gq or gk:
            r = channel_dot(dMV, y=MV)                 # sum_j dA_ij A_ij
            DA = channel_dot(dMV, v=plane_dot(VV2))    # sum_j dA_ij
            dqn, nr, cr = _vec((N, Nc), Q), _vec((N, Nc), Q), _vec((N, Nc), Q)
            lib.vst_attn_bwd_rows(ptr(r), ptr(DA), ptr(qn), ptr(c), ptr(e), ptr(dqn), ptr(nr), ptr(cr), N * Nc, Ns,
                                  stream())
            dS = attn_gemm(dMV, Nc, 2 * dv, VV2, Ns, rb=c, cg=ks, ra=nr, role=role)  # (dA - r) c ks
            if gq:
                dQ = gemm_abt(Km, dS, role=role)  # [N][d][Nc]
                lib.vst_norm_grad_add(ptr(dQ), ptr(dqn), ptr(qn), ptr(Qm), N, d, Nc, stream())
                dQ = dQ.view(Q.shape)
            if gk:
                dK = bmm_at_b(Qm, d, Nc, True, dS, Ns, role=role)  # [N][d][Ns]
                dMVc = _empty(dMV.shape, dMV)
                lib.vst_scale_cols(ptr(dMV), ptr(c), ptr(dMVc), N, 2 * dv, Nc, stream())
                Z = gemm_abt(dMVc, Qm, role=role)  # [N][2dv][d]
                Y = bmm_at_b(Z, d, 2 * dv, False, VV2, Ns, role=role)  # [N][d][Ns]
                dkn = _vec((N, Ns), K)
                lib.vst_attn_dkn(ptr(Km), ptr(Y), ptr(plane_dot(Qm, cr)), ptr(ks), ptr(dkn), N, d, Ns, stream())
                lib.vst_norm_grad_add(ptr(dK), ptr(dkn), ptr(kn), ptr(Km), N, d, Ns, stream())
                dK = dK.view(K.shape)
        return dQ, dK, dV, None, None, None


def _softmax_block(Qm, Km, c0, C, role):
    """A rows c0 .. c0+C-1: softmax_rows(Q[:, :, c0:c0+C]^T K)  [N][C][Ns]."""
    N, d, Nc = Qm.shape
    Ns = Km.shape[2]
    Qb = Qm if (c0 == 0 and C == Nc) else copy_cols(Qm, c0, C)
    S = bmm_at_b(Qb, C, d, False, Km, Ns, role=role)
    A, _ = attention_rows(S, SOFTMAX)
    return A


# ---------------------------------------------------------------------------------------------
# Cosine attention in linear form.  CosineSimilarity (AA/network.py:111-125) is
#   A_ij = s_ij / sum_j s_ij,  s_ij = qh_i . kh_j + 1,  qh = q / ||q||, kh = k / ||k||
# so with U = [V; V^2] (2dv x Ns) the two moments AdaAttN needs (AA/network.py:209-213) are
#   [M; E2]_i = sum_j A_ij U_j = (G^T qh_i + us) / rs_i,   G = Kh U^T (d x 2dv),  us = sum_j U_j,
#   rs_i = qh_i . ksum + Ns,  ksum = sum_j kh_j
# -- an exact re-association of the reference's bmm(A, V) / bmm(A, V**2): the Nc x Ns matrix A is
# never formed (HBM O(N d) instead of O(Nc Ns)) and the products cost 2 Ns d 2dv + 2 Nc d 2dv
# instead of 2 Nc Ns (d + 2dv) FLOPs (17x fewer at 256x512 level 3, 4x more per 2x resolution
# instead of 16x).  The backward is the same algebra transposed (all GEMMs of d x 2dv operands):
#   dRh = dMV / rs;  te = rs^-1 sum_v dMV MV (= -d rs);  dqh = G dRh - ksum te;  dG = Qh dRh^T;
#   dus = sum_i dRh;  dksum = -Qh te;  dkh = dG U + dksum;  dU = dG^T Kh + dus;
#   dV = dU[:dv] + 2 V dU[dv:];  dq = (dqh - qh (qh . dqh)) / ||q||  (likewise k).
# The style side (K, V) may carry fewer images than Q: Q image n attends to K / V image n % Nk
# (the train_video step's two content frames share one style encoding), and its gradients are
# summed over the repeats.
def _repeat(x, r):
    """x [Nk, ...] repeated r times along the batch (plane-copy kernel); x itself when r == 1."""
    if r == 1:
        return x
    out = torch.empty((r * x.shape[0],) + tuple(x.shape[1:]), device=x.device, dtype=torch.float32)
    for i in range(r):
        ops.copy_into(x, out[i * x.shape[0]:(i + 1) * x.shape[0]])
    return out


def _sum_repeats(x, r):
    if r == 1:
        return x
    per = x[: x.shape[0] // r].numel()
    out = torch.empty((x.shape[0] // r,) + tuple(x.shape[1:]), device=x.device, dtype=torch.float32)
    lib.vst_sum_repeats(ptr(x), ptr(out), r, per, stream())
    return out


def _axpy(x, u=None, v=None, w=None, alpha=1.0, out=None):
    """out[n][m][p] = (x + alpha u[n][m] v[n][p]) w[n][p] over x viewed [N][M][P]."""
    N, M = x.shape[:2]
    P = x[0, 0].numel()
    out = x if out is None else out
    lib.vst_outer_axpy(ptr(x), ptr(u), ptr(v), ptr(w), float(alpha), ptr(out), N, M, P, stream())
    return out


def _normalized(x, nrm_inv):
    return _axpy(x, w=nrm_inv, out=_empty(x.shape, x))


def _normalize_bwd(xh, dxh, nrm_inv):
    N, C, P = xh.shape
    t = channel_dot(xh, y=dxh)
    out = _empty(xh.shape, xh)
    lib.vst_normalize_cols_bwd(ptr(xh), ptr(dxh), ptr(t), ptr(nrm_inv), ptr(out), N, C, P, stream())
    return out


def _neg(x):
    """-x (a small per-row vector) with the library's affine kernel: x + (-2) x, exact."""
    out = _empty(x.shape, x)
    lib.vst_outer_axpy(ptr(x), ptr(x), None, None, -2.0, ptr(out), 1, x.numel(), 1, stream())
    return out


def _recip(x):
    y = _empty(x.shape, x)
    lib.vst_reciprocal(ptr(x), ptr(y), x.numel(), stream())
    return y


class LinearCosineAttnFn(Function):
    """out = sqrt(clamp(E2 - M^2, 1e-6)) * cn + M with [M; E2] the cosine-attention moments in
    linear form (see above); gradients for Q, K, V."""

    @staticmethod
    def forward(ctx, Q, K, V, cn):
        Nq, d, h, w = Q.shape
        Nk, _, hs, ws = K.shape
        dv = V.shape[1]
        Nc, Ns = h * w, hs * ws
        if (K.shape[1] != d or V.shape != (Nk, dv, hs, ws) or cn.shape != (Nq, dv, h, w) or Nq % Nk):
            raise VstError(f"adaattn: Q{tuple(Q.shape)} K{tuple(K.shape)} V{tuple(V.shape)} c{tuple(cn.shape)}")
        Q, K, V, cn = (ops._check(t, "adaattn operand", 4) for t in (Q, K, V, cn))
        r = Nq // Nk
        role = "attn_" + COSINE
        Qm, Km = Q.view(Nq, d, Nc), K.view(Nk, d, Ns)
        qn = channel_norm(Qm)
        qs, ks = _recip(qn), _recip(channel_norm(Km))
        Qh, Kh = _normalized(Qm, qs), _normalized(Km, ks)
        U = _empty((Nk, 2 * dv, Ns), V)
        lib.vst_square_concat(ptr(V), ptr(U), Nk, dv * Ns, stream())
        G = gemm_abt(Kh, U, role=role)                       # [Nk][d][2dv]
        ksum, us = plane_dot(Kh), plane_dot(U)              # [Nk][d], [Nk][2dv]
        Gr, ksr, usr = _repeat(G, r), _repeat(ksum, r), _repeat(us, r)
        qk = channel_dot(Qm, v=ksr)                         # q . ksum  [Nq][Nc]
        rinv = _empty(qk.shape, qk)
        lib.vst_attn_fwd_rows(ptr(qk), ptr(qn), ptr(_empty(qk.shape, qk)), ptr(rinv), qk.numel(), Ns,
                              stream())                     # 1 / rs = 1 / (q . ksum / ||q|| + Ns)
        MV = attn_gemm(Gr, 2 * dv, d, Qh, Nc, rb=None, cg=rinv, ra=usr, role=role)  # (G^T qh + us) / rs
        out = _empty((Nq, dv, h, w), V)
        lib.vst_adaattn_out(ptr(MV), ptr(cn), ptr(out), Nq, dv * Nc, stream())
        ctx.dims = (Nq, Nk, d, dv, Nc, Ns, (h, w), (hs, ws))
        if any(ctx.needs_input_grad[:3]):
            ctx.save_for_backward(V, cn, Qh, Kh, qs, ks, U, Gr, ksr, MV, rinv)
        return out

    @staticmethod
    def backward(ctx, dout):
        V, cn, Qh, Kh, qs, ks, U, Gr, ksr, MV, rinv = ctx.saved_tensors
        Nq, Nk, d, dv, Nc, Ns, hw, hws = ctx.dims
        r = Nq // Nk
        role = "attn_" + COSINE
        if ctx.needs_input_grad[3]:
            raise VstError("adaattn: gradient w.r.t. the content features (norm_v(c_x)) is not on the reference path")
        dRh = _empty(MV.shape, MV)                          # dMV / rs, in the out-backward's pass
        lib.vst_adaattn_out_bwd_scaled(ptr(dout.contiguous()), ptr(MV), ptr(cn), ptr(rinv), ptr(dRh), Nq, dv * Nc, Nc,
                                       stream())
        te = channel_dot(dRh, y=MV)                         # rs^-1 sum_v dMV MV
        dG = _sum_repeats(gemm_abt(Qh, dRh, role=role), r)  # [Nk][d][2dv]
        dQ = dK = dV = None
        if ctx.needs_input_grad[0]:
            dQh = bmm_at_b(Gr, d, 2 * dv, True, dRh, Nc, role=role)  # G dRh  [Nq][d][Nc]
            _axpy(dQh, u=ksr, v=te, alpha=-1.0)
            dQ = _normalize_bwd(Qh, dQh, qs).view(Nq, d, *hw)
        if ctx.needs_input_grad[1]:
            dks = _sum_repeats(plane_dot(Qh, te), r)       # -dksum
            dKh = attn_gemm(dG, d, 2 * dv, U, Ns, rb=None, cg=None, ra=_neg(dks), role=role, transpose=True)  # dG U + dksum
            dK = _normalize_bwd(Kh, dKh, ks).view(Nk, d, *hws)
        if ctx.needs_input_grad[2]:
            dus = _sum_repeats(plane_dot(dRh), r)          # [Nk][2dv]
            dU = attn_gemm(dG, 2 * dv, d, Kh, Ns, rb=None, cg=None, ra=dus, role=role)  # dG^T Kh + dus
            dV = _empty(V.shape, V)
            lib.vst_square_concat_bwd(ptr(dU), ptr(V), ptr(dV), Nk, dv * Ns, stream())
        return dQ, dK, dV, None


def adaattn(Q, K, V, cn, activation=COSINE, block_rows=None):
    """AdaAttN attention + modulation (AA/network.py:191-220 after the 1x1 convs).  Cosine: the
    linear form (no Nc x Ns matrix; K / V may hold a divisor of Q's batch, broadcast over repeats);
    softmax: attention formed in blocks of query rows (block_rows; default from
    SOFTMAX_BLOCK_BYTES)."""
    if activation == COSINE:
        return LinearCosineAttnFn.apply(Q, K, V, cn)
    if K.shape[0] != Q.shape[0]:
        raise VstError("adaattn (softmax): Q and K/V batches must match")
    return AdaAttnFn.apply(Q, K, V, cn, activation, block_rows)


_AFFINE_ID = {}


def instance_norm_plain(x, eps=1e-5):
    """nn.InstanceNorm2d(C, affine=False) (running stats off): the affine IN kernel with w=1, b=0."""
    C = x.shape[1]
    key = (x.device, C)
    wb = _AFFINE_ID.get(key)
    if wb is None:
        wb = _AFFINE_ID[key] = tuple(ops.persistent_full(x, (C, 1.0), (C, 0.0)))
    return ops.instance_norm(x, ops.constant(wb[0]), ops.constant(wb[1]), eps=eps)
