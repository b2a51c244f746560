/*
 * vst_hip.h — C ABI of libvst_hip.so, the MI355X (gfx950 / CDNA4) kernels of the
 * video-style-transfer training hot path (ReCoNet step: stylizer conv stack, frozen VGG feature
 * pass, Gram / temporal / TV losses, Adam).
 *
 * The reference (Maboroshi0327/Video-Style-Transfer) has no native layer: every entry below
 * replaces an implicit PyTorch/ATen kernel behind one of the reference's Python call sites,
 * cited per entry as RC/<file>:<line> (RC/ = "Real-time-Coherent-Video-Style-Transfer-Network-
 * (ReCoNet)/").  The Python module API that mirrors the reference (`network.py`,
 * `utilities.py`) calls these through ctypes (video-style-transfer_amd/vst/_lib.py).
 *
 * Conventions
 *   - Tensors: contiguous NCHW fp32 device pointers owned by the caller (PyTorch's caching
 *     allocator). The library never allocates or frees device memory; scratch comes in through
 *     `workspace`/`ws`/`partial` arguments sized by the documented formulas.
 *   - `stream`: a hipStream_t passed as void*; every call is asynchronous on it, no host sync,
 *     so whole steps can be captured into a hipGraph.
 *   - Return: 0 on success, negative VST_E* on invalid arguments, positive hipError_t on a
 *     launch failure.  No exceptions cross the ABI.
 */
#ifndef VST_HIP_H
#define VST_HIP_H

#ifdef __cplusplus
extern "C" {
#endif

/* ---- library ------------------------------------------------------------------------------ */
int vst_version(void);
const char* vst_strerror(int code);
/* Build provenance: the first 16 hex digits of the sha256 of the sorted csrc/ *.hip, *.h and Makefile
 * followed by include/vst_hip.h, taken at build time (csrc/Makefile BUILD_ID; vst/_lib.py
 * source_build_id() computes the same digest over the tree it runs from and refuses a library whose
 * id differs). */
const char* vst_build_id(void);

/* GEMM arithmetic: a per-call argument `mode` of every conv / Gram / attention GEMM entry and of
 * every entry that writes a packed A operand.  The library holds no mode state: calls with
 * different modes may run concurrently on different streams / threads.  A packed operand is only
 * valid for GEMM calls with the mode it was packed with.
 *   VST_GEMM_F32     exact fp32 MFMA (v_mfma_f32_32x32x2_f32), products exact, fp32 accumulate;
 *   VST_GEMM_BF16X3  fp32 operands split into hi + lo bf16, hi*hi + hi*lo + lo*hi on
 *                    v_mfma_f32_32x32x16_bf16 with fp32 accumulation (per-product error ~2^-16);
 *   VST_GEMM_BF16    hi*hi only (reduced precision, BASELINE config 5's half-precision MFMA path);
 *   VST_GEMM_BF16X6  three-way hi + mid + lo split, the six products of order >= 2^-16 (per-product
 *                    error ~2^-24, fp32-class); packed operands are 1.5x the fp32 size
 *                    (Kpad*Mpad*3/2 floats).
 *   VST_GEMM_F16     one fp16 product per fp32 product (v_mfma_f32_32x32x16_f16, 11-bit significand,
 *                    ~2^-11 per operand rounding, fp32 accumulate): BASELINE config 5's fp16 MFMA
 *                    path.  fp16's range ends at 65504 and its normal range at 6.1e-5, so the caller
 *                    keeps operands inside it (the trainers scale the loss, hence every backward
 *                    operand, by a dynamic power of two -- initial 2^12, halved on an Inf / NaN
 *                    gradient, doubled after 2000 clean steps -- and vst_adam_loss_scaled unscales).
 * VST_GEMM_KBLOCK may be or-ed into the mode of a conv pack + GEMM pair (both must carry it):
 * channel-block-major, tap-minor K order (16 channels x every tap, then the next 16 channels), which
 * keeps each block's re-read source rows L2-resident; the sums then run in a different order.
 * 3x3 stride-1 convs under VST_GEMM_KBLOCK (bf16x6 / bf16 / fp16) run on the halo-tiled kernel
 * (the source patch of an output tile staged once per 16-channel block for all nine taps); its
 * results are bitwise those of the per-tap kernel.  VST_GEMM_PERTAP or-ed into a GEMM call's mode
 * selects the per-tap kernel instead (an explicit per-call choice for A/B measurement and the
 * equivalence test; pack entries ignore it).
 * A bf16x6 / bf16x3 / bf16 / fp16 halo launch whose grid would not fill the chip (fewer than 512 blocks:
 * AdaAttN config 4's decoder, VGG19 conv4 / conv5) is split over the 16-channel blocks (split-K) when the
 * caller passes a workspace (fp16 launches too since round 5; tests/test_gpu_adaattn.py
 * test_f16_step_order_insensitive holds the fp16 step's tolerance under that summation-order change):
 * the slices' raw sums go to the CALLER's `workspace` (vst_conv_splitk_workspace bytes,
 * 16-byte aligned), and a reduce kernel on the same stream adds them in slice order (deterministic)
 * and applies the epilogue -- equal to the unsplit result up to fp32 summation order.  A launch given
 * a smaller (or NULL) workspace runs unsplit, so ws_bytes = 0 is always valid.
 * VST_GEMM_NOSPLIT or-ed into the mode keeps such a launch unsplit (the bitwise test against the
 * per-tap kernel).
 * An unknown mode returns VST_EINVAL (-1). */
#define VST_GEMM_F32 0
#define VST_GEMM_BF16X3 1
#define VST_GEMM_BF16 2
#define VST_GEMM_BF16X6 3
#define VST_GEMM_F16 4
#define VST_GEMM_KBLOCK 16
#define VST_GEMM_PERTAP 32
#define VST_GEMM_NOSPLIT 64

/* ---- convolution (implicit GEMM on MFMA, arithmetic per the `mode` argument) ---------------
 * Replaces: ReflectionPad2d + Conv2d (RC/network.py:68-75), nearest x2 interpolate + pad + conv
 * (RC/network.py:114-120), torchvision VGG Conv2d(3x3, pad 1) + ReLU (RC/network.py:12-24),
 * and their autograd backward (dgrad / wgrad), the conv1 bias add and ConvTanh's
 * tanh(y/255)*150+127.5 (RC/network.py:83-85) as epilogues.
 *
 * Weights are re-packed tap-major into A[k][m] (k = (kh*KW+kw)*C + c, leading dim Mpad, rows
 * padded to Kpad with zeros):  forward: m = cout, c = cin;  transposed (dgrad): m = cin, c = cout;
 * split_kh (row-split forward for tiny Cout): m = cout*KH + kh, k = kw*Cin + ci.
 */
int vst_conv_pack_dims(int M, int K, int* Mpad, int* Kpad);
int vst_pack_weight(const float* w, float* packed, int Cout, int Cin, int KH, int KW, int transposed, int split_kh,
                    int Mpad, int Kpad, int mode, void* stream);
/* out[n][m][Ho][Wo] = epi(sum_k A[k][m] * gather(src[n], k, pixel)).
 * gmode 0: reflect pad, 1: zero pad (forward gather y = oy*stride + kh - pad on the x`up` grid);
 * gmode 2: transposed gather (dgrad) ty = oy + pad - kh, valid iff ty % stride == 0.
 * epi bits: 1 bias, 2 relu, 4 reconet-tanh (aux: tanh value, may be NULL), 8 mask (out *= mask>0),
 * 16 accumulate into out.  a_batch_stride > 0: per-image A (Gram backward).
 * gmask (may be NULL, same shape as src): gathered values are zeroed where gmask <= 0 — the
 * ReLU backward of the layer that produced src, fused into the dgrad gather.
 * workspace / ws_bytes: split-K scratch (see VST_GEMM_NOSPLIT above); NULL / 0 runs unsplit. */
int vst_conv_gemm(const float* src, const float* wpack, const float* bias, const float* mask, float* out, int N,
                  int Cs, int Hs, int Ws, int M, int K, int Ho, int Wo, int KH, int KW, int gmode, int stride, int pad,
                  int up, int epi, long a_batch_stride, float* aux, const float* gmask, void* workspace, long ws_bytes,
                  int mode, void* stream);
/* Bytes of split-K workspace the conv GEMM launch with these arguments uses (0: it never splits).
 * The geometry is vst_conv_gemm_padx's (Cs = source channels, M = output rows, Ho x Wo = output
 * grid); for vst_conv_dgrad_padout pass (N, Cout, Cin, H + 2 pad, W + 2 pad, KS, KS, gmode 2, stride 1,
 * pad 0, pad_x 0, up 1, epi 128 | (mask ? 8 : 0), 0, mode).  Pure host arithmetic, no GPU call. */
long vst_conv_splitk_workspace(int N, int Cs, int M, int Ho, int Wo, int KH, int KW, int gmode, int stride, int pad,
                               int pad_x, int up, int epi, long a_batch_stride, int mode);
/* row-split forward epilogue: out[n][co][y][x] = epi(bias + sum_kh P[n][co*KH+kh][y+kh][x]) where P
 * [N][Cout*KH][H+KH-1][W] came from vst_conv_gemm(KH=1, KW=K, split_kh pack) over the padded rows
 * (RC/network.py:169 deconv3 = ConvTanh(48, 3, 9): 27 GEMM rows instead of 3 padded to 32) */
int vst_rowsplit_reduce(const float* P, const float* bias, float* out, float* aux, int N, int Cout, int KH, int H,
                        int W, int epi, void* stream);
/* stride-2 reflect-pad data gradient (RC/network.py:158-159 conv2/conv3 backward) as ONE
 * transposed GEMM over all four parity phases of the padded input grid: GEMM row m = ci*4 + 2a + b
 * computes padded pixel (2I+a, 2J+b) from the ceil(KS/2)^2 window dY[I-t][J-s] (A packed by
 * vst_pack_weight_phase2: Mpad/Kpad from vst_conv_pack_dims(4*Cin, ceil(KS/2)^2*Cout)).  The
 * epilogue writes interior pixels straight into dx [N][Cin][H][W] and the reflect-pad border into
 * border [N][Cin][H+2p][W+2p] (only its border is written/read); vst_fold_border then adds the
 * border's reflections into dx.  gmask (optional, dY-shaped) gates dY by (gmask > 0). */
int vst_pack_weight_phase2(const float* w, float* packed, int Cout, int Cin, int KS, int Mpad, int Kpad, int mode, void* stream);
int vst_conv_dgrad_s2(const float* dy, const float* wpack, const float* gmask, float* dx, float* border, int N,
                      int Cout, int Ho, int Wo, int Cin, int H, int W, int KS, int pad, int mode, void* stream);
/* mask (optional, dx-shaped): the fold adds only where mask > 0 (the producer's ReLU backward fused
 * into a masked data gradient: the GEMM epilogue already zeroed dx there) */
int vst_fold_border(const float* border, const float* mask, float* dx, long NC, int H, int W, int pad, void* stream);
/* data gradient of a 3x3 stride-1 pad-1 conv with 1..4 output channels (the AdaAttN decoder's last conv,
 * AA/network.py:99), in exact fp32 on the VALU: dx = [mask > 0] * (the interior of the transposed conv
 * of dy over the padded grid); reflect != 0 adds the padded grid's ring through `border`
 * ([N][Cin][H+2][W+2], only its ring is written) and vst_fold_border.  w: [Cout][Cin][3][3];
 * Cin even, W % 4 == 0, W >= 8; mask NULL or dx-shaped. */
int vst_conv_dgrad_thin(const float* dy, const float* w, const float* mask, float* dx, float* border, int N, int Cout,
                        int Cin, int H, int W, int reflect, void* stream);
/* Thin-channel convolutions (RC/network.py:155 conv1 = ConvLayer(3, 48, 9), :169 deconv3 =
 * ConvTanh(48, 3, 9) backward, VGG conv1_1): a tensor with C*K <= Cu channels is kw-unfolded,
 *   out[n][c*K + kw][y][v] = src[n][c][y][v + sgn*kw + off]  (reflect or zero outside; zero channels
 *   past C*K), Cu a multiple of 16,
 * so the conv becomes a Kx1 conv over Cu channels on the 16-channel k-tile path:
 *   forward:  vst_unfold_kw(x, sgn=+1, off=-pad, Wout=W) then vst_conv_gemm_padx(KH=K, KW=1,
 *             pad_x=0) with A from vst_pack_weight_kwu(transposed=0);
 *   dgrad (thin Cout, stride 1): vst_unfold_kw(dy, sgn=-1, off=0, Wout=Wu, zero) then
 *             vst_conv_dgrad_padout_kwu with A from vst_pack_weight_kwu(transposed=1), then
 *             vst_fold_border; Wu = W+2p rounded up to a multiple of 4 (the unfold's float4 rows: the
 *             AdaAttN decoder's last conv, 1024 + 2 wide at config 5). */
/* Direct 3x3 conv of a 3-channel image, stride 1, pad 1 (reflect or zero), out = [relu](conv + b) in
 * exact fp32 on the VALU (VGG conv1_1, RC/network.py:17 / AA/vgg19.py:19; b may be NULL).
 * w: [Cout][3][3][3] (PyTorch layout).  The output-write-bound layer skips the unfold + K = 48 GEMM. */
int vst_conv_cin3_k3(const float* x, const float* w, const float* b, float* out, int N, int H, int W, int Cout,
                     int reflect, int relu, void* stream);
int vst_unfold_kw(const float* src, float* out, int N, int C, int H, int Ws, int Wout, int K, int Cu, int sgn, int off,
                  int reflect, void* stream);
int vst_pack_weight_kwu(const float* w, float* packed, int Cout, int Cin, int K, int Cu, int transposed, int Mpad,
                        int Kpad, int mode, void* stream);
int vst_conv_gemm_padx(const float* src, const float* wpack, const float* bias, const float* mask, float* out, int N,
                       int Cs, int Hs, int Ws, int M, int K, int Ho, int Wo, int KH, int KW, int gmode, int stride,
                       int pad, int pad_x, int up, int epi, long a_batch_stride, float* aux, const float* gmask,
                       void* workspace, long ws_bytes, int mode, void* stream);
int vst_conv_dgrad_padout_kwu(const float* dyu, const float* wpack, const float* mask, float* dx, float* border, int N,
                              int Cu, int Ho, int Cin, int H, int W, int KS, int pad, int mode, void* stream);
/* data gradient of a zero-padded stride-1 KxK conv with few input channels (VGG conv1_1, 64 -> 3):
 * P = tap-split 1x1 transposed GEMM (vst_conv_gemm with A = vst_pack_weight of w viewed as
 * [Cout][Cin*K*K][1][1], transposed; rows (c, kh, kw)), then
 *   dx[n][c][y][x] (+)= sum_{kh,kw} P[n][(c*K+kh)*K+kw][y+pad-kh][x+pad-kw]  (zero outside). */
int vst_tapsum(const float* P, float* dx, int N, int C, int H, int W, int K, int pad, int accumulate, void* stream);
/* stride-1 reflect-pad data gradient (ResidualBlock / ConvTanh backward, RC/network.py:72-75,
 * 145-150, 83-85; the AdaAttN decoder's Conv / ConvReLU, AA/network.py:11-33): the transposed GEMM
 * (A = vst_pack_weight(transposed=1)) runs over the padded grid (H+2p) x (W+2p); interior pixels go
 * straight into dx, the p-wide border into border [N][Cin][H+2p][W+2p]; then vst_fold_border.
 * mask (optional, dx-shaped; the same pointer to vst_fold_border): dx is written only where
 * mask > 0 (the ReLU backward of a conv+ReLU producing this conv's input, fused). */
int vst_conv_dgrad_padout(const float* dy, const float* wpack, const float* mask, float* dx, float* border, int N,
                          int Cout, int Ho, int Wo, int Cin, int H, int W, int KS, int pad, void* workspace,
                          long ws_bytes, int mode, void* stream);
/* Reflect-pad dgrad without the padded grid (ConvLayer / UpsampleConvLayer backward,
 * RC/network.py:72-75,114-120): core = vst_conv_gemm on the unpadded grid (up=1: GM_TRANSPOSED,
 * pad=KS/2; up=2: GM_ZERO stride 2, pad KS-1-KS/2, KS+1 taps with the weights of
 * vst_pack_weight_upsum), ring = the KS/2-wide border of the padded-grid gradient
 * (vst_dgrad_ring over the [Cout][Cin][KS][KS] weight; ring = N*Cin*vst_dgrad_ring_size floats in
 * four segments top/bottom/left/right), folded into dx's border band by vst_fold_ring
 * (accumulates). */
int vst_pack_weight_upsum(const float* w, float* packed, int Cout, int Cin, int KS, int Mpad, int Kpad, int mode, void* stream);
int vst_dgrad_ring_splits(int Cout, int KS);
long vst_dgrad_ring_size(int Hv, int Wv, int KS, int Cout);
int vst_dgrad_ring(const float* dy, const float* w, float* ring, int N, int Cout, int Cin, int KS, int Hv, int Wv,
                   void* stream);
int vst_fold_ring(const float* ring, float* dx, long NC, int Hs, int Ws, int KS, int up, int Cout, void* stream);

/* adjoint of (nearest x`up` upsample -> ReflectionPad2d(pad)): dpad [NC][Hs*up+2p][Ws*up+2p] -> dx [NC][Hs][Ws] */
int vst_fold_reflect(const float* dpad, float* dx, long NC, int Hs, int Ws, int pad, int up, int accumulate,
                     void* stream);
/* weight gradient, split-K over output pixels with deterministic slab reduction;
 * workspace / ws_floats: at least vst_conv_wgrad_workspace(same geometry and mode) floats.  A workspace
 * smaller than that but at least vst_wgrad_workspace(N, Cout, KH*KW*Cin, Ho*Wo) (the row-tiled kernel's
 * need) runs the row-tiled kernel; a smaller one returns VST_EINVAL.  3x3 stride-1 pad-1 convs over
 * 32-channel multiples with 16-multiple widths (ResidualBlock, the AdaAttN decoder) run on the halo
 * weight gradient under the split-product modes (bf16x6 / bf16 / fp16): one block owns all nine taps
 * of 32 input channels and walks a 16-column strip down the rows, the source rows in an LDS ring (each
 * loaded and split once instead of nine times).  VST_GEMM_PERTAP in `mode` selects the row-tiled
 * kernel instead (same sums, other fp32 summation order).  Cout <= 4 (the AdaAttN decoder's last conv,
 * 64 -> 3) with 3x3 stride-1 pad-1, Cin % 4 == 0, Ws % 4 == 0: a VALU kernel in exact fp32 whatever the
 * mode (each source row loaded once, deterministic slab sums; PERTAP selects the GEMM here too). */
long vst_wgrad_workspace(int N, int M, int J, int HWo);
long vst_conv_wgrad_workspace(int N, int Cin, int Hs, int Ws, int Cout, int Ho, int Wo, int KH, int KW, int gmode,
                              int stride, int pad, int up, int mode);
int vst_conv_wgrad(const float* dy, const float* x, float* dw, float* workspace, long ws_floats, int N, int Cin,
                   int Hs, int Ws, int Cout, int Ho, int Wo, int KH, int KW, int gmode, int stride, int pad, int up,
                   int accumulate, int mode, void* stream);
/* same for a stride-1 reflect-padded KxK conv with tiny Cout (row-split, GEMM rows (co,kh));
 * workspace floats = vst_wgrad_workspace(N, Cout*K, K*Cin, (H+K-1)*W) */
int vst_conv_wgrad_rowsplit(const float* dy, const float* x, float* dw, float* workspace, int N, int Cin, int H,
                            int W, int Cout, int K, int accumulate, int mode, void* stream);

/* forward of nearest-x2 upsample -> ReflectionPad2d(1) -> Conv2d(k3, stride 1) [+bias]
 * (UpsampleConvLayer, RC/network.py:114-120; replaces F.interpolate + pad + conv2d): one
 * phase-stacked 2x2 GEMM over the (H+1) x (W+1) source grid (2.25x fewer MACs).
 * w2 [4*Cout][Cin][2][2] = vst_up2_phase_weights(w [Cout][Cin][3][3]); wpack = vst_pack_weight of
 * w2 (Cout' = 4*Cout, KH = KW = 2, same mode); out [N][Cout][2H][2W] */
int vst_up2_phase_weights(const float* w, float* w2, int Cout, int Cin, void* stream);
int vst_conv_up2_fwd(const float* x, const float* wpack, const float* bias, float* out, int N, int Cin, int H, int W,
                     int Cout, int mode, void* stream);
/* weight gradient of nearest-x2 upsample -> ReflectionPad2d(1) -> Conv2d(k=3, stride 1)
 * (UpsampleConvLayer, RC/network.py:114-120; replaces autograd's conv2d weight backward of that
 * layer): one phase-stacked 2x2 GEMM on the source grid, 2.25x fewer MACs than the virtual-grid
 * wgrad.  dy [N][Cout][2H][2W], x [N][Cin][H][W] (pre-upsample), dw [Cout][Cin][3][3];
 * workspace floats = vst_conv_wgrad_up2_workspace(N, Cin, H, W, Cout) */
long vst_conv_wgrad_up2_workspace(int N, int Cin, int H, int W, int Cout);
int vst_conv_wgrad_up2(const float* dy, const float* x, float* dw, float* workspace, int N, int Cin, int H, int W,
                       int Cout, int accumulate, int mode, void* stream);

/* ---- Gram matrix (RC/utilities.py:93-98): G[n] = F[n] F[n]^T * scale ----------------------
 * workspace floats = vst_wgrad_workspace(N, C, C, HW) */
int vst_gram(const float* f, float* g, float* workspace, int N, int C, int HW, float scale, int mode, void* stream);
/* Gram backward, part 1: S[n] = scale * (gG[n] + gG[n]^T) written as a packed A [Kpad][Mpad]
 * (zero padded); part 2: dF = S F via vst_conv_gemm(KS=1, a_batch_stride=Kpad*Mpad)
 * (bmm backward of RC/utilities.py:97) */
int vst_symmetrize(const float* g, float* S, int N, int C, int Kpad, int Mpad, float scale, int mode, void* stream);

/* ---- InstanceNorm2d(affine) [+ReLU] [+residual] (RC/network.py:91-97, 140-150) ------------
 * stats: [N*C][2] (mean, rstd) saved for backward. */
int vst_instnorm_fwd(const float* x, const float* w, const float* b, const float* res, float* y, float* stats, int N,
                     int C, int HW, float eps, int relu, void* stream);
/* partial: N*C*3 floats; gw, gb, gbias_prev (sum of gx = grad of the feeding conv's bias) may be NULL.
 * relu: the ReLU mask is the pre-activation recomputed from x and b (bit-identical to the forward's)
 * when y is NULL, else y > 0 -- valid only when the forward had no residual add (y = relu(.) + res). */
int vst_instnorm_bwd(const float* gy, const float* x, const float* y, const float* b, const float* stats,
                     const float* w, float* gx, float* gw, float* gb, float* gbias_prev, float* partial, int N, int C,
                     int HW, int relu, int accumulate, void* stream);
/* out[c] (+)= sum_{n,i} x[n][c][i]; partial: N*C floats (conv bias gradient) */
int vst_channel_sum(const float* x, float* out, float* partial, int N, int C, int HW, int accumulate, void* stream);

/* ---- VGG MaxPool2d(2, 2) (RC/network.py:12-24 via torchvision features) -------------------- */
int vst_maxpool2x2_fwd(const float* x, float* y, long NC, int H, int W, void* stream);
/* relu_mask: gx also masked by x > 0 (x = ReLU output consumed only by this pool) */
int vst_maxpool2x2_bwd(const float* x, const float* gy, float* gx, long NC, int H, int W, int relu_mask, void* stream);
/* VGG slice boundary (a ReLU output x feeding both the losses and the next slice's pool):
 * gx = [relu_mask: (x > 0) *] (pool_bwd(gy) + addend) in one pass; gy or addend may be NULL */
int vst_maxpool2x2_bwd_add(const float* x, const float* gy, const float* addend, float* gx, long NC, int H, int W,
                           int relu_mask, void* stream);

/* ---- flow warp (RC/utilities.py:39-57) / occlusion mask (RC/utilities.py:60-90) ------------
 * warp_bwd scatters with float atomics into gx (zero it first or accumulate). */
int vst_warp_fwd(const float* x, const float* flo, float* out, int B, int C, int H, int W, void* stream);
int vst_warp_bwd(const float* gout, const float* flo, float* gx, int B, int C, int H, int W, void* stream);
/* warp backward in gather form (no float atomics on the gradient, deterministic): the bilinear taps
 * are inverted per image into per-source-pixel lists (CSR: a count pass, a scan, a fill pass) in
 * `workspace` (vst_warp_bwd_workspace bytes, 16-B aligned), then each source pixel sums its entries
 * over all channels in increasing output-pixel order -- bitwise reproducible run to run; gx is
 * overwritten (accumulate=0) or added to. */
long vst_warp_bwd_workspace(int B, int H, int W);
int vst_warp_bwd_gather(const float* gout, const float* flo, float* gx, void* workspace, int B, int C, int H, int W,
                        int accumulate, void* stream);
int vst_flow_warp_mask(const float* flo01, const float* flo10, float* mask, int B, int H, int W, float threshold,
                       void* stream);
/* F.interpolate(mode="bilinear", align_corners=False) (RC/train_single/train_candy.py:91,97);
 * optional per-channel scale (chscale[C], device) and binarize (> 0) epilogues */
int vst_resize_bilinear(const float* x, float* out, long NC, int C, int H, int W, int Ho, int Wo,
                        const float* chscale, int binarize, long out_bs, const float* addend, void* stream);
/* adjoint, as a deterministic gather (gx fully written); gout images gout_bs floats apart (0: dense)
 * (AA/network.py:59,80,85,90,94 decoder upsampling backward) */
int vst_resize_bilinear_bwd(const float* gout, float* gx, long NC, int C, int H, int W, int Ho, int Wo, long gout_bs,
                            void* stream);
/* the same pair with explicit coordinate scales (input pixels per output pixel, > 0): output pixel d
 * reads source (d + 0.5) * scale - 0.5.  vst_resize_bilinear uses H / Ho and W / Wo; F.interpolate
 * with scale_factor=s (AA/network.py:49-60 ConvReluInterpolate, any s) uses 1 / s with
 * Ho = floor(H s), which differs from H / Ho when H s is not a whole number */
int vst_resize_bilinear_scaled(const float* x, float* out, long NC, int C, int H, int W, int Ho, int Wo, float scale_y,
                               float scale_x, const float* chscale, int binarize, long out_bs, const float* addend,
                               void* stream);
int vst_resize_bilinear_scaled_bwd(const float* gout, float* gx, long NC, int C, int H, int W, int Ho, int Wo,
                                   float scale_y, float scale_x, long gout_bs, void* stream);
/* adjoint of the x2 upsample (Ho = 2H, Wo = 2W) of the decoder (AA/network.py:59,80,85,90,94), with
 * the fixed 4-tap weights per axis; ymask (optional, the upsample's input = a ReLU output): gx = 0
 * where ymask <= 0, i.e. the producer ConvReLU's ReLU backward fused in (AA/network.py:28-33).  W odd or
 * unaligned pointers fall back to the generic gather (VST_EUNSUPPORTED if a mask was asked for) */
int vst_upsample2x_bwd(const float* gout, const float* ymask, float* gx, long NC, int C, int H, int W, long gout_bs,
                       void* stream);

/* ---- losses (RC/train_single/train_candy.py:90-145) ----------------------------------------
 * ws: >= 2048 floats; out: 3 floats {loss, weight/denom, denom count}.  Backward reads gout[0]
 * and out[1] from device memory. */
/* mode 0 FTL: sum m*(a-b)^2 / nnz, m = mask>0 broadcast over C;  mode 1 OTL: a=styled2, b=warped
 * styled1, c=img2, d=warped img1, sum m*((a-b) - lum(c-d))^2 / nnz */
int vst_masked_sqdiff_fwd(int mode, const float* a, const float* b, const float* c, const float* d,
                          const float* mask, int N, int C, long HW, float weight, float* ws, float* out, void* stream);
int vst_masked_sqdiff_bwd(int mode, const float* a, const float* b, const float* c, const float* d,
                          const float* mask, int N, int C, long HW, const float* gout, const float* out, float* ga,
                          float* gb, void* stream);
/* weight * mean((a - b[i % nb])^2) (nn.MSELoss, train_candy.py:45,127-137) */
int vst_mse_fwd(const float* a, const float* b, long n, long nb, float weight, float* ws, float* out, void* stream);
int vst_mse_bwd(const float* a, const float* b, long n, long nb, const float* gout, const float* out, float* ga,
                float* gb, void* stream);
/* weight * sum of squared right/down differences (train_candy.py:141-145) */
int vst_tv_fwd(const float* s, long NC, int H, int W, float weight, float* ws, float* out, void* stream);
int vst_tv_bwd(const float* s, long NC, int H, int W, const float* gout, const float* out, float* gs, void* stream);

/* out = {weight * sum(x[0:n]), weight, 0} */
int vst_sum_scaled(const float* x, long n, float weight, float* ws, float* out, void* stream);

/* ---- AdaAttN (AA/network.py:102-251, AA/lossfn.py:5-53) --------------------------------------
 * Cosine attention (CosineSimilarity, the train_video path) is never materialised: its two moments
 * [M; E2] = (G^T q^ + sum u) / (q^ . sum k^ + Ns), G = K^ [V; V^2]^T, are formed in linear form
 *  from vst_gemm_abt / vst_attn_gemm products, vst_outer_axpy, vst_attn_fwd_rows and
 * vst_square_concat, with the transposed algebra in the backward.  The softmax activation (the image
 * trainer) keeps the materialised path: S = Q^T K per image ([N][Nc][Ns] fp32), vst_softmax_rows,
 * [M;E2] and the backward products on the same GEMM entries. */
/* out[n][m][j] = scale * sum_r a[n][m][r] b[n][j][r]; workspace = vst_wgrad_workspace(N, M, J, R) */
int vst_gemm_abt(const float* a, const float* b, float* out, float* workspace, int N, int M, int J, int R, float scale,
                 int mode, void* stream);
/* packed A operand from row-major X[k][m] (transpose 0) or X[m][k] (transpose 1), per batch */
int vst_pack_matrix(const float* x, float* packed, int B, int M, int K, int transpose, int Mpad, int Kpad, long x_bs,
                    int mode, void* stream);
/* out[n][p] = ||x[n][:][p]||_2 (LA.vector_norm over channels, AA/network.py:121-122) */
int vst_channel_norm(const float* x, float* out, int N, int C, int P, void* stream);
/* A = (S/(qn_i kn_j) + 1) / rowsum_i  (CosineSimilarity, AA/network.py:123-124) */
int vst_cos_attn_rows(const float* S, const float* qn, const float* kn, float* A, float* rowsum, int N, int Nc, int Ns,
                      void* stream);
/* backward: dS = d(raw Q^T K), dqn, dkn; S_t overwritten; part = N*ceil(Nc/64)*Ns floats */
int vst_cos_attn_rows_bwd(const float* dA, const float* A, float* S_t, const float* qn, const float* kn,
                          const float* rowsum, float* dS, float* dqn, float* dkn, float* part, int N, int Nc, int Ns,
                          void* stream);
/* A = softmax(S) over rows of Ns (Softmax activation, AA/network.py:102-108) and its backward
 * dS = A (dA - rowsum(dA A)); dS may alias dA */
int vst_softmax_rows(const float* S, float* A, long rows, int Ns, void* stream);
int vst_softmax_rows_bwd(const float* dA, const float* A, float* dS, long rows, int Ns, void* stream);
/* x[n][c][p] += s[n][p] / nrm[n][p] * y[n][c][p] */
int vst_norm_grad_add(float* x, const float* s, const float* nrm, const float* y, int N, int C, int P, void* stream);
/* VV2[n] = [V[n]; V[n]^2] and its backward dV = dV + 2 V dV2 */
int vst_square_concat(const float* V, float* VV2, int N, long per, void* stream);
int vst_square_concat_bwd(const float* dVV2, const float* V, float* dV, int N, long per, void* stream);
/* out = sqrt(clamp(E2 - M^2, 1e-6)) * IN(c_x) + M, MV[n] = [M; E2] (AA/network.py:209-220) */
int vst_adaattn_out(const float* MV, const float* cn, float* out, int N, long per, void* stream);
int vst_adaattn_out_bwd(const float* dout, const float* MV, const float* cn, float* dMV, int N, long per, void* stream);
/* the same, both halves of dMV times colscale[n][p] (per = dv * P): dRh = dMV / rs of the linear-form
 * cosine attention (attention.py LinearCosineAttnFn) in the same pass */
int vst_adaattn_out_bwd_scaled(const float* dout, const float* MV, const float* cn, const float* colscale, float* dMV,
                               int N, long per, int P, void* stream);
/* per-plane mean / unbiased std (global_stylized_loss, AA/lossfn.py:5-17) and backward */
int vst_plane_meanstd(const float* x, float* mean, float* std_, long NC, int HW, void* stream);
int vst_plane_meanstd_bwd(const float* x, const float* mean, const float* std_, const float* gmean, const float* gstd,
                          float* gx, long NC, int HW, void* stream);
/* per-plane L2 norm and its gradient add x += s/nrm * y */
int vst_plane_norm(const float* x, float* out, long NC, int HW, void* stream);
int vst_plane_norm_grad(float* x, const float* s, const float* nrm, const float* y, long NC, int HW, void* stream);
/* image_similarity_loss (AA/lossfn.py:25-53) on precomputed C x C products and norms;
 * partial[n][i] = sum_j |Dn_c - Dn_cs|_ij / hw (N*C floats); backward w.r.t. the stylised side (dG, dun, dvn fully written, fixed summation order) */
int vst_simloss(const float* Gc, const float* unc, const float* vnc, const float* Gs, const float* uns,
                const float* vns, float* colc, float* cols, float* partial, int N, int C, int HW, void* stream);
int vst_simloss_bwd(const float* Gc, const float* unc, const float* vnc, const float* Gs, const float* uns,
                    const float* vns, const float* colc, const float* cols, const float* gout, float weight, float* dG,
                    float* dun, float* dvn, int N, int C, int HW, void* stream);

/* Cosine attention without the S matrix (analytic row/column statistics, see adaattn.hip):
 * vst_attn_gemm: per-image 1x1 GEMM with the affine epilogue out = (acc + ra_m) rb_m cg_p + rd_m
 * (A = S c ks + e in the forward, dS = (dA - r) c ks in the backward); plane_dot: out[n][c] =
 * sum_p x w; channel_dot: out[n][p] = sum_c x (v[n][c] | y[n][c][p]); attn_fwd_rows: c =
 * 1/(rowsum qn), e = 1/rowsum from qkbar; attn_bwd_rows: dqn, -r, c r; scale_cols: y = x c[p];
 * attn_dkn: dkn_j = -ks_j^2 sum_c K[c][j](Y[c][j] - qt[c]). */
int vst_attn_gemm(const float* src, const float* apack, float* out, int N, int K, int P, int M, long a_batch_stride,
                  const float* ra, const float* rb, const float* rd, const float* cg, int mode, void* stream);
int vst_plane_dot(const float* x, const float* w, float* out, int N, int C, int P, void* stream);
int vst_channel_dot(const float* x, const float* v, const float* y, float* out, int N, int C, int P, void* stream);
int vst_attn_fwd_rows(const float* qkbar, const float* qn, float* c, float* e, long n, int Ns, void* stream);
int vst_reciprocal(const float* x, float* y, long n, void* stream);
int vst_attn_bwd_rows(const float* r, const float* DA, const float* qn, const float* c, const float* e, float* dqn,
                      float* nr, float* cr, long n, int Ns, void* stream);
int vst_scale_cols(const float* x, const float* c, float* y, int N, int R, int P, void* stream);
int vst_attn_dkn(const float* K, const float* Y, const float* qt, const float* ks, float* dkn, int N, int d, int Ns,
                 void* stream);

/* Cosine attention in linear form (A = diag(1/rowsum) (Qhat^T Khat + 1) never formed, see
 * video-style-transfer_amd/vst/adaattn/attention.py):
 * vst_outer_axpy: out[n][m][p] = (x[n][m][p] + alpha * u[n][m] * v[n][p]) * w[n][p]  (u, v, w may be
 *   NULL: no term / 1 / 1; out may alias x);
 * vst_sum_repeats: out[i] = sum_{r < R} x[r * per + i] (gradient of an operand broadcast over R
 *   repeats of a batch: the style side shared by both content frames);
 * vst_normalize_cols_bwd: out = (dxh - xh * t[n][p]) * s[n][p], the adjoint of column normalisation
 *   xh = x / ||x|| (t = sum_c xh dxh, s = 1 / ||x||). */
int vst_outer_axpy(const float* x, const float* u, const float* v, const float* w, float alpha, float* out, int N, int M,
                   long P, void* stream);
int vst_sum_repeats(const float* x, float* out, int R, long per, void* stream);
int vst_normalize_cols_bwd(const float* xh, const float* dxh, const float* t, const float* s, float* out, int N, int C,
                           long P, void* stream);

/* dst[n][0:per] = src[n][0:per] with batch strides (channel concat / split, AA/network.py:87) */
int vst_copy_planes(const float* src, long src_bs, float* dst, long dst_bs, int N, long per, void* stream);
/* D = 1 - G / (un_i vn_j + 1e-6) (cosine_distance forward) */
int vst_cosdist(const float* G, const float* un, const float* vn, float* D, int N, int C, void* stream);

/* ---- elementwise ---------------------------------------------------------------------------
 * vgg_normalize (RC/utilities.py:101-106): out = (x/255 - mean)/std, inplace_scale: x <- x/255 */
int vst_vgg_normalize(float* x, float* out, int N, int HW, int inplace_scale, void* stream);
int vst_vgg_normalize_bwd(const float* gout, const float* gscaled, float* gx, int N, int HW, void* stream);
/* ReLU backward: gx = gy * (y > 0) */
int vst_relu_bwd(const float* gy, const float* y, float* gx, long n, void* stream);
/* ReLU backward of an output with two consumers (a VGG19 slice output that is both a loss feature and
 * the next slice's input, AA/vgg19.py:39-63): gx = (g1 + g2) * (y > 0) in one pass, replacing
 * autograd's sum of the two gradients and the producer's separate ReLU backward; g2 may be NULL */
int vst_relu_bwd_add(const float* g1, const float* g2, const float* y, float* gx, long n, void* stream);
/* ConvTanh backward from the saved tanh value (prenorm: fold vgg_normalize's backward in) */
int vst_tanh_out_bwd(const float* gy, const float* t, float* gv, long total, long HW, int prenorm, void* stream);

/* ---- optimizer: torch.optim.Adam defaults over one flat parameter buffer
 * (RC/train_single/train_candy.py:44,152); gscale multiplies the gradient (1/world_size) */
int vst_adam(float* p, const float* g, float* m, float* v, long n, float lr, float b1, float b2, float eps,
             long step, float gscale, void* stream);

/* Adam under a dynamic loss scale (the fp16 policy's overflow guard; the reference steps in fp32
 * every batch, AA/train_video.py:121-122, RC/train_single/train_candy.py:151-152, and needs none):
 * one device-side pass flags any Inf / NaN in g; on a flagged step nothing is updated (p, m, v and
 * the Adam step count untouched) and the scale is multiplied by `backoff`; a clean step is
 * vst_adam with g * world_scale / scale, its step count read from the state, and the scale grows by
 * `growth` after `growth_interval` clean steps in a row.  No host synchronisation.
 * state: 8 floats, [0] scale (seed of the next backward), [1] clean steps since the last change,
 * [2] Adam step count, [3] last step skipped (0/1), [4] step_size, [5] sqrt(bias correction 2),
 * [6] last gradient factor, [7] skipped steps in total.  ws: >= VST_SCALER_WS floats; g 16-B aligned. */
#define VST_SCALER_WS 1024
int vst_adam_loss_scaled(float* p, const float* g, float* m, float* v, long n, float lr, float b1, float b2,
                         float eps, float world_scale, float* state, float* ws, int growth_interval, float growth,
                         float backoff, void* stream);

/* ---- RTNSTV (RT/train.py, RT/network.py) --------------------------------------------------
 * sqrt-TV regulariser (RT/train.py:57-61): out[0] = weight * mean over (nc, y < H-1, x < W-1) of
 * sqrt(clamp((s[y][x+1]-s[y][x])^2 + (s[y+1][x]-s[y][x])^2, 1e-8)); ws/out as vst_tv_fwd */
int vst_tv_sqrt_fwd(const float* s, long NC, int H, int W, float weight, float* ws, float* out, void* stream);
int vst_tv_sqrt_bwd(const float* s, long NC, int H, int W, const float* gout, const float* out, float* gs,
                    void* stream);
/* stylizer output (RT/network.py:93 after the Tanh Conv): y = (tanh(v) + 1) / 2 * 255 (image = 1)
 * or y = tanh(v) (image = 0, a standalone nn.Tanh); t = tanh(v) is kept for the backward */
int vst_tanh_image_fwd(const float* v, float* y, float* t, long n, int image, void* stream);
int vst_tanh_image_bwd(const float* gy, const float* t, float* gv, long n, int image, void* stream);

/* ---- video frames (ReCoNet inference, RC/utilities.py:108-235) -----------------------------
 * cvframe_to_tensor (RC/utilities.py:108-123, the tensor half; cv2.resize stays on the host):
 * frames = N x H x W x 3 uint8 (cv2 BGR order), out = N x 3 x H x W fp32, out = (b / 255) * 255
 * (ToTensor then .mul(255)); swap_rb = 1 applies cv2.COLOR_BGR2RGB. */
int vst_frames_to_tensor(const void* frames, float* out, int N, int H, int W, int swap_rb, void* stream);
/* Inference.__iter__ (RC/utilities.py:213-227): y (N x 3 x H x W fp32) -> clamp(0, 255) ->
 * HWC -> cv2.COLOR_RGB2BGR (swap_rb = 1) -> astype(uint8) (truncation) into frames; clamped
 * (may be NULL) receives the clamped fp32 tensor (calculate_mse's styled frame). */
int vst_tensor_to_frames(const float* y, float* clamped, void* frames, int N, int H, int W, int swap_rb,
                         void* stream);
/* calculate_mse (RC/utilities.py:151-161): out[0] = mean(((x1 - x0) - (y1 - y0))^2) over n
 * elements, computed on the device (workspace: VST_FRAME_MSE_WS_BYTES bytes). */
#define VST_FRAME_MSE_WS_BYTES 16384
int vst_frame_diff_mse(const float* x0, const float* x1, const float* y0, const float* y1, long n, void* workspace,
                       float* out, void* stream);

/* ---- frame-pair preparation of the flow datasets (RC/datasets.py:114-155, 210-251) ----------
 * Pillow Image.resize(size, BILINEAR) coefficient tables for one axis (Pillow Resample.c
 * precompute_coeffs + normalize_coeffs_8bpc, host-side, no GPU): bounds = out_size x {min, count},
 * kk = out_size x ksize 22-bit fixed-point taps.  Returns 0, or the needed ksize (> 0) when
 * ksize_cap is too small. */
int vst_pil_bilinear_coeffs(int in_size, int out_size, int* bounds, int* kk, int ksize_cap);
/* src = N x Hs x Ws x C uint8 (PIL raster, C = 3 for .convert("RGB") frames, 1 for the motion
 * boundary images); tables from vst_pil_bilinear_coeffs on the device.  mode 0: out = N x C x Ho x Wo
 * fp32 = toTensor255 of the resized image (RC/datasets.py:116-118); mode 1 (C = 1): out = N x Ho x Wo
 * flow mask, multiplied in place by the motion mask 1 - (resized != 0) (RC/datasets.py:138-144). */
int vst_pil_resize_u8(const void* src, float* out, int N, int Hs, int Ws, int C, int Ho, int Wo, const void* hbounds,
                      const void* hk, int hks, const void* vbounds, const void* vk, int vks, int mode, void* stream);
/* raw = N x Hs x Ws x Cr float32 PFM payloads in file order (bottom-up rows; byte-swapped on the
 * fly when big_endian) -> out = N x 2 x Ho x Wo: flipud, [:-1] channel drop (first 2 channels),
 * F.interpolate(bilinear, align_corners=False), channel 0 * sx, channel 1 * sy
 * (RC/datasets.py:121-136; the reference scales x by Ho/Hs and y by Wo/Ws). */
int vst_flow_prep(const void* raw, float* out, int N, int Hs, int Ws, int Cr, int big_endian, int Ho, int Wo,
                  float sx, float sy, void* stream);
/* flowlib.readPFM (RC/flowlib.py:34-64), host-side: header parse ("PF" -> 3 channels, "Pf" -> 1;
 * "W H" line as re '^(\d+)\s(\d+)\s$'; scale < 0 -> little-endian).  Errors carry the reference's
 * messages ("Not a PFM file.", "Malformed PFM header."); the payload must hold exactly
 * W*H*channels floats (np.reshape raised otherwise).  vst_pfm_read copies the raw payload bytes. */
int vst_pfm_read_header(const char* path, int* width, int* height, int* channels, int* big_endian, int* offset,
                        float* scale);
int vst_pfm_read(const char* path, void* dst, long bytes, int offset);

/* ---- gradient sums / fills -----------------------------------------------------------------
 * out[i] = ((a[i] + b[i]) + c[i]) + d[i] over n floats, NULL addends skipped (a..d: at least one);
 * out may be one of the addends.  The autograd gradient sum of a tensor with several consumers
 * (vst/ops.py ForkFn: ResidualBlock's input, RC/network.py:136-150; the feature map and the stylised
 * frame, RC/train_single/train_candy.py:100-145; loss-term sums) -- the ATen add it replaces summed
 * two at a time.  vst_fill: x[i] = value (the flat gradient's zeroing before each step). */
int vst_sum4(const float* a, const float* b, const float* c, const float* d, float* out, long n, void* stream);
int vst_fill(float* x, long n, float value, void* stream);

/* ---- profiling ---------------------------------------------------------------------------
 * an empty kernel (vst_marker_kernel) on `stream`: marks a region boundary in rocprofv3 traces
 * (bench.py launches one before its timed steps; tools/pmc_traffic.py --after-marker) */
int vst_marker(void* stream);
/* test only: one wave on `stream` that sleeps iters x 8128 cycles (about 3.5 us each at 2.4 GHz), so
 * the work enqueued after it on that stream starts late; the stream-ordering tests
 * (tests/test_gpu_streams.py) put it in front of each cross-stream hand-off of the training step.
 * iters < 0: VST_EINVAL. */
int vst_test_delay(long iters, void* stream);
/* test only: `blocks` x 256 lanes of three kernels with 256 B / 1280 B / 4608 B private (scratch)
 * segments each write `value` over their whole private array on `stream`, so the scratch slots the
 * next kernels with register spills get on that stream hold `value` (a NaN) -- a kernel that read a
 * private slot before writing it would then show it (tools/f16_repro.py --poison-scratch). */
int vst_test_scratch_poison(long blocks, float value, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* VST_HIP_H */
