// Implicit-GEMM convolution on fp32 MFMA (v_mfma_f32_32x32x2_f32) for gfx950.
//
//   out[n][m][p] = epi( sum_k  Apack[k][m] * gather(src[n], k, p) )
//
// One kernel serves every "weights x im2col" product of the ReCoNet / VGG training step:
//   * forward conv, reflection or zero padding, stride 1/2, optional nearest x2 upsample folded
//     into the gather (RC/network.py:72-75, 114-120; VGG features conv3x3 pad 1),
//   * data-gradient (transposed gather, stride-divisibility test) into the padded/virtual input
//     grid, followed by `fold_reflect` (reflection-pad + upsample adjoint),
//   * 1x1 products with a per-image A (Gram backward dF = S F, RC/utilities.py:93-98).
// K is ordered tap-major / channel-minor, k = (kh*KW + kw)*Cs + c, so when Cs % 16 == 0 a whole
// 16-deep k-tile shares one tap and the reflect/zero/upsample index math is done once per tile.
//
// Tile: 4 waves (256 threads); each wave owns TM x TN 32x32 accumulators (WM x WN waves).
// LDS: A[BK][BM] and B[BK][BN], double buffered; global->register prefetch of tile t+1 overlaps
// the MFMAs of tile t; one barrier per k-tile.
#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "conv_gemm_kernel.h"
#include "conv_halo_kernel.h"
#include "vst_common.h"
#include "vst_hip.h"

using namespace vstk;

namespace {

// sum of the split-K slices part[s][n][m][p] (s in order: deterministic), then the conv epilogue.
// Grid: x = pixel chunks of 4 x 256, y = n * M + m.
template <bool VEC>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(ConvParams P, int N) {
  const int row = blockIdx.y, n = row / P.M, m = row - n * P.M;
  const int HWo = P.Ho * P.Wo;
  const long slice = (long)N * P.M * HWo;
  const float* src = P.part + (long)row * HWo;
  const int p0 = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (p0 >= HWo) return;
  float v[4];
  if constexpr (VEC) {
    float4 a = *reinterpret_cast<const float4*>(src + p0);
    v[0] = a.x, v[1] = a.y, v[2] = a.z, v[3] = a.w;
    for (int s = 1; s < P.ksplit; ++s) {
      const float4 b = *reinterpret_cast<const float4*>(src + s * slice + p0);
      v[0] += b.x, v[1] += b.y, v[2] += b.z, v[3] += b.w;
    }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[i] = 0.f;
      if (p0 + i < HWo)
        for (int s = 0; s < P.ksplit; ++s) v[i] += src[s * slice + p0 + i];
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (p0 + i < HWo) conv_epilogue_elem(P, n, m, p0 + i, v[i]);
}

// slices for a halo launch of `wgs` blocks over `nblk` 16-channel blocks: none when the grid
// already fills the chip; otherwise the fewest equal slices (>= 3 blocks each) that reach two
// blocks per CU, at most four per CU
int halo_ksplit(long wgs, int nblk) {
  if (wgs >= 512) return 1;
  int best = 1;
  for (int s : {2, 3, 4, 6, 8}) {
    if (nblk % s || nblk / s < 3 || wgs * s > 1024) continue;
    best = s;
    if (wgs * s >= 512) break;
  }
  return best;
}

// ---------------------------------------------------------------------------------------------
// fwd:        A[k = (kh*KW+kw)*Cin + ci][m = co]
// transposed: A[k = (kh*KW+kw)*Cout + co][m = ci]        (data gradient)
// split_kh:   A[k = kw*Cin + ci][m = co*KH + kh]          (row-split GEMM for tiny Cout, see vst_hip.h)
// bsplit: write the bf16 hi/lo layout of the bf16 GEMM modes (vst_common.h apack_store)
__global__ void pack_weight_kernel(const float* __restrict__ w, float* __restrict__ out, int Cout, int Cin, int KH,
                                   int KW, int transposed, int split_kh, int Mpad, int Kpad, int bsplit) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)Mpad * Kpad;
  if (idx >= total) return;
  int m = (int)(idx % Mpad);
  int k = (int)(idx / Mpad);
  float v = 0.f;
  if (split_kh) {
    if (m < Cout * KH && k < KW * Cin) {
      int kw, ci;
      kdecode(k, Cin, KW, kw, ci, bsplit >> 4);
      const int co = m / KH, kh = m % KH;
      v = w[(((long)co * Cin + ci) * KH + kh) * KW + kw];
    }
  } else {
    int Ck = transposed ? Cout : Cin;  // channel count inside the k index
    int Mm = transposed ? Cin : Cout;
    if (m < Mm && k < KH * KW * Ck) {
      int tap, c;
      kdecode(k, Ck, KH * KW, tap, c, bsplit >> 4);
      int kh = tap / KW, kw = tap % KW;
      int co = transposed ? c : m, ci = transposed ? m : c;
      v = w[(((long)co * Cin + ci) * KH + kh) * KW + kw];
    }
  }
  apack_store(out, k, m, Mpad, v, bsplit);
}

// adjoint of (nearest x`up` upsample -> ReflectionPad2d(pad)): dpad [NC][Hv+2p][Wv+2p] -> dx [NC][Hs][Ws]
// padded-grid sources of virtual coordinate u: the direct one and up to two reflections
// (fixed register slots, -1 = none: no dynamically indexed arrays -> no scratch)
struct Src3 {
  int a, b, c;
};
__device__ __forceinline__ Src3 reflect_sources(int u, int n_v, int pad) {
  Src3 s;
  s.a = u + pad;
  s.b = (u >= 1 && u <= pad) ? pad - u : -1;
  s.c = (u >= n_v - 1 - pad && u <= n_v - 2) ? 2 * (n_v - 1) - u + pad : -1;
  return s;
}

__device__ __forceinline__ float fold_row(const float* __restrict__ r, const Src3& cx) {
  float v = r[cx.a];
  if (cx.b >= 0) v += r[cx.b];
  if (cx.c >= 0) v += r[cx.c];
  return v;
}

// grid: x over the pixels of one plane, y over planes (grid-stride)
__global__ void fold_reflect_kernel(const float* __restrict__ dpad, float* __restrict__ dx, int NC, int Hs, int Ws,
                                    int pad, int up, int accumulate) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= Hs * Ws) return;
  const int xs = p % Ws, ys = p / Ws;
  const int Hv = Hs * up, Wv = Ws * up;
  const int Hp = Hv + 2 * pad, Wp = Wv + 2 * pad;
  for (int nc = blockIdx.y; nc < NC; nc += gridDim.y) {
    const float* d = dpad + (long)nc * Hp * Wp;
    float s = 0.f;
    for (int dy = 0; dy < up; ++dy) {
      const Src3 ry = reflect_sources(ys * up + dy, Hv, pad);
      for (int dxx = 0; dxx < up; ++dxx) {
        const Src3 cx = reflect_sources(xs * up + dxx, Wv, pad);
        s += fold_row(d + (long)ry.a * Wp, cx);
        if (ry.b >= 0) s += fold_row(d + (long)ry.b * Wp, cx);
        if (ry.c >= 0) s += fold_row(d + (long)ry.c * Wp, cx);
      }
    }
    float* o = dx + (long)nc * Hs * Ws + p;
    if (accumulate) s += *o;
    *o = s;
  }
}

// Stride-2 data gradient, all four parity phases stacked in one transposed GEMM (EPI_PHASE2):
// padded-input pixel (2I+a, 2J+b) receives taps kh = a + 2t, kw = b + 2s from dY[I-t][J-s], so with
// the window t, s < ceil(KS/2) over dY the A operand is k = (t*KW2 + s)*Cout + co, m = ci*4 + 2a + b,
// zero where a + 2t or b + 2s falls outside the kernel.
__global__ void pack_phase2_kernel(const float* __restrict__ w, float* __restrict__ out, int Cout, int Cin, int KS,
                                   int Mpad, int Kpad, int bsplit) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)Mpad * Kpad) return;
  int m = (int)(idx % Mpad);
  int k = (int)(idx / Mpad);
  const int K2 = (KS + 1) / 2;
  float v = 0.f;
  if (m < 4 * Cin && k < K2 * K2 * Cout) {
    int tap, co;
    kdecode(k, Cout, K2 * K2, tap, co, bsplit >> 4);
    const int t = tap / K2, sx = tap % K2;
    const int ci = m >> 2, kh = ((m >> 1) & 1) + 2 * t, kw = (m & 1) + 2 * sx;
    if (kh < KS && kw < KS) v = w[(((long)co * Cin + ci) * KS + kh) * KS + kw];
  }
  apack_store(out, k, m, Mpad, v, bsplit);
}

// kw-unfold of a thin-channel tensor (Cin*K <= Cu, e.g. 3-channel images under a 9x9 kernel):
//   out[n][c*K + kw][y][v] = src[n][c][y][xs],  xs = v + sgn*kw + off  (reflect or zero outside),
// channels c*K + kw >= C*K are zero.  A conv over `out` with a Kx1 kernel (pad_x = 0) then runs on
// the 16-channel k-tile path instead of a per-element tap decode over 3 channels.
__global__ void unfold_kw_kernel(const float* __restrict__ src, float* __restrict__ out, int N, int C, int H, int Ws,
                                 int Wout, int K, int Cu, int Cg, int sgn, int off, int reflect) {
  // one thread per 4 consecutive outputs (float4 store; Wout % 4 == 0) of all K unfolded rows of one
  // source row: grid.y = (n, channel group cg, y), the group's rows cu = cg*K + kw (kw < K, cu < Cu;
  // groups cg >= C write the zero channels).  The K rows re-read one source row segment from L1.
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (4 * q >= Wout) return;
  const int row = blockIdx.y + gridDim.y * blockIdx.z;
  if (row >= N * Cg * H) return;
  const int y = row % H, t = row / H, cg = t % Cg, n = t / Cg;
  const float* sr = src + (((long)n * C + (cg < C ? cg : 0)) * H + y) * Ws;
  float* orow = out + (((long)n * Cu + cg * K) * H + y) * Wout + 4 * q;
  const long ostride = (long)H * Wout;
  for (int kw = 0; kw < K && cg * K + kw < Cu; ++kw) {
    float v4[4] = {0.f, 0.f, 0.f, 0.f};
    if (cg < C) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        int xs = 4 * q + e + sgn * kw + off;
        if (reflect) {
          xs = abs(xs);
          xs = xs >= Ws ? 2 * Ws - 2 - xs : xs;
        }
        // (reflect: single reflections only; anything further reads 0, never out of bounds)
        v4[e] = (xs >= 0 && xs < Ws) ? sr[xs] : 0.f;
      }
    }
    *reinterpret_cast<f32x4*>(orow + kw * ostride) = f32x4{v4[0], v4[1], v4[2], v4[3]};
  }
}

// dx[n][c][y][x] (+)= sum_{kh,kw} P[n][(c*K + kh)*K + kw][y + pad - kh][x + pad - kw]  (zero outside):
// the data gradient of a zero-padded stride-1 KxK conv with few input channels, after the tap-split
// 1x1 GEMM P = W^T dY (rows (c, kh, kw): 27 GEMM rows for VGG conv1_1 instead of 3 padded to 32)
__global__ void tapsum_kernel(const float* __restrict__ P, float* __restrict__ dx, int N, int C, int H, int W, int K,
                              int pad, int accumulate) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long HW = (long)H * W;
  if (idx >= (long)N * C * HW) return;
  const long q = idx % HW, nc = idx / HW;
  const int y = (int)(q / W), x = (int)(q % W);
  const int c = (int)(nc % C), n = (int)(nc / C);
  const float* pb = P + ((long)n * C * K * K + (long)c * K * K) * HW;
  float s = 0.f;
  for (int kh = 0; kh < K; ++kh) {
    const int yy = y + pad - kh;
    if (yy < 0 || yy >= H) continue;
    for (int kw = 0; kw < K; ++kw) {
      const int xx = x + pad - kw;
      if (xx >= 0 && xx < W) s += pb[(long)(kh * K + kw) * HW + (long)yy * W + xx];
    }
  }
  dx[idx] = accumulate ? dx[idx] + s : s;
}

// A operand over a kw-unfolded source: k = kh*Cu + c*K + kw (c < Cc, the unfolded tensor's channel),
// fwd: m = co, Cc = Cin; transposed (data gradient): m = ci, Cc = Cout
__global__ void pack_kwu_kernel(const float* __restrict__ w, float* __restrict__ out, int Cout, int Cin, int K, int Cu,
                                int transposed, int Mpad, int Kpad, int bsplit) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)Mpad * Kpad) return;
  const int m = (int)(idx % Mpad);
  const int k = (int)(idx / Mpad);
  const int Mm = transposed ? Cin : Cout, Cc = transposed ? Cout : Cin;
  float v = 0.f;
  if (m < Mm && k < K * Cu) {
    int kh, cu;
    kdecode(k, Cu, K, kh, cu, bsplit >> 4);
    const int c = cu / K, kw = cu - (cu / K) * K;
    if (c < Cc) {
      const int co = transposed ? c : m, ci = transposed ? m : c;
      v = w[(((long)co * Cin + ci) * K + kh) * K + kw];
    }
  }
  apack_store(out, k, m, Mpad, v, bsplit);
}

// dx (+)= the reflect-pad border of the padded-grid gradient (the interior went straight to dx):
// one thread per element of dx's border band (rows/cols within pad+1 of an edge)
__global__ void fold_border_kernel(const float* __restrict__ border, const float* __restrict__ mask,
                                   float* __restrict__ dx, int NC, int Hs, int Ws, int pad) {
  const int nb = pad < Hs / 2 ? pad + 1 : Hs;  // band rows at each edge (rows 0..pad and Hs-1-pad..Hs-1)
  const int band_rows = nb >= Hs ? Hs : 2 * nb;
  const int nbc = pad < Ws / 2 ? pad + 1 : Ws;
  const int band_cols = nbc >= Ws ? Ws : 2 * nbc;
  const long per_plane = (long)band_rows * Ws + (long)(Hs - band_rows) * band_cols;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= per_plane * NC) return;
  const int nc = (int)(idx / per_plane);
  int q = (int)(idx - (long)nc * per_plane), y, x;
  if (q < band_rows * Ws) {
    const int r = q / Ws;
    x = q - r * Ws;
    y = (band_rows == Hs || r < nb) ? r : Hs - band_rows + r;
  } else {
    q -= band_rows * Ws;
    const int r = q / band_cols, c = q - r * band_cols;
    y = nb + r;
    x = (band_cols == Ws || c < nbc) ? c : Ws - band_cols + c;
  }
  const int Hp = Hs + 2 * pad, Wp = Ws + 2 * pad;
  const float* b = border + (long)nc * Hp * Wp;
  const Src3 ry = reflect_sources(y, Hs, pad), cx = reflect_sources(x, Ws, pad);
  // every (row source, column source) pair except (direct, direct) is a border position
  float s = 0.f;
  const int us[3] = {ry.a, ry.b, ry.c}, vs[3] = {cx.a, cx.b, cx.c};
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      if ((i | j) && us[i] >= 0 && vs[j] >= 0) s += b[(long)us[i] * Wp + vs[j]];
  const long o = ((long)nc * Hs + y) * Ws + x;
  if (mask && !(mask[o] > 0.f)) return;  // masked: the epilogue already wrote 0
  dx[o] += s;
}

}  // namespace

extern "C" {

int vst_version(void) { return 400; }

#ifndef VST_BUILD_ID
#define VST_BUILD_ID "unknown"
#endif
const char* vst_build_id(void) { return VST_BUILD_ID; }


const char* vst_strerror(int code) {
  if (code == VST_OK) return "success";
  if (code == VST_EINVAL) return "vst: invalid argument";
  if (code == VST_EUNSUPPORTED) return "vst: unsupported configuration";
  if (code == VST_EIO) return "vst: cannot open file";
  if (code == VST_EPFM_MAGIC) return "Not a PFM file.";
  if (code == VST_EPFM_HEADER) return "Malformed PFM header.";
  if (code == VST_EPFM_SIZE) return "PFM data size does not match its header";
  return hipGetErrorString((hipError_t)code);
}

int vst_conv_pack_dims(int M, int K, int* Mpad, int* Kpad) {
  VST_CHECK_ARG(M > 0 && K > 0 && Mpad && Kpad);
  int bm = cfg_bm(select_cfg(M));
  *Mpad = (M + bm - 1) / bm * bm;
  *Kpad = (K + BK - 1) / BK * BK;
  return VST_OK;
}

int vst_pack_weight(const float* w, float* packed, int Cout, int Cin, int KH, int KW, int transposed, int split_kh,
                    int Mpad, int Kpad, int mode, void* stream) {
  VST_CHECK_ARG(vst_mode_ok(mode));
  VST_CHECK_ARG(w && packed && Cout > 0 && Cin > 0 && KH > 0 && KW > 0 && !(transposed && split_kh));
  long total = (long)Mpad * Kpad;
  pack_weight_kernel<<<ceil_div(total, 256), 256, 0, (hipStream_t)stream>>>(
      w, packed, Cout, Cin, KH, KW, transposed, split_kh, Mpad, Kpad, apack_split(mode));
  return vst_launch_status();
}

}  // extern "C"

// floats of one packed A operand of an M x K GEMM in `mode` (vst_conv_pack_dims padding; bf16x6
// blocks are 1.5x): per-image packs must be at least this far apart
static long apack_floats(int M, int K, int mode) {
  const int bm = cfg_bm(select_cfg(M));
  const long f = (long)((M + bm - 1) / bm * bm) * ((K + BK - 1) / BK * BK);
  return vst_mode_arith(mode) == VST_GEMM_BF16X6 ? f * 3 / 2 : f;
}

// Halo-kernel plan of a conv GEMM launch (shared by the launch and vst_conv_splitk_workspace, so the
// workspace a caller is told to supply is exactly what the launch will use): the halo block config
// (0 = the per-tap kernel runs) and the split-K slice count S (1 = unsplit).
struct HaloPlan {
  int hcfg, S, tiles, mpad;
};
static HaloPlan halo_plan(int N, int Cs, int M, int Ho, int Wo, int KH, int KW, int gmode, int stride, int pad,
                          int pad_x, int up, int epi, long a_batch_stride, int mode, bool gmask_free = true) {
  HaloPlan hp{0, 1, 0, 0};
  const int am = vst_mode_arith(mode);
  // (the packed A carries vst_conv_pack_dims' Mpad; the halo block's M tile must divide it)
  const int pack_bm = cfg_bm(select_cfg(M));
  hp.mpad = (M + pack_bm - 1) / pack_bm * pack_bm;
  const int hcfg = halo_cfg(M, hp.mpad);
  // 3x3 taps (stride 1, reflect / zero / transposed gathers), or the 2x2 phase-stacked GEMMs
  // (EPI_PHASE2: the stride-2 data gradient's transposed gather, the up2 forward's edge clamp)
  const bool ph2 = (epi & EPI_PHASE2) != 0;
  // 9 x 1 over a kw-unfolded operand (column pad 0): the 64- / 128-row block selections only
  const bool k91 = !ph2 && KH == 9 && KW == 1 && pad_x == 0 && gmask_free && (hcfg == HALO_M64 || hcfg == HALO_M128) &&
                   (gmode == GM_REFLECT || gmode == GM_TRANSPOSED);
  // 1 x 9 over the reflect-padded rows (ConvTanh's row-split forward: 27 rows in a 32-row pack)
  const bool k19 = !ph2 && KH == 1 && KW == 9 && pad_x == pad && gmask_free && hp.mpad == 32 && gmode == GM_REFLECT &&
                   epi == 0;
  const int hcfg19 = k19 ? H1x4S : hcfg;
  const bool taps_ok = ph2 ? (KH == 2 && KW == 2 && (gmode == GM_TRANSPOSED || gmode == GM_CLAMP) && gmask_free)
                       : (k91 || k19) ? true
                             : (KH == 3 && KW == 3 && (gmode == GM_REFLECT || gmode == GM_ZERO || gmode == GM_TRANSPOSED));
  const bool halo = hcfg19 && !(mode & VST_GEMM_PERTAP) && (mode & VST_GEMM_KBLOCK) && taps_ok &&
                    stride == 1 && up == 1 && Cs % 16 == 0 && (pad_x == pad || k91) && a_batch_stride == 0 &&
                    !(epi & EPI_AFFINE) &&
                    (am == VST_GEMM_BF16X6 || am == VST_GEMM_BF16X3 || am == VST_GEMM_BF16 || am == VST_GEMM_F16);
  if (!halo) return hp;
  hp.hcfg = hcfg19;
  const int bm = 32 * halo_wm(hcfg19), th = 4 * halo_wn(hcfg19);
  hp.tiles = ((Wo + HTW - 1) / HTW) * ((Ho + th - 1) / th);
  // split-K when the grid is too small for the chip (AdaAttN config 4's decoder and VGG19 conv4 /
  // conv5 layers: 128-384 blocks); every split launch matches its unsplit launch to <= 3e-6
  // (tools/split_diag.py).  Not for the phase-stacked epilogue (the reduce writes plain / padded-grid
  // outputs only).
  if (!ph2 && !(mode & VST_GEMM_NOSPLIT))
    hp.S = halo_ksplit((long)hp.tiles * (hp.mpad / bm) * N, Cs / 16);
  return hp;
}

// bytes of split-K workspace a planned launch needs (0: unsplit)
static long splitk_bytes(const HaloPlan& hp, int N, int M, int Ho, int Wo) {
  return hp.S > 1 ? (long)hp.S * N * M * Ho * Wo * (long)sizeof(float) : 0;
}

static int conv_gemm_launch(const float* src, const float* wpack, const float* bias, const float* mask, float* out,
                            int N, int Cs, int Hs, int Ws, int M, int K, int Ho, int Wo, int KH, int KW, int gmode,
                            int stride, int pad, int pad_x, int up, int epi, long a_batch_stride, float* aux,
                            const float* gmask, int mode, void* stream, const float* ep_ra = nullptr,
                            const float* ep_rb = nullptr, const float* ep_rd = nullptr,
                            const float* ep_cg = nullptr, float* ph_border = nullptr, int ph_H = 0, int ph_W = 0,
                            int ph_pad = 0, void* workspace = nullptr, long ws_bytes = 0) {
  ConvParams P;
  P.ph_border = ph_border;
  P.ph_H = ph_H;
  P.ph_W = ph_W;
  P.ph_pad = ph_pad;
  P.src = src;
  P.wpack = wpack;
  P.bias = bias;
  P.mask = mask;
  P.gmask = gmask;
  P.out = out;
  P.aux = aux;
  P.a_batch_stride = a_batch_stride;
  P.Cs = Cs;
  P.Hs = Hs;
  P.Ws = Ws;
  P.M = M;
  int cfg = widen_cfg(select_cfg(M), (long)Ho * Wo);
  {
    // 256-row tiles for 256-multiple M on the single-product paths (then A-direct below).  Not under
    // bf16x3: its 256 x 128 LDS-A tile spills 63 VGPRs (eight accumulator fragments and two pieces per
    // operand); the 128-row tile ran config 5 at 128.4 / 128.1 ms against 128.5 / 129.6 (A/B/A/B on one
    // box, the AdaAttN attention projections)
    const int am = vst_mode_arith(mode);
    if (cfg == T128 && M % 256 == 0 && (am == VST_GEMM_BF16 || am == VST_GEMM_F16)) cfg = T256;
    // bf16x6 A-direct blocks: 64-, 128- and 256-row tiles always, the 192-row tile for data
    // gradients only (its forward keeps the LDS-A tile: DESIGN.md §4.2 item 3)
    const bool dg = gmode == GM_TRANSPOSED;
    if (am == VST_GEMM_BF16X6) {
      if (cfg == T128 && M % 256 == 0) cfg = T256A;
      if (cfg == T128) cfg = T128A;
      if (cfg == T64W || cfg == T64) cfg = T64A;
      if (cfg == T192 && dg) cfg = T192A;
    }
    // single-product modes (bf16, fp16): A-direct blocks with two k-tiles per stage -- the LDS-A
    // tiles stage 256 weight rows x 32 B per k-tile through LDS for 8 MFMAs per wave, which puts
    // their LDS store traffic past the array's write rate
    if (am == VST_GEMM_BF16 || am == VST_GEMM_F16) {
      if (cfg == T256) cfg = T256A;
      if (cfg == T128) cfg = M % 256 == 0 ? T256A : T128A;
      if (cfg == T64W || cfg == T64) cfg = T64A;
      if (cfg == T192) cfg = T192A;
    }
  }
  // 3x3 stride-1 convs in the channel-blocked K order: the halo-tiled kernel (conv_halo_kernel.h),
  // one A-direct wave per 32 weight rows -- 2 / 4 / 6 / 8 waves as the per-tap kernel's blocks
  const int am = vst_mode_arith(mode);
  const HaloPlan hp =
      halo_plan(N, Cs, M, Ho, Wo, KH, KW, gmode, stride, pad, pad_x, up, epi, a_batch_stride, mode, gmask == nullptr);
  if (hp.hcfg) {
    const int hcfg = hp.hcfg, bm = 32 * halo_wm(hcfg);
    P.Mpad = hp.mpad;
    P.K = K;
    P.Kpad = (K + BK - 1) / BK * BK;
    P.Ho = Ho;
    P.Wo = Wo;
    P.KH = KH;
    P.KW = KW;
    P.gmode = gmode;
    P.stride = 1;
    P.pad = pad;
    P.pad_x = pad_x;
    P.up = 1;
    P.epi = epi;
    P.ep_ra = P.ep_rb = P.ep_rd = P.ep_cg = nullptr;
    P.fd_Wo = make_fastdiv(Wo);
    P.fd_Cs = make_fastdiv(Cs);
    P.fd_KW = make_fastdiv(KW);
    P.kb = 1;
    hipStream_t st = (hipStream_t)stream;
    // the split's slices go to the caller's workspace (vst_conv_splitk_workspace bytes); a launch
    // given less runs unsplit -- same result up to fp32 summation order
    const long need = splitk_bytes(hp, N, M, Ho, Wo);
    int S = 1;
    if (need > 0 && workspace && ws_bytes >= need && ((uintptr_t)workspace & 15) == 0) {
      S = hp.S;
      P.part = (float*)workspace;
      P.ksplit = S;
    }
    dim3 grid(hp.tiles, P.Mpad / bm, N * S);
    const bool gm = gmask != nullptr;
    if (am == VST_GEMM_BF16X6) launch_halo_prec<3>(gm, hcfg, KH, grid, st, P);
    else if (am == VST_GEMM_F16) launch_halo_prec<4>(gm, hcfg, KH, grid, st, P);
    else if (am == VST_GEMM_BF16X3) launch_halo_prec<1>(gm, hcfg, KH, grid, st, P);
    else launch_halo_prec<2>(gm, hcfg, KH, grid, st, P);
    if (S > 1) {
      const int HWo = Ho * Wo;
      dim3 rgrid((HWo + 1023) / 1024, N * M);
      if (HWo % 4 == 0) splitk_reduce_kernel<true><<<rgrid, 256, 0, st>>>(P, N);
      else splitk_reduce_kernel<false><<<rgrid, 256, 0, st>>>(P, N);
    }
    return vst_launch_status();
  }
  int bm = cfg_bm(cfg), bn = cfg_bn(cfg);
  P.Mpad = (M + bm - 1) / bm * bm;
  P.K = K;
  P.Kpad = (K + BK - 1) / BK * BK;
  P.Ho = Ho;
  P.Wo = Wo;
  P.KH = KH;
  P.KW = KW;
  P.gmode = gmode;
  P.stride = stride;
  P.pad = pad;
  P.pad_x = pad_x;
  P.up = up;
  P.epi = epi;
  P.ep_ra = ep_ra;
  P.ep_rb = ep_rb;
  P.ep_rd = ep_rd;
  P.ep_cg = ep_cg;
  P.fd_Wo = make_fastdiv(Wo);
  P.fd_Cs = make_fastdiv(Cs);
  P.fd_KW = make_fastdiv(KW);
  P.kb = (mode & VST_GEMM_KBLOCK) ? 1 : 0;
  dim3 grid(ceil_div((long)Ho * Wo, bn), P.Mpad / bm, N);
  const bool cfast = (Cs % 16) == 0, gm = gmask != nullptr;
  hipStream_t st = (hipStream_t)stream;
  switch (vst_mode_arith(mode)) {
    case VST_GEMM_F32: launch_prec<0>(cfast, gm, cfg, grid, st, P); break;
    case VST_GEMM_BF16: launch_prec<2>(cfast, gm, cfg, grid, st, P); break;
    case VST_GEMM_BF16X6: launch_prec<3>(cfast, gm, cfg, grid, st, P); break;
    case VST_GEMM_F16: launch_prec<4>(cfast, gm, cfg, grid, st, P); break;
    default: launch_prec<1>(cfast, gm, cfg, grid, st, P); break;
  }
  return vst_launch_status();
}

// Direct 3x3 convolution of a 3-channel image (VGG conv1_1: Conv2d(3, Cout, 3, padding=1) [+ReLU],
// RC/network.py:17, AA/vgg19.py:19), stride 1, zero or reflect pad 1.  27 MACs per output: the
// layer is bound by its output write, so it runs on the VALU in exact fp32 (fmaf chain from the
// bias over (ci, kh, kw)) instead of an unfold pass + a K = 48 GEMM.  One thread per pixel, all
// output channels; the 27 inputs stay in registers, the weights are wave-uniform (scalar loads),
// each output plane is written by consecutive lanes (coalesced rows).
template <bool REFLECT>
__global__ __launch_bounds__(256) void cin3_conv3_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                         const float* __restrict__ b, float* __restrict__ out, int H,
                                                         int W, int Cout, int relu) {
  const int n = blockIdx.z, y = blockIdx.y;
  const int px = blockIdx.x * 256 + threadIdx.x;
  if (px >= W) return;
  const float* xn = x + (long)n * 3 * H * W;
  float v[27];
#pragma unroll
  for (int kh = 0; kh < 3; ++kh) {
    int yy = y + kh - 1;
    bool oky = true;
    if (REFLECT) yy = yy < 0 ? -yy : (yy >= H ? 2 * H - 2 - yy : yy);
    else oky = yy >= 0 && yy < H;
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      int xx = px + kw - 1;
      bool ok = oky;
      if (REFLECT) xx = xx < 0 ? -xx : (xx >= W ? 2 * W - 2 - xx : xx);
      else ok = ok && xx >= 0 && xx < W;
#pragma unroll
      for (int ci = 0; ci < 3; ++ci) v[ci * 9 + kh * 3 + kw] = ok ? xn[((long)ci * H + yy) * W + xx] : 0.f;
    }
  }
  float* o = out + ((long)n * Cout * H + y) * W + px;
  const long cstride = (long)H * W;
  for (int co = 0; co < Cout; ++co) {
    const float* wc = w + co * 27;
    float a = b ? b[co] : 0.f;
#pragma unroll
    for (int t = 0; t < 27; ++t) a = fmaf(wc[t], v[t], a);
    if (relu) a = fmaxf(a, 0.f);
    o[co * cstride] = a;
  }
}

// The same convolution, four consecutive pixels per thread (W % 4 == 0): pixel pairs go through packed
// fp32 FMAs (v_pk_fma_f32: two fmaf per instruction, the same fused operations in the same order, so
// the output is bitwise that of cin3_conv3_kernel) and each output row segment is one 16-byte store.
// The one-pixel kernel issued 27 VALU FMAs and a 4-byte store per output: at 64 output channels it
// ran at half the HBM write rate (config 5: 0.73 ms for a 2.1 GB output).
template <bool REFLECT>
__global__ __launch_bounds__(256) void cin3_conv3_x4_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                            const float* __restrict__ b, float* __restrict__ out,
                                                            int H, int W, int Cout, int relu) {
  const int n = blockIdx.z, y = blockIdx.y;
  const int px0 = 4 * (blockIdx.x * 256 + threadIdx.x);
  if (px0 >= W) return;
  const float* xn = x + (long)n * 3 * H * W;
  // v[ci][kh][c]: source columns px0 - 1 .. px0 + 4
  float v[3][3][6];
#pragma unroll
  for (int kh = 0; kh < 3; ++kh) {
    int yy = y + kh - 1;
    bool oky = true;
    if (REFLECT) yy = yy < 0 ? -yy : (yy >= H ? 2 * H - 2 - yy : yy);
    else oky = yy >= 0 && yy < H;
    int xl = px0 - 1, xr = px0 + 4;
    bool okl = oky, okr = oky;
    if (REFLECT) {
      xl = xl < 0 ? 1 : xl;
      xr = xr >= W ? W - 2 : xr;
    } else {
      okl = okl && xl >= 0;
      okr = okr && xr < W;
    }
#pragma unroll
    for (int ci = 0; ci < 3; ++ci) {
      const float* row = xn + ((long)ci * H + (oky ? yy : 0)) * W;
      const f32x4 m = oky ? *reinterpret_cast<const f32x4*>(row + px0) : f32x4{0.f, 0.f, 0.f, 0.f};
      v[ci][kh][0] = okl ? row[xl] : 0.f;
      v[ci][kh][1] = m[0];
      v[ci][kh][2] = m[1];
      v[ci][kh][3] = m[2];
      v[ci][kh][4] = m[3];
      v[ci][kh][5] = okr ? row[xr] : 0.f;
    }
  }
  float* o = out + ((long)n * Cout * H + y) * W + px0;
  const long cstride = (long)H * W;
  for (int co = 0; co < Cout; ++co) {
    const float* wc = w + co * 27;
    const float bc = b ? b[co] : 0.f;
    f32x2 a01 = {bc, bc}, a23 = {bc, bc};
#pragma unroll
    for (int ci = 0; ci < 3; ++ci)
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const float wt = wc[ci * 9 + kh * 3 + kw];
          const f32x2 ww = {wt, wt};
          a01 = __builtin_elementwise_fma(ww, f32x2{v[ci][kh][kw], v[ci][kh][kw + 1]}, a01);
          a23 = __builtin_elementwise_fma(ww, f32x2{v[ci][kh][kw + 2], v[ci][kh][kw + 3]}, a23);
        }
    f32x4 r = {a01[0], a01[1], a23[0], a23[1]};
    if (relu) {
#pragma unroll
      for (int e = 0; e < 4; ++e) r[e] = fmaxf(r[e], 0.f);
    }
    *reinterpret_cast<f32x4*>(o + co * cstride) = r;
  }
}

extern "C" {

int vst_conv_gemm(const float* src, const float* wpack, const float* bias, const float* mask, float* out, int N,
                  int Cs, int Hs, int Ws, int M, int K, int Ho, int Wo, int KH, int KW, int gmode, int stride, int pad,
                  int up, int epi, long a_batch_stride, float* aux, const float* gmask, void* workspace, long ws_bytes,
                  int mode, void* stream) {
  VST_CHECK_ARG(vst_mode_ok(mode));
  return vst_conv_gemm_padx(src, wpack, bias, mask, out, N, Cs, Hs, Ws, M, K, Ho, Wo, KH, KW, gmode, stride, pad, pad,
                            up, epi, a_batch_stride, aux, gmask, workspace, ws_bytes, mode, stream);
}

long vst_conv_splitk_workspace(int N, int Cs, int M, int Ho, int Wo, int KH, int KW, int gmode, int stride, int pad,
                               int pad_x, int up, int epi, long a_batch_stride, int mode) {
  if (!vst_mode_ok(mode) || N <= 0 || Cs <= 0 || M <= 0 || Ho <= 0 || Wo <= 0) return 0;
  const HaloPlan hp = halo_plan(N, Cs, M, Ho, Wo, KH, KW, gmode, stride, pad, pad_x, up, epi, a_batch_stride, mode);
  return hp.hcfg ? splitk_bytes(hp, N, M, Ho, Wo) : 0;
}

int vst_conv_gemm_padx(const float* src, const float* wpack, const float* bias, const float* mask, float* out, int N,
                       int Cs, int Hs, int Ws, int M, int K, int Ho, int Wo, int KH, int KW, int gmode, int stride,
                       int pad, int pad_x, int up, int epi, long a_batch_stride, float* aux, const float* gmask,
                       void* workspace, long ws_bytes, int mode, void* stream) {
  VST_CHECK_ARG(vst_mode_ok(mode));
  VST_CHECK_ARG(ws_bytes >= 0 && (workspace || ws_bytes == 0));
  VST_CHECK_ARG(src && wpack && out && N > 0 && Cs > 0 && Hs > 0 && Ws > 0 && M > 0 && Ho > 0 && Wo > 0);
  VST_CHECK_ARG(K == KH * KW * Cs && KH > 0 && KW > 0);
  VST_CHECK_ARG(gmode >= 0 && gmode <= 2 && (stride == 1 || stride == 2) && (up == 1 || up == 2));
  VST_CHECK_ARG(!((epi & EPI_BIAS) && !bias) && !((epi & EPI_MASK) && !mask));
  if (gmode == GM_REFLECT) VST_CHECK_ARG(pad < Hs * up && pad_x < Ws * up);
  VST_CHECK_ARG(pad >= 0 && pad_x >= 0);
  VST_CHECK_ARG(a_batch_stride == 0 || a_batch_stride >= apack_floats(M, K, mode));
  return conv_gemm_launch(src, wpack, bias, mask, out, N, Cs, Hs, Ws, M, K, Ho, Wo, KH, KW, gmode, stride, pad, pad_x,
                          up, epi, a_batch_stride, aux, gmask, mode, stream, nullptr, nullptr, nullptr, nullptr,
                          nullptr, 0, 0, 0, workspace, ws_bytes);
}

// out[n][m][p] = (sum_k A[n][k][m] B[n][k][p] + ra[n][m]) * rb[n][m] * cg[n][p] + rd[n][m]
// (A packed per image, a_batch_stride floats apart; B = src [N][K][P]; ra, rd may be NULL)
int vst_attn_gemm(const float* src, const float* apack, float* out, int N, int K, int P, int M, long a_batch_stride,
                  const float* ra, const float* rb, const float* rd, const float* cg, int mode, void* stream) {
  VST_CHECK_ARG(vst_mode_ok(mode));
  VST_CHECK_ARG(src && apack && out && rb && cg && N > 0 && K > 0 && P > 0 && M > 0);
  VST_CHECK_ARG(a_batch_stride == 0 || a_batch_stride >= apack_floats(M, K, mode));
  return conv_gemm_launch(src, apack, nullptr, nullptr, out, N, K, 1, P, M, K, 1, P, 1, 1, GM_ZERO, 1, 0, 0, 1,
                          EPI_AFFINE, a_batch_stride, nullptr, nullptr, mode, stream, ra, rb, rd, cg);
}

int vst_pack_weight_phase2(const float* w, float* packed, int Cout, int Cin, int KS, int Mpad, int Kpad,
                           int mode, void* stream) {
  VST_CHECK_ARG(vst_mode_ok(mode));
  VST_CHECK_ARG(w && packed && Cout > 0 && Cin > 0 && KS > 0 && Mpad >= 4 * Cin);
  VST_CHECK_ARG(Kpad >= (KS + 1) / 2 * ((KS + 1) / 2) * Cout);
  long total = (long)Mpad * Kpad;
  pack_phase2_kernel<<<ceil_div(total, 256), 256, 0, (hipStream_t)stream>>>(
      w, packed, Cout, Cin, KS, Mpad, Kpad, apack_split(mode));
  return vst_launch_status();
}

int vst_conv_dgrad_s2(const float* dy, const float* wpack, const float* gmask, float* dx, float* border, int N,
                      int Cout, int Ho, int Wo, int Cin, int H, int W, int KS, int pad, int mode, void* stream) {
  VST_CHECK_ARG(vst_mode_ok(mode));
  VST_CHECK_ARG(dy && wpack && dx && border && N > 0 && Cout > 0 && Ho > 0 && Wo > 0 && Cin > 0 && KS > 0);
  VST_CHECK_ARG(pad >= 0 && pad < H && pad < W && Ho == (H + 2 * pad - KS) / 2 + 1 && Wo == (W + 2 * pad - KS) / 2 + 1);
  const int K2 = (KS + 1) / 2;
  const int Hc = (H + 2 * pad + 1) / 2, Wc = (W + 2 * pad + 1) / 2;
  return conv_gemm_launch(dy, wpack, nullptr, nullptr, dx, N, Cout, Ho, Wo, 4 * Cin, K2 * K2 * Cout, Hc, Wc, K2, K2,
                          GM_TRANSPOSED, 1, 0, 0, 1, EPI_PHASE2, 0, nullptr, gmask, mode, stream, nullptr, nullptr, nullptr,
                          nullptr, border, H, W, pad);
}

// Forward of nearest-x2 upsample -> ReflectionPad2d(1) -> Conv2d(k3, stride 1) (UpsampleConvLayer,
// RC/network.py:114-120) as ONE phase-stacked 2x2 GEMM on the source grid: output pixel (2i'-a, 2j'-b)
// = sum_{eh,ew,ci} W2[(co, 1-a, 1-b)][ci][eh][ew] * x[ci][clamp(i'-1+eh)][clamp(j'-1+ew)] over the
// (H+1) x (W+1) grid of (i', j'); the reflect border of the virtual grid is the edge clamp, W2 holds
// the phase's tap sums (vst_up2_phase_weights).  16 instead of 36 MACs per (co, ci, source pixel);
// the EPI_PHASE2 epilogue scatters the four phase rows of each channel to their output pixels (+bias).
__global__ void up2_phase_weights_kernel(const float* __restrict__ w, float* __restrict__ w2, int Cout, int Cin) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;  // over [Cout][4][Cin][2][2]
  const long total = (long)Cout * 16 * Cin;
  if (idx >= total) return;
  const int ew = (int)(idx & 1), eh = (int)((idx >> 1) & 1);
  long t = idx >> 2;
  const int ci = (int)(t % Cin);
  t /= Cin;
  const int ph = (int)(t & 3), co = (int)(t >> 2);
  const int a = 1 - (ph >> 1), b = 1 - (ph & 1);  // row phase (a', b') = (1-a, 1-b)
  const float* wc = w + ((long)co * Cin + ci) * 9;
  float s = 0.f;
  for (int kh = 0; kh < 3; ++kh) {
    if (((a + kh + 1) >> 1) - a != eh) continue;
    for (int kw = 0; kw < 3; ++kw)
      if (((b + kw + 1) >> 1) - b == ew) s += wc[kh * 3 + kw];
  }
  w2[idx] = s;
}

int vst_up2_phase_weights(const float* w, float* w2, int Cout, int Cin, void* stream) {
  VST_CHECK_ARG(w && w2 && Cout > 0 && Cin > 0);
  const long total = (long)Cout * 16 * Cin;
  up2_phase_weights_kernel<<<ceil_div(total, 256), 256, 0, (hipStream_t)stream>>>(w, w2, Cout, Cin);
  return vst_launch_status();
}

int vst_conv_up2_fwd(const float* x, const float* wpack, const float* bias, float* out, int N, int Cin, int H, int W,
                     int Cout, int mode, void* stream) {
  VST_CHECK_ARG(vst_mode_ok(mode));
  VST_CHECK_ARG(x && wpack && out && N > 0 && Cin > 0 && H > 0 && W > 0 && Cout > 0);
  return conv_gemm_launch(x, wpack, bias, nullptr, out, N, Cin, H, W, 4 * Cout, 4 * Cin, H + 1, W + 1, 2, 2, GM_CLAMP,
                          1, 1, 1, 1, EPI_PHASE2 | (bias ? EPI_BIAS : 0), 0, nullptr, nullptr, mode, stream, nullptr,
                          nullptr, nullptr, nullptr, nullptr, 2 * H, 2 * W, 1);
}

int vst_conv_cin3_k3(const float* x, const float* w, const float* b, float* out, int N, int H, int W, int Cout,
                     int reflect, int relu, void* stream) {
  VST_CHECK_ARG(x && w && out && N > 0 && H > 1 && W > 1 && Cout > 0);
  hipStream_t st = (hipStream_t)stream;
  if (W % 4 == 0 && W >= 8 && (((uintptr_t)x | (uintptr_t)out) & 15) == 0) {
    dim3 g4(ceil_div(W / 4, 256), H, N);
    if (reflect) cin3_conv3_x4_kernel<true><<<g4, 256, 0, st>>>(x, w, b, out, H, W, Cout, relu);
    else cin3_conv3_x4_kernel<false><<<g4, 256, 0, st>>>(x, w, b, out, H, W, Cout, relu);
    return vst_launch_status();
  }
  dim3 grid(ceil_div(W, 256), H, N);
  if (reflect) cin3_conv3_kernel<true><<<grid, 256, 0, st>>>(x, w, b, out, H, W, Cout, relu);
  else cin3_conv3_kernel<false><<<grid, 256, 0, st>>>(x, w, b, out, H, W, Cout, relu);
  return vst_launch_status();
}

int vst_unfold_kw(const float* src, float* out, int N, int C, int H, int Ws, int Wout, int K, int Cu, int sgn, int off,
                  int reflect, void* stream) {
  VST_CHECK_ARG(src && out && N > 0 && C > 0 && H > 0 && Ws > 0 && Wout > 0 && K > 0 && Cu >= C * K);
  VST_CHECK_ARG((sgn == 1 || sgn == -1) && !(reflect && Ws < 2) && Wout % 4 == 0);
  const int Cg = (Cu + K - 1) / K;
  VST_CHECK_ARG((long)N * Cu * H < (1L << 31));
  const long rows = (long)N * Cg * H;
  const unsigned gy = (unsigned)(rows < 65535 ? rows : 65535);
  // block = the row's float4 columns rounded up to whole wavefronts (at most 256)
  const int bx = (Wout / 4 + 63) / 64 * 64 < 256 ? (Wout / 4 + 63) / 64 * 64 : 256;
  dim3 g(ceil_div(Wout / 4, bx), gy, (unsigned)((rows + gy - 1) / gy));
  unfold_kw_kernel<<<g, bx, 0, (hipStream_t)stream>>>(src, out, N, C, H, Ws, Wout, K, Cu, Cg, sgn, off, reflect);
  return vst_launch_status();
}

int vst_tapsum(const float* P, float* dx, int N, int C, int H, int W, int K, int pad, int accumulate, void* stream) {
  VST_CHECK_ARG(P && dx && N > 0 && C > 0 && H > 0 && W > 0 && K > 0 && pad >= 0);
  const long total = (long)N * C * H * W;
  tapsum_kernel<<<ceil_div(total, 256), 256, 0, (hipStream_t)stream>>>(P, dx, N, C, H, W, K, pad, accumulate);
  return vst_launch_status();
}

int vst_pack_weight_kwu(const float* w, float* packed, int Cout, int Cin, int K, int Cu, int transposed, int Mpad,
                        int Kpad, int mode, void* stream) {
  VST_CHECK_ARG(vst_mode_ok(mode));
  VST_CHECK_ARG(w && packed && Cout > 0 && Cin > 0 && K > 0 && Cu >= (transposed ? Cout : Cin) * K);
  VST_CHECK_ARG(Mpad >= (transposed ? Cin : Cout) && Kpad >= K * Cu);
  const long total = (long)Mpad * Kpad;
  pack_kwu_kernel<<<ceil_div(total, 256), 256, 0, (hipStream_t)stream>>>(w, packed, Cout, Cin, K, Cu, transposed, Mpad,
                                                                         Kpad, apack_split(mode));
  return vst_launch_status();
}

int vst_conv_dgrad_padout_kwu(const float* dyu, const float* wpack, const float* mask, float* dx, float* border, int N,
                              int Cu, int Ho, int Cin, int H, int W, int KS, int pad, int mode, void* stream) {
  VST_CHECK_ARG(vst_mode_ok(mode));
  VST_CHECK_ARG(dyu && wpack && dx && border && N > 0 && Cu % 16 == 0 && Cin > 0 && KS > 0 && pad >= 0 && pad < H &&
                pad < W && Ho == H + 2 * pad - KS + 1);
  // dyu rows are Wu = Wp rounded up to 4 wide (vst_unfold_kw's float4 rows); the GEMM covers Wp columns
  const int Hp = H + 2 * pad, Wp = W + 2 * pad, Wu = (Wp + 3) / 4 * 4;
  return conv_gemm_launch(dyu, wpack, nullptr, mask, dx, N, Cu, Ho, Wu, Cin, KS * Cu, Hp, Wp, KS, 1, GM_TRANSPOSED, 1,
                          0, 0, 1, EPI_PADOUT | (mask ? EPI_MASK : 0), 0, nullptr, nullptr, mode, stream, nullptr,
                          nullptr, nullptr, nullptr, border, H, W, pad);
}

int vst_conv_dgrad_padout(const float* dy, const float* wpack, const float* mask, float* dx, float* border, int N,
                          int Cout, int Ho, int Wo, int Cin, int H, int W, int KS, int pad, void* workspace,
                          long ws_bytes, int mode, void* stream) {
  VST_CHECK_ARG(vst_mode_ok(mode));
  VST_CHECK_ARG(ws_bytes >= 0 && (workspace || ws_bytes == 0));
  VST_CHECK_ARG(dy && wpack && dx && border && N > 0 && Cout > 0 && Cin > 0 && KS > 0 && pad >= 0 && pad < H &&
                pad < W && Ho == H + 2 * pad - KS + 1 && Wo == W + 2 * pad - KS + 1);
  return conv_gemm_launch(dy, wpack, nullptr, mask, dx, N, Cout, Ho, Wo, Cin, KS * KS * Cout, H + 2 * pad,
                          W + 2 * pad, KS, KS, GM_TRANSPOSED, 1, 0, 0, 1, EPI_PADOUT | (mask ? EPI_MASK : 0), 0, nullptr,
                          nullptr, mode, stream, nullptr, nullptr, nullptr, nullptr, border, H, W, pad, workspace,
                          ws_bytes);
}

int vst_fold_border(const float* border, const float* mask, float* dx, long NC, int H, int W, int pad, void* stream) {
  VST_CHECK_ARG(border && dx && NC > 0 && H > 0 && W > 0 && pad >= 0 && pad < H && pad < W);
  if (pad == 0) return VST_OK;
  const int nb = pad < H / 2 ? pad + 1 : H, nbc = pad < W / 2 ? pad + 1 : W;
  const int br = nb >= H ? H : 2 * nb, bc = nbc >= W ? W : 2 * nbc;
  const long total = ((long)br * W + (long)(H - br) * bc) * NC;
  fold_border_kernel<<<ceil_div(total, 256), 256, 0, (hipStream_t)stream>>>(border, mask, dx, (int)NC, H, W, pad);
  return vst_launch_status();
}

int vst_fold_reflect(const float* dpad, float* dx, long NC, int Hs, int Ws, int pad, int up, int accumulate,
                     void* stream) {
  VST_CHECK_ARG(dpad && dx && NC > 0 && Hs > 0 && Ws > 0 && pad >= 0 && (up == 1 || up == 2));
  dim3 g(ceil_div((long)Hs * Ws, 256), (unsigned)(NC < 65535 ? NC : 65535));
  fold_reflect_kernel<<<g, 256, 0, (hipStream_t)stream>>>(dpad, dx, (int)NC, Hs, Ws, pad, up, accumulate);
  return vst_launch_status();
}

}  // extern "C"

// ---------------------------------------------------------------------------------------------
// Row-split forward for convs with few output channels (ConvTanh 48->3, k9, RC/network.py:169):
// the GEMM computes P[(co,kh)][q_y][x] = sum_{ci,kw} W[co][ci][kh][kw] Xpad[ci][q_y][x+kw] over the
// (H+KH-1) padded rows (27 useful rows of 32 instead of 3), this kernel finishes
//   out[co][y][x] = epi(bias[co] + sum_kh P[(co,kh)][y+kh][x])
namespace {
__global__ void rowsplit_reduce_kernel(const float* __restrict__ P, const float* __restrict__ bias,
                                       float* __restrict__ out, float* __restrict__ aux, int N, int Cout, int KH, int H,
                                       int W, int epi) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)N * Cout * H * W;
  if (idx >= total) return;
  int x = (int)(idx % W);
  long t = idx / W;
  int y = (int)(t % H);
  t /= H;
  int co = (int)(t % Cout);
  long n = t / Cout;
  const int Hq = H + KH - 1;
  const float* p = P + ((n * Cout + co) * KH * (long)Hq + y) * W + x;
  float s = 0.f;
  for (int kh = 0; kh < KH; ++kh) s += p[((long)kh * Hq + kh) * W];
  float v = s;
  if (epi & EPI_BIAS) v += bias[co];
  if (epi & EPI_RELU) v = fmaxf(v, 0.f);
  if (epi & EPI_TANH) {
    const float th = tanhf(v / 255.0f);
    if (aux) aux[idx] = th;
    v = th * 150.0f + 127.5f;
  }
  out[idx] = v;
}
}  // namespace

extern "C" int vst_rowsplit_reduce(const float* P, const float* bias, float* out, float* aux, int N, int Cout, int KH,
                                   int H, int W, int epi, void* stream) {
  VST_CHECK_ARG(P && out && N > 0 && Cout > 0 && KH > 0 && H > 0 && W > 0 && !((epi & EPI_BIAS) && !bias));
  long total = (long)N * Cout * H * W;
  rowsplit_reduce_kernel<<<ceil_div(total, 256), 256, 0, (hipStream_t)stream>>>(P, bias, out, aux, N, Cout, KH, H, W,
                                                                                epi);
  return vst_launch_status();
}

// ---------------------------------------------------------------------------------------------
// Reflect-pad data gradient without the padded grid (RC/network.py:72-75 ConvLayer and
// :114-120 UpsampleConvLayer backward).  dXpad = full correlation of dY with the flipped
// weights over the padded (virtual, upsampled) grid; dX = fold of dXpad.  Split:
//   * core: the directly-mapped part, one GEMM on the UNPADDED grid (rows aligned with the
//     activations; for nearest x2 upsampling the 2x2 fold is folded into a stride-2 GEMM with
//     (KS+1)^2 tap-summed weights, 2.25x fewer MACs than the upsampled-grid GEMM);
//   * ring: the p-wide border of dXpad (reflected copies), computed here and folded into the
//     2p-wide border band of dX.
namespace {

// Summed-tap packed weight for the up=2 core: W'[jh][jw] = sum W[kh][kw] over
// kh in {KS-1-jh, KS-jh}, kw in {KS-1-jw, KS-jw} (valid ones); transposed A: m = ci, k = (jh*(KS+1)+jw)*Cout + co
__global__ void pack_upsum_kernel(const float* __restrict__ w, float* __restrict__ out, int Cout, int Cin, int KS,
                                  int Mpad, int Kpad, int bsplit) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)Mpad * Kpad) return;
  const int m = (int)(idx % Mpad);
  const int k = (int)(idx / Mpad);
  const int KU = KS + 1;
  float v = 0.f;
  if (m < Cin && k < KU * KU * Cout) {
    int tap, co;
    kdecode(k, Cout, KU * KU, tap, co, bsplit >> 4);
    const int jh = tap / KU, jw = tap % KU;
    const float* wp = w + ((long)co * Cin + m) * KS * KS;
    for (int a = 0; a < 2; ++a) {
      const int kh = KS - 1 - jh + a;
      if (kh < 0 || kh >= KS) continue;
      for (int b = 0; b < 2; ++b) {
        const int kw = KS - 1 - jw + b;
        if (kw < 0 || kw >= KS) continue;
        v += wp[kh * KS + kw];
      }
    }
  }
  apack_store(out, k, m, Mpad, v, bsplit);
}

// The ring of the padded-grid gradient, stored as four segments (each written by one GEMM):
// top [NC][p][Wv+2p], bottom [NC][p][Wv+2p], left [NC][Hv][p], right [NC][Hv][p].
struct Ring {
  const float *top, *bot, *left, *right;
  int Hv, Wv, p, S;
  long slab;  // floats between split-K slabs
};

// value of padded-grid position (u, v) if it lies on the ring (returns false for core positions)
__device__ __forceinline__ bool ring_at(const Ring& R, long nc, int u, int v, float& val) {
  const int p = R.p, Wp = R.Wv + 2 * p;
  const float* q;
  if (u < p) {
    q = R.top + (nc * p + u) * Wp + v;
  } else if (u >= R.Hv + p) {
    q = R.bot + (nc * p + (u - R.Hv - p)) * Wp + v;
  } else if (v < p) {
    q = R.left + (nc * R.Hv + (u - p)) * p + v;
  } else if (v >= R.Wv + p) {
    q = R.right + (nc * R.Hv + (u - p)) * p + (v - R.Wv - p);
  } else {
    return false;
  }
  float a = 0.f;
  for (int z = 0; z < R.S; ++z) a += q[z * R.slab];
  val = a;
  return true;
}

// dx (+)= ring contributions, for the border band of dX only (each element written by one thread)
__global__ void fold_ring_kernel(Ring RG, float* __restrict__ dx, int NC, int Hs, int Ws, int up, int bt, int bb,
                                 int ct, int cb) {
  const int nb = (bt + bb) * Ws + (Hs - bt - bb) * (ct + cb);
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nb) return;
  int y, x;
  if (t < bt * Ws) {
    y = t / Ws;
    x = t % Ws;
  } else if (t < (bt + bb) * Ws) {
    y = Hs - bb + (t - bt * Ws) / Ws;
    x = (t - bt * Ws) % Ws;
  } else {
    const int q = t - (bt + bb) * Ws;
    y = bt + q / (ct + cb);
    const int c = q % (ct + cb);
    x = c < ct ? c : Ws - cb + (c - ct);
  }
  const int p = RG.p;
  for (int nc = blockIdx.y; nc < NC; nc += gridDim.y) {
    float s = 0.f;
    for (int dy = 0; dy < up; ++dy) {
      const Src3 ry = reflect_sources(y * up + dy, RG.Hv, p);
      for (int dxx = 0; dxx < up; ++dxx) {
        const Src3 cx = reflect_sources(x * up + dxx, RG.Wv, p);
        const int us[3] = {ry.a, ry.b, ry.c};
        const int vs[3] = {cx.a, cx.b, cx.c};
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
          for (int j = 0; j < 3; ++j) {
            float v;
            if (us[i] >= 0 && vs[j] >= 0 && ring_at(RG, nc, us[i], vs[j], v)) s += v;
          }
      }
    }
    dx[((long)nc * Hs + y) * Ws + x] += s;
  }
}

// Ring of the padded-grid gradient as 4p lines (top rows, bottom rows, left and right columns of
// the border), each a small GEMM  out[ci][i] = sum_{co, taps} W[co][ci][kh][kw] dY[co][u_i-kh][v_i-kw]
// over the taps that can reach the line (rows: kh <= u resp. kh >= u-Hv+1; columns: kw likewise).
// Block: 64 positions x 64 input channels, 16-deep k-chunks staged in LDS, 4x4 outputs per thread.
__global__ __launch_bounds__(256) void dgrad_ring_kernel(const float* __restrict__ dy, const float* __restrict__ w,
                                                         float* __restrict__ ring, int N, int Cout, int Cin, int KS,
                                                         int Hv, int Wv, int S) {
  __shared__ float As[16][64 + 4];
  __shared__ float Bs[16][64 + 4];
  const int p = KS / 2, Wp = Wv + 2 * p;
  const int line = blockIdx.z % (4 * p), sidx = (blockIdx.z / (4 * p)) % S, n = blockIdx.z / (4 * p * S);
  const int seg = line / p, li = line % p;  // 0 top, 1 bottom, 2 left, 3 right
  const int len = seg < 2 ? Wp : Hv;
  const int i0 = blockIdx.x * 64, ci0 = blockIdx.y * 64;
  if (i0 >= len) return;
  // line geometry: position i -> (u, v)
  const int u0 = seg == 0 ? li : (seg == 1 ? Hv + p + li : p);
  const int v0 = seg == 2 ? li : (seg == 3 ? Wv + p + li : 0);
  const int du = seg < 2 ? 0 : 1, dv = seg < 2 ? 1 : 0;
  int kh0 = 0, kh1 = KS - 1, kw0 = 0, kw1 = KS - 1;
  if (seg == 0) kh1 = u0;
  if (seg == 1) kh0 = u0 - Hv + 1;
  if (seg == 2) kw1 = v0;
  if (seg == 3) kw0 = v0 - Wv + 1;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  float acc[4][4] = {};
  const long dplane = (long)Hv * Wv;
  const float* dyn = dy + (long)n * Cout * dplane;
  // loader roles: A: co row = t>>4 (16), ci = (t&15)*4..+3 ; B: co row = t>>4, positions (t&15)*4..+3
  const int lr = threadIdx.x >> 4, lc = (threadIdx.x & 15) * 4;
  // flattened (kh, kw, co-chunk) iteration space, split S ways across blocks (slab sidx)
  const int nch = (Cout + 15) / 16, nkw = kw1 - kw0 + 1;
  const int T = (kh1 - kh0 + 1) * nkw * nch;
  const int t0 = (int)((long)T * sidx / S), t1 = (int)((long)T * (sidx + 1) / S);
  for (int it = t0; it < t1; ++it) {
        const int cch = it % nch, tap = it / nch;
        const int kh = kh0 + tap / nkw, kw = kw0 + tap % nkw;
        const int co = cch * 16 + lr;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int ci = ci0 + lc + j;
          As[lr][lc + j] = (co < Cout && ci < Cin) ? w[(((long)co * Cin + ci) * KS + kh) * KS + kw] : 0.f;
          const int i = i0 + lc + j;
          const int uu = u0 + du * i - kh, vv = v0 + dv * i - kw;
          const bool ok = co < Cout && i < len && uu >= 0 && uu < Hv && vv >= 0 && vv < Wv;
          Bs[lr][lc + j] = ok ? dyn[co * dplane + (long)uu * Wv + vv] : 0.f;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const float4 a = *reinterpret_cast<const float4*>(&As[k][ty * 4]);
          const float4 bq = *reinterpret_cast<const float4*>(&Bs[k][tx * 4]);
          const float av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {bq.x, bq.y, bq.z, bq.w};
#pragma unroll
          for (int x = 0; x < 4; ++x)
#pragma unroll
            for (int y = 0; y < 4; ++y) acc[x][y] += av[x] * bv[y];
        }
      }
  // segment layout: top/bottom [NC][p][Wp], left/right [NC][Hv][p]; slab sidx after the others
  const long NC = (long)N * Cin;
  const long segtb = (long)p * Wp, seglr = (long)Hv * p;
  ring += (long)sidx * NC * (2 * segtb + 2 * seglr);
#pragma unroll
  for (int x = 0; x < 4; ++x) {
    const int ci = ci0 + ty * 4 + x;
    if (ci >= Cin) continue;
    const long nc = (long)n * Cin + ci;
#pragma unroll
    for (int y = 0; y < 4; ++y) {
      const int i = i0 + tx * 4 + y;
      if (i >= len) continue;
      long o;
      if (seg == 0) o = nc * segtb + (long)li * Wp + i;
      else if (seg == 1) o = NC * segtb + nc * segtb + (long)li * Wp + i;
      else if (seg == 2) o = 2 * NC * segtb + nc * seglr + (long)i * p + li;
      else o = 2 * NC * segtb + NC * seglr + nc * seglr + (long)i * p + li;
      ring[o] = acc[x][y];
    }
  }
}

}  // namespace

extern "C" {

int vst_pack_weight_upsum(const float* w, float* packed, int Cout, int Cin, int KS, int Mpad, int Kpad, int mode, void* stream) {
  VST_CHECK_ARG(vst_mode_ok(mode));
  VST_CHECK_ARG(w && packed && Cout > 0 && Cin > 0 && KS > 0 && Mpad >= Cin && Kpad >= (KS + 1) * (KS + 1) * Cout);
  long total = (long)Mpad * Kpad;
  pack_upsum_kernel<<<ceil_div(total, 256), 256, 0, (hipStream_t)stream>>>(w, packed, Cout, Cin, KS, Mpad, Kpad,
                                                                           apack_split(mode));
  return vst_launch_status();
}

// split-K ways of the ring GEMMs: <= ~8 k-chunk iterations per block
int vst_dgrad_ring_splits(int Cout, int KS) {
  const int p = KS / 2;
  const long tmax = (long)(p + 1) * KS * ((Cout + 15) / 16);
  long S = (tmax + 7) / 8;
  return (int)(S < 1 ? 1 : (S > 8 ? 8 : S));
}

// floats per (n, ci) plane of the ring buffer, all split-K slabs included
long vst_dgrad_ring_size(int Hv, int Wv, int KS, int Cout) {
  const int p = KS / 2;
  return (2L * p * (Wv + 2 * p) + 2L * Hv * p) * vst_dgrad_ring_splits(Cout, KS);
}

// ring = N*Cin*vst_dgrad_ring_size floats (segment layout of fold_ring_kernel)
int vst_dgrad_ring(const float* dy, const float* w, float* ring, int N, int Cout, int Cin, int KS, int Hv, int Wv,
                   void* stream) {
  VST_CHECK_ARG(dy && w && ring && N > 0 && Cout > 0 && Cin > 0 && (KS & 1) && KS > 1 && Hv > KS && Wv > KS);
  const int p = KS / 2, S = vst_dgrad_ring_splits(Cout, KS);
  VST_CHECK_ARG((long)N * 4 * p * S <= 65535);
  dim3 g(ceil_div(max(Wv + 2 * p, Hv), 64), ceil_div(Cin, 64), N * 4 * p * S);
  dgrad_ring_kernel<<<g, 256, 0, (hipStream_t)stream>>>(dy, w, ring, N, Cout, Cin, KS, Hv, Wv, S);
  return vst_launch_status();
}

int vst_fold_ring(const float* ring, float* dx, long NC, int Hs, int Ws, int KS, int up, int Cout, void* stream) {
  const int p = KS / 2;
  VST_CHECK_ARG(ring && dx && NC > 0 && (up == 1 || up == 2) && (KS & 1) && KS > 1);
  const int Hv = Hs * up, Wv = Ws * up;
  // virtual rows with reflected sources: [1, p] and [Hv-1-p, Hv-2]
  const int bt = p / up + 1, bb = Hs - (Hv - 1 - p) / up;
  const int ct = p / up + 1, cb = Ws - (Wv - 1 - p) / up;
  VST_CHECK_ARG(bt + bb <= Hs && ct + cb <= Ws && Hv > 2 * p + 1 && Wv > 2 * p + 1);
  const int Wp = Wv + 2 * p;
  Ring RG;
  RG.top = ring;
  RG.bot = RG.top + NC * p * Wp;
  RG.left = RG.bot + NC * p * Wp;
  RG.right = RG.left + NC * Hv * p;
  RG.Hv = Hv;
  RG.Wv = Wv;
  RG.p = p;
  RG.S = vst_dgrad_ring_splits(Cout, KS);
  RG.slab = NC * (2L * p * Wp + 2L * Hv * p);
  const int nb = (bt + bb) * Ws + (Hs - bt - bb) * (ct + cb);
  dim3 g(ceil_div(nb, 256), (unsigned)(NC < 65535 ? NC : 65535));
  fold_ring_kernel<<<g, 256, 0, (hipStream_t)stream>>>(RG, dx, (int)NC, Hs, Ws, up, bt, bb, ct, cb);
  return vst_launch_status();
}

}  // extern "C"
