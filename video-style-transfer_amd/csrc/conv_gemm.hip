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
// K is ordered tap-major / channel-minor, k = (kh*KS + kw)*Cs + c, so when Cs % 16 == 0 a whole
// 16-deep k-tile shares one tap and the reflect/zero/upsample index math is done once per tile.
//
// Tile: 4 waves (256 threads); each wave owns TM x TN 32x32 accumulators (WM x WN waves).
// LDS: A[BK][BM] and B[BK][BN], double buffered; global->register prefetch of tile t+1 overlaps
// the MFMAs of tile t; one barrier per k-tile.
#include "vst_common.h"
#include "vst_hip.h"

namespace {

constexpr int BK = 16;
constexpr int NT = 256;

struct ConvParams {
  const float* src;
  const float* wpack;
  const float* bias;
  const float* mask;
  const float* gmask;
  float* out;
  float* aux;
  long a_batch_stride;
  int Cs, Hs, Ws;
  int M, Mpad, K, Kpad;
  int Ho, Wo;
  int KS, gmode, stride, pad, up;
  int epi;
  FastDiv fd_Wo, fd_Cs, fd_KS;
};

enum { GM_REFLECT = 0, GM_ZERO = 1, GM_TRANSPOSED = 2 };
enum { EPI_BIAS = 1, EPI_RELU = 2, EPI_TANH = 4, EPI_MASK = 8, EPI_ACCUM = 16 };

// source offset (within one channel plane) of tap (kh,kw) for output pixel (oy,ox); -1 if zero
__device__ __forceinline__ int gather_offset(const ConvParams& P, int oy, int ox, int kh, int kw) {
  if (P.gmode == GM_TRANSPOSED) {
    int ty = oy + P.pad - kh, tx = ox + P.pad - kw;
    if (ty < 0 || tx < 0) return -1;
    if (P.stride == 2) {
      if ((ty | tx) & 1) return -1;
      ty >>= 1;
      tx >>= 1;
    }
    if (ty >= P.Hs || tx >= P.Ws) return -1;
    return ty * P.Ws + tx;
  }
  int Hv = P.Hs * P.up, Wv = P.Ws * P.up;
  int y = oy * P.stride + kh - P.pad, x = ox * P.stride + kw - P.pad;
  if (P.gmode == GM_REFLECT) {
    y = y < 0 ? -y : y;
    y = y >= Hv ? 2 * Hv - 2 - y : y;
    x = x < 0 ? -x : x;
    x = x >= Wv ? 2 * Wv - 2 - x : x;
  } else if (y < 0 || y >= Hv || x < 0 || x >= Wv) {
    return -1;
  }
  if (P.up == 2) {
    y >>= 1;
    x >>= 1;
  }
  return y * P.Ws + x;
}

template <int WM, int TM, int WN, int TN, bool CFAST>
__global__ __launch_bounds__(NT) void conv_gemm_kernel(ConvParams P) {
  constexpr int BM = WM * TM * 32;
  constexpr int BN = WN * TN * 32;
  constexpr int A_F4 = BK * BM / 4;          // float4 per A tile
  constexpr int A_PER = (A_F4 + NT - 1) / NT;
  constexpr int ROWSTEP = NT / BN;           // B rows covered per pass
  constexpr int B_PER = BK / ROWSTEP;        // B elements per thread per tile
  static_assert(NT % BN == 0 && BK % ROWSTEP == 0, "tile");

  __shared__ float As[2][BK][BM];
  __shared__ float Bs[2][BK][BN];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int lo = lane & 31, hi = lane >> 5;
  const int wm = wave / WN, wn = wave % WN;
  const int n = blockIdx.z;
  const int m0 = blockIdx.y * BM;
  const int p0 = blockIdx.x * BN;
  const int HWo = P.Ho * P.Wo;
  const long plane = (long)P.Hs * P.Ws;
  const float* src_n = P.src + (long)n * P.Cs * plane;
  const float* gm_n = P.gmask ? P.gmask + (long)n * P.Cs * plane : nullptr;
  const float* A = P.wpack + (long)n * P.a_batch_stride;

  // this thread's B column (fixed for the whole k loop)
  const int bcol = tid % BN;
  const int brow0 = tid / BN;
  const int p = p0 + bcol;
  const bool pvalid = p < HWo;
  int oy = 0, ox = 0;
  if (pvalid) {
    oy = (int)fdiv((uint32_t)p, P.fd_Wo);
    ox = p - oy * P.Wo;
  }

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  float4 ra[A_PER];
  float rb[B_PER];
  const int ntiles = P.Kpad / BK;

  auto load_tile = [&](int t) {
    const int k0 = t * BK;
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      int idx = tid + i * NT;
      if (idx < A_F4) {
        int kk = idx / (BM / 4), mm = (idx % (BM / 4)) * 4;
        ra[i] = *reinterpret_cast<const float4*>(A + (long)(k0 + kk) * P.Mpad + m0 + mm);
      }
    }
    if (CFAST) {
      // whole tile shares one tap (Cs % BK == 0): scalar tap decode, one offset per thread
      const int tap = k0 / P.Cs;
      const int c0 = k0 - tap * P.Cs;
      const int kh = tap / P.KS, kw = tap - (tap / P.KS) * P.KS;
      int off = pvalid ? gather_offset(P, oy, ox, kh, kw) : -1;
      const long base = (long)(c0 + brow0) * plane + off;
#pragma unroll
      for (int i = 0; i < B_PER; ++i) {
        float v = 0.f;
        if (off >= 0) {
          v = src_n[base + (long)i * ROWSTEP * plane];
          if (gm_n && !(gm_n[base + (long)i * ROWSTEP * plane] > 0.f)) v = 0.f;
        }
        rb[i] = v;
      }
    } else {
#pragma unroll
      for (int i = 0; i < B_PER; ++i) {
        int k = k0 + brow0 + i * ROWSTEP;
        float v = 0.f;
        if (pvalid && k < P.K) {
          int tap = (int)fdiv((uint32_t)k, P.fd_Cs);
          int c = k - tap * P.Cs;
          int kh = (int)fdiv((uint32_t)tap, P.fd_KS);
          int kw = tap - kh * P.KS;
          int off = gather_offset(P, oy, ox, kh, kw);
          if (off >= 0) {
            v = src_n[(long)c * plane + off];
            if (gm_n && !(gm_n[(long)c * plane + off] > 0.f)) v = 0.f;
          }
        }
        rb[i] = v;
      }
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      int idx = tid + i * NT;
      if (idx < A_F4) {
        int kk = idx / (BM / 4), mm = (idx % (BM / 4)) * 4;
        *reinterpret_cast<float4*>(&As[buf][kk][mm]) = ra[i];
      }
    }
#pragma unroll
    for (int i = 0; i < B_PER; ++i) Bs[buf][brow0 + i * ROWSTEP][bcol] = rb[i];
  };

  load_tile(0);
  store_tile(0);
  __syncthreads();

  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    if (t + 1 < ntiles) load_tile(t + 1);
#pragma unroll
    for (int s = 0; s < BK / 2; ++s) {
      float a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = As[buf][2 * s + hi][(wm * TM + i) * 32 + lo];
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = Bs[buf][2 * s + hi][(wn * TN + j) * 32 + lo];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (t + 1 < ntiles) store_tile(buf ^ 1);
    __syncthreads();
  }

  // epilogue: C/D map of 32x32 MFMA: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
  float* out_n = P.out + (long)n * P.M * HWo;
  const float* mask_n = P.mask ? P.mask + (long)n * P.M * HWo : nullptr;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int pp = p0 + (wn * TN + j) * 32 + lo;
    if (pp >= HWo) continue;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + (wm * TM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * hi;
        if (m >= P.M) continue;
        float v = acc[i][j][r];
        if (P.epi & EPI_BIAS) v += P.bias[m];
        if (P.epi & EPI_RELU) v = fmaxf(v, 0.f);
        const long o = (long)m * HWo + pp;
        if (P.epi & EPI_TANH) {
          const float t = tanhf(v / 255.0f);
          if (P.aux) P.aux[(long)n * P.M * HWo + o] = t;
          v = t * 150.0f + 127.5f;
        }
        if (P.epi & EPI_MASK) v = mask_n[o] > 0.f ? v : 0.f;
        if (P.epi & EPI_ACCUM) v += out_n[o];
        out_n[o] = v;
      }
    }
  }
}

// tile configurations (BM x BN)
enum TileCfg { T32 = 0, T64, T96, T128, T192 };

static int select_cfg(int M) {
  if (M <= 32) return T32;
  if (M <= 64) return T64;
  if (M <= 96) return T96;
  if (M % 192 == 0 && M % 128 != 0) return T192;
  return T128;
}
static int cfg_bm(int c) {
  const int bm[] = {32, 64, 96, 128, 192};
  return bm[c];
}
static int cfg_bn(int c) { return c == T32 ? 256 : 128; }

template <bool CF>
static void launch_cfg(int cfg, dim3 grid, hipStream_t st, const ConvParams& P) {
  switch (cfg) {
    case T32: conv_gemm_kernel<1, 1, 4, 2, CF><<<grid, NT, 0, st>>>(P); break;
    case T64: conv_gemm_kernel<1, 2, 4, 1, CF><<<grid, NT, 0, st>>>(P); break;
    case T96: conv_gemm_kernel<1, 3, 4, 1, CF><<<grid, NT, 0, st>>>(P); break;
    case T128: conv_gemm_kernel<2, 2, 2, 2, CF><<<grid, NT, 0, st>>>(P); break;
    default: conv_gemm_kernel<2, 3, 2, 2, CF><<<grid, NT, 0, st>>>(P); break;
  }
}

// ---------------------------------------------------------------------------------------------
__global__ void pack_weight_kernel(const float* __restrict__ w, float* __restrict__ out, int Cout, int Cin, int KS,
                                   int transposed, int Mpad, int Kpad) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)Mpad * Kpad;
  if (idx >= total) return;
  int m = (int)(idx % Mpad);
  int k = (int)(idx / Mpad);
  int Ck = transposed ? Cout : Cin;   // channel count inside the k index
  int Mm = transposed ? Cin : Cout;
  float v = 0.f;
  if (m < Mm && k < KS * KS * Ck) {
    int tap = k / Ck, c = k % Ck;
    int kh = tap / KS, kw = tap % KS;
    int co = transposed ? c : m, ci = transposed ? m : c;
    v = w[(((long)co * Cin + ci) * KS + kh) * KS + kw];
  }
  out[idx] = v;
}

// adjoint of (nearest x`up` upsample -> ReflectionPad2d(pad)): dpad [NC][Hv+2p][Wv+2p] -> dx [NC][Hs][Ws]
__device__ __forceinline__ int reflect_sources(int u, int n_v, int pad, int* src) {
  int c = 0;
  src[c++] = u + pad;
  if (u >= 1 && u <= pad) src[c++] = pad - u;
  if (u >= n_v - 1 - pad && u <= n_v - 2) src[c++] = 2 * (n_v - 1) - u + pad;
  return c;
}

__global__ void fold_reflect_kernel(const float* __restrict__ dpad, float* __restrict__ dx, long NC, int Hs, int Ws,
                                    int pad, int up, int accumulate) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = NC * Hs * Ws;
  if (idx >= total) return;
  int xs = (int)(idx % Ws);
  long t = idx / Ws;
  int ys = (int)(t % Hs);
  long nc = t / Hs;
  int Hv = Hs * up, Wv = Ws * up;
  int Hp = Hv + 2 * pad, Wp = Wv + 2 * pad;
  const float* d = dpad + nc * Hp * Wp;
  float s = 0.f;
  for (int dy = 0; dy < up; ++dy) {
    int rows[3];
    int nr = reflect_sources(ys * up + dy, Hv, pad, rows);
    for (int dxx = 0; dxx < up; ++dxx) {
      int cols[3];
      int ncl = reflect_sources(xs * up + dxx, Wv, pad, cols);
      for (int a = 0; a < nr; ++a)
        for (int b = 0; b < ncl; ++b) s += d[(long)rows[a] * Wp + cols[b]];
    }
  }
  if (accumulate) s += dx[idx];
  dx[idx] = s;
}

}  // namespace

extern "C" {

int vst_version(void) { return 100; }

const char* vst_strerror(int code) {
  if (code == VST_OK) return "success";
  if (code == VST_EINVAL) return "vst: invalid argument";
  if (code == VST_EUNSUPPORTED) return "vst: unsupported configuration";
  return hipGetErrorString((hipError_t)code);
}

int vst_conv_pack_dims(int M, int K, int* Mpad, int* Kpad) {
  VST_CHECK_ARG(M > 0 && K > 0 && Mpad && Kpad);
  int bm = cfg_bm(select_cfg(M));
  *Mpad = (M + bm - 1) / bm * bm;
  *Kpad = (K + BK - 1) / BK * BK;
  return VST_OK;
}

int vst_pack_weight(const float* w, float* packed, int Cout, int Cin, int KS, int transposed, int Mpad, int Kpad,
                    void* stream) {
  VST_CHECK_ARG(w && packed && Cout > 0 && Cin > 0 && KS > 0);
  long total = (long)Mpad * Kpad;
  pack_weight_kernel<<<ceil_div(total, 256), 256, 0, (hipStream_t)stream>>>(w, packed, Cout, Cin, KS, transposed, Mpad,
                                                                            Kpad);
  return vst_launch_status();
}

int vst_conv_gemm(const float* src, const float* wpack, const float* bias, const float* mask, float* out, int N,
                  int Cs, int Hs, int Ws, int M, int K, int Ho, int Wo, int KS, int gmode, int stride, int pad,
                  int up, int epi, long a_batch_stride, float* aux, const float* gmask, void* stream) {
  VST_CHECK_ARG(src && wpack && out && N > 0 && Cs > 0 && Hs > 0 && Ws > 0 && M > 0 && Ho > 0 && Wo > 0);
  VST_CHECK_ARG(K == KS * KS * Cs);
  VST_CHECK_ARG(gmode >= 0 && gmode <= 2 && (stride == 1 || stride == 2) && (up == 1 || up == 2));
  VST_CHECK_ARG(!((epi & EPI_BIAS) && !bias) && !((epi & EPI_MASK) && !mask));
  if (gmode == GM_REFLECT) VST_CHECK_ARG(pad < Hs * up && pad < Ws * up);
  ConvParams P;
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
  int cfg = select_cfg(M);
  int bm = cfg_bm(cfg), bn = cfg_bn(cfg);
  P.Mpad = (M + bm - 1) / bm * bm;
  P.K = K;
  P.Kpad = (K + BK - 1) / BK * BK;
  P.Ho = Ho;
  P.Wo = Wo;
  P.KS = KS;
  P.gmode = gmode;
  P.stride = stride;
  P.pad = pad;
  P.up = up;
  P.epi = epi;
  P.fd_Wo = make_fastdiv(Wo);
  P.fd_Cs = make_fastdiv(Cs);
  P.fd_KS = make_fastdiv(KS);
  dim3 grid(ceil_div((long)Ho * Wo, bn), P.Mpad / bm, N);
  bool cfast = (Cs % BK) == 0;
  if (cfast)
    launch_cfg<true>(cfg, grid, (hipStream_t)stream, P);
  else
    launch_cfg<false>(cfg, grid, (hipStream_t)stream, P);
  return vst_launch_status();
}

int vst_fold_reflect(const float* dpad, float* dx, long NC, int Hs, int Ws, int pad, int up, int accumulate,
                     void* stream) {
  VST_CHECK_ARG(dpad && dx && NC > 0 && Hs > 0 && Ws > 0 && pad >= 0 && (up == 1 || up == 2));
  long total = NC * Hs * Ws;
  fold_reflect_kernel<<<ceil_div(total, 256), 256, 0, (hipStream_t)stream>>>(dpad, dx, NC, Hs, Ws, pad, up,
                                                                             accumulate);
  return vst_launch_status();
}

}  // extern "C"
