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
#include <cstdlib>
#include <cstring>

#include "vst_common.h"
#include "vst_hip.h"

namespace {

__device__ __forceinline__ f32x4 mk4(float a, float b, float c, float d) {
  f32x4 v = {a, b, c, d};
  return v;
}

#ifndef VST_CONV_BK
#define VST_CONV_BK 16
#endif
constexpr int BK = VST_CONV_BK;  // k-tile depth (multiple of 16)
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
  int KH, KW, gmode, stride, pad, up;
  int pad_x;  // column padding (= pad except for the dgrad ring segments)
  int epi;
  // EPI_AFFINE: v = (acc + ra[n][m]) * rb[n][m] * cg[n][p] + rd[n][m]  (ra, rd optional)
  const float *ep_ra, *ep_rb, *ep_rd, *ep_cg;
  FastDiv fd_Wo, fd_Cs, fd_KW;
};

enum { GM_REFLECT = 0, GM_ZERO = 1, GM_TRANSPOSED = 2 };
enum { EPI_BIAS = 1, EPI_RELU = 2, EPI_TANH = 4, EPI_MASK = 8, EPI_ACCUM = 16, EPI_AFFINE = 32 };

// source offset (within one channel plane) of tap (kh,kw) for output pixel (oy,ox); -1 if zero
// (select-only arithmetic: no divergent branches inside the k loop)
__device__ __forceinline__ int gather_offset(const ConvParams& P, int oy, int ox, int kh, int kw) {
  if (P.gmode == GM_TRANSPOSED) {
    int ty = oy + P.pad - kh, tx = ox + P.pad_x - kw;
    bool ok = ty >= 0 && tx >= 0;
    if (P.stride == 2) {
      ok = ok && !((ty | tx) & 1);
      ty >>= 1;
      tx >>= 1;
    }
    ok = ok && ty < P.Hs && tx < P.Ws;
    return ok ? ty * P.Ws + tx : -1;
  }
  const int Hv = P.Hs * P.up, Wv = P.Ws * P.up;
  int y = oy * P.stride + kh - P.pad, x = ox * P.stride + kw - P.pad_x;
  bool ok = true;
  if (P.gmode == GM_REFLECT) {
    y = abs(y);
    y = y >= Hv ? 2 * Hv - 2 - y : y;
    x = abs(x);
    x = x >= Wv ? 2 * Wv - 2 - x : x;
  } else {
    ok = y >= 0 && y < Hv && x >= 0 && x < Wv;
  }
  const int sh = P.up - 1;
  return ok ? (y >> sh) * P.Ws + (x >> sh) : -1;
}

// float4 slot (row*4 + quad) of A-tile element idx: 8 consecutive lanes take 8 consecutive rows of
// one quad, so each 8-lane ds_write_b128 group hits 8 distinct 4-bank slots (rows are 20 dwords
// apart; bank = dword mod 32) -- the plain row-major order put rows r and r+1's quads 0 and 3 on
// the same banks (2-way conflict on every A store).  The wave still covers whole 64-B rows.
__device__ __forceinline__ int a_slot(int idx) {
  const int row = (idx & 7) | ((idx >> 5) << 3), quad = (idx >> 3) & 3;
  return row * 4 + quad;
}

template <int WM, int TM, int WN, int TN, bool CFAST, bool GM, int MINW, int PREC>
__global__ __launch_bounds__(NT, MINW) void conv_gemm_kernel(ConvParams P) {
  constexpr int BM = WM * TM * 32;
  constexpr int BN = WN * TN * 32;
  constexpr int A_F4 = BK * BM / 4;          // float4 per A tile
  constexpr int A_PER = (A_F4 + NT - 1) / NT;
  constexpr int ROWSTEP = NT / BN;           // B rows covered per pass
  constexpr int B_PER = BK / ROWSTEP;        // B elements per thread per tile
  constexpr int KSTEPS = BK / 2;
  // k rows of this thread's B elements: fp32 MFMA (32x32x2: lane half h takes k = 2s + h) ->
  // k = brow0 + ROWSTEP*i; bf16 MFMA (32x32x16: lane half h takes k = 8h..8h+7) -> contiguous
  // k = brow0*B_PER + i, so each thread packs its own bf16 pairs
  constexpr int KSTEP = PREC ? 1 : ROWSTEP;
  static_assert(NT % BN == 0 && BK % ROWSTEP == 0, "tile");

  static_assert(BK == 16, "packed A layout assumes 16-deep k-tiles");
  constexpr int LS = 20;  // LDS row: [hi][s] 16 floats + 4 pad (conflict-free ds_read_b128 / ds_write_b128)
  __shared__ __attribute__((aligned(16))) float As[2][BM][LS];
  __shared__ __attribute__((aligned(16))) float Bs[2][BN][LS];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int lo = lane & 31, hi = lane >> 5;
  const int wm = wave / WN, wn = wave % WN;
  // XCD-aware work order: M tile fastest, then pixel tile, then image, so the blocks that share a
  // source panel (and its halo rows) run on one XCD's L2
  const int gx = gridDim.x, gy = gridDim.y;
  const int wk = xcd_remap(blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z), gx * gy * gridDim.z);
  const int rest = wk / gy;
  const int n = rest / gx;
  const int m0 = (wk - rest * gy) * BM;
  const int p0 = (rest - n * gx) * BN;
  const int HWo = P.Ho * P.Wo;
  const long plane = (long)P.Hs * P.Ws;
  const float* src_n = P.src + (long)n * P.Cs * plane;
  const float* gm_n = GM ? P.gmask + (long)n * P.Cs * plane : nullptr;
  const float* A = P.wpack + (long)n * P.a_batch_stride;

  // this thread's B column (fixed for the whole k loop)
  const int bcol = tid % BN;
  const int brow0 = tid / BN;
  const int krow0 = PREC ? brow0 * B_PER : brow0;
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

  f32x4 ra[A_PER];
  float rb[B_PER];
  float rg[GM ? B_PER : 1];
  // buffer descriptors over this image's source planes (wave-uniform inputs only)
  const int plane_i = P.Hs * P.Ws;
  const uint32_t src_bytes = (uint32_t)P.Cs * (uint32_t)plane_i * 4u;
  constexpr int OOR = 0x7ffffff0;  // any offset >= num_records reads 0
  const __amdgpu_buffer_rsrc_t srd = __builtin_amdgcn_make_buffer_rsrc((void*)src_n, (short)0, (int)src_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t gsrd =
      __builtin_amdgcn_make_buffer_rsrc((void*)(GM ? gm_n : src_n), (short)0, (int)src_bytes, 0x00020000);
  const int ntiles = P.Kpad / BK;

  // Issue every global load of tile t without branches (out-of-range taps read a clamped, valid
  // address and are zeroed at LDS-store time), so the loads stay in flight across the MFMAs.
  auto load_tile = [&](int t) {
    const int k0 = t * BK;
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      int idx = tid + i * NT;
      if (A_F4 % NT == 0 || idx < A_F4) {
        ra[i] = *reinterpret_cast<const f32x4*>(A + ((long)t * P.Mpad + m0) * 16 + 4 * a_slot(idx));
      }
    }
    if (CFAST) {
      // every 16-row group of the tile shares one tap (Cs % 16 == 0): scalar tap decode, one
      // offset per thread per group; out-of-range taps use an offset past the buffer end, which
      // the buffer-load range check turns into 0 (no branch, no select)
      constexpr int NG = BK / 16, PER_G = B_PER / NG;
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        const int kg = k0 + 16 * g;
        const int tap = kg / P.Cs;
        const int c0 = kg - tap * P.Cs;
        const int kh = tap / P.KW, kw = tap - (tap / P.KW) * P.KW;
        const int off0 = gather_offset(P, oy, ox, kh, kw);
        const bool ok = pvalid && kg < P.K && off0 >= 0;
        const int vo = ok ? ((c0 + (PREC ? brow0 * PER_G : brow0)) * plane_i + off0) * 4 : OOR;
        const int vstep = ok ? KSTEP * plane_i * 4 : 0;
#pragma unroll
        for (int i = 0; i < PER_G; ++i) {
          rb[g * PER_G + i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(srd, vo + i * vstep, 0, 0));
          if (GM) rg[g * PER_G + i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(gsrd, vo + i * vstep, 0, 0));
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < B_PER; ++i) {
        const int k = k0 + krow0 + i * KSTEP;
        const int kc = k < P.K ? k : 0;
        const int tap = (int)fdiv((uint32_t)kc, P.fd_Cs);
        const int c = kc - tap * P.Cs;
        const int kh = (int)fdiv((uint32_t)tap, P.fd_KW);
        const int kw = tap - kh * P.KW;
        const int off0 = gather_offset(P, oy, ox, kh, kw);
        const bool ok = pvalid && k < P.K && off0 >= 0;
        const int vo = ok ? (c * plane_i + off0) * 4 : OOR;
        rb[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(srd, vo, 0, 0));
        if (GM) rg[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(gsrd, vo, 0, 0));
      }
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      int idx = tid + i * NT;
      if (A_F4 % NT == 0 || idx < A_F4) {
        const int sl = a_slot(idx);
        *reinterpret_cast<f32x4*>(&As[buf][sl >> 2][(sl & 3) * 4]) = ra[i];
      }
    }
    float bv[B_PER];
#pragma unroll
    for (int i = 0; i < B_PER; ++i) bv[i] = GM ? (rg[i] > 0.f ? rb[i] : 0.f) : rb[i];
    if constexpr (PREC != 0) {  // bf16 row: [hi k0..15][lo k0..15], this thread's k contiguous
      uint32_t h[B_PER / 2], l[B_PER / 2];
#pragma unroll
      for (int q = 0; q < B_PER / 2; ++q) split_bf16x2(bv[2 * q], bv[2 * q + 1], h[q], l[q]);
      uint32_t* d = reinterpret_cast<uint32_t*>(&Bs[buf][bcol][0]);
      if constexpr (ROWSTEP == 2) {  // k = 8*brow0 .. 8*brow0+7
        *reinterpret_cast<u32x4*>(d + 4 * brow0) = u32x4{h[0], h[1], h[2], h[3]};
        if (PREC == 1) *reinterpret_cast<u32x4*>(d + 8 + 4 * brow0) = u32x4{l[0], l[1], l[2], l[3]};
      } else {                       // k = 0..15
        *reinterpret_cast<u32x4*>(d) = u32x4{h[0], h[1], h[2], h[3]};
        *reinterpret_cast<u32x4*>(d + 4) = u32x4{h[4], h[5], h[6], h[7]};
        if (PREC == 1) {
          *reinterpret_cast<u32x4*>(d + 8) = u32x4{l[0], l[1], l[2], l[3]};
          *reinterpret_cast<u32x4*>(d + 12) = u32x4{l[4], l[5], l[6], l[7]};
        }
      }
    } else if constexpr (ROWSTEP == 2) {  // rows k = brow0 + 2i: hi = brow0, s = i -> 8 contiguous floats
      float* d = &Bs[buf][bcol][brow0 * 8];
      *reinterpret_cast<f32x4*>(d) = mk4(bv[0], bv[1], bv[2], bv[3]);
      *reinterpret_cast<f32x4*>(d + 4) = mk4(bv[4], bv[5], bv[6], bv[7]);
    } else {             // ROWSTEP == 1: rows k = i
      float* d = &Bs[buf][bcol][0];
      *reinterpret_cast<f32x4*>(d) = mk4(bv[0], bv[2], bv[4], bv[6]);
      *reinterpret_cast<f32x4*>(d + 4) = mk4(bv[8], bv[10], bv[12], bv[14]);
      *reinterpret_cast<f32x4*>(d + 8) = mk4(bv[1], bv[3], bv[5], bv[7]);
      *reinterpret_cast<f32x4*>(d + 12) = mk4(bv[9], bv[11], bv[13], bv[15]);
    }
  };

  load_tile(0);
  store_tile(0);
  __syncthreads();

  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    if (t + 1 < ntiles) load_tile(t + 1);
    if constexpr (PREC != 0) {
      mfma_bf16_ktile<TM, TN, PREC, LS>(acc, As[buf], Bs[buf], wm * TM * 32, wn * TN * 32, lane);
    } else {
      // each lane's 8 k-steps of every fragment: two ds_read_b128 per fragment, then the MFMA chain
      f32x4 a[TM][2], b[TN][2];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const float* r = &As[buf][(wm * TM + i) * 32 + lo][hi * 8];
        a[i][0] = *reinterpret_cast<const f32x4*>(r);
        a[i][1] = *reinterpret_cast<const f32x4*>(r + 4);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const float* r = &Bs[buf][(wn * TN + j) * 32 + lo][hi * 8];
        b[j][0] = *reinterpret_cast<const f32x4*>(r);
        b[j][1] = *reinterpret_cast<const f32x4*>(r + 4);
      }
#pragma unroll
      for (int s = 0; s < KSTEPS; ++s)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] =
                __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][s >> 2][s & 3], b[j][s >> 2][s & 3], acc[i][j], 0, 0, 0);
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
        if (P.epi & EPI_AFFINE) {
          const long rm = (long)n * P.M + m;
          v = (v + (P.ep_ra ? P.ep_ra[rm] : 0.f)) * P.ep_rb[rm] * P.ep_cg[(long)n * HWo + pp] +
              (P.ep_rd ? P.ep_rd[rm] : 0.f);
        }
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
enum TileCfg { T32 = 0, T64, T96, T128, T192, T64W, T96W };

static int select_cfg(int M) {
  if (M <= 32) return T32;
  if (M <= 64) return T64;
  if (M <= 96) return T96;
  if (M % 192 == 0 && M % 128 != 0) return T192;
  return T128;
}
static int cfg_bm(int c) {
  const int bm[] = {32, 64, 96, 128, 192, 64, 96};
  return bm[c];
}
static int cfg_bn(int c) { return (c == T32 || c == T64W || c == T96W) ? 256 : 128; }
#ifndef VST_WIDE
#define VST_WIDE 1
#endif
// 64/96-row tiles on large pixel grids: 256-column tiles (twice the MFMAs per A fragment)
static int widen_cfg(int c, long HWo) {
  if (!VST_WIDE || HWo < 8192) return c;
  return c == T64 ? T64W : (c == T96 ? T96W : c);
}

#ifndef VST_MINW_T128
#define VST_MINW_T128 4
#endif
#ifndef VST_MINW_T192
#define VST_MINW_T192 2
#endif
#ifndef VST_MINW_SMALL
#define VST_MINW_SMALL 4
#endif

template <bool CF, bool GMK, int PR>
static void launch_cfg(int cfg, dim3 grid, hipStream_t st, const ConvParams& P) {
  switch (cfg) {
    case T32: conv_gemm_kernel<1, 1, 4, 2, CF, GMK, 3, PR><<<grid, NT, 0, st>>>(P); break;
    case T64: conv_gemm_kernel<1, 2, 4, 1, CF, GMK, VST_MINW_SMALL, PR><<<grid, NT, 0, st>>>(P); break;
    case T96: conv_gemm_kernel<1, 3, 4, 1, CF, GMK, VST_MINW_SMALL, PR><<<grid, NT, 0, st>>>(P); break;
    case T64W: conv_gemm_kernel<1, 2, 4, 2, CF, GMK, 3, PR><<<grid, NT, 0, st>>>(P); break;
    case T96W: conv_gemm_kernel<1, 3, 4, 2, CF, GMK, 2, PR><<<grid, NT, 0, st>>>(P); break;
    case T128: conv_gemm_kernel<2, 2, 2, 2, CF, GMK, VST_MINW_T128, PR><<<grid, NT, 0, st>>>(P); break;
    default: conv_gemm_kernel<2, 3, 2, 2, CF, GMK, VST_MINW_T192, PR><<<grid, NT, 0, st>>>(P); break;
  }
}

template <int PR>
static void launch_prec(bool cfast, bool gm, int cfg, dim3 grid, hipStream_t st, const ConvParams& P) {
  if (cfast)
    gm ? launch_cfg<true, true, PR>(cfg, grid, st, P) : launch_cfg<true, false, PR>(cfg, grid, st, P);
  else
    gm ? launch_cfg<false, true, PR>(cfg, grid, st, P) : launch_cfg<false, false, PR>(cfg, grid, st, P);
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
      int co = m / KH, kh = m % KH, kw = k / Cin, ci = k % Cin;
      v = w[(((long)co * Cin + ci) * KH + kh) * KW + kw];
    }
  } else {
    int Ck = transposed ? Cout : Cin;  // channel count inside the k index
    int Mm = transposed ? Cin : Cout;
    if (m < Mm && k < KH * KW * Ck) {
      int tap = k / Ck, c = k % Ck;
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

// Stride-2 data gradient, parity class (py, px): only taps kh = py + 2i, kw = px + 2j reach
// padded-input pixels (2yy+py, 2xx+px), and they read dY[yy - i][xx - j].  Packed as a
// transposed A: k = (i*nkw + j)*Cout + co, m = ci.
__global__ void pack_parity_kernel(const float* __restrict__ w, float* __restrict__ out, int Cout, int Cin, int KS,
                                   int py, int px, int Mpad, int Kpad, int bsplit) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)Mpad * Kpad) return;
  int m = (int)(idx % Mpad);
  int k = (int)(idx / Mpad);
  const int nkh = (KS - py + 1) / 2, nkw = (KS - px + 1) / 2;
  float v = 0.f;
  if (m < Cin && k < nkh * nkw * Cout) {
    int tap = k / Cout, co = k % Cout;
    int i = tap / nkw, j = tap % nkw;
    v = w[(((long)co * Cin + m) * KS + py + 2 * i) * KS + px + 2 * j];
  }
  apack_store(out, k, m, Mpad, v, bsplit);
}

// fold_reflect over the 4 parity-class planes [class (a,b)][NC][Hc_a][Wc_b] of the padded grid
struct Cls4 {
  const float *c00, *c01, *c10, *c11;
  int w0, w1;
};
__device__ __forceinline__ float parity_at(const Cls4& c, int yp, int xp) {
  const bool ya = yp & 1, xb = xp & 1;
  const float* base = ya ? (xb ? c.c11 : c.c10) : (xb ? c.c01 : c.c00);
  return base[(yp >> 1) * (xb ? c.w1 : c.w0) + (xp >> 1)];
}

// grid: x over the pixels of one plane, y over planes (grid-stride)
__global__ void fold_reflect_parity_kernel(const float* __restrict__ cls, float* __restrict__ dx, int NC, int Hs,
                                           int Ws, int pad, int accumulate) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= Hs * Ws) return;
  const int xs = p % Ws, ys = p / Ws;
  const int Hp = Hs + 2 * pad, Wp = Ws + 2 * pad;
  const int Hc0 = (Hp + 1) / 2, Hc1 = Hp / 2;
  const int Wc0 = (Wp + 1) / 2, Wc1 = Wp / 2;
  const long s01 = (long)NC * Hc0 * Wc0, s10 = s01 + (long)NC * Hc0 * Wc1, s11 = s10 + (long)NC * Hc1 * Wc0;
  const Src3 ry = reflect_sources(ys, Hs, pad), cx = reflect_sources(xs, Ws, pad);
  for (int nc = blockIdx.y; nc < NC; nc += gridDim.y) {
    const Cls4 c = {cls + (long)nc * Hc0 * Wc0, cls + s01 + (long)nc * Hc0 * Wc1, cls + s10 + (long)nc * Hc1 * Wc0,
                    cls + s11 + (long)nc * Hc1 * Wc1, Wc0, Wc1};
    float s = 0.f;
#define VST_ROW(yp)                                         \
  {                                                         \
    s += parity_at(c, yp, cx.a);                        \
    if (cx.b >= 0) s += parity_at(c, yp, cx.b);         \
    if (cx.c >= 0) s += parity_at(c, yp, cx.c);         \
  }
    VST_ROW(ry.a);
    if (ry.b >= 0) VST_ROW(ry.b);
    if (ry.c >= 0) VST_ROW(ry.c);
#undef VST_ROW
    float* o = dx + (long)nc * Hs * Ws + p;
    if (accumulate) s += *o;
    *o = s;
  }
}

}  // namespace

extern "C" {

int vst_version(void) { return 101; }

static int g_gemm_mode = -1;

int vst_set_gemm_mode(int mode) {
  VST_CHECK_ARG(mode == VST_GEMM_F32 || mode == VST_GEMM_BF16X3 || mode == VST_GEMM_BF16);
  g_gemm_mode = mode;
  return VST_OK;
}

int vst_get_gemm_mode(void) { return vst_gemm_mode_internal(); }

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

int vst_pack_weight(const float* w, float* packed, int Cout, int Cin, int KH, int KW, int transposed, int split_kh,
                    int Mpad, int Kpad, void* stream) {
  VST_CHECK_ARG(w && packed && Cout > 0 && Cin > 0 && KH > 0 && KW > 0 && !(transposed && split_kh));
  long total = (long)Mpad * Kpad;
  pack_weight_kernel<<<ceil_div(total, 256), 256, 0, (hipStream_t)stream>>>(
      w, packed, Cout, Cin, KH, KW, transposed, split_kh, Mpad, Kpad, vst_gemm_mode_internal() != VST_GEMM_F32);
  return vst_launch_status();
}

}  // extern "C"

// initial mode from the environment: VST_GEMM_MODE = f32 | bf16x3 (default) | bf16
int vst_gemm_mode_internal() {
  if (g_gemm_mode < 0) {
    const char* e = getenv("VST_GEMM_MODE");
    int m = VST_GEMM_BF16X3;
    if (e && !strcmp(e, "f32")) m = VST_GEMM_F32;
    if (e && !strcmp(e, "bf16")) m = VST_GEMM_BF16;
    g_gemm_mode = m;
  }
  return g_gemm_mode;
}

static int conv_gemm_launch(const float* src, const float* wpack, const float* bias, const float* mask, float* out,
                            int N, int Cs, int Hs, int Ws, int M, int K, int Ho, int Wo, int KH, int KW, int gmode,
                            int stride, int pad, int pad_x, int up, int epi, long a_batch_stride, float* aux,
                            const float* gmask, void* stream, const float* ep_ra = nullptr,
                            const float* ep_rb = nullptr, const float* ep_rd = nullptr,
                            const float* ep_cg = nullptr) {
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
  int cfg = widen_cfg(select_cfg(M), (long)Ho * Wo);
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
  dim3 grid(ceil_div((long)Ho * Wo, bn), P.Mpad / bm, N);
  const bool cfast = (Cs % 16) == 0, gm = gmask != nullptr;
  hipStream_t st = (hipStream_t)stream;
  switch (vst_gemm_mode_internal()) {
    case VST_GEMM_F32: launch_prec<0>(cfast, gm, cfg, grid, st, P); break;
    case VST_GEMM_BF16: launch_prec<2>(cfast, gm, cfg, grid, st, P); break;
    default: launch_prec<1>(cfast, gm, cfg, grid, st, P); break;
  }
  return vst_launch_status();
}

extern "C" {

int vst_conv_gemm(const float* src, const float* wpack, const float* bias, const float* mask, float* out, int N,
                  int Cs, int Hs, int Ws, int M, int K, int Ho, int Wo, int KH, int KW, int gmode, int stride, int pad,
                  int up, int epi, long a_batch_stride, float* aux, const float* gmask, void* stream) {
  VST_CHECK_ARG(src && wpack && out && N > 0 && Cs > 0 && Hs > 0 && Ws > 0 && M > 0 && Ho > 0 && Wo > 0);
  VST_CHECK_ARG(K == KH * KW * Cs && KH > 0 && KW > 0);
  VST_CHECK_ARG(gmode >= 0 && gmode <= 2 && (stride == 1 || stride == 2) && (up == 1 || up == 2));
  VST_CHECK_ARG(!((epi & EPI_BIAS) && !bias) && !((epi & EPI_MASK) && !mask));
  if (gmode == GM_REFLECT) VST_CHECK_ARG(pad < Hs * up && pad < Ws * up);
  return conv_gemm_launch(src, wpack, bias, mask, out, N, Cs, Hs, Ws, M, K, Ho, Wo, KH, KW, gmode, stride, pad, pad, up,
                          epi, a_batch_stride, aux, gmask, stream);
}

// out[n][m][p] = (sum_k A[n][k][m] B[n][k][p] + ra[n][m]) * rb[n][m] * cg[n][p] + rd[n][m]
// (A packed per image, a_batch_stride floats apart; B = src [N][K][P]; ra, rd may be NULL)
int vst_attn_gemm(const float* src, const float* apack, float* out, int N, int K, int P, int M, long a_batch_stride,
                  const float* ra, const float* rb, const float* rd, const float* cg, void* stream) {
  VST_CHECK_ARG(src && apack && out && rb && cg && N > 0 && K > 0 && P > 0 && M > 0);
  return conv_gemm_launch(src, apack, nullptr, nullptr, out, N, K, 1, P, M, K, 1, P, 1, 1, GM_ZERO, 1, 0, 0, 1,
                          EPI_AFFINE, a_batch_stride, nullptr, nullptr, stream, ra, rb, rd, cg);
}

int vst_pack_weight_parity(const float* w, float* packed, int Cout, int Cin, int KS, int py, int px, int Mpad, int Kpad,
                           void* stream) {
  VST_CHECK_ARG(w && packed && Cout > 0 && Cin > 0 && KS > 0 && (py == 0 || py == 1) && (px == 0 || px == 1));
  long total = (long)Mpad * Kpad;
  pack_parity_kernel<<<ceil_div(total, 256), 256, 0, (hipStream_t)stream>>>(
      w, packed, Cout, Cin, KS, py, px, Mpad, Kpad, vst_gemm_mode_internal() != VST_GEMM_F32);
  return vst_launch_status();
}

int vst_fold_reflect_parity(const float* cls, float* dx, long NC, int Hs, int Ws, int pad, int accumulate,
                            void* stream) {
  VST_CHECK_ARG(cls && dx && NC > 0 && Hs > 0 && Ws > 0 && pad >= 0 && pad < Hs && pad < Ws);
  dim3 g(ceil_div((long)Hs * Ws, 256), (unsigned)(NC < 65535 ? NC : 65535));
  fold_reflect_parity_kernel<<<g, 256, 0, (hipStream_t)stream>>>(cls, dx, (int)NC, Hs, Ws, pad, accumulate);
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
    const int tap = k / Cout, co = k % Cout;
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

int vst_pack_weight_upsum(const float* w, float* packed, int Cout, int Cin, int KS, int Mpad, int Kpad, void* stream) {
  VST_CHECK_ARG(w && packed && Cout > 0 && Cin > 0 && KS > 0 && Mpad >= Cin && Kpad >= (KS + 1) * (KS + 1) * Cout);
  long total = (long)Mpad * Kpad;
  pack_upsum_kernel<<<ceil_div(total, 256), 256, 0, (hipStream_t)stream>>>(w, packed, Cout, Cin, KS, Mpad, Kpad,
                                                                           vst_gemm_mode_internal() != VST_GEMM_F32);
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
