// Implicit-GEMM convolution kernel template (shared by the per-precision translation units
// conv_gemm_p{0,1,2}.hip, which each instantiate one GEMM arithmetic mode, and conv_gemm.hip,
// which holds the host launcher and the C ABI).  See conv_gemm.hip for the algorithm.
#pragma once

#include "vst_common.h"

namespace vstk {

__device__ __forceinline__ f32x4 mk4(float a, float b, float c, float d) {
  f32x4 v = {a, b, c, d};
  return v;
}

constexpr int BK = 16;  // k-tile depth
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
  // EPI_PHASE2 (stride-2 data gradient, all four parity phases in one GEMM): row m = ci*4 + 2a + b,
  // pixel (I, J) of the phase grid -> padded-grid position (2I + a, 2J + b); interior positions go
  // straight to dx [N][M/4][ph_H][ph_W], the reflect-pad border to ph_border [N][M/4][Hp][Wp].
  // (The nearest-x2 forward, vst_conv_up2_fwd, uses the same map with ph_pad = 1, + bias, and no
  // border buffer: its out-of-range phase positions are dropped.)
  // EPI_PADOUT (stride-1 data gradient over the padded grid): row m = ci, pixel (u, v) of the
  // padded grid, same interior / border split.
  float* ph_border;
  int ph_H, ph_W, ph_pad;
  FastDiv fd_Wo, fd_Cs, fd_KW;
  int kb;  // channel-blocked K order (VST_GEMM_KBLOCK, vst_common.h kdecode)
  // split-K of the halo kernel (conv_halo_kernel.h): blockIdx.z = n * ksplit + s, slice s sums its
  // share of the 16-channel blocks into part[s][n][M][Ho Wo] (raw accumulators); the reduce kernel
  // adds the slices in order and applies the epilogue
  int ksplit = 1;
  float* part = nullptr;
};

enum { GM_REFLECT = 0, GM_ZERO = 1, GM_TRANSPOSED = 2, GM_CLAMP = 3 };
enum { EPI_BIAS = 1, EPI_RELU = 2, EPI_TANH = 4, EPI_MASK = 8, EPI_ACCUM = 16, EPI_AFFINE = 32, EPI_PHASE2 = 64, EPI_PADOUT = 128 };

// source offset (within one channel plane) of tap (kh,kw) for output pixel (oy,ox); -1 if zero.
// Straight-line code: the three border rules of the forward gathers are all evaluated and the
// block-uniform gmode picks one through bit masks (an if / else-if chain on gmode compiled into a
// ~60-instruction branch ladder executed per k-tile, since the channel-blocked K walk changes the
// tap every tile).
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
  const int y0 = oy * P.stride + kh - P.pad, x0 = ox * P.stride + kw - P.pad_x;
  int yr = abs(y0), xr = abs(x0);  // reflect
  yr = yr >= Hv ? 2 * Hv - 2 - yr : yr;
  xr = xr >= Wv ? 2 * Wv - 2 - xr : xr;
  const int yc = min(max(y0, 0), Hv - 1), xc = min(max(x0, 0), Wv - 1);  // edge clamp
  const int mr = -(int)(P.gmode == GM_REFLECT), mc = -(int)(P.gmode == GM_CLAMP), mz = ~(mr | mc);
  const int y = (yr & mr) | (yc & mc) | (y0 & mz), x = (xr & mr) | (xc & mc) | (x0 & mz);
  const bool inb = (unsigned)y0 < (unsigned)Hv && (unsigned)x0 < (unsigned)Wv;
  const int sh = P.up - 1;
  const int off = (y >> sh) * P.Ws + (x >> sh);
  return (inb || mz == 0) ? off : -1;
}

// Epilogue of the implicit-GEMM conv kernels (conv_gemm_kernel, conv_halo_kernel): the C/D map of
// the 32x32 MFMA (col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)); fragment (i, j) holds rows
// mrow0 + 32i + row and the output pixel pix[j] (linear oy*Wo + ox; -1: outside the output)
template <int TM, int TN>
__device__ __forceinline__ void conv_epilogue(const ConvParams& P, const f32x16 (&acc)[TM][TN], int n, int mrow0,
                                              const int (&pix)[TN], int hi) {
  const int HWo = P.Ho * P.Wo;
  float* out_n = P.out + (long)n * P.M * HWo;
  const float* mask_n = P.mask ? P.mask + (long)n * P.M * HWo : nullptr;
  // plain outputs [+ bias] [-> ReLU] of a full row tile (every forward conv but ConvTanh's, the
  // attention / Gram GEMMs): per weight fragment, the bias of each of the lane's 16 rows loaded once,
  // not per pixel fragment, and no per-element epi / row-range branches -- the general path below is
  // ~16k instructions of branchy code, which on the shallow layers (64 channels: four channel blocks)
  // outweighed the k loop.  Same operations in the same order per element: bitwise the general path's
  if ((P.epi & ~(EPI_BIAS | EPI_RELU)) == 0 && mrow0 + TM * 32 <= P.M) {
    const bool relu = (P.epi & EPI_RELU) != 0, has_b = (P.epi & EPI_BIAS) != 0;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      float bv[16];
      int mo[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = mrow0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hi;
        bv[r] = has_b ? P.bias[m] : 0.f;
        mo[r] = m * HWo;  // (< 2^31: one image's output)
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if (pix[j] < 0) continue;
        float* o = out_n + pix[j];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float v = acc[i][j][r];
          if (has_b) v += bv[r];
          if (relu) v = fmaxf(v, 0.f);
          o[mo[r]] = v;
        }
      }
    }
    return;
  }
  if (P.epi & (EPI_PHASE2 | EPI_PADOUT)) {
    // PHASE2: the 4 consecutive rows of a C-register group are the 4 phases of one channel
    const bool ph2 = P.epi & EPI_PHASE2;
    const int Cx = ph2 ? P.M >> 2 : P.M, Hp = P.ph_H + 2 * P.ph_pad, Wp = P.ph_W + 2 * P.ph_pad;
    float* dx_n = P.out + (long)n * Cx * P.ph_H * P.ph_W;
    float* bd_n = P.ph_border + (long)n * Cx * Hp * Wp;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int pp = pix[j];
      if (pp < 0) continue;
      const int I = (int)fdiv((uint32_t)pp, P.fd_Wo), J = pp - I * P.Wo;
      if (!ph2) {  // one padded-grid pixel per column: one interior/border decision for all rows
        const int y = I - P.ph_pad, x = J - P.ph_pad;
        const bool in = y >= 0 && y < P.ph_H && x >= 0 && x < P.ph_W;
        float* base = in ? dx_n + (long)y * P.ph_W + x : bd_n + (long)I * Wp + J;
        const long cstride = in ? (long)P.ph_H * P.ph_W : (long)Hp * Wp;
        // EPI_MASK: interior values gated by the dx-shaped mask (the border keeps the raw values;
        // vst_fold_border applies the same mask when it folds them in)
        const float* mk = (in && (P.epi & EPI_MASK)) ? P.mask + (long)n * Cx * P.ph_H * P.ph_W + (long)y * P.ph_W + x
                                                      : nullptr;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int ci = mrow0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hi;
            if (ci < Cx) base[ci * cstride] = (mk && !(mk[ci * cstride] > 0.f)) ? 0.f : acc[i][j][r];
          }
        continue;
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int mb = mrow0 + i * 32 + 8 * g + 4 * hi;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int ci = ph2 ? mb >> 2 : mb + r;
            const int u = ph2 ? 2 * I + (r >> 1) : I, v = ph2 ? 2 * J + (r & 1) : J;
            if (ci >= Cx) continue;
            const int y = u - P.ph_pad, x = v - P.ph_pad;
            const float val = acc[i][j][4 * g + r] + ((P.epi & EPI_BIAS) ? P.bias[ci] : 0.f);
            if (y >= 0 && y < P.ph_H && x >= 0 && x < P.ph_W)
              dx_n[((long)ci * P.ph_H + y) * P.ph_W + x] = val;
            else if (P.ph_border && u < Hp && v < Wp)
              bd_n[((long)ci * Hp + u) * Wp + v] = val;
          }
        }
      }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int pp = pix[j];
    if (pp < 0) continue;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = mrow0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hi;
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

// conv_epilogue for one output element (row m, output pixel pp of image n) given its accumulated
// value: the paths the halo kernel can take (no EPI_AFFINE, no EPI_PHASE2), for the split-K reduce.
__device__ __forceinline__ void conv_epilogue_elem(const ConvParams& P, int n, int m, int pp, float v) {
  const int HWo = P.Ho * P.Wo;
  if (P.epi & EPI_PADOUT) {
    const int I = (int)fdiv((uint32_t)pp, P.fd_Wo), J = pp - I * P.Wo;
    const int y = I - P.ph_pad, x = J - P.ph_pad;
    if (y >= 0 && y < P.ph_H && x >= 0 && x < P.ph_W) {
      const long o = ((long)n * P.M + m) * P.ph_H * P.ph_W + (long)y * P.ph_W + x;
      P.out[o] = ((P.epi & EPI_MASK) && !(P.mask[o] > 0.f)) ? 0.f : v;
    } else {
      const int Hp = P.ph_H + 2 * P.ph_pad, Wp = P.ph_W + 2 * P.ph_pad;
      P.ph_border[(((long)n * P.M + m) * Hp + I) * Wp + J] = v;
    }
    return;
  }
  if (P.epi & EPI_BIAS) v += P.bias[m];
  if (P.epi & EPI_RELU) v = fmaxf(v, 0.f);
  const long o = ((long)n * P.M + m) * HWo + pp;
  if (P.epi & EPI_TANH) {
    const float t = tanhf(v / 255.0f);
    if (P.aux) P.aux[o] = t;
    v = t * 150.0f + 127.5f;
  }
  if (P.epi & EPI_MASK) v = P.mask[o] > 0.f ? v : 0.f;
  if (P.epi & EPI_ACCUM) v += P.out[o];
  P.out[o] = v;
}

// float4 slot (row*4 + quad) of A-tile element idx: 8 consecutive lanes take 8 consecutive rows of
// one quad, so each 8-lane ds_write_b128 group hits 8 distinct 4-bank slots (rows are 20 dwords
// apart; bank = dword mod 32) -- the plain row-major order put rows r and r+1's quads 0 and 3 on
// the same banks (2-way conflict on every A store).  The wave still covers whole 64-B rows.
__device__ __forceinline__ int a_slot(int idx) {
  const int row = (idx & 7) | ((idx >> 5) << 3), quad = (idx >> 3) & 3;
  return row * 4 + quad;
}

// hi-half A slots (PREC 2: two float4 per row): slot = row*2 + quad, 8 consecutive lanes on 8
// consecutive rows of one quad (rows 20 dwords apart: distinct 4-bank groups per 8-lane store)
__device__ __forceinline__ int a_slot2(int idx) {
  const int row = (idx & 7) | ((idx >> 4) << 3), quad = (idx >> 3) & 1;
  return row * 2 + quad;
}

// bf16x6 A slots (six float4 per 96-B packed row, LDS rows 28 dwords apart): slot = row*6 + six with
// 8 consecutive lanes on 8 consecutive rows of one float4 column (28 r mod 32 = 0, 28, 24, .., 4:
// distinct 4-bank groups per 8-lane ds_write_b128).  The plain row-major order (idx / 6, idx % 6) put
// lane 7 of each group back on lane 0's banks (profiles/r06_mfma_busy_reconet.json: 1.6 conflict
// cycles per LDS instruction on the 192-row LDS-A tile).  A wave still loads whole 768-B runs of rows.
__device__ __forceinline__ int a_slot6(int idx) {
  const int row = (idx & 7) | ((idx / 48) << 3), six = (idx >> 3) % 6;
  return row * 6 + six;
}

// ADIR (bf16x6 only): the packed weights go straight from memory into each wave's MFMA A operand
// registers (one buffer_load_b128 per 32-row fragment and piece, next tile prefetched a k-step
// ahead) instead of through LDS: no A stores to LDS (the stores were the largest non-MFMA cost of
// the k loop, tools/gemm_bench.py ablations) and no A reads from it.  With WN > 1 the waves of one
// wave row fetch the same fragments (WN x the A bytes, from L2: the packed weights of a layer are
// at most a few MB).
// Block = WM x WN waves (4 on the LDS-A path; 2, 6 or 8 with A-direct, where the threads that
// divide the B tile evenly -- all of them for 2, 4 and 8 waves, the first 256 for 6 -- gather and
// split it and every wave reads it).
// KD: k-tiles per LDS stage (one barrier per KD tiles; the loads of the next KD tiles are in flight
// across the MFMAs of the current KD).  The single-product modes (bf16, fp16) do one MFMA per
// fragment pair, so at KD 1 their k loop is paced by the barrier and the LDS round trip of every
// 16-deep tile rather than by the MFMAs; KD 2 halves both per MFMA.
// One stage of global loads is in flight (the loads of stage s+1 across the MFMAs of stage s).  A
// two-stage variant (round 3, `PF = 2`) measured slower and computed wrong gradients in the
// train_video step; it was removed rather than shipped behind a switch.
template <int WM, int TM, int WN, int TN, bool CFAST, bool GM, int MINW, int PREC, bool ADIR = false, int KD = 1>
__global__ __launch_bounds__(WM * WN * 64, MINW) void conv_gemm_kernel(ConvParams P) {
  static_assert(!ADIR || PREC >= 2, "A-direct: bf16x6, bf16, fp16");
  static_assert(ADIR || WM * WN == 4, "LDS-A path: 4 waves");
  constexpr int BM = WM * TM * 32;
  constexpr int BN = WN * TN * 32;
  constexpr int NTT = WM * WN * 64;          // threads per block
  constexpr int NBT = (NTT % BN == 0 && BK % (NTT / BN) == 0) ? NTT : NT;  // B-tile threads
  // A block per (k-tile, row): 16 fp32 / 16 hi + 16 lo bf16 (64 B); bf16x6: + 16 mid bf16 (96 B)
  constexpr int AW = PREC == 3 ? 24 : 16;    // dwords per (k-tile, row)
  // single bf16 (PREC 2) reads only the hi half of each packed 64-B block: the lo half is never an
  // MFMA operand, so it is neither loaded nor stored to LDS (half the A bytes of the bf16 path)
  constexpr int AWL = (PREC == 2 || PREC == 4) ? 8 : AW;  // dwords per (k-tile, row) actually staged
  constexpr int A_F4 = BM * AWL / 4;         // float4 per A tile
  constexpr int A_PER = (A_F4 + NT - 1) / NT;
  constexpr int ROWSTEP = NBT / BN;          // B rows covered per pass
  constexpr int B_PER = BK / ROWSTEP;        // B elements per thread per tile
  constexpr int KSTEPS = BK / 2;
  // k rows of this thread's B elements: fp32 MFMA (32x32x2: lane half h takes k = 2s + h) ->
  // k = brow0 + ROWSTEP*i; bf16 MFMA (32x32x16: lane half h takes k = 8h..8h+7) -> contiguous
  // k = brow0*B_PER + i, so each thread packs its own bf16 pairs
  constexpr int KSTEP = PREC ? 1 : ROWSTEP;
  static_assert(NBT % BN == 0 && BK % ROWSTEP == 0, "tile");
  const bool bthread = NTT == NBT || threadIdx.x < NBT;  // wave-uniform

  static_assert(BK == 16, "packed A layout assumes 16-deep k-tiles");
  static_assert(KD == 1 || KD == 2, "k-tiles per stage");
  // LDS row: the staged block + 4 pad dwords (12, 20 or 28 dwords: conflict-free ds_read_b128 over
  // the 4 x 16-lane groups / 64 banks, and ds_write_b128 over the 8 x 8-lane groups / 32 banks)
  constexpr int LS = AWL + 4;
  __shared__ __attribute__((aligned(16))) float As[2][KD][ADIR ? 1 : BM][LS];
  __shared__ __attribute__((aligned(16))) float Bs[2][KD][BN][LS];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int lo = lane & 31, hi = lane >> 5;
  const int wm = wave / WN, wn = wave % WN;
  // XCD-aware work order: M tile fastest, then pixel tile, then image, so the blocks that share a
  // source panel (and its halo rows) run on one XCD's L2
  const int gx = gridDim.x, gy = gridDim.y;
  const int wk = xcd_remap(blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z), gx * gy * gridDim.z);
  // (integer division is VALU work: readfirstlane keeps the results scalar, so the buffer
  // descriptors built from them stay in SGPRs -- no waterfall loops around the loads)
  const int rest = __builtin_amdgcn_readfirstlane(wk / gy);
  const int n = __builtin_amdgcn_readfirstlane(rest / gx);
  const int m0 = __builtin_amdgcn_readfirstlane((wk - rest * gy) * BM);
  const int p0 = __builtin_amdgcn_readfirstlane((rest - n * gx) * BN);
  const int HWo = P.Ho * P.Wo;
  const long plane = (long)P.Hs * P.Ws;
  const float* src_n = P.src + (long)n * P.Cs * plane;
  const float* gm_n = GM ? P.gmask + (long)n * P.Cs * plane : nullptr;
  const float* A = P.wpack + (long)n * P.a_batch_stride;

  // this thread's B column (fixed for the whole k loop)
  // ROWSTEP 4 (8-wave blocks; one ds_write_b64 per piece): lanes 8j..8j+7 of a 32-lane chunk take
  // 8 consecutive columns with row group j, so each 16-lane store group hits 16 distinct 2-bank
  // pairs (the plain tid % BN order put columns r and r+8 on the same banks: 2-way conflicts).
  // The gather then reads 8 consecutive pixels per 8 lanes instead of 64 per wave.
  const int bcol = ROWSTEP == 4 ? ((tid & 7) | ((tid >> 5) << 3)) % BN : tid % BN;
  const int brow0 = ROWSTEP == 4 ? (tid >> 3) & 3 : tid / BN;
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

  f32x4 ra0[KD][A_PER];
  float rb0[KD][B_PER];
  float rg0[KD][GM ? B_PER : 1];
  // buffer descriptors over this image's source planes (wave-uniform inputs only)
  const int plane_i = P.Hs * P.Ws;
  const uint32_t src_bytes = (uint32_t)P.Cs * (uint32_t)plane_i * 4u;
  constexpr int OOR = 0x7ffffff0;  // any offset >= num_records reads 0
  const __amdgpu_buffer_rsrc_t srd = uniform_rsrc(src_n, src_bytes);
  const __amdgpu_buffer_rsrc_t gsrd = uniform_rsrc(GM ? gm_n : src_n, src_bytes);
  const int ntiles = P.Kpad / BK;
  // A (packed weights) through a buffer descriptor too: per thread a FIXED byte offset inside the
  // tile (its float4 slot), per tile a scalar offset -- no per-tile VALU address math, and the
  // threads past a partial tile's last float4 read the out-of-range zero (their store is skipped)
  // instead of branching around the load
  const __amdgpu_buffer_rsrc_t asrd = uniform_rsrc(A, (uint32_t)((long)P.Kpad / BK * P.Mpad * AW * 4));
  int a_voff[A_PER];
#pragma unroll
  for (int i = 0; i < A_PER; ++i) {
    const int idx = tid + i * NT;
    a_voff[i] = (A_F4 % NT == 0 || idx < A_F4)
                    ? (AWL == 8 ? (a_slot2(idx) >> 1) * AW * 4 + (a_slot2(idx) & 1) * 16
                                : 16 * (AW == 16 ? a_slot(idx) : a_slot6(idx)))
                    : OOR;
  }
  // A-direct: lane (r, h) of fragment i, piece p reads the 16 B at dword 8p + 4h of packed row
  // m0 + (wm*TM + i)*32 + r (same layout the LDS path copies: [hi k0..15][mid][lo] per row)
  int ad_voff[ADIR ? TM : 1];
#pragma unroll
  for (int i = 0; i < (ADIR ? TM : 1); ++i) ad_voff[i] = (((wm * TM + i) * 32 + lo) * AW + 4 * hi) * 4;
  bf16x8_t arN[KD][ADIR ? TM : 1][3], arC[KD][ADIR ? TM : 1][3];

  // CFAST walk, tiles in k order: tap-major -- the (tap, channel) position advances by 16 channels
  // per tile and the gather offset is decoded once per tap (wave-uniform branch); channel-blocked
  // (P.kb) -- the tap advances every tile, its offset decoded per tile (the tap is a scalar, so the
  // decode is a few VALU ops per thread), the channel block every KH*KW tiles
  const bool blocked = CFAST && kblocked(P.Cs, P.kb);
  const int ntap = P.KH * P.KW;
  int st_tap = 0, st_c0 = 0, st_vbase = 0;
  bool st_ok = false;

  // Issue every global load of tile t without branches (out-of-range taps read a clamped, valid
  // address and are zeroed at LDS-store time), so the loads stay in flight across the MFMAs.
  auto load_tile = [&](int t, f32x4 (&ra)[A_PER], float (&rb)[B_PER], float (&rg)[GM ? B_PER : 1],
                       bf16x8_t (&arn)[ADIR ? TM : 1][3]) {
    const int k0 = t * BK;
    const int a_soff = __builtin_amdgcn_readfirstlane(((t * P.Mpad + m0) * AW) * 4);
    if constexpr (ADIR) {
      // bf16x6: the hi / mid / lo pieces (32 B apart); bf16 / fp16: the hi piece only
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int pc = 0; pc < (PREC == 3 ? 3 : 1); ++pc)
          arn[i][pc] = __builtin_bit_cast(bf16x8_t, __builtin_amdgcn_raw_buffer_load_b128(asrd, ad_voff[i], a_soff + 32 * pc, 0));
    } else
#pragma unroll
    for (int i = 0; i < A_PER; ++i)
      ra[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(asrd, a_voff[i], a_soff, 0));
    if (!bthread) {
    } else if (CFAST) {
      // every 16-row group of the tile shares one tap (Cs % 16 == 0): scalar tap decode, one
      // offset per thread per group; out-of-range taps use an offset past the buffer end, which
      // the buffer-load range check turns into 0 (no branch, no select)
      // (Cs % 16 == 0, so K = taps * Cs is a whole number of tiles and every tile is in range)
      static_assert(BK == 16, "one tap per k-tile");
      (void)k0;
      if (blocked || st_c0 == 0) {
        const int kh = (int)fdiv((uint32_t)st_tap, P.fd_KW), kw = st_tap - kh * P.KW;
        const int off0 = gather_offset(P, oy, ox, kh, kw);
        st_ok = pvalid && off0 >= 0;
        st_vbase = ((PREC ? brow0 * B_PER : brow0) * plane_i + off0) * 4;
      }
      // one address VGPR per tile; the thread's B_PER channels differ by a uniform stride, which
      // goes into the scalar offset (an out-of-range base stays out of range: OOR + the largest
      // stride does not wrap 32 bits for any plane that fits the 2^31 B descriptor)
      const int vo = st_ok ? st_vbase + st_c0 * plane_i * 4 : OOR;
      const int sstep = __builtin_amdgcn_readfirstlane(KSTEP * plane_i * 4);
#pragma unroll
      for (int i = 0; i < B_PER; ++i) {
        rb[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(srd, vo, i * sstep, 0));
        if (GM) rg[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(gsrd, vo, i * sstep, 0));
      }
      // advance in select form: a branchy in-place update (`++st_tap` under one flag, `st_c0 += 16`
      // under the other) was folded into a select of POINTERS to the two walk variables, which
      // pushed them to scratch and put a flat load/store with vmcnt(0) -- a full drain of the tile
      // prefetch -- into every k-step
      const int tap1 = st_tap + 1, c1 = st_c0 + 16;
      const bool wrap = blocked ? tap1 == ntap : c1 == P.Cs;
      const int nt = blocked ? (wrap ? 0 : tap1) : (wrap ? tap1 : st_tap);
      const int nc = blocked ? (wrap ? c1 : st_c0) : (wrap ? 0 : c1);
      st_tap = nt;
      st_c0 = nc;
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
  auto store_tile = [&](float (*Asb)[LS], float (*Bsb)[LS], const f32x4 (&ra)[A_PER], const float (&rb)[B_PER],
                        const float (&rg)[GM ? B_PER : 1]) {
#pragma unroll
    for (int i = 0; i < (ADIR ? 0 : A_PER); ++i) {
      int idx = tid + i * NT;
      if (A_F4 % NT == 0 || idx < A_F4) {
        if (AWL == 8) {
          const int sl = a_slot2(idx);
          *reinterpret_cast<f32x4*>(&Asb[sl >> 1][(sl & 1) * 4]) = ra[i];
        } else if (AW == 16) {
          const int sl = a_slot(idx);
          *reinterpret_cast<f32x4*>(&Asb[sl >> 2][(sl & 3) * 4]) = ra[i];
        } else {
          const int sl = a_slot6(idx);
          *reinterpret_cast<f32x4*>(&Asb[sl / 6][(sl % 6) * 4]) = ra[i];
        }
      }
    }
    if (!bthread) return;
    float bv[B_PER];
#pragma unroll
    for (int i = 0; i < B_PER; ++i) bv[i] = GM ? (rg[i] > 0.f ? rb[i] : 0.f) : rb[i];
    if constexpr (PREC == 3) {  // bf16x6 row: [hi k0..15][mid k0..15][lo k0..15]
      uint32_t h[B_PER / 2], m[B_PER / 2], l[B_PER / 2];
#pragma unroll
      for (int q = 0; q < B_PER / 2; ++q) {
        split3_bf16x2(bv[2 * q], bv[2 * q + 1], h[q], m[q], l[q]);
      }
      uint32_t* d = reinterpret_cast<uint32_t*>(&Bsb[bcol][0]);
      if constexpr (ROWSTEP == 4) {  // k = 4*brow0 .. 4*brow0+3: one b64 per piece
#pragma unroll
        for (int part = 0; part < 3; ++part) {
          const uint32_t* v = part == 0 ? h : (part == 1 ? m : l);
          *reinterpret_cast<u32x2*>(d + 8 * part + 2 * brow0) = u32x2{v[0], v[1]};
        }
      } else if constexpr (ROWSTEP == 2) {
#pragma unroll
        for (int part = 0; part < 3; ++part) {
          const uint32_t* v = part == 0 ? h : (part == 1 ? m : l);
          *reinterpret_cast<u32x4*>(d + 8 * part + 4 * brow0) = u32x4{v[0], v[1], v[2], v[3]};
        }
      } else {
#pragma unroll
        for (int part = 0; part < 3; ++part) {
          const uint32_t* v = part == 0 ? h : (part == 1 ? m : l);
          *reinterpret_cast<u32x4*>(d + 8 * part) = u32x4{v[0], v[1], v[2], v[3]};
          *reinterpret_cast<u32x4*>(d + 8 * part + 4) = u32x4{v[4], v[5], v[6], v[7]};
        }
      }
    } else if constexpr (PREC != 0) {  // bf16 row: [hi k0..15][lo k0..15], this thread's k contiguous
      uint32_t h[B_PER / 2], l[B_PER / 2];
#pragma unroll
      for (int q = 0; q < B_PER / 2; ++q) split2<PREC>(bv[2 * q], bv[2 * q + 1], h[q], l[q]);
      uint32_t* d = reinterpret_cast<uint32_t*>(&Bsb[bcol][0]);
      if constexpr (ROWSTEP == 4) {  // k = 4*brow0 .. 4*brow0+3 (8-wave blocks): one b64 per piece
        *reinterpret_cast<u32x2*>(d + 2 * brow0) = u32x2{h[0], h[1]};
        if (PREC == 1) *reinterpret_cast<u32x2*>(d + 8 + 2 * brow0) = u32x2{l[0], l[1]};
      } else if constexpr (ROWSTEP == 2) {  // k = 8*brow0 .. 8*brow0+7
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
      float* d = &Bsb[bcol][brow0 * 8];
      *reinterpret_cast<f32x4*>(d) = mk4(bv[0], bv[1], bv[2], bv[3]);
      *reinterpret_cast<f32x4*>(d + 4) = mk4(bv[4], bv[5], bv[6], bv[7]);
    } else {             // ROWSTEP == 1: rows k = i
      float* d = &Bsb[bcol][0];
      *reinterpret_cast<f32x4*>(d) = mk4(bv[0], bv[2], bv[4], bv[6]);
      *reinterpret_cast<f32x4*>(d + 4) = mk4(bv[8], bv[10], bv[12], bv[14]);
      *reinterpret_cast<f32x4*>(d + 8) = mk4(bv[1], bv[3], bv[5], bv[7]);
      *reinterpret_cast<f32x4*>(d + 12) = mk4(bv[9], bv[11], bv[13], bv[15]);
    }
  };

  auto compute_tile = [&](int buf, int d) {
    if constexpr (ADIR && PREC == 3) {
      mfma_bf16x6_ktile_ra<TM, TN, LS>(acc, arC[d], Bs[buf][d], wn * TN * 32, lane);
    } else if constexpr (ADIR) {
      mfma_single_ktile_ra<TM, TN, PREC, LS>(acc, arC[d], Bs[buf][d], wn * TN * 32, lane);
    } else if constexpr (PREC == 3) {
      mfma_bf16x6_ktile<TM, TN, LS>(acc, As[buf][d], Bs[buf][d], wm * TM * 32, wn * TN * 32, lane);
    } else if constexpr (PREC != 0) {
      mfma_bf16_ktile<TM, TN, PREC, LS>(acc, As[buf][d], Bs[buf][d], wm * TM * 32, wn * TN * 32, lane);
    } else {
      // each lane's 8 k-steps of every fragment: two ds_read_b128 per fragment, then the MFMA chain
      f32x4 a[TM][2], b[TN][2];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const float* r = &As[buf][d][(wm * TM + i) * 32 + lo][hi * 8];
        a[i][0] = *reinterpret_cast<const f32x4*>(r);
        a[i][1] = *reinterpret_cast<const f32x4*>(r + 4);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const float* r = &Bs[buf][d][(wn * TN + j) * 32 + lo][hi * 8];
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
  };

  // the loads of tile t+1 are in flight across the MFMAs of tile t (a second register set for
  // tile t+2 measured no gain: the loop is not waiting on global latency)
  // (A-direct: the A registers of tile t+1 land with the B loads the store waits for, then become
  // the current set -- register moves after that wait, no extra drain)
  auto rotate_a = [&]() {
    if constexpr (ADIR) {
#pragma unroll
      for (int d = 0; d < KD; ++d)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int pc = 0; pc < (PREC == 3 ? 3 : 1); ++pc) arC[d][i][pc] = arN[d][i][pc];
    }
  };
  // a stage = KD consecutive k-tiles (tile order is the walk order of load_tile, so stages are
  // loaded in order); the tiles of a short last stage are neither loaded, stored nor computed
  // (ntiles is block-uniform)
  const int nst = (ntiles + KD - 1) / KD;
  auto load_stage = [&](int s) {
#pragma unroll
    for (int d = 0; d < KD; ++d)
      if (d == 0 || s * KD + d < ntiles) load_tile(s * KD + d, ra0[d], rb0[d], rg0[d], arN[d]);
  };
  auto store_stage = [&](int buf, int s) {
#pragma unroll
    for (int d = 0; d < KD; ++d)
      if (d == 0 || s * KD + d < ntiles) store_tile(As[buf][d], Bs[buf][d], ra0[d], rb0[d], rg0[d]);
  };
  auto compute_stage = [&](int s) {
#pragma unroll
    for (int d = 0; d < KD; ++d)
      if (d == 0 || s * KD + d < ntiles) compute_tile(s & 1, d);
  };
  load_stage(0);
  store_stage(0, 0);
  rotate_a();
  __syncthreads();
  for (int s = 0; s < nst; ++s) {
    if (s + 1 < nst) load_stage(s + 1);
    compute_stage(s);
    if (s + 1 < nst) store_stage((s & 1) ^ 1, s + 1);
    if (s + 1 < nst) rotate_a();
    __syncthreads();
  }

  int pix[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int pp = p0 + (wn * TN + j) * 32 + lo;
    pix[j] = pp < HWo ? pp : -1;
  }
  conv_epilogue<TM, TN>(P, acc, n, m0 + wm * TM * 32, pix, hi);
}

// tile configurations (BM x BN)
// T64A / T192A / T256A: bf16x6 A-direct blocks of 2 / 6 / 8 waves (32 weight rows x 128 pixels per
// wave)
enum TileCfg { T32 = 0, T64, T96, T128, T192, T64W, T96W, T256, T64A, T192A, T256A, T128A };

inline int select_cfg(int M) {
  if (M <= 32) return T32;
  if (M <= 64) return T64;
  if (M <= 96) return T96;
  if (M % 192 == 0 && M % 128 != 0) return T192;
  return T128;
}
inline int cfg_bm(int c) {
  const int bm[] = {32, 64, 96, 128, 192, 64, 96, 256, 64, 192, 256, 128};
  return bm[c];
}
inline int cfg_bn(int c) { return (c == T32 || c == T64W || c == T96W) ? 256 : 128; }
// 64/96-row tiles on large pixel grids: 256-column tiles (twice the MFMAs per A fragment)
inline int widen_cfg(int c, long HWo) {
  if (HWo < 8192) return c;
  return c == T64 ? T64W : (c == T96 ? T96W : c);
}

// waves per SIMD the tiles' registers must allow (occupancy targets, measured per tile)
constexpr int MINW_T128 = 4, MINW_T256 = 2, MINW_T192 = 2, MINW_SMALL = 4;
constexpr int MINW_T128_BF = 3;  // bf16 paths: the hi/lo conversion temporaries push the 2x2-accumulator tile past 128 VGPRs
constexpr int MINW_ADIR = 3, MINW_A256 = 4;  // A-direct tiles (one wave per 32 weight rows, 128 pixels per block)

// two k-tiles per stage for the single-product modes on the 128- and 256-row tiles; the smaller
// tiles keep one (their two-tile stages exceed the register budget of their occupancy target).
// Compile-time only: the library has one tested kernel per (shape, mode) -- no run-time switches.
template <int WM, int TM, int WN, int TN, bool CF, bool GMK, int MINW, int PR, bool ADIR = false, bool KD2OK = false>
static void launch_k(dim3 grid, hipStream_t st, const ConvParams& P) {
  constexpr int KD = (KD2OK && (PR == 2 || PR == 4)) ? 2 : 1;
  conv_gemm_kernel<WM, TM, WN, TN, CF, GMK, MINW, PR, ADIR, KD><<<grid, WM * WN * 64, 0, st>>>(P);
}

template <bool CF, bool GMK, int PR>
static void launch_cfg(int cfg, dim3 grid, hipStream_t st, const ConvParams& P) {
  constexpr bool AD = PR == 3 || PR == 2 || PR == 4;  // A-direct tiles: bf16x6, bf16, fp16
  switch (cfg) {
    case T32: launch_k<1, 1, 4, 2, CF, GMK, 3, PR>(grid, st, P); break;
    case T64: launch_k<1, 2, 4, 1, CF, GMK, MINW_SMALL, PR>(grid, st, P); break;
    case T64A:
      if constexpr (AD) launch_k<2, 1, 1, 4, CF, GMK, MINW_ADIR, PR, true, true>(grid, st, P);
      break;
    case T192A:
      if constexpr (AD) launch_k<6, 1, 1, 4, CF, GMK, 3, PR, true, true>(grid, st, P);
      break;
    case T256A:  // all eight waves gather the B tile (4 elements each)
      if constexpr (AD) launch_k<8, 1, 1, 4, CF, GMK, MINW_A256, PR, true, true>(grid, st, P);
      break;
    case T96: launch_k<1, 3, 4, 1, CF, GMK, MINW_SMALL, PR>(grid, st, P); break;
    case T64W: launch_k<1, 2, 4, 2, CF, GMK, 3, PR>(grid, st, P); break;
    case T96W: launch_k<1, 3, 4, 2, CF, GMK, 2, PR>(grid, st, P); break;
    case T128: launch_k<2, 2, 2, 2, CF, GMK, PR ? MINW_T128_BF : MINW_T128, PR, false, true>(grid, st, P); break;
    case T128A:  // four A-direct waves of 32 rows x 128 pixels
      if constexpr (AD) launch_k<4, 1, 1, 4, CF, GMK, MINW_ADIR, PR, true, true>(grid, st, P);
      break;
    case T256:  // bf16x3 / bf16 / fp16 only (launch side): 4x2 accumulators per wave, twice the MFMAs per gathered B element
      if constexpr (PR == 1 || PR == 2 || PR == 4) launch_k<2, 4, 2, 2, CF, GMK, MINW_T256, PR, false, true>(grid, st, P);
      break;
    default: launch_k<2, 3, 2, 2, CF, GMK, MINW_T192, PR>(grid, st, P); break;
  }
}

template <int PR>
void launch_prec(bool cfast, bool gm, int cfg, dim3 grid, hipStream_t st, const ConvParams& P) {
  if (cfast)
    gm ? launch_cfg<true, true, PR>(cfg, grid, st, P) : launch_cfg<true, false, PR>(cfg, grid, st, P);
  else
    gm ? launch_cfg<false, true, PR>(cfg, grid, st, P) : launch_cfg<false, false, PR>(cfg, grid, st, P);
}


extern template void launch_prec<0>(bool, bool, int, dim3, hipStream_t, const ConvParams&);
extern template void launch_prec<1>(bool, bool, int, dim3, hipStream_t, const ConvParams&);
extern template void launch_prec<2>(bool, bool, int, dim3, hipStream_t, const ConvParams&);
extern template void launch_prec<3>(bool, bool, int, dim3, hipStream_t, const ConvParams&);
extern template void launch_prec<4>(bool, bool, int, dim3, hipStream_t, const ConvParams&);

}  // namespace vstk
