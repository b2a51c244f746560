// Split-K "activation-gradient x im2col(input)^T" GEMM on MFMA (fp32 32x32x2, or bf16x3 / bf16x6 /
// bf16 split products on 32x32x16 bf16, per the call's `mode` argument).
//
//   slab[z][m][j] = sum_{r in chunk z}  A[n][m][r] * gather(src[n], j, r)
//
// Serves the conv weight gradient (dW[co][(kh,kw,ci)], RC/network.py:70 Conv2d backward) and the
// Gram matrix F F^T (RC/utilities.py:93-98, 1x1, A == src).  The reduction runs over output
// pixels r of ONE image per block (grid.z = N * S splits); partial slabs are summed by
// `wgrad_reduce` (into PyTorch's [co][ci][kh][kw] order) or `gram_reduce` (per image, scaled),
// which keeps the result deterministic (no float atomics).
#include <cstdlib>

#include <type_traits>

#include "vst_common.h"
#include "vst_hip.h"
#include "thin.h"
#include "wgrad_halo.h"

namespace {

constexpr int BK = 16;  // pixels per k-tile
constexpr int NT = 256;

struct WgParams {
  const float* a;    // [N][M][Ho][Wo]
  const float* src;  // [N][Cs][Hs][Ws]
  float* slab;       // [N*S][Mpad][Jpad]
  int M, Mpad, J, Jpad;
  int Cs, Hs, Ws, Ho, Wo;
  int KH, KW, gmode, stride, pad, up;
  int pad_x;  // column padding (= pad)
  int S, chunk;
  int asplit, Ha;  // row-split A gather: m = co*asplit + kh reads a[co][oy-kh][ox] (a has Ha rows)
  FastDiv fd_Wo, fd_Cs, fd_KW;
};

// TAP: the block's columns are input channels of ONE tap (kh, kw) (grid.x = taps x channel
// tiles), so the im2col offset of a pixel is computed once per pixel instead of once per
// (pixel, column) -- the per-element index math otherwise dominates the bf16 MFMA loop.
template <int WM, int TM, int WN, int TN, bool AV, int MINW, int PREC, bool TAP>
__global__ __launch_bounds__(NT, MINW) void wgrad_kernel(WgParams P) {
  constexpr int BM = WM * TM * 32;
  constexpr int BN = WN * TN * 32;
  // LDS row: fp32 [hi][s] (k = 2s + hi) / bf16 [hi k][lo k] / bf16x6 [hi k][mid k][lo k]; + 4 pad
  constexpr int LS = PREC == 3 ? 28 : 20;
  constexpr int A_F4 = BM * BK / 4;            // vector path: float4 per A tile
  constexpr int A_PV = (A_F4 + NT - 1) / NT;
  // scalar element map: PAIR consecutive pixels per thread (the bf16 paths pack a thread's two
  // pixels into one dword), CPT rows (A) / columns (B) per pass
  constexpr int PAIR = PREC ? 2 : 1;
  constexpr int CPT = NT * PAIR / BK;          // 16 (fp32) or 32 (bf16)
  constexpr int NCOL = BN / CPT;               // B columns per thread
  constexpr int NAR = BM / CPT;                // A rows per thread (scalar path)
  static_assert(BK == 16, "LDS layout assumes 16-pixel k-tiles");
  static_assert(BN % CPT == 0 && BM % CPT == 0, "tile");

  __shared__ __attribute__((aligned(16))) float As[2][BM][LS];
  __shared__ __attribute__((aligned(16))) float Bs[2][BN][LS];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int lo = lane & 31, hi = lane >> 5;
  const int wm = wave / WN, wn = wave % WN;
  // XCD-aware work order (column tile fastest, then row tile, then (image, split)): the tiles of
  // one split-K chunk share its A rows and source pixels, so they run on one XCD's L2
  const int gx = gridDim.x, gy = gridDim.y;
  const int wk = xcd_remap(blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z), gx * gy * gridDim.z);
  // (readfirstlane: keep the block coordinates, and the buffer descriptors built from them, scalar)
  const int rest = __builtin_amdgcn_readfirstlane(wk / gx), bz = __builtin_amdgcn_readfirstlane(rest / gy);
  const int bx = wk - rest * gx;
  const int j0 = __builtin_amdgcn_readfirstlane(bx * BN);
  // TAP: bx = tap * nct + channel tile
  const int nct = (P.Cs + BN - 1) / BN;
  const int tap = TAP ? __builtin_amdgcn_readfirstlane(bx / nct) : 0;
  const int ci0 = TAP ? __builtin_amdgcn_readfirstlane((bx - tap * nct) * BN) : 0;
  const int tkh = TAP ? tap / P.KW : 0, tkw = TAP ? tap - (tap / P.KW) * P.KW : 0;
  const int m0 = __builtin_amdgcn_readfirstlane((rest - bz * gy) * BM);
  const int n = __builtin_amdgcn_readfirstlane(bz / P.S);
  const int sidx = bz - n * P.S;
  const int HWo = P.Ho * P.Wo;
  const int r_begin = sidx * P.chunk;
  const int r_end = min(HWo, r_begin + P.chunk);
  const int plane = P.Hs * P.Ws;
  const long a_img = P.asplit ? (long)(P.M / P.asplit) * P.Ha * P.Wo : (long)P.M * HWo;
  const float* a_n = P.a + (long)n * a_img;
  const float* src_n = P.src + (long)n * P.Cs * plane;
  constexpr int OOR = 0x7ffffff0;
  const __amdgpu_buffer_rsrc_t asrd = uniform_rsrc(a_n, (uint32_t)(a_img * 4));
  const __amdgpu_buffer_rsrc_t bsrd = uniform_rsrc(src_n, (uint32_t)((long)P.Cs * plane * 4));

  const int rr = PREC ? (tid % (BK / 2)) * 2 : tid % BK;  // this thread's (first) pixel within a k-tile
  const int cc = PREC ? tid / (BK / 2) : tid / BK;        // base row / column

  // CONS (Cs % NCOL == 0, wave-uniform): this thread's NCOL columns are consecutive channels of
  // one tap (LDS rows cc*NCOL + i), so each pixel's reflect/zero index math is done once for all
  // of them; otherwise the columns are cc + i*CPT, each decoded on its own.
  const bool cons = !TAP && P.Cs % NCOL == 0;
  const int crow0 = cons ? cc * NCOL : cc, cstep = cons ? 1 : CPT;

  // decode this thread's B columns once: (ci, kh, kw) packed, -1 if j >= J
  // (TAP: the channel's plane offset in elements, -1 if ci >= Cs)
  int jdesc[NCOL];
#pragma unroll
  for (int i = 0; i < NCOL; ++i) {
    if (TAP) {
      const int ci = ci0 + cc + i * CPT;
      jdesc[i] = ci < P.Cs ? ci * plane : -1;
      continue;
    }
    int j = j0 + crow0 + i * cstep;
    int d = -1;
    if (j < P.J) {
      int tap = (int)fdiv((uint32_t)j, P.fd_Cs);
      int ci = j - tap * P.Cs;
      int kh = (int)fdiv((uint32_t)tap, P.fd_KW);
      int kw = tap - kh * P.KW;
      d = ci | (kh << 16) | (kw << 24);
    }
    jdesc[i] = d;
  }

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  f32x4 rav[AV ? A_PV : 1];
  float ras[AV ? 1 : NAR * PAIR];
  float rb[NCOL * PAIR];
  const int ntiles = r_end > r_begin ? (r_end - r_begin + BK - 1) / BK : 0;
  const int Hv = P.Hs * P.up, Wv = P.Ws * P.up;
  const int sh = P.up - 1;

  auto a_offset = [&](int m, int r) -> int {  // element offset of A[m][r] or OOR
    if (m >= P.M || r >= r_end) return OOR;
    if (!P.asplit) return m * HWo + r;
    const int oy = (int)fdiv((uint32_t)r, P.fd_Wo), ox = r - oy * P.Wo;
    const int co = m / P.asplit, kh = m - co * P.asplit;
    const int yy = oy - kh;
    return (yy >= 0 && yy < P.Ha) ? (co * P.Ha + yy) * P.Wo + ox : OOR;
  };

  auto load_tile = [&](int t) {
    const int rt = r_begin + t * BK;
    if constexpr (AV) {
#pragma unroll
      for (int i = 0; i < A_PV; ++i) {
        const int idx = tid + i * NT;
        if (A_F4 % NT == 0 || idx < A_F4) {
          const int off = a_offset(m0 + (idx >> 2), rt + 4 * (idx & 3));
          rav[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(asrd, off == OOR ? OOR : off * 4, 0, 0));
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < NAR; ++i)
#pragma unroll
        for (int q = 0; q < PAIR; ++q) {
          const int off = a_offset(m0 + cc + i * CPT, rt + rr + q);
          ras[i * PAIR + q] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(asrd, off == OOR ? OOR : off * 4, 0, 0));
        }
    }
#pragma unroll
    for (int q = 0; q < PAIR; ++q) {
      const int r = rt + rr + q;
      const bool rv = r < r_end;
      const int oy = (int)fdiv((uint32_t)r, P.fd_Wo), ox = r - oy * P.Wo;
      const int by = oy * P.stride - P.pad, bx = ox * P.stride - P.pad_x;
      if (TAP) {  // one source offset per pixel, shared by all of this thread's channels
        int y = by + tkh, x = bx + tkw;
        bool ok = rv;
        if (P.gmode == 0) {
          y = abs(y);
          y = min(y, 2 * Hv - 2 - y);
          x = abs(x);
          x = min(x, 2 * Wv - 2 - x);
        } else {
          ok = ok && y >= 0 && y < Hv && x >= 0 && x < Wv;
        }
        const int off = (y >> sh) * P.Ws + (x >> sh);
#pragma unroll
        for (int i = 0; i < NCOL; ++i) {
          const int vo = ok && jdesc[i] >= 0 ? (jdesc[i] + off) * 4 : OOR;
          rb[i * PAIR + q] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(bsrd, vo, 0, 0));
        }
        continue;
      }
      if (cons) {  // one tap for all of this thread's columns (J % NCOL == 0: all valid or none)
        const int d = jdesc[0];
        const int ci = d & 0xffff, kh = (d >> 16) & 0xff, kw = d >> 24;
        int y = by + kh, x = bx + kw;
        bool ok = rv && d >= 0;
        if (P.gmode == 0) {
          y = abs(y);
          y = min(y, 2 * Hv - 2 - y);
          x = abs(x);
          x = min(x, 2 * Wv - 2 - x);
        } else {
          ok = ok && y >= 0 && y < Hv && x >= 0 && x < Wv;
        }
        const int vo = ok ? (ci * plane + (y >> sh) * P.Ws + (x >> sh)) * 4 : OOR;
        const int vstep = ok ? plane * 4 : 0;
#pragma unroll
        for (int i = 0; i < NCOL; ++i)
          rb[i * PAIR + q] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(bsrd, vo + i * vstep, 0, 0));
        continue;
      }
#pragma unroll
      for (int i = 0; i < NCOL; ++i) {
        const int d = jdesc[i];
        const int ci = d & 0xffff, kh = (d >> 16) & 0xff, kw = d >> 24;
        int y = by + kh, x = bx + kw;
        bool ok = rv && d >= 0;
        if (P.gmode == 0) {
          y = abs(y);
          y = min(y, 2 * Hv - 2 - y);
          x = abs(x);
          x = min(x, 2 * Wv - 2 - x);
        } else {
          ok = ok && y >= 0 && y < Hv && x >= 0 && x < Wv;
        }
        const int vo = ok ? (ci * plane + (y >> sh) * P.Ws + (x >> sh)) * 4 : OOR;
        rb[i * PAIR + q] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(bsrd, vo, 0, 0));
      }
    }
  };
  // one thread's two consecutive pixels of a bf16 row, split per PREC
  auto store_pair = [&](uint32_t* row, float a, float b) {
    uint32_t h, l;
    if constexpr (PREC == 3) {
      uint32_t md;
      split3_bf16x2(a, b, h, md, l);
      row[8 + (rr >> 1)] = md;
      row[16 + (rr >> 1)] = l;
    } else {
      split2<PREC>(a, b, h, l);
      if (PREC == 1) row[8 + (rr >> 1)] = l;
    }
    row[rr >> 1] = h;
  };
  auto store_tile = [&](int buf) {
    if constexpr (PREC == 0) {
      if constexpr (AV) {
#pragma unroll
        for (int i = 0; i < A_PV; ++i) {
          const int idx = tid + i * NT;
          if (A_F4 % NT == 0 || idx < A_F4) {
            const int m = idx >> 2, q = idx & 3;  // pixels 4q..4q+3 -> (s, hi) = (2q,0),(2q,1),(2q+1,0),(2q+1,1)
            float* row = &As[buf][m][0];
            *reinterpret_cast<f32x2*>(&row[2 * q]) = f32x2{rav[i][0], rav[i][2]};
            *reinterpret_cast<f32x2*>(&row[8 + 2 * q]) = f32x2{rav[i][1], rav[i][3]};
          }
        }
      } else {
#pragma unroll
        for (int i = 0; i < NAR; ++i) As[buf][cc + i * CPT][(rr & 1) * 8 + (rr >> 1)] = ras[i];
      }
#pragma unroll
      for (int i = 0; i < NCOL; ++i) Bs[buf][crow0 + i * cstep][(rr & 1) * 8 + (rr >> 1)] = rb[i];
    } else {  // bf16 rows [hi px 0..15][lo px 0..15]
      if constexpr (AV) {
#pragma unroll
        for (int i = 0; i < A_PV; ++i) {
          const int idx = tid + i * NT;
          if (A_F4 % NT == 0 || idx < A_F4) {
            const int m = idx >> 2, q = idx & 3;  // pixels 4q..4q+3 -> bf16 slots 4q..4q+3 = dwords 2q, 2q+1
            uint32_t h0, l0, h1, l1;
            uint32_t* row = reinterpret_cast<uint32_t*>(&As[buf][m][0]);
            if constexpr (PREC == 3) {
              uint32_t m0, m1;
              split3_bf16x2(rav[i][0], rav[i][1], h0, m0, l0);
              split3_bf16x2(rav[i][2], rav[i][3], h1, m1, l1);
              *reinterpret_cast<u32x2*>(row + 8 + 2 * q) = u32x2{m0, m1};
              *reinterpret_cast<u32x2*>(row + 16 + 2 * q) = u32x2{l0, l1};
            } else {
              split2<PREC>(rav[i][0], rav[i][1], h0, l0);
              split2<PREC>(rav[i][2], rav[i][3], h1, l1);
              if (PREC == 1) *reinterpret_cast<u32x2*>(row + 8 + 2 * q) = u32x2{l0, l1};
            }
            *reinterpret_cast<u32x2*>(row + 2 * q) = u32x2{h0, h1};
          }
        }
      } else {
#pragma unroll
        for (int i = 0; i < NAR; ++i) store_pair(reinterpret_cast<uint32_t*>(&As[buf][cc + i * CPT][0]), ras[2 * i], ras[2 * i + 1]);
      }
#pragma unroll
      for (int i = 0; i < NCOL; ++i) store_pair(reinterpret_cast<uint32_t*>(&Bs[buf][crow0 + i * cstep][0]), rb[2 * i], rb[2 * i + 1]);
    }
  };

  if (ntiles > 0) {
    load_tile(0);
    store_tile(0);
  }
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    if (t + 1 < ntiles) load_tile(t + 1);
    if constexpr (PREC == 3) {
      mfma_bf16x6_ktile<TM, TN, LS>(acc, As[buf], Bs[buf], wm * TM * 32, wn * TN * 32, lane);
    } else if constexpr (PREC != 0) {
      mfma_bf16_ktile<TM, TN, PREC, LS>(acc, As[buf], Bs[buf], wm * TM * 32, wn * TN * 32, lane);
    } else {
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
      for (int s = 0; s < BK / 2; ++s)
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

  float* slab = P.slab + (long)bz * P.Mpad * P.Jpad;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    int jj = j0 + (wn * TN + j) * 32 + lo;
    if (TAP) {
      const int ci = ci0 + (wn * TN + j) * 32 + lo;
      if (ci >= P.Cs) continue;
      jj = tap * P.Cs + ci;
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + (wm * TM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * hi;
        slab[(long)m * P.Jpad + jj] = acc[i][j][r];
      }
  }
}

// ---------------------------------------------------------------------------------------------
// Row-tiled weight-gradient GEMM (the path for every KxK conv / Gram / A*B^T whose output rows are
// a multiple of 16 pixels wide): a k-tile is 16 consecutive pixels of ONE output row, so its row
// index oy and first column ox0 are block-uniform scalars advanced once per tile.
//   * each thread owns ONE B column j = (tap, ci) for the whole loop (decoded once) and 8 of the
//     tile's 16 pixels: per tile it computes one source row (reflect / zero, nearest-x2 shift) and
//     one base offset, and loads its 8 source elements with immediate offsets (contiguous for
//     stride 1; stride 2 / upsample 2 have their own straight-line forms; a tile whose 8-pixel
//     window crosses the left / right border decodes per element);
//   * A (dY rows) loads are two float4 per (row, 8-pixel half) at a FIXED per-thread offset plus a
//     per-tile scalar offset;
//   * both operands are split (per PREC) in registers and stored with one ds_write_b128 per
//     section; 8 consecutive lanes take 8 consecutive LDS rows, so the 28- / 20-dword row stride
//     puts them on 8 distinct 4-bank groups (conflict-free).
struct Wg2Params {
  const float* a;    // [N][M][HWo]
  const float* src;  // [N][Cs][Hs][Ws]
  float* slab;       // [N*S][Mpad][Jpad]
  int M, Mpad, J, Jpad;
  int Cs, Hs, Ws, Ho, Wo;
  int KH, KW, stride, pad, up;
  int S, chunk;
  int asplit, Ha;  // row-split A (vst_conv_wgrad_rowsplit): m = co*asplit + kh reads a[co][oy-kh][ox], a has Ha rows
};

// KD: k-tiles per LDS stage (one barrier per KD tiles); two for the single-product modes, whose
// k loop does 4-6 MFMAs per wave and tile and is otherwise paced by the per-tile barrier
// (one stage of loads in flight; the round-3 two-stage variant measured no gain and was removed)
template <int WM, int TM, int WN, int TN, int MINW, int PREC, int GMODE, int KD = 1, bool S1 = false>
__global__ __launch_bounds__(WM * WN * 64, MINW) void wgrad2_kernel(Wg2Params P) {
  constexpr int NTH = WM * WN * 64;
  constexpr int BM = WM * TM * 32;
  constexpr int BN = WN * TN * 32;
  // LDS row: the staged k-tile + 4 pad dwords (bf16 / fp16 stage only their 8-dword hi half)
  constexpr int LS = (PREC == 2 || PREC == 4) ? 12 : (PREC == 3 ? 28 : 20);
  // A task = AQ consecutive pixels of one dY row.  8 (two float4) unless 2*BM tasks would leave
  // some waves with one task more than others (the 192-row tile: 384 tasks on 256 threads): then 4,
  // so every thread splits the same number of elements (3 x 4 A + 8 B) and no wave waits at the
  // barrier for the others' extra split work
  constexpr int AQ = ((2 * BM) % NTH != 0 && (4 * BM) % NTH == 0) ? 4 : 8;
  constexpr int APARTS = BK / AQ;
  constexpr int A_TASKS = APARTS * BM, A_IT = (A_TASKS + NTH - 1) / NTH;
  constexpr int B_TASKS = 2 * BN, B_IT = (B_TASKS + NTH - 1) / NTH;
  constexpr int OOR = 0x7ffffff0;
  static_assert(BK == 16, "16-pixel k-tiles");

  __shared__ __attribute__((aligned(16))) float As[2][KD][BM][LS];
  __shared__ __attribute__((aligned(16))) float Bs[2][KD][BN][LS];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int gx = gridDim.x, gy = gridDim.y;
  const int wk = xcd_remap(blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z), gx * gy * gridDim.z);
  const int rest = __builtin_amdgcn_readfirstlane(wk / gx), bz = __builtin_amdgcn_readfirstlane(rest / gy);
  const int j0 = __builtin_amdgcn_readfirstlane((wk - rest * gx) * BN);
  const int m0 = __builtin_amdgcn_readfirstlane((rest - bz * gy) * BM);
  const int n = __builtin_amdgcn_readfirstlane(bz / P.S);
  const int sidx = bz - n * P.S;
  const int HWo = P.Ho * P.Wo;
  const int r_begin = sidx * P.chunk;
  const int r_end = min(HWo, r_begin + P.chunk);
  const int ntiles = r_end > r_begin ? (r_end - r_begin) / BK : 0;
  const int plane = P.Hs * P.Ws;
  const long a_img = P.asplit ? (long)(P.M / P.asplit) * P.Ha * P.Wo : (long)P.M * HWo;
  const float* a_n = P.a + (long)n * a_img;
  const float* src_n = P.src + (long)n * P.Cs * plane;
  const __amdgpu_buffer_rsrc_t asrd = uniform_rsrc(a_n, (uint32_t)(a_img * 4));
  const __amdgpu_buffer_rsrc_t bsrd = uniform_rsrc(src_n, (uint32_t)((long)P.Cs * plane * 4));
  const int Hv = S1 ? P.Hs : P.Hs * P.up, Wv = S1 ? P.Ws : P.Ws * P.up, sh = P.up - 1;

  // A tasks: (row, half) with 8 consecutive lanes on 8 consecutive rows of one half.  Row-split A:
  // a_voff is the (possibly negative) byte offset of a[co][-kh][8*half]; per tile the row oy - kh
  // is checked and the tile offset added in the vector offset
  int a_voff[A_IT], a_row[A_IT], a_half[A_IT], a_kh[A_IT];
#pragma unroll
  for (int i = 0; i < A_IT; ++i) {
    const int q = tid + i * NTH;
    a_row[i] = (q & 7) + 8 * (q / (8 * APARTS));
    a_half[i] = (q >> 3) % APARTS;  // part index (half for AQ = 8, quarter for AQ = 4)
    const int m = m0 + a_row[i];
    const bool ok = q < A_TASKS && m < P.M;
    if (P.asplit) {
      const int co = m / P.asplit, kh = m - co * P.asplit;
      a_kh[i] = ok ? kh : -(1 << 20);  // an invalid row never passes the per-tile row check
      a_voff[i] = ((co * P.Ha - kh) * P.Wo + AQ * a_half[i]) * 4;
    } else {
      a_kh[i] = 0;
      a_voff[i] = ok ? (m * HWo + AQ * a_half[i]) * 4 : OOR;
    }
  }
  // B tasks: column c = q % BN (consecutive lanes -> consecutive columns), half = q / BN
  int b_col[B_IT], b_half[B_IT], b_kh[B_IT], b_kw[B_IT], b_cbase[B_IT];
  bool b_ok[B_IT];
#pragma unroll
  for (int i = 0; i < B_IT; ++i) {
    const int q = tid + i * NTH;
    b_col[i] = q % BN;
    b_half[i] = q / BN;
    const int j = j0 + b_col[i];
    b_ok[i] = q < B_TASKS && j < P.J;
    const int jj = b_ok[i] ? j : 0;
    const int tap = jj / P.Cs, ci = jj - tap * P.Cs;
    b_kh[i] = tap / P.KW;
    b_kw[i] = tap - b_kh[i] * P.KW;
    b_cbase[i] = ci * plane;
  }

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  f32x4 RA[KD][A_IT][2];  // the prefetched stage's registers
  float RB[KD][B_IT][8];
  // tile position (scalar): output row oy, first column ox0
  int t_oy = __builtin_amdgcn_readfirstlane(r_begin / P.Wo);
  int t_ox = __builtin_amdgcn_readfirstlane(r_begin - t_oy * P.Wo);

  auto load_tile = [&](f32x4 (&ra)[A_IT][2], float (&rb)[B_IT][8], int t) {
    const int soff = __builtin_amdgcn_readfirstlane((r_begin + t * BK) * 4);
#pragma unroll
    for (int i = 0; i < A_IT; ++i) {
      if (!S1 && P.asplit) {  // wave-uniform branch
        const int ya = t_oy - a_kh[i];
        const int vo = (ya >= 0 && ya < P.Ha) ? a_voff[i] + soff : OOR;
        ra[i][0] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(asrd, vo, 0, 0));
        if (AQ == 8) ra[i][1] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(asrd, vo + 16, 0, 0));
      } else {
        ra[i][0] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(asrd, a_voff[i], soff, 0));
        if (AQ == 8)
          ra[i][1] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(asrd, a_voff[i] + 16, soff, 0));
      }
    }
#pragma unroll
    for (int i = 0; i < B_IT; ++i) {
      const int stride = S1 ? 1 : P.stride, up = S1 ? 1 : P.up;
      int yv = t_oy * stride + b_kh[i] - P.pad;
      bool ok = b_ok[i];
      if (GMODE == 0) {
        yv = abs(yv);
        yv = min(yv, 2 * Hv - 2 - yv);
      } else if (GMODE == 2) {  // edge clamp (the phase-stacked nearest-x2 weight gradient)
        yv = min(max(yv, 0), Hv - 1);
      } else {
        ok = ok && yv >= 0 && yv < Hv;
      }
      const int rowoff = b_cbase[i] + (S1 ? yv : yv >> sh) * P.Ws;
      const int xv0 = (t_ox + 8 * b_half[i]) * stride + b_kw[i] - P.pad;
      const int xv7 = xv0 + 7 * stride;
      if (xv0 >= 0 && xv7 < Wv) {  // interior window: one base, immediate offsets
        if (up == 2) {             // nearest x2: 8 virtual columns over 4-5 source columns
          const int vo = ok ? (rowoff + (xv0 >> 1)) * 4 : OOR;
          float s[5];
#pragma unroll
          for (int e = 0; e < 5; ++e) s[e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(bsrd, vo + 4 * e, 0, 0));
          const bool odd = xv0 & 1;
#pragma unroll
          for (int e = 0; e < 8; ++e) rb[i][e] = odd ? s[(e + 1) >> 1] : s[e >> 1];
        } else if (stride == 2) {
          const int vo = ok ? (rowoff + xv0) * 4 : OOR;
#pragma unroll
          for (int e = 0; e < 8; ++e) rb[i][e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(bsrd, vo + 8 * e, 0, 0));
        } else {
          // stride 1: the 8 source elements are contiguous -> two 16-byte loads (dword-aligned;
          // gfx950 buffer loads take unaligned addresses)
          const int vo = ok ? (rowoff + xv0) * 4 : OOR;
          const f32x4 a0 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(bsrd, vo, 0, 0));
          const f32x4 a1 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(bsrd, vo + 16, 0, 0));
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            rb[i][e] = a0[e];
            rb[i][4 + e] = a1[e];
          }
        }
      } else {  // border window: per element
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          int xv = xv0 + e * stride;
          bool oke = ok;
          if (GMODE == 0) {
            xv = abs(xv);
            xv = min(xv, 2 * Wv - 2 - xv);
          } else if (GMODE == 2) {
            xv = min(max(xv, 0), Wv - 1);
          } else {
            oke = oke && xv >= 0 && xv < Wv;
          }
          const int vo = oke ? (rowoff + (S1 ? xv : xv >> sh)) * 4 : OOR;
          rb[i][e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(bsrd, vo, 0, 0));
        }
      }
    }
  };

  // 8 consecutive k (pixels 8*half .. 8*half+7) of one LDS row, in the layout of PREC
  auto store8 = [&](float* row, int half, const float* v) {
    if constexpr (PREC == 0) {  // fp32 [hi][s]: k = 2s + hi -> even k at dwords 4*half.., odd at 8 + 4*half..
      *reinterpret_cast<f32x4*>(row + 4 * half) = f32x4{v[0], v[2], v[4], v[6]};
      *reinterpret_cast<f32x4*>(row + 8 + 4 * half) = f32x4{v[1], v[3], v[5], v[7]};
    } else if constexpr (PREC == 3) {
      uint32_t h[4], md[4], l[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) split3_bf16x2(v[2 * q], v[2 * q + 1], h[q], md[q], l[q]);
      uint32_t* d = reinterpret_cast<uint32_t*>(row) + 4 * half;
      *reinterpret_cast<u32x4*>(d) = u32x4{h[0], h[1], h[2], h[3]};
      *reinterpret_cast<u32x4*>(d + 8) = u32x4{md[0], md[1], md[2], md[3]};
      *reinterpret_cast<u32x4*>(d + 16) = u32x4{l[0], l[1], l[2], l[3]};
    } else {
      uint32_t h[4], l[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) split2<PREC>(v[2 * q], v[2 * q + 1], h[q], l[q]);
      uint32_t* d = reinterpret_cast<uint32_t*>(row) + 4 * half;
      *reinterpret_cast<u32x4*>(d) = u32x4{h[0], h[1], h[2], h[3]};
      if (PREC == 1) *reinterpret_cast<u32x4*>(d + 8) = u32x4{l[0], l[1], l[2], l[3]};
    }
  };
  // 4 consecutive k (pixels 4*part .. 4*part+3) of one LDS row: one ds_write_b64 per section
  // (8 consecutive lanes on 8 rows 28 / 20 dwords apart, two parts per 16-lane group: distinct banks)
  auto store4 = [&](float* row, int part, const f32x4& v) {
    uint32_t* d = reinterpret_cast<uint32_t*>(row) + 2 * part;
    if constexpr (PREC == 0) {
      *reinterpret_cast<f32x2*>(row + 2 * part) = f32x2{v[0], v[2]};
      *reinterpret_cast<f32x2*>(row + 8 + 2 * part) = f32x2{v[1], v[3]};
    } else if constexpr (PREC == 3) {
      uint32_t h0, m0, l0, h1, m1, l1;
      split3_bf16x2(v[0], v[1], h0, m0, l0);
      split3_bf16x2(v[2], v[3], h1, m1, l1);
      *reinterpret_cast<u32x2*>(d) = u32x2{h0, h1};
      *reinterpret_cast<u32x2*>(d + 8) = u32x2{m0, m1};
      *reinterpret_cast<u32x2*>(d + 16) = u32x2{l0, l1};
    } else {
      uint32_t h0, l0, h1, l1;
      split2<PREC>(v[0], v[1], h0, l0);
      split2<PREC>(v[2], v[3], h1, l1);
      *reinterpret_cast<u32x2*>(d) = u32x2{h0, h1};
      if (PREC == 1) *reinterpret_cast<u32x2*>(d + 8) = u32x2{l0, l1};
    }
  };
  auto store_tile = [&](int buf, int s, const f32x4 (&ra)[A_IT][2], const float (&rb)[B_IT][8]) {
#pragma unroll
    for (int i = 0; i < A_IT; ++i) {
      if (AQ == 4) {
        if (A_TASKS % NTH == 0 || tid + i * NTH < A_TASKS) store4(&As[buf][s][a_row[i]][0], a_half[i], ra[i][0]);
      } else if (A_TASKS % NTH == 0 || tid + i * NTH < A_TASKS) {
        const float v[8] = {ra[i][0][0], ra[i][0][1], ra[i][0][2], ra[i][0][3],
                            ra[i][1][0], ra[i][1][1], ra[i][1][2], ra[i][1][3]};
        store8(&As[buf][s][a_row[i]][0], a_half[i], v);
      }
    }
#pragma unroll
    for (int i = 0; i < B_IT; ++i)
      if (B_TASKS % NTH == 0 || tid + i * NTH < B_TASKS) store8(&Bs[buf][s][b_col[i]][0], b_half[i], rb[i]);
  };
  auto advance = [&]() {
    t_ox += BK;
    if (t_ox == P.Wo) {
      t_ox = 0;
      ++t_oy;
    }
  };

  const int lo = lane & 31, hi = lane >> 5;
  auto mfma_tile = [&](int buf, int d) {
    if constexpr (PREC == 3) {
      mfma_bf16x6_ktile<TM, TN, LS>(acc, As[buf][d], Bs[buf][d], wm * TM * 32, wn * TN * 32, lane);
    } else if constexpr (PREC != 0) {
      mfma_bf16_ktile<TM, TN, PREC, LS>(acc, As[buf][d], Bs[buf][d], wm * TM * 32, wn * TN * 32, lane);
    } else {
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
      for (int s = 0; s < BK / 2; ++s)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] =
                __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][s >> 2][s & 3], b[j][s >> 2][s & 3], acc[i][j], 0, 0, 0);
    }
  };

  // a stage = KD consecutive k-tiles in walk order (loaded in order: load_tile's row walk advances
  // per tile); the tiles of a short last stage are neither loaded, stored nor computed (ntiles is
  // block-uniform)
  const int nst = (ntiles + KD - 1) / KD;
  auto load_stage = [&](int st) {
#pragma unroll
    for (int d = 0; d < KD; ++d)
      if (d == 0 || st * KD + d < ntiles) {
        load_tile(RA[d], RB[d], st * KD + d);
        advance();
      }
  };
  auto store_stage = [&](int buf, int st) {
#pragma unroll
    for (int d = 0; d < KD; ++d)
      if (d == 0 || st * KD + d < ntiles) store_tile(buf, d, RA[d], RB[d]);
  };
  auto compute_stage = [&](int st) {
#pragma unroll
    for (int d = 0; d < KD; ++d)
      if (d == 0 || st * KD + d < ntiles) mfma_tile(st & 1, d);
  };
  if (ntiles > 0) {
    load_stage(0);
    store_stage(0, 0);
  }
  __syncthreads();
  for (int st = 0; st < nst; ++st) {
    if (st + 1 < nst) load_stage(st + 1);
    compute_stage(st);
    if (st + 1 < nst) store_stage((st & 1) ^ 1, st + 1);
    __syncthreads();
  }

  float* slab = P.slab + (long)bz * P.Mpad * P.Jpad;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int jj = j0 + (wn * TN + j) * 32 + lo;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + (wm * TM + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * hi;
        slab[(long)m * P.Jpad + jj] = acc[i][j][r];
      }
  }
}

// *N: 256-column variants, W64H: a 64 x 64 block for J <= 64 (the 64-channel Gram matrices, VGG16
// relu1_2: the 64 x 128 block spent half its MFMAs and B staging on the padded columns); row-tiled
// kernel only
enum { W32 = 0, W64, W96, W128, W192, W64N, W96N, W64H };
static int wsel(int M) {
  if (M <= 32) return W32;
  if (M <= 64) return W64;
  if (M <= 96) return W96;
  if (M % 192 == 0 && M % 128 != 0) return W192;
  return W128;
}
static int wbm(int c) {
  const int bm[] = {32, 64, 96, 128, 192};
  return bm[c];
}
constexpr int WBN = 128;

// out[co][ci][kh][kw] (+)= scale * sum_z slab[z][co][(kh*KW+kw)*Cs+ci]
// rowsplit: slab rows are m = co*KH + kh and columns j = kw*Cs + ci
__global__ void wgrad_reduce_kernel(const float* __restrict__ slab, float* __restrict__ out, int nslab, int Cout,
                                    int Mpad, int Jpad, int Cs, int KH, int KW, int rowsplit, float scale,
                                    int accumulate) {
  // threads walk the slab order (ci fastest: coalesced slab reads, the dominant traffic) and
  // scatter into PyTorch's [co][ci][kh][kw] order
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)Cout * Cs * KH * KW;
  if (idx >= total) return;
  int ci = (int)(idx % Cs);
  long t = idx / Cs;
  int kw = (int)(t % KW);
  t /= KW;
  int kh = (int)(t % KH);
  int co = (int)(t / KH);
  long off = rowsplit ? (long)(co * KH + kh) * Jpad + kw * Cs + ci : (long)co * Jpad + (kh * KW + kw) * Cs + ci;
  long zs = (long)Mpad * Jpad;
  float s = 0.f;
#pragma unroll 8
  for (int z = 0; z < nslab; ++z) s += slab[off + z * zs];
  s *= scale;
  const long o = (((long)co * Cs + ci) * KH + kh) * KW + kw;
  if (accumulate) s += out[o];
  out[o] = s;
}

// out[n][i][j] = scale * sum_{s<S} slab[n*S+s][i][j],  i < M, j < J
__global__ void gram_reduce_kernel(const float* __restrict__ slab, float* __restrict__ out, int N, int S, int M, int J,
                                   int Mpad, int Jpad, float scale) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)N * M * J;
  if (idx >= total) return;
  int j = (int)(idx % J);
  long t = idx / J;
  int i = (int)(t % M);
  int n = (int)(t / M);
  long zs = (long)Mpad * Jpad;
  const float* p = slab + (long)n * S * zs + (long)i * Jpad + j;
  float s = 0.f;
  for (int z = 0; z < S; ++z) s += p[z * zs];
  out[idx] = s * scale;
}

template <bool AV, int PR, bool TAP>
static void launch_wg_t(int c, dim3 g, hipStream_t st, const WgParams& P) {
  switch (c) {
    case W32: wgrad_kernel<1, 1, 4, 1, AV, 4, PR, TAP><<<g, NT, 0, st>>>(P); break;
    case W64: wgrad_kernel<1, 2, 4, 1, AV, 4, PR, TAP><<<g, NT, 0, st>>>(P); break;
    case W96: wgrad_kernel<1, 3, 4, 1, AV, 4, PR, TAP><<<g, NT, 0, st>>>(P); break;
    case W128: wgrad_kernel<2, 2, 2, 2, AV, 3, PR, TAP><<<g, NT, 0, st>>>(P); break;  // 4 per CU spills (128-VGPR cap)
    default: wgrad_kernel<2, 3, 2, 2, AV, 2, PR, TAP><<<g, NT, 0, st>>>(P); break;
  }
}

template <int PR>
static void launch_wg_p(bool av, bool tap, int c, dim3 g, hipStream_t st, const WgParams& P) {
  if (tap)
    av ? launch_wg_t<true, PR, true>(c, g, st, P) : launch_wg_t<false, PR, true>(c, g, st, P);
  else
    av ? launch_wg_t<true, PR, false>(c, g, st, P) : launch_wg_t<false, PR, false>(c, g, st, P);
}

static void launch_wg(int c, bool tap, dim3 g, int mode, hipStream_t st, const WgParams& P) {
  // float4 A loads need 4 consecutive pixels in one row segment (and, for the row-split gather,
  // in one output row)
  const bool av = (P.Ho * P.Wo) % 4 == 0 && (!P.asplit || P.Wo % 4 == 0);
  switch (vst_mode_arith(mode)) {
    case VST_GEMM_F32: launch_wg_p<0>(av, tap, c, g, st, P); break;
    case VST_GEMM_BF16: launch_wg_p<2>(av, tap, c, g, st, P); break;
    case VST_GEMM_BF16X6: launch_wg_p<3>(av, tap, c, g, st, P); break;
    case VST_GEMM_F16: launch_wg_p<4>(av, tap, c, g, st, P); break;
    default: launch_wg_p<1>(av, tap, c, g, st, P); break;
  }
}

static int wminw(int c) {  // resident blocks per CU of each configuration (its launch bound)
  return c == W192 ? 2 : (c == W128 ? 3 : 4);
}

// Split-K count: minimise (waves of blocks) x (k-tiles per block + fixed cost) plus the slab
// reduction traffic, i.e. fill the 256 CUs evenly without over-splitting.
static int plan_splits(long tiles, int N, int HWo, int c, long Mpad, long Jpad) {
  const long slots = 256L * wminw(c);
  const long ktiles = (HWo + BK - 1) / BK;
  const double t_tile = wminw(c) * 2.0 * wbm(c) * WBN * BK / 0.44e12;  // s per k-tile per block
  long maxs = (HWo + 2 * BK - 1) / (2 * BK);                        // >= 2 k-tiles per split
  if (maxs > 64) maxs = 64;
  if (maxs < 1) maxs = 1;
  int best = 1;
  double best_t = 1e30;
  for (int S = 1; S <= maxs; ++S) {
    const long blocks = tiles * N * S;
    const long waves = (blocks + slots - 1) / slots;
    const long kt = ((HWo + S - 1) / S + BK - 1) / BK;
    const double t = waves * (kt + 4) * t_tile + (double)N * S * Mpad * Jpad * 8.0 / 4e12;
    if (t < best_t * 0.995) {
      best_t = t;
      best = S;
    }
  }
  (void)ktiles;
  return best;
}

template <int PR, int GMD, int KD, bool S1>
static void launch_wg2_pks(int c, dim3 g, hipStream_t st, const Wg2Params& P) {
  switch (c) {
    case W32: wgrad2_kernel<1, 1, 4, 1, 4, PR, GMD, KD, S1><<<g, NT, 0, st>>>(P); break;
    case W64: wgrad2_kernel<1, 2, 4, 1, 4, PR, GMD, KD, S1><<<g, NT, 0, st>>>(P); break;
    case W96: wgrad2_kernel<1, 3, 4, 1, 4, PR, GMD, KD, S1><<<g, NT, 0, st>>>(P); break;
    case W128: wgrad2_kernel<2, 2, 2, 2, 3, PR, GMD, KD, S1><<<g, NT, 0, st>>>(P); break;
    case W64N: wgrad2_kernel<1, 2, 4, 2, 2, PR, GMD, KD, S1><<<g, NT, 0, st>>>(P); break;
    case W96N: wgrad2_kernel<1, 3, 4, 2, 2, PR, GMD, KD, S1><<<g, NT, 0, st>>>(P); break;
    case W64H: wgrad2_kernel<1, 2, 2, 1, 4, PR, GMD, KD, S1><<<g, 128, 0, st>>>(P); break;
    default: wgrad2_kernel<2, 3, 2, 2, 2, PR, GMD, KD, S1><<<g, NT, 0, st>>>(P); break;
  }
}
// S1: stride 1, no upsampling, plain A rows (every layer but conv2 / conv3, the row-split and the
// up2 phase GEMMs) -- the gather without the run-time stride / upsample / row-split paths, whose
// merged branches cost the k loop waits on its own prefetch (residual layer 0.58 -> 0.50 ms)
template <int PR, int GMD, int KD>
static void launch_wg2_pk(int c, dim3 g, hipStream_t st, const Wg2Params& P) {
  if (P.stride == 1 && P.up == 1 && !P.asplit) launch_wg2_pks<PR, GMD, KD, true>(c, g, st, P);
  else launch_wg2_pks<PR, GMD, KD, false>(c, g, st, P);
}

// k-tiles per stage for the single-product modes (compile-time: one tested kernel per mode)
constexpr int WKD_SP = 2;
template <int PR, int GMD>
static void launch_wg2_p(int c, dim3 g, hipStream_t st, const Wg2Params& P) {
  launch_wg2_pk<PR, GMD, (PR == 2 || PR == 4) ? WKD_SP : 1>(c, g, st, P);
}

template <int GMD>
static void launch_wg2(int c, dim3 g, int mode, hipStream_t st, const Wg2Params& P) {
  switch (vst_mode_arith(mode)) {
    case VST_GEMM_F32: launch_wg2_p<0, GMD>(c, g, st, P); break;
    case VST_GEMM_BF16: launch_wg2_p<2, GMD>(c, g, st, P); break;
    case VST_GEMM_BF16X6: launch_wg2_p<3, GMD>(c, g, st, P); break;
    case VST_GEMM_F16: launch_wg2_p<4, GMD>(c, g, st, P); break;
    default: launch_wg2_p<1, GMD>(c, g, st, P); break;
  }
}

// row-tiled kernel applies: output rows a multiple of 16 wide (plain or row-split A gather), and
// every source offset within the 2^31 B buffer range
static bool wg2_ok(int asplit, int Wo) {
  (void)asplit;
  return Wo % BK == 0;
}

static int run_wg(const float* a, const float* src, float* slab, int N, int M, int Cs, int Hs, int Ws, int Ho, int Wo,
                  int KH, int KW, int gmode, int stride, int pad, int up, int S, int asplit, int Ha, int mode,
                  hipStream_t st) {
  if (wg2_ok(asplit, Wo)) {
    Wg2Params Q;
    Q.a = a;
    Q.src = src;
    Q.slab = slab;
    Q.M = M;
    const int c = wsel(M);
    Q.Mpad = (M + wbm(c) - 1) / wbm(c) * wbm(c);
    Q.J = KH * KW * Cs;
    Q.Jpad = (Q.J + WBN - 1) / WBN * WBN;
    Q.Cs = Cs;
    Q.Hs = Hs;
    Q.Ws = Ws;
    Q.Ho = Ho;
    Q.Wo = Wo;
    Q.KH = KH;
    Q.KW = KW;
    Q.stride = stride;
    Q.pad = pad;
    Q.up = up;
    Q.S = S;
    Q.asplit = asplit;
    Q.Ha = Ha;
    Q.chunk = ((Ho * Wo + S - 1) / S + BK - 1) / BK * BK;
    // 64- / 96-row tiles over more than 128 columns: 256-column blocks when that pads J no further
    // (ReCoNet conv1 J = 243, conv2 J = 432): the dY rows are split once per 256 columns instead of
    // per 128, and each wave runs twice the MFMAs per k-tile.  Same Mpad / Jpad / split count, so
    // the slab layout and the workspace size do not change.
    int cw = c;
    if ((c == W64 || c == W96) && Q.J > WBN && Q.Jpad % (2 * WBN) == 0) cw = c == W64 ? W64N : W96N;
    // J <= 64 on a 64-row tile: one 64 x 64 block per M tile (the slab keeps its 128-column stride;
    // its columns >= J are never written nor read)
    if (c == W64 && Q.J <= 64) cw = W64H;
    dim3 g(cw == W64H ? 1 : Q.Jpad / (cw == c ? WBN : 2 * WBN), Q.Mpad / wbm(c), N * S);
    if (gmode == 0) launch_wg2<0>(cw, g, mode, st, Q);
    else if (gmode == 2) launch_wg2<2>(cw, g, mode, st, Q);
    else launch_wg2<1>(cw, g, mode, st, Q);
    return vst_launch_status();
  }
  WgParams P;
  P.a = a;
  P.src = src;
  P.slab = slab;
  P.M = M;
  int c = wsel(M);
  P.Mpad = (M + wbm(c) - 1) / wbm(c) * wbm(c);
  P.J = KH * KW * Cs;
  P.Jpad = (P.J + WBN - 1) / WBN * WBN;
  P.Cs = Cs;
  P.Hs = Hs;
  P.Ws = Ws;
  P.Ho = Ho;
  P.Wo = Wo;
  P.KH = KH;
  P.KW = KW;
  P.gmode = gmode;
  P.stride = stride;
  P.pad = pad;
  P.pad_x = pad;
  P.up = up;
  P.S = S;
  P.asplit = asplit;
  P.Ha = Ha;
  int HWo = Ho * Wo;
  P.chunk = ((HWo + S - 1) / S + BK - 1) / BK * BK;
  P.fd_Wo = make_fastdiv(Wo);
  P.fd_Cs = make_fastdiv(Cs);
  P.fd_KW = make_fastdiv(KW);
  // tap-uniform column tiles when the channels fill whole 128-column tiles (VGG / AdaAttN decoder
  // widths; measured slower for the ReCoNet widths 48/96/192, whose padded tiles waste MFMAs)
  const bool tap = !asplit && KH * KW > 1 && Cs % WBN == 0;
  const int gxn = tap ? KH * KW * ((Cs + WBN - 1) / WBN) : P.Jpad / WBN;
  dim3 g(gxn, P.Mpad / wbm(c), N * S);
  launch_wg(c, tap, g, mode, st, P);
  return vst_launch_status();
}

static int splits_for(int N, int M, long J, int HWo) {
  int c = wsel(M);
  long Mpad = (M + wbm(c) - 1) / wbm(c) * wbm(c);
  long Jpad = (J + WBN - 1) / WBN * WBN;
  int S = plan_splits((Mpad / wbm(c)) * (Jpad / WBN), N, HWo, c, Mpad, Jpad);
  const int maxs = (HWo + 2 * BK - 1) / (2 * BK);
  return S < maxs ? S : (maxs > 0 ? maxs : 1);
}

// ---------------------------------------------------------------------------------------------
// Weight gradient of nearest-x2 upsample -> ReflectionPad2d(1) -> Conv2d(k3) (UpsampleConvLayer,
// RC/network.py:114-120) as a phase-stacked 2x2 GEMM on the SOURCE grid.  Output pixel (2i+a, 2j+b)
// with tap (kh, kw) reads source pixel (i + d(a,kh), j + d(b,kw)), d(a,k) = floor((a+k-1)/2), and the
// reflect border of the virtual grid is an edge clamp on the source grid.  Re-indexing phase a by
// i' = i + a makes the source offset i' - 1 + e with e = e(a,k) = floor((a+k+1)/2) - a in {0, 1}
// for every phase, so ONE GEMM with
//   rows    m = (co, a, b)                       A[m][i'][j'] = dy[co][2i'-a][2j'-b]  (0 outside)
//   columns j = (eh, ew, ci)                     B = x[ci][clamp(i'-1+eh)][clamp(j'-1+ew)]
//   K       = the (H+1) x Wp grid of (i', j')    (Wp = W+1 rounded up to the 16-pixel k-tile)
// gives every (phase, tap) product: 16 (phase, e) pairs per (co, ci) instead of the 36 (phase, tap)
// pairs of the virtual-grid GEMM (2.25x fewer MACs), with M = 4*Cout rows (48 -> 192, 96 -> 384)
// filling whole tiles.  dW[co][ci][kh][kw] = sum_{a,b} P[(co,a,b)][(e(a,kh), e(b,kw), ci)].
// one thread per (nc, a, i', 4-column group j'..j'+3): both b planes from the dy row 2i'-a
// (two aligned float4 + one scalar load, two float4 stores; odd W, whose rows start only 8-B
// aligned, takes the per-element loads)
__global__ void up2_phase_planes_kernel(const float* __restrict__ dy, float* __restrict__ A, long NC, int H, int W,
                                        int Wp) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int Wq = Wp >> 2;
  const long total = NC * 2 * (H + 1) * Wq;
  if (idx >= total) return;
  const int jq = (int)(idx % Wq);
  long t = idx / Wq;
  const int i = (int)(t % (H + 1));
  t /= H + 1;
  const int a = (int)(t & 1);
  const long nc = t >> 1;
  const int y = 2 * i - a, j = 4 * jq, W2 = 2 * W;
  float e[9];  // dy[y][2j - 1 .. 2j + 7]
  if (y >= 0 && y < 2 * H) {
    const float* row = dy + (nc * 2 * H + y) * W2;
    if ((W & 1) == 0 && 2 * j + 8 <= W2) {  // even W: the row starts 16-B aligned (2W % 4 == 0)
      const f32x4 v0 = *reinterpret_cast<const f32x4*>(row + 2 * j);
      const f32x4 v1 = *reinterpret_cast<const f32x4*>(row + 2 * j + 4);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        e[1 + q] = v0[q];
        e[5 + q] = v1[q];
      }
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) e[1 + q] = 2 * j + q < W2 ? row[2 * j + q] : 0.f;
    }
    e[0] = (j > 0 && 2 * j - 1 < W2) ? row[2 * j - 1] : 0.f;
  } else {
#pragma unroll
    for (int q = 0; q < 9; ++q) e[q] = 0.f;
  }
  // plane (a, b) row i: element j' = dy[y][2j' - b]
  float* p0 = A + (((nc * 4 + 2 * a) * (H + 1) + i) * Wp + j);
  float* p1 = p0 + (long)(H + 1) * Wp;
  *reinterpret_cast<f32x4*>(p0) = f32x4{e[1], e[3], e[5], e[7]};
  *reinterpret_cast<f32x4*>(p1) = f32x4{e[0], e[2], e[4], e[6]};
}

__global__ void up2_wgrad_reduce_kernel(const float* __restrict__ slab, float* __restrict__ out, int nslab, int Cout,
                                        int Mpad, int Jpad, int Cin, int accumulate) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;  // (co, kh, kw, ci), ci fastest
  const long total = (long)Cout * 9 * Cin;
  if (idx >= total) return;
  const int ci = (int)(idx % Cin);
  long t = idx / Cin;
  const int kw = (int)(t % 3);
  t /= 3;
  const int kh = (int)(t % 3);
  const int co = (int)(t / 3);
  const long zs = (long)Mpad * Jpad;
  float s = 0.f;
  for (int z = 0; z < nslab; ++z) {
    const float* sl = slab + z * zs;
#pragma unroll
    for (int ph = 0; ph < 4; ++ph) {
      const int a = ph >> 1, b = ph & 1;
      const int eh = ((a + kh + 1) >> 1) - a, ew = ((b + kw + 1) >> 1) - b;
      s += sl[(long)(co * 4 + ph) * Jpad + (eh * 2 + ew) * Cin + ci];
    }
  }
  const long o = (((long)co * Cin + ci) * 3 + kh) * 3 + kw;
  if (accumulate) s += out[o];
  out[o] = s;
}

static int up2_wp(int W) { return (W + 1 + BK - 1) / BK * BK; }

}  // namespace

extern "C" {

// workspace floats of vst_conv_wgrad_up2: slab + the four phase planes of dY
long vst_conv_wgrad_up2_workspace(int N, int Cin, int H, int W, int Cout) {
  const int M = 4 * Cout, J = 4 * Cin, Wp = up2_wp(W);
  return vst_wgrad_workspace(N, M, J, (H + 1) * Wp) + (long)N * M * (H + 1) * Wp;
}

// dW of nearest-x2 upsample + reflect pad 1 + 3x3 conv; dy [N][Cout][2H][2W], x [N][Cin][H][W]
int vst_conv_wgrad_up2(const float* dy, const float* x, float* dw, float* workspace, int N, int Cin, int H, int W,
                       int Cout, int accumulate, int mode, void* stream) {
  VST_CHECK_ARG(vst_mode_ok(mode));
  VST_CHECK_ARG(dy && x && dw && workspace && N > 0 && Cin > 0 && Cout > 0 && H > 0 && W > 0);
  const int M = 4 * Cout, J = 4 * Cin, Wp = up2_wp(W), Hq = H + 1;
  VST_CHECK_ARG(wg2_ok(0, Wp));
  const int S = splits_for(N, M, J, Hq * Wp);
  const int c = wsel(M);
  const long Mpad = (M + wbm(c) - 1) / wbm(c) * wbm(c), Jpad = ((long)J + WBN - 1) / WBN * WBN;
  float* slab = workspace;
  float* planes = workspace + (long)N * S * Mpad * Jpad;
  hipStream_t st = (hipStream_t)stream;
  const long np = (long)N * Cout * 2 * Hq * (Wp / 4);
  up2_phase_planes_kernel<<<ceil_div(np, 256), 256, 0, st>>>(dy, planes, (long)N * Cout, H, W, Wp);
  int rc = vst_launch_status();
  if (rc) return rc;
  rc = run_wg(planes, x, slab, N, M, Cin, H, W, Hq, Wp, 2, 2, 2, 1, 1, 1, S, 0, 0, mode, st);
  if (rc) return rc;
  const long total = (long)Cout * 9 * Cin;
  up2_wgrad_reduce_kernel<<<ceil_div(total, 256), 256, 0, st>>>(slab, dw, N * S, Cout, (int)Mpad, (int)Jpad, Cin,
                                                               accumulate);
  return vst_launch_status();
}

// workspace (floats) needed by vst_conv_wgrad / vst_conv_wgrad_rowsplit / vst_gram
long vst_wgrad_workspace(int N, int M, int J, int HWo) {
  int c = wsel(M);
  long Mpad = (M + wbm(c) - 1) / wbm(c) * wbm(c);
  long Jpad = (J + WBN - 1) / WBN * WBN;
  return (long)N * splits_for(N, M, J, HWo) * Mpad * Jpad;
}

// the halo weight gradient (wgrad_halo.hip) applies: 3x3 stride-1 pad-1 over 32-channel blocks and
// 16-column strips, a split-product mode, unless the call asks for the row-tiled kernel
static bool use_wgrad_halo(int Cout, int Cin, int Hs, int Ws, int Ho, int Wo, int KH, int KW, int gmode, int stride,
                           int pad, int up, int mode) {
  return !(mode & VST_GEMM_PERTAP) && Ho == Hs && Wo == Ws &&
         wgrad_halo_ok(Cout, Cin, Hs, Ws, KH, KW, stride, pad, up, gmode, mode);
}

long vst_conv_wgrad_workspace(int N, int Cin, int Hs, int Ws, int Cout, int Ho, int Wo, int KH, int KW, int gmode,
                              int stride, int pad, int up, int mode) {
  if (N <= 0 || Cin <= 0 || Cout <= 0 || Ho <= 0 || Wo <= 0 || KH <= 0 || KW <= 0 || !vst_mode_ok(mode)) return 0;
  if (vst_thin_wgrad_ok(Cout, Cin, Hs, Ws, Ho, Wo, KH, KW, gmode, stride, pad, up, mode))
    return vst_thin_wgrad_floats(N, Cout, Cin, Hs, Ws);
  if (use_wgrad_halo(Cout, Cin, Hs, Ws, Ho, Wo, KH, KW, gmode, stride, pad, up, mode))
    return wgrad_halo_slab_floats(N, Cin, wgrad_halo_plan(N, Cout, Cin, Hs, Ws, mode));
  return vst_wgrad_workspace(N, Cout, KH * KW * Cin, Ho * Wo);
}

int vst_conv_wgrad(const float* dy, const float* x, float* dw, float* workspace, long ws_floats, int N, int Cin,
                   int Hs, int Ws, int Cout, int Ho, int Wo, int KH, int KW, int gmode, int stride, int pad, int up,
                   int accumulate, int mode, void* stream) {
  VST_CHECK_ARG(vst_mode_ok(mode));
  VST_CHECK_ARG(dy && x && dw && workspace && N > 0 && Cin > 0 && Cout > 0 && Ho > 0 && Wo > 0 && KH > 0 && KW > 0);
  VST_CHECK_ARG((gmode == 0 || gmode == 1) && (stride == 1 || stride == 2) && (up == 1 || up == 2));
  // at most 4 output channels: the VALU kernel (exact fp32, whatever the mode's MFMA arithmetic),
  // given the workspace vst_conv_wgrad_workspace names for it
  if (vst_thin_wgrad_ok(Cout, Cin, Hs, Ws, Ho, Wo, KH, KW, gmode, stride, pad, up, mode) &&
      ws_floats >= vst_thin_wgrad_floats(N, Cout, Cin, Hs, Ws))
    return vst_thin_wgrad_launch(dy, x, dw, workspace, N, Cin, Hs, Ws, Cout, gmode, accumulate, (hipStream_t)stream);
  const long rowtiled_floats = vst_wgrad_workspace(N, Cout, KH * KW * Cin, Ho * Wo);
  bool halo = use_wgrad_halo(Cout, Cin, Hs, Ws, Ho, Wo, KH, KW, gmode, stride, pad, up, mode);
  // a workspace sized for the row-tiled kernel (the pre-halo rule) but smaller than the halo slabs
  // runs row-tiled; one smaller than both is refused
  if (halo && ws_floats < wgrad_halo_slab_floats(N, Cin, wgrad_halo_plan(N, Cout, Cin, Hs, Ws, mode))) halo = false;
  VST_CHECK_ARG(halo || ws_floats >= rowtiled_floats);
  if (halo) {
    const WhPlan p = wgrad_halo_plan(N, Cout, Cin, Hs, Ws, mode);
    hipStream_t st = (hipStream_t)stream;
    int rc = wgrad_halo_launch(p, dy, x, workspace, N, Cout, Cin, Hs, Ws, gmode, mode, st);
    if (rc) return rc;
    const long total = (long)Cout * 9 * Cin;
    wgrad_reduce_kernel<<<ceil_div(total, 256), 256, 0, st>>>(workspace, dw, p.NB, Cout, p.Mpad, 9 * Cin, Cin, 3, 3, 0,
                                                             1.0f, accumulate);
    return vst_launch_status();
  }
  long J = (long)KH * KW * Cin;
  int S = splits_for(N, Cout, J, Ho * Wo);
  hipStream_t st = (hipStream_t)stream;
  int rc = run_wg(dy, x, workspace, N, Cout, Cin, Hs, Ws, Ho, Wo, KH, KW, gmode, stride, pad, up, S, 0, 0, mode, st);
  if (rc) return rc;
  int c = wsel(Cout);
  long Mpad = (Cout + wbm(c) - 1) / wbm(c) * wbm(c), Jpad = (J + WBN - 1) / WBN * WBN;
  long total = (long)Cout * J;
  wgrad_reduce_kernel<<<ceil_div(total, 256), 256, 0, st>>>(workspace, dw, N * S, Cout, (int)Mpad, (int)Jpad, Cin, KH,
                                                           KW, 0, 1.0f, accumulate);
  return vst_launch_status();
}

// Weight gradient of a stride-1 reflect-padded KxK conv with few output channels (ConvTanh 48->3,
// k9, RC/network.py:169): GEMM rows m = (co, kh) (27 for 3x9 instead of 3 padded to 32), columns
// j = (kw, ci), reduction over the (H+K-1) x W grid of padded rows q:
//   dW[co][ci][kh][kw] = sum_q dy[co][q_y - kh][q_x] * Xpad[ci][q_y][q_x + kw]
int vst_conv_wgrad_rowsplit(const float* dy, const float* x, float* dw, float* workspace, int N, int Cin, int H,
                            int W, int Cout, int K, int accumulate, int mode, void* stream) {
  VST_CHECK_ARG(vst_mode_ok(mode));
  VST_CHECK_ARG(dy && x && dw && workspace && N > 0 && Cin > 0 && Cout > 0 && K > 0 && (K & 1) && K / 2 < H &&
                K / 2 < W);
  const int M = Cout * K, J = K * Cin, Hq = H + K - 1;
  int S = splits_for(N, M, J, Hq * W);
  hipStream_t st = (hipStream_t)stream;
  int rc = run_wg(dy, x, workspace, N, M, Cin, H, W, Hq, W, 1, K, 0, 1, K / 2, 1, S, K, H, mode, st);
  if (rc) return rc;
  int c = wsel(M);
  long Mpad = (M + wbm(c) - 1) / wbm(c) * wbm(c), Jpad = ((long)J + WBN - 1) / WBN * WBN;
  long total = (long)Cout * Cin * K * K;
  wgrad_reduce_kernel<<<ceil_div(total, 256), 256, 0, st>>>(workspace, dw, N * S, Cout, (int)Mpad, (int)Jpad, Cin, K, K,
                                                           1, 1.0f, accumulate);
  return vst_launch_status();
}

// G[n] = F[n] F[n]^T * scale,  F = [N][C][H*W]
int vst_gram(const float* f, float* g, float* workspace, int N, int C, int HW, float scale, int mode, void* stream) {
  VST_CHECK_ARG(vst_mode_ok(mode));
  VST_CHECK_ARG(f && g && workspace && N > 0 && C > 0 && HW > 0);
  int S = splits_for(N, C, C, HW);
  hipStream_t st = (hipStream_t)stream;
  int rc = run_wg(f, f, workspace, N, C, C, 1, HW, 1, HW, 1, 1, 1, 1, 0, 1, S, 0, 0, mode, st);
  if (rc) return rc;
  int c = wsel(C);
  long Mpad = (C + wbm(c) - 1) / wbm(c) * wbm(c), Jpad = (C + WBN - 1) / WBN * WBN;
  long total = (long)N * C * C;
  gram_reduce_kernel<<<ceil_div(total, 256), 256, 0, st>>>(workspace, g, N, S, C, C, (int)Mpad, (int)Jpad, scale);
  return vst_launch_status();
}

// out[n][m][j] = scale * sum_r a[n][m][r] * b[n][j][r]   (per-image A B^T; AdaAttN moments,
// attention query gradient, cosine-distance C x C products)
int vst_gemm_abt(const float* a, const float* b, float* out, float* workspace, int N, int M, int J, int R, float scale,
                 int mode, void* stream) {
  VST_CHECK_ARG(vst_mode_ok(mode));
  VST_CHECK_ARG(a && b && out && workspace && N > 0 && M > 0 && J > 0 && R > 0);
  int S = splits_for(N, M, J, R);
  hipStream_t st = (hipStream_t)stream;
  int rc = run_wg(a, b, workspace, N, M, J, 1, R, 1, R, 1, 1, 1, 1, 0, 1, S, 0, 0, mode, st);
  if (rc) return rc;
  int c = wsel(M);
  long Mpad = (M + wbm(c) - 1) / wbm(c) * wbm(c), Jpad = ((long)J + WBN - 1) / WBN * WBN;
  long total = (long)N * M * J;
  gram_reduce_kernel<<<ceil_div(total, 256), 256, 0, st>>>(workspace, out, N, S, M, J, (int)Mpad, (int)Jpad, scale);
  return vst_launch_status();
}

}  // extern "C"
