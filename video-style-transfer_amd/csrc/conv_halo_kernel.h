// 3x3 stride-1 convolution with the input patch staged once per 16-channel block ("halo" tiles).
//
// The per-tap implicit GEMM (conv_gemm_kernel) gathers, splits and stores a fresh B tile for every
// 16-deep k-tile: with the channel-blocked K order (VST_GEMM_KBLOCK) the nine k-tiles of one
// channel block are the nine taps, i.e. the same source pixels shifted -- each input element is
// gathered, split into its bf16 pieces and written to LDS nine times, with a barrier per tap.
// Here a block owns a TH x TW output tile (4 rows x 32 columns = 128 pixels) and, per 16-channel
// block, stages the (TH+2) x (TW+2) source patch ONCE (gather with the reflect / zero border
// folded in, optional ReLU mask of the data gradient applied, split, one LDS store per piece); the
// nine taps then read their B fragments from that patch at shifted positions (compile-time LDS
// offsets) -- one gather + split + store + barrier per 9 k-tiles instead of per k-tile.  The A
// operand (packed weights) goes straight from memory into each wave's MFMA registers, one tap
// ahead (the A-direct scheme of conv_gemm_kernel: one wave per 32 weight rows).
//
// The k-tile sequence (channel block major, tap minor) and the per-k-tile MFMA sequence are those of
// conv_gemm_kernel under VST_GEMM_KBLOCK, so the two kernels produce bitwise-identical results
// (tests/test_gpu_halo.py).  Covers every 3x3 stride-1 conv on the training paths: VGG16 / VGG19
// convs (zero pad 1, RC/network.py:9-40, AA/vgg19.py:19-37), ReCoNet / AdaAttN residual and decoder
// convs (reflect pad 1, RC/network.py:72-75,145-150, AA/network.py:9-33), and their data gradients
// (the transposed gather over dY, zero pad; RC ResidualBlock's over the padded grid, EPI_PADOUT).
#pragma once
#include "conv_gemm_kernel.h"

namespace vstk {

// taps of A preloaded ahead of the patch on the double-buffered single-product tiles (conv_halo_kernel):
// five keep the 4- and 8-wave tiles at 126 / 116 VGPRs (4 waves per SIMD); config 5, fp16 kernel trace:
// 8-wave 763 -> 726 us, 4-wave 951 -> 921 us against one (profiles/r06_thin_halo_c5_kernel_summary.txt,
// profiles/r06_apre_c5_kernel_summary.txt)
constexpr int HALO_APRE_DB = 5;
// and under the split products (bf16x6 / bf16x3: 12 / 8 VGPRs a tap) on the 3x3 one-buffer and 8-wave
// tiles; the 4-wave double-buffered and the 9x1 / 1x9 tiles keep one (their registers would cost a
// wave per SIMD)
constexpr int HALO_APRE_SPLIT = 2;
constexpr int HTW = 32;  // output tile width (one MFMA column block); each wave covers 4 rows of it

// One tap of a wave's 32 x 128 tile: the B fragments of output row j (LDS pixel rows jstride apart)
// stream through a two-deep register ring -- fragment j+1's reads are issued before fragment j's
// MFMAs -- instead of all TN fragments up front (24 fewer live VGPRs: the 4-wave-per-SIMD budget)
template <int TN, int PREC, int LS>
__device__ __forceinline__ void halo_tap(f32x16 (&acc)[1][TN], const bf16x8_t (&ar)[1][3], const float (*B)[LS],
                                         int lane, int jstride) {
  constexpr int NPC = PREC == 3 ? 3 : PREC == 1 ? 2 : 1;
  const int r = lane & 31, h = lane >> 5;
  bf16x8_t b[2][3];
  auto load = [&](int j, bf16x8_t (&d)[3]) {
    const float* p = &B[j * jstride + r][4 * h];
#pragma unroll
    for (int pc = 0; pc < NPC; ++pc) d[pc] = *reinterpret_cast<const bf16x8_t*>(p + 8 * pc);
  };
  load(0, b[0]);
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    if (j + 1 < TN) load(j + 1, b[(j + 1) & 1]);
    const bf16x8_t(&c)[3] = b[j & 1];
    f32x16 a = acc[0][j];
    if constexpr (PREC == 3) {
      a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ar[0][2], c[0], a, 0, 0, 0);
      a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ar[0][1], c[1], a, 0, 0, 0);
      a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ar[0][0], c[2], a, 0, 0, 0);
      a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ar[0][1], c[0], a, 0, 0, 0);
      a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ar[0][0], c[1], a, 0, 0, 0);
      a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ar[0][0], c[0], a, 0, 0, 0);
    } else if constexpr (PREC == 1) {  // bf16x3: lo*hi + hi*lo + hi*hi (mfma_bf16_ktile's order)
      a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ar[0][1], c[0], a, 0, 0, 0);
      a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ar[0][0], c[1], a, 0, 0, 0);
      a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ar[0][0], c[0], a, 0, 0, 0);
    } else if constexpr (PREC == 4) {
      a = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8_t, ar[0][0]), __builtin_bit_cast(f16x8_t, c[0]),
                                                 a, 0, 0, 0);
    } else {
      a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ar[0][0], c[0], a, 0, 0, 0);
    }
    acc[0][j] = a;
  }
}

// Block = WM x WN waves: wave (wm, wn) computes weight rows m0 + 32 wm .. +31 for output rows
// oy0 + 4 wn .. +3 (TN = 4 fragments of 32 pixels), so the tile is TH = 4 WN rows x 32 columns and
// the patch (TH + 2) x 34 pixels.  DB: double-buffered patch (the next channel block's stores need
// no second barrier) or one buffer (half the LDS: more blocks per CU, two barriers per block).
// PREC 3: bf16x6 (three bf16 pieces per value); 1: bf16x3 (hi / lo pieces, three products); 2 / 4:
// single bf16 / fp16 product (one piece).
// One 16-channel block per stage (one barrier per block).  (Several blocks per stage, meant to cover
// the single-product modes' first-touch gathers, measured slower -- fp16 VGG + residual shapes 2.38 ms
// at one block, 2.58 at 2, 2.61 at 4: the larger stage halves the resident blocks per CU,
// profiles/r04_halo_kc.txt -- and was removed in round 5.)
// KH x KW taps: 3 x 3 (the 3x3 stride-1 convs); 2 x 2 (the phase-stacked GEMMs of the stride-2 data
// gradient and the nearest-x2 upsample forward, EPI_PHASE2 -- patch (TH + 1) x 33, four taps); 9 x 1
// (the 9x9 layers over a kw-unfolded operand: ReCoNet conv1's forward and ConvTanh's data gradient,
// RC/network.py:78-85,158 -- patch (TH + 8) x 32, nine row taps, column pad P.pad_x = 0); 1 x 9
// (ConvTanh's row-split forward, RC/network.py:78-85: GEMM rows (co, kh), nine column taps over the
// reflect-padded rows -- patch TH x 40, on the 32-row block H1x4S).
template <int WM, int WN, int MINW, int PREC, bool GM, bool DB, int PD = 1, int KH = 3, int KW = KH>
__global__ __launch_bounds__(WM * WN * 64, MINW) void conv_halo_kernel(ConvParams P) {
  static_assert(PREC >= 1 && PREC <= 4, "halo kernel: bf16x3, bf16x6, bf16 or fp16 products");
  static_assert((KH == KW && (KH == 2 || KH == 3)) || (KH == 9 && KW == 1) || (KH == 1 && KW == 9),
                "halo kernel: 2x2, 3x3, 9x1 or 1x9 taps");
  constexpr int TM = 1, TN = 4, NTAP = KH * KW;
  constexpr int TH = 4 * WN, HPH = TH + KH - 1, HPW = HTW + KW - 1, HPP = HPH * HPW;
  constexpr int NTT = WM * WN * 64;
  constexpr int BM = WM * 32;
  constexpr int AW = PREC == 3 ? 24 : 16;  // packed A dwords per (k-tile, row) (vst_common.h apack_store)
  constexpr int NPC = PREC == 3 ? 3 : PREC == 1 ? 2 : 1;  // bf16 pieces per value in the patch
  constexpr int LS = NPC * 8 + 4;          // LDS dwords per patch pixel (+4 pad: conflict-free b128 reads)
  constexpr int NTASK = 2 * HPP;           // (patch pixel, channel octet)
  constexpr int TIT = (NTASK + NTT - 1) / NTT;
  constexpr int NBUF = DB ? 2 : 1;
  constexpr int OOR = 0x7ffffff0;
  __shared__ __attribute__((aligned(16))) float Ps[NBUF][HPP][LS];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int lo = lane & 31, hi = lane >> 5;
  const int wm = wave % WM, wn = wave / WM;
  // work order: M tile fastest, then pixel tile, then image (XCD-aware: the M tiles of one pixel
  // tile share its patch through one L2)
  const int gx = gridDim.x, gy = gridDim.y;
  const int wk = xcd_remap(blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z), gx * gy * gridDim.z);
  const int rest = __builtin_amdgcn_readfirstlane(wk / gy);
  const int nz = __builtin_amdgcn_readfirstlane(rest / gx);
  const int m0 = __builtin_amdgcn_readfirstlane((wk - rest * gy) * BM);
  const int tile = __builtin_amdgcn_readfirstlane(rest - nz * gx);
  // split-K: image n, slice s of the channel blocks (ConvParams::ksplit)
  const int n = __builtin_amdgcn_readfirstlane(nz / P.ksplit), ks = nz - n * P.ksplit;
  const int tiles_x = (P.Wo + HTW - 1) / HTW;
  const int ty = __builtin_amdgcn_readfirstlane(tile / tiles_x);
  const int oy0 = ty * TH, ox0 = (tile - ty * tiles_x) * HTW;
  // forward: source row oy - pad + kh; data gradient (transposed, stride 1): dY row oy + pad - kh
  const bool tr = P.gmode == GM_TRANSPOSED;
  const int y0 = oy0 + (tr ? P.pad - (KH - 1) : -P.pad), x0 = ox0 + (tr ? P.pad_x - (KW - 1) : -P.pad_x);

  const int plane = P.Hs * P.Ws;
  const long plane_l = (long)plane;
  const float* src_n = P.src + (long)n * P.Cs * plane_l;
  const uint32_t src_bytes = (uint32_t)P.Cs * (uint32_t)plane * 4u;
  const __amdgpu_buffer_rsrc_t srd = uniform_rsrc(src_n, src_bytes);
  const __amdgpu_buffer_rsrc_t gsrd = uniform_rsrc(GM ? P.gmask + (long)n * P.Cs * plane_l : src_n, src_bytes);
  const float* A = P.wpack + (long)n * P.a_batch_stride;
  const __amdgpu_buffer_rsrc_t asrd = uniform_rsrc(A, (uint32_t)((long)P.Kpad / BK * P.Mpad * AW * 4));
  const int ad_voff = ((wm * 32 + lo) * AW + 4 * hi) * 4;

  // this thread's patch tasks: pixel q (consecutive lanes -> consecutive pixels of a patch row),
  // channel octet o; the source offset of channel 8o of the block, or OOR (zero / outside)
  int t_voff[TIT], t_lds[TIT];
#pragma unroll
  for (int it = 0; it < TIT; ++it) {
    const int t = tid + it * NTT;
    const int o = t >= HPP ? 1 : 0, q = t - o * HPP;
    const int py = q / HPW, px = q - py * HPW;
    int y = y0 + py, x = x0 + px;
    if (P.gmode == GM_REFLECT) {
      y = abs(y);
      y = y >= P.Hs ? 2 * P.Hs - 2 - y : y;
      x = abs(x);
      x = x >= P.Ws ? 2 * P.Ws - 2 - x : x;
    } else if (P.gmode == GM_CLAMP) {  // (the up2 phase forward: the reflect border of the virtual grid)
      y = min(max(y, 0), P.Hs - 1);
      x = min(max(x, 0), P.Ws - 1);
    }
    const bool ok = t < NTASK && (unsigned)y < (unsigned)P.Hs && (unsigned)x < (unsigned)P.Ws;
    t_voff[it] = ok ? ((8 * o) * plane + y * P.Ws + x) * 4 : OOR;
    t_lds[it] = t < NTASK ? q * LS + 4 * o : -1;
  }
  const int cstep = __builtin_amdgcn_readfirstlane(plane * 4);  // bytes between channels

  f32x16 acc[TM][TN];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[0][j][r] = 0.f;

  const int nst_all = P.Cs / 16;
  const int st0 = __builtin_amdgcn_readfirstlane(ks * nst_all / P.ksplit);
  const int nst = __builtin_amdgcn_readfirstlane((ks + 1) * nst_all / P.ksplit);  // (this slice's end)
  float rv[TIT][8];
  float rgv[TIT][GM ? 8 : 1];
  // stage s = channel block s.  The prefetch of the stage after the last one is issued too, with every
  // offset out of range (the loads return zeros without touching memory): a prefetch under a branch
  // made the waitcnt pass merge its two paths conservatively -- the first tap's MFMA then waited for
  // the whole next patch (s_waitcnt vmcnt(1) behind 24 patch loads), so no gather ever overlapped the
  // taps
  auto load_into = [&](int st, auto& R, auto& G) {
    const bool live = st < nst;
    const int cb_off = __builtin_amdgcn_readfirstlane((live ? st : 0) * 16 * plane * 4);
#pragma unroll
    for (int it = 0; it < TIT; ++it) {
      const int vo = live ? t_voff[it] : OOR;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        R[it][i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(srd, vo, cb_off + i * cstep, 0));
        if constexpr (GM)
          G[it][i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(gsrd, vo, cb_off + i * cstep, 0));
      }
    }
  };
  auto store_from = [&](int buf, auto& R, auto& G) {
#pragma unroll
    for (int it = 0; it < TIT; ++it) {
      if (NTASK % NTT != 0 && t_lds[it] < 0) continue;
      float v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = GM ? (G[it][i] > 0.f ? R[it][i] : 0.f) : R[it][i];
      uint32_t* d = reinterpret_cast<uint32_t*>(&Ps[buf][0][0]) + t_lds[it];
      if constexpr (PREC == 3) {
        uint32_t h[4], md[4], l[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) split3_bf16x2(v[2 * q], v[2 * q + 1], h[q], md[q], l[q]);
        *reinterpret_cast<u32x4*>(d) = u32x4{h[0], h[1], h[2], h[3]};
        *reinterpret_cast<u32x4*>(d + 8) = u32x4{md[0], md[1], md[2], md[3]};
        *reinterpret_cast<u32x4*>(d + 16) = u32x4{l[0], l[1], l[2], l[3]};
      } else {
        uint32_t h[4], l[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) split2<PREC>(v[2 * q], v[2 * q + 1], h[q], l[q]);
        *reinterpret_cast<u32x4*>(d) = u32x4{h[0], h[1], h[2], h[3]};
        if constexpr (PREC == 1) *reinterpret_cast<u32x4*>(d + 8) = u32x4{l[0], l[1], l[2], l[3]};
      }
    }
  };
  // A fragments of k-tile kt (channel block cb, tap t: kt = NTAP cb + t under the blocked K order)
  bf16x8_t arN[TM][3], arC[TM][3];
  auto load_a = [&](int kt, bf16x8_t (&ar)[TM][3]) {
    const int a_soff = __builtin_amdgcn_readfirstlane(((kt * P.Mpad + m0) * AW) * 4);
#pragma unroll
    for (int pc = 0; pc < NPC; ++pc)
      ar[0][pc] = __builtin_bit_cast(bf16x8_t, __builtin_amdgcn_raw_buffer_load_b128(asrd, ad_voff, a_soff + 32 * pc, 0));
  };

  // The A fragments of the first APRE taps of a stage are loaded at the end of the previous stage,
  // ahead of the next patch's loads; later taps load theirs one tap ahead.  Vector-memory loads complete
  // in issue order, so a per-tap A load issued after the patch prefetch makes its tap wait for the whole
  // patch: with per-tap loads from tap 1 on, the prefetch overlapped one tap of nine.  APRE: all nine
  // taps on the single-product one-buffer tiles (3 waves per SIMD), five on the single-product
  // double-buffered ones and two (or one) under the split products (two or three pieces a tap), each
  // within the register budget of its tile's occupancy.
  constexpr int APRE = NPC == 1 ? (!DB ? NTAP : HALO_APRE_DB)
                                : ((KH == 3 && KW == 3 && (!DB || WM * WN >= 8)) ? HALO_APRE_SPLIT : 1);
  bf16x8_t arS[APRE > 1 ? APRE : 1][3];
  auto load_stage_a = [&](int cb) {
    const int c = cb < nst ? cb : 0;  // (past the slice: a harmless reload, unbranched)
#pragma unroll
    for (int t = 0; t < APRE; ++t) {
      const int a_soff = __builtin_amdgcn_readfirstlane((((NTAP * c + t) * P.Mpad + m0) * AW) * 4);
#pragma unroll
      for (int pc = 0; pc < NPC; ++pc)
        arS[t][pc] =
            __builtin_bit_cast(bf16x8_t, __builtin_amdgcn_raw_buffer_load_b128(asrd, ad_voff, a_soff + 32 * pc, 0));
    }
  };
  // the taps of every channel block of stage st, B fragments from patch buffer buf
  auto taps = [&](int cb, int buf) {
#pragma unroll
    for (int t = 0; t < NTAP; ++t) {
      const int kh = t / KW, kw = t % KW;
      const int ph = tr ? KH - 1 - kh : kh, pw = tr ? KW - 1 - kw : kw;  // (tr is block-uniform)
      // B fragments of tap t: output row 4 wn + j of the tile reads patch row 4 wn + j + ph,
      // columns lo + pw
      const float(*Bt)[LS] = &Ps[buf][(4 * wn + ph) * HPW + pw];
      if constexpr (APRE == 1) {
        // per-tap loads throughout: the last tap loads the next stage's first (past the slice's last
        // k-tile: a harmless reload of k-tile 0, unbranched)
        const int kt_next = t < NTAP - 1 ? NTAP * cb + t + 1 : (cb + 1 < nst ? NTAP * (cb + 1) : 0);
        load_a(kt_next, arN);
        halo_tap<TN, PREC, LS>(acc, arC, Bt, lane, HPW);
#pragma unroll
        for (int pc = 0; pc < NPC; ++pc) arC[0][pc] = arN[0][pc];
      } else {
        if (t + 1 >= APRE && t + 1 < NTAP) load_a(NTAP * cb + t + 1, arN);
        if (t < APRE) {
          const bf16x8_t a1[1][3] = {{arS[t][0], arS[t][1], arS[t][2]}};
          halo_tap<TN, PREC, LS>(acc, a1, Bt, lane, HPW);
        } else {
          halo_tap<TN, PREC, LS>(acc, arC, Bt, lane, HPW);
        }
        if (t + 1 >= APRE && t + 1 < NTAP) {
#pragma unroll
          for (int pc = 0; pc < NPC; ++pc) arC[0][pc] = arN[0][pc];
        }
      }
    }
  };
  load_into(st0, rv, rgv);
  if constexpr (APRE == 1) load_a(NTAP * st0, arC);
  else load_stage_a(st0);
  store_from(0, rv, rgv);
  if constexpr (PD == 1) {
    __syncthreads();
    for (int st = st0; st < nst; ++st) {
      const int buf = DB ? ((st - st0) & 1) : 0;
      load_into(st + 1, rv, rgv);
      // (the loads stay ahead of the taps: no code motion across, and the store below is unconditional
      // -- under `if (st + 1 < nst)` the IR sink pass moved the loads into that branch, after the taps)
      __builtin_amdgcn_sched_barrier(0);
      taps(st, buf);
      if constexpr (!DB) __syncthreads();  // every wave is done reading the one buffer
      store_from(DB ? buf ^ 1 : 0, rv, rgv);  // (after the last stage: zeros into a buffer nobody reads)
      if constexpr (APRE > 1) load_stage_a(st + 1);
      __syncthreads();
    }
  } else {
    // two patches in flight: stage st + 2's loads are issued before stage st's taps, into the
    // register set stage st + 1 is not stored from (the two sets alternate, loop unrolled by two)
    static_assert(PD == 2 && DB, "depth-2 patch prefetch: double-buffered tiles");
    float rvN[TIT][8];
    float rgvN[TIT][GM ? 8 : 1];
    load_into(st0 + 1, rv, rgv);
    __syncthreads();
    auto stage = [&](int st, auto& Rs, auto& Gs, auto& Rl, auto& Gl) {
      const int buf = (st - st0) & 1;
      load_into(st + 2, Rl, Gl);
      __builtin_amdgcn_sched_barrier(0);
      taps(st, buf);
      store_from(buf ^ 1, Rs, Gs);
      if constexpr (APRE > 1) load_stage_a(st + 1);
      __syncthreads();
    };
    // (pairs in the loop, an odd last stage after it: no branch around a stage inside the loop)
    int st = st0;
    for (; st + 1 < nst; st += 2) {
      stage(st, rv, rgv, rvN, rgvN);
      stage(st + 1, rvN, rgvN, rv, rgv);
    }
    if (st < nst) stage(st, rv, rgv, rvN, rgvN);
  }

  int pix[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int oy = oy0 + 4 * wn + j, ox = ox0 + lo;
    pix[j] = (oy < P.Ho && ox < P.Wo) ? oy * P.Wo + ox : -1;
  }
  if (P.ksplit > 1) {  // raw partial sums of this slice: part[ks][n][m][pixel]
    const long HWo = (long)P.Ho * P.Wo;
    float* pt = P.part + (long)(ks * (gridDim.z / P.ksplit) + n) * P.M * HWo;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      if (pix[j] < 0) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * hi;
        if (m < P.M) pt[m * HWo + pix[j]] = acc[0][j][r];
      }
    }
    return;
  }
  conv_epilogue<TM, TN>(P, acc, n, m0 + wm * 32, pix, hi);
}

// Block shape per layer width (M = weight rows): WM x WN waves, M tile 32 WM.  The packed A carries
// vst_conv_pack_dims' Mpad, which the M tile must divide (halo_cfg returns 0 otherwise).
// Measured per layer shape (tools/gemm_bench.py, one box, bf16x6 / fp16; profiles/r04_halo_shapes.txt):
//   M = 64  (VGG conv1_x, 256x512): 2x2 one buffer 746-758 us < 2x2 double 878 < 2x1 902 < per-tap 1071
//   M = 128 (VGG conv2_x): 4x1 619-664 < 4x2 685 < per-tap 751
//   M = 192 (ReCoNet residual, 64x128): 2x4 one buffer 354-391 us (fp16 110-118) < per-tap 413-452
//           (LDS-A tile) < 3x2 415-428, 6x1 428, 3x1 448; re-measured on one box:
//           2x2 one buffer 339 us (fp16 121) < 2x4 one buffer 363 (125) < 3x1 one buffer 379 (121);
//           the padded-grid data gradient 474 us on 2x2 one buffer (544 on 2x4): config 3 46.12 ms
//           with it on the halo kernel vs 46.61 per-tap (profiles/r04_halo_m192.txt)
//   2x4 one-buffer everywhere: 128-row layers 839 us, 256-row 695-770; 4x2 one-buffer: 932-1172 --
//   both slower than 4x1 / 8x1 (profiles/r04_halo_shapes.txt)
//   M = 256-multiples (VGG conv3_x / conv4_x): 8x1, 268-274 TF/s vs per-tap 233-245
// block shape of 64-, 128-, 192-row and 256-multiple layers (HaloCfg below)
constexpr int HALO_M64 = 3, HALO_M128 = 4, HALO_M192 = 3, HALO_M256 = 8;
// WM x WN waves (S: one patch buffer)
enum HaloCfg { H2x1 = 1, H2x2, H2x2S, H4x1, H4x2, H6x1, H3x2, H8x1, H2x4S, H3x1S, H3x2S, H4x2S, H1x4S };
constexpr int halo_wm_c(int c) { return c == H1x4S ? 1 : c == H2x1 || c == H2x2 || c == H2x2S || c == H2x4S ? 2
                                      : c == H4x1 || c == H4x2 || c == H4x2S ? 4 : c == H6x1 ? 6 : c == H8x1 ? 8 : 3; }
constexpr int halo_wn_c(int c) { return c == H2x4S || c == H1x4S ? 4 : (c == H2x2 || c == H2x2S || c == H4x2 || c == H3x2 || c == H3x2S || c == H4x2S) ? 2 : 1; }
constexpr bool halo_db_c(int c) { return !(c == H2x2S || c == H2x4S || c == H3x1S || c == H3x2S || c == H4x2S || c == H1x4S); }
inline int halo_wm(int c) { return halo_wm_c(c); }
inline int halo_wn(int c) { return halo_wn_c(c); }
// 0: the per-tap kernel (the M tile would not divide the pack's Mpad).  (The bf16x6 residual data
// gradient over the padded grid -- 66 x 130, a fifth of a 32-column tile grid wasted -- is slower than
// per-tap on the 2x4 block and faster on the 2x2 one, measured above: it runs here.)
inline int halo_cfg(int M, int pack_mpad) {
  int c;
  if (M <= 64) c = HALO_M64;
  else if (M % 256 == 0) c = HALO_M256;
  else if (M % 192 == 0 && M % 128 != 0) c = HALO_M192;
  else c = HALO_M128;
  return pack_mpad % (32 * halo_wm(c)) == 0 ? c : 0;
}

// waves per SIMD of the single-product one-buffer tiles: 3 -- the stage's nine A fragments (36 VGPRs) and
// the patch prefetch in flight across the taps do not fit 4 waves' 128 VGPRs without spills (round 5,
// with the prefetch sunk behind the taps by the compiler and per-tap A loads: 3 measured 142.31 vs
// 141.5 ms at 4)
constexpr int HALO_SMINW_SP = 3;
// patches in flight for the single-product double-buffered tiles: one.  The second register set (round 4)
// bought its gain through the compiler's placement of the first one's loads; with the loads pinned ahead
// of the taps and the taps' A loads ahead of them, a second patch in flight would still be waited for by
// the first per-tap A load after it (vector loads complete in order)
constexpr int HALO_PD = 1;
template <int C, int PR, bool GM, int KH = 3, int KW = KH>
void launch_halo_c(dim3 grid, hipStream_t st, const ConvParams& P) {
  constexpr int WM = halo_wm_c(C), WN = halo_wn_c(C);
  // waves per SIMD the registers must allow: one-buffer tiles 4 for the single-product modes (their
  // LDS admits 16 waves per CU) but 3 for bf16x6, whose three-piece fragments spill at the 128-VGPR
  // budget (measured: the spilling 2x2 tile 1088 us vs 758 us at 3 waves per SIMD on the 64-row VGG
  // layer; fp16 at 4 waves 118 us vs 150 us at 3 on the residual layer); 3 for 4-wave double-
  // buffered tiles, 2 for the 6- and 8-wave double-buffered ones
  constexpr int MINW = !halo_db_c(C) ? (PR == 3 || PR == 1 ? 3 : HALO_SMINW_SP) : (WM * WN <= 4 ? 3 : 2);
  // depth-2 patch prefetch (round 4: config 5 145.07 -> 141.5 ms, profiles/r04_halo_pd.txt) is off
  // (HALO_PD above)
  constexpr int PD = (PR != 3 && halo_db_c(C) && WM * WN >= 8) ? HALO_PD : 1;
  conv_halo_kernel<WM, WN, MINW, PR, GM, halo_db_c(C), PD, KH, KW><<<grid, WM * WN * 64, 0, st>>>(P);
}

// only the block shapes the build's selection can reach are instantiated
template <int PR, bool GM>
void launch_halo(int c, dim3 grid, hipStream_t st, const ConvParams& P) {
  if (c == HALO_M64) launch_halo_c<HALO_M64, PR, GM>(grid, st, P);
  else if (c == HALO_M128) launch_halo_c<HALO_M128, PR, GM>(grid, st, P);
  else if (c == HALO_M192) launch_halo_c<HALO_M192, PR, GM>(grid, st, P);
  else launch_halo_c<HALO_M256, PR, GM>(grid, st, P);
}

// the 2x2 phase-stacked GEMMs (no gather mask on their paths): M = 4 x channels, the 128- and 192-row
// selections (ReCoNet deconv1 / conv3: 384 rows; deconv2 / conv2: 192)
template <int PR>
void launch_halo2(int c, dim3 grid, hipStream_t st, const ConvParams& P) {
  if (c == HALO_M192) launch_halo_c<HALO_M192, PR, false, 2>(grid, st, P);
  else if (c == HALO_M128) launch_halo_c<HALO_M128, PR, false, 2>(grid, st, P);
  else if (c == HALO_M64) launch_halo_c<HALO_M64, PR, false, 2>(grid, st, P);
  else launch_halo_c<HALO_M256, PR, false, 2>(grid, st, P);
}

// the 9 x 1 GEMMs over kw-unfolded operands (48 weight rows: the 64-row selection; 128 for other widths)
template <int PR>
void launch_halo91(int c, dim3 grid, hipStream_t st, const ConvParams& P) {
  if (c == HALO_M64) launch_halo_c<HALO_M64, PR, false, 9, 1>(grid, st, P);
  else launch_halo_c<HALO_M128, PR, false, 9, 1>(grid, st, P);
}

// the 1 x 9 GEMM of the row-split forward (27 weight rows (co, kh) in a 32-row pack): one 32-row wave
// column, four wave rows (16 output rows per tile), one patch buffer
template <int PR>
void launch_halo19(dim3 grid, hipStream_t st, const ConvParams& P) {
  launch_halo_c<H1x4S, PR, false, 1, 9>(grid, st, P);
}

template <int PR>
void launch_halo_prec(bool gm, int c, int kh, dim3 grid, hipStream_t st, const ConvParams& P) {
  if (kh == 2) launch_halo2<PR>(c, grid, st, P);
  else if (kh == 9) launch_halo91<PR>(c, grid, st, P);
  else if (kh == 1) launch_halo19<PR>(grid, st, P);
  else gm ? launch_halo<PR, true>(c, grid, st, P) : launch_halo<PR, false>(c, grid, st, P);
}

extern template void launch_halo_prec<1>(bool, int, int, dim3, hipStream_t, const ConvParams&);
extern template void launch_halo_prec<2>(bool, int, int, dim3, hipStream_t, const ConvParams&);
extern template void launch_halo_prec<3>(bool, int, int, dim3, hipStream_t, const ConvParams&);
extern template void launch_halo_prec<4>(bool, int, int, dim3, hipStream_t, const ConvParams&);

}  // namespace vstk
