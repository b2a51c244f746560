// Weight gradient of a 3x3 stride-1 pad-1 convolution (reflect or zero border) with the input rows
// staged once for all nine taps ("halo" weight gradient).
//
//   dW[co][ci][kh][kw] = sum_{n, y, x} dY[n][co][y][x] * X[n][ci][y + kh - 1][x + kw - 1]
//
// RC/network.py:72-75 (ResidualBlock convs, RC/network.py:136-150), AA/network.py:9-33 (the AdaAttN
// decoder's Conv / ConvReLU): the weight half of their Conv2d backward.
//
// The row-tiled kernel (wgrad2_kernel) owns one tap per GEMM column: for every 16-pixel k-tile each
// of the nine taps gathers its own shifted copy of the source window and splits it into bf16 pieces,
// so every input element is loaded and split nine times per output row that reads it.  Here a block
// owns ALL nine taps of a 32-channel block (288 GEMM columns) and walks a strip of the output DOWN its
// rows, one strip row (KT k-tiles of 16 pixels: 16 columns under bf16x6, 32 / 64 under the single
// products, wh_kt) per step:
//   * the source rows y - 1, y, y + 1 sit in a four-slot LDS ring, so each step loads and splits ONE
//     new source row (strip width + 2 columns) per channel -- the other two were staged by the previous
//     steps;
//   * each staged row is written as three copies shifted by kw = 0, 1, 2 columns, so every tap's B
//     fragment is an aligned 16-byte LDS read (the odd shift re-pairs the split bf16 dwords with
//     v_alignbit, no second split);
//   * the dY tile (A operand, BM rows x 16 pixels) is split once per step and shared by the nine taps.
// Wave (wm, kh) computes weight rows m0 + 32 wm .. +31 for the three taps (kh, 0..2) of its row.
// Each block accumulates G consecutive (strip, row chunk) segments of one image into a private slab
// [Mpad][9 Cs] (the split-K slab layout of wgrad2_kernel: column j = (kh*3 + kw)*Cs + ci), and
// wgrad_reduce_kernel sums the slabs in a fixed order (deterministic, no atomics).
#include "vst_common.h"
#include "wgrad_halo.h"

namespace {

constexpr int WH_BK = 16;  // pixels per k-tile (one output row of a 16-column strip)
constexpr int WH_CB = 32;  // input channels per block (one MFMA column tile per tap)

// waves per SIMD the registers must allow: 3 (two 6-wave blocks or one 12-wave block per CU).  The
// single-product modes wait on their staging loads most of the time (config 5: 80 % of wave time), but
// twice the resident blocks does not help: fp16 decoder shapes (tools/wgrad_bench.py, one box) at 3 /
// 5 / 6 waves per SIMD: 512 ch 1.46 / 1.46 / 1.30 ms, 256 ch 1.43 / 1.43 / 1.65, 128 ch 1.69 / 1.68 /
// 2.00, 64 ch 3.62 / 5.09 / 5.26 (twice the slabs to write and reduce, and the blocks' rows no longer
// share one XCD's L2); config 5 139.0 -> 142.8 ms at 6.  Nor does a barrier per two output rows of a
// 16-column strip (6 MFMAs per wave per step instead of 3, an eight-slot source ring): 512 / 256 / 128
// / 64 ch 1.46 / 1.60 / 1.78 / 3.64 ms against 1.46 / 1.54 / 1.68 / 3.65 -- the 64-byte dY and source
// row pieces of a 16-column strip, half a cache line each, are what the waves wait on: wider strips
// for the single products (wh_kt below) are what helps.
constexpr int WH_WAVES = 3;

// k-tiles (16-pixel column groups) per strip row: two (bf16x6, and the single-product modes on the
// 6-wave 64-row blocks), four (single products on the 12-wave 128-row blocks) -- a 32-column strip row
// is a whole 128-byte line of dY and of x, and 3 KT (x the mode's products) MFMAs per wave per barrier.
// fp16 decoder shapes (tools/wgrad_bench.py, one box; 16 / 32 / 64 columns): 512 ch 1.46 / 1.50 / 1.41
// ms, 256 ch 1.53 / 1.46 / 1.37, 128 ch 1.67 / 1.55 / 1.45, 64 ch (64 rows) 3.65 / 2.68 / 2.76, 128 -> 64
// ch (64 rows) 1.11 / 0.81 / 1.16 (the 64-column strips' LDS leaves one 6-wave block per CU); bf16x6
// (16 / 32 columns): residual 192 ch 0.595 / 0.578 (row-tiled 0.619), decoder 512 ch 2.87 / 2.75,
// 256 ch 2.87 / 2.78, 128 ch 3.18 / 2.96, 64 ch 5.71 / 4.52
constexpr int wh_kt(int prec, int wm) { return prec == 3 ? 2 : (wm == 4 ? 4 : 2); }

template <int WM, int PREC, int GMODE>
__global__ __launch_bounds__(WM * 3 * 64, WH_WAVES) void wgrad_halo_kernel(WhParams P) {
  static_assert(PREC == 2 || PREC == 3 || PREC == 4, "halo wgrad: bf16x6, bf16 or fp16 products");
  constexpr int NTH = WM * 3 * 64;
  constexpr int BM = WM * 32;
  constexpr int NPC = PREC == 3 ? 3 : 1;   // bf16 pieces per value
  constexpr int LS = NPC * 8 + 4;          // LDS dwords per (row | channel) of a k-tile (+4: conflict-free)
  constexpr int KT = wh_kt(PREC, WM);     // k-tiles per strip row (strip = 16 KT columns)
  constexpr int A_TASKS = 4 * BM;          // (row, 4-pixel quarter) per k-tile: waves 0 .. 2 WM - 1
  constexpr int B_WAVE = A_TASKS / 64;     // the 128 (channel, 4-pixel quarter) B tasks: the next two waves
  constexpr int NRV = KT * 6 > 10 ? KT * 6 : 10;  // staged floats per thread (A 4 per k-tile, B 6)
  constexpr int OOR = 0x7ffffff0;
  static_assert(B_WAVE + 2 <= WM * 3, "staging waves");

  __shared__ __attribute__((aligned(16))) float As[2][KT][BM][LS];
  __shared__ __attribute__((aligned(16))) float Bs[4][3][KT][WH_CB][LS];  // [ring slot][kw copy][k-tile][channel]

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int lo = lane & 31, hi = lane >> 5;
  const int wm = wave % WM, kh = wave / WM;

  // work order: channel block fastest, then M tile, then (image, slab): the channel blocks of one
  // segment share its dY rows through one XCD's L2
  const int gx = gridDim.x, gy = gridDim.y;
  const int wk = xcd_remap(blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z), gx * gy * gridDim.z);
  const int rest = __builtin_amdgcn_readfirstlane(wk / gx), bz = __builtin_amdgcn_readfirstlane(rest / gy);
  const int c0 = __builtin_amdgcn_readfirstlane((wk - rest * gx) * WH_CB);
  const int m0 = __builtin_amdgcn_readfirstlane((rest - bz * gy) * BM);
  const int H = P.H, W = P.W, HW = H * W;
  // (the image's buffer descriptors, rebuilt per segment: segments of one block may span images)
  __amdgpu_buffer_rsrc_t asrd, xsrd;

  // staging task of this thread, wave-uniform kind (no divergent A / B paths inside a wave)
  const bool is_b = wave == B_WAVE || wave == B_WAVE + 1;
  const int bt = tid - 64 * B_WAVE;  // B task: (channel, quarter)
  const int at = tid;   // A task: (row, quarter)
  const bool a_ok = at < A_TASKS;
  // (a 16-lane store group = 8 rows x 2 quarters: its ds_write_b64 cover 32 distinct banks with the
  // 28-dword row stride, where 16 rows of one quarter would hit each bank pair twice)
  const int a_row = a_ok ? 8 * ((at >> 4) >> 1) + (at & 7) : 0;
  const int a_q = a_ok ? 2 * ((at >> 4) & 1) + ((at >> 3) & 1) : 0;
  const bool a_live = a_ok && m0 + a_row < P.M;
  const int a_voff = a_live ? ((m0 + a_row) * HW + 4 * a_q) * 4 : OOR;
  const int b_c = 8 * ((bt >> 4) & 3) + (bt & 7), b_q = 2 * ((bt >> 6) & 1) + ((bt >> 3) & 1);  // (same grouping)
  const int b_cbase = (c0 + b_c) * HW;

  f32x16 acc[3];
#pragma unroll
  for (int j = 0; j < 3; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;

  float rv0[NRV], rv1[NRV];  // staged values of one step; bf16x6 keeps two steps in flight

  // source row / column maps (reflect or zero border); -1 = zero
  auto src_row = [&](int yy) -> int {
    if (GMODE == 0) {
      yy = yy < 0 ? -yy : yy;
      return yy >= H ? 2 * H - 2 - yy : yy;
    }
    return (yy >= 0 && yy < H) ? yy : -1;
  };
  auto src_col = [&](int xx) -> int {
    if (GMODE == 0) {
      xx = xx < 0 ? -xx : xx;
      return xx >= W ? 2 * W - 2 - xx : xx;
    }
    return (xx >= 0 && xx < W) ? xx : -1;
  };

  // global loads of one step's staging, per k-tile t: the dY quarter row (A task) of output row y, or
  // the 6 source values x[c][row(yb)][ox0 + 16 t + 4q - 1 .. + 4] (B task) of logical source row yb
  auto load_a = [&](float (&rv)[NRV], int y, int ox0) {
#pragma unroll
    for (int t = 0; t < KT; ++t) {
      const int soff = __builtin_amdgcn_readfirstlane((y * W + ox0 + WH_BK * t) * 4);
      const f32x4 v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(asrd, a_voff, soff, 0));
#pragma unroll
      for (int e = 0; e < 4; ++e) rv[4 * t + e] = v[e];
    }
  };
  auto load_b1 = [&](float* rv, int yb, int ox0) {
    const int sy = src_row(yb);
    const int x0 = ox0 + 4 * b_q - 1;
    if (sy >= 0 && x0 >= 0 && x0 + 5 < W) {
      const int vo = (b_cbase + sy * W + x0) * 4;
      const f32x4 v0 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xsrd, vo, 0, 0));
      const f32x2 v1 = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(xsrd, vo + 16, 0, 0));
#pragma unroll
      for (int e = 0; e < 4; ++e) rv[e] = v0[e];
      rv[4] = v1[0];
      rv[5] = v1[1];
    } else {
#pragma unroll
      for (int e = 0; e < 6; ++e) {
        const int sx = src_col(x0 + e);
        const int vo = (sy >= 0 && sx >= 0) ? (b_cbase + sy * W + sx) * 4 : OOR;
        rv[e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xsrd, vo, 0, 0));
      }
    }
  };
  auto load_b = [&](float (&rv)[NRV], int yb, int ox0) {
#pragma unroll
    for (int t = 0; t < KT; ++t) load_b1(rv + 6 * t, yb, ox0 + WH_BK * t);
  };
  auto load_stage = [&](float (&rv)[NRV], int y, int yb, int ox0) {
    if (is_b) load_b(rv, yb, ox0);
    else if (a_ok) load_a(rv, y, ox0);
  };

  // split a pair into the mode's pieces (packed dwords, element 0 low)
  auto split_pair = [&](float u, float v, uint32_t (&d)[3]) {
    if constexpr (PREC == 3) {
      split3_bf16x2(u, v, d[0], d[1], d[2]);
    } else {
      uint32_t l;
      split2<PREC>(u, v, d[0], l);
    }
  };
  auto store_a = [&](const float (&rv)[NRV], int buf) {
    if (!a_ok) return;
#pragma unroll
    for (int t = 0; t < KT; ++t) {
      uint32_t p0[3], p1[3];
      split_pair(rv[4 * t], rv[4 * t + 1], p0);
      split_pair(rv[4 * t + 2], rv[4 * t + 3], p1);
      uint32_t* d = reinterpret_cast<uint32_t*>(&As[buf][t][a_row][0]) + 2 * a_q;
#pragma unroll
      for (int pc = 0; pc < NPC; ++pc) *reinterpret_cast<u32x2*>(d + 8 * pc) = u32x2{p0[pc], p1[pc]};
    }
  };
  // copy kw holds x[ox0 + i + kw - 1], i = 4q .. 4q + 3: from the quarter's 6 values v = x[ox0 + 4q - 1 ..]
  // copies 0 and 2 are the pairs (v0 v1)(v2 v3) and (v2 v3)(v4 v5); copy 1 re-pairs them
  auto store_b = [&](const float (&rv)[NRV], int slot) {
#pragma unroll
    for (int t = 0; t < KT; ++t) {
      uint32_t p[3][3];
#pragma unroll
      for (int q = 0; q < 3; ++q) split_pair(rv[6 * t + 2 * q], rv[6 * t + 2 * q + 1], p[q]);
#pragma unroll
      for (int pc = 0; pc < NPC; ++pc) {
        const int o = 8 * pc + 2 * b_q;
        *reinterpret_cast<u32x2*>(reinterpret_cast<uint32_t*>(&Bs[slot][0][t][b_c][0]) + o) = u32x2{p[0][pc], p[1][pc]};
        *reinterpret_cast<u32x2*>(reinterpret_cast<uint32_t*>(&Bs[slot][2][t][b_c][0]) + o) = u32x2{p[1][pc], p[2][pc]};
        *reinterpret_cast<u32x2*>(reinterpret_cast<uint32_t*>(&Bs[slot][1][t][b_c][0]) + o) =
            u32x2{__builtin_amdgcn_alignbit(p[1][pc], p[0][pc], 16), __builtin_amdgcn_alignbit(p[2][pc], p[1][pc], 16)};
      }
    }
  };
  auto store_stage = [&](const float (&rv)[NRV], int buf, int slot) {
    if (is_b) store_b(rv, slot);
    else store_a(rv, buf);
  };

  // the three taps (kh, kw = 0..2) of this wave for strip row y, k-tiles t = 0 .. KT-1 (A buffer buf)
  auto compute = [&](int y, int buf) {
    const int slot = (y + kh + 3) & 3;  // logical source row y + kh - 1
#pragma unroll
    for (int t = 0; t < KT; ++t) {
    const float* ap = &As[buf][t][wm * 32 + lo][4 * hi];
    bf16x8_t af[3];
#pragma unroll
    for (int pc = 0; pc < NPC; ++pc) af[pc] = *reinterpret_cast<const bf16x8_t*>(ap + 8 * pc);
    bf16x8_t bfr[3][3];
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const float* bp = &Bs[slot][kw][t][lo][4 * hi];
#pragma unroll
      for (int pc = 0; pc < NPC; ++pc) bfr[kw][pc] = *reinterpret_cast<const bf16x8_t*>(bp + 8 * pc);
    }
    if constexpr (KT == 1) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      f32x16 c = acc[kw];
      if constexpr (PREC == 3) {
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[2], bfr[kw][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[1], bfr[kw][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0], bfr[kw][2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[1], bfr[kw][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0], bfr[kw][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0], bfr[kw][0], c, 0, 0, 0);
      } else if constexpr (PREC == 4) {
        c = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8_t, af[0]),
                                                   __builtin_bit_cast(f16x8_t, bfr[kw][0]), c, 0, 0, 0);
      } else {
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0], bfr[kw][0], c, 0, 0, 0);
      }
      acc[kw] = c;
    }
    }
  };

  // this block's segments: its share [T bz / NB, T (bz + 1) / NB) of the T = N x strips x row chunks
  // segments of the tile pair, image-major, then strip, then chunk (consecutive segments of a block
  // are neighbouring strips of one image)
  const int nstrip = W / (WH_BK * KT);
  const int nseg = nstrip * P.nchunk;
  const int T = P.N * nseg;
  const int g0 = __builtin_amdgcn_readfirstlane((int)((long)T * bz / P.NB));
  const int g1 = __builtin_amdgcn_readfirstlane((int)((long)T * (bz + 1) / P.NB));
  for (int g = g0; g < g1; ++g) {
    const int n = g / nseg, gi = g - n * nseg;
    const int strip = gi / P.nchunk, chunk = gi - strip * P.nchunk;
    asrd = uniform_rsrc(P.a + (long)n * P.M * HW, (uint32_t)((long)P.M * HW * 4));
    xsrd = uniform_rsrc(P.x + (long)n * P.Cs * HW, (uint32_t)((long)P.Cs * HW * 4));
    const int ox0 = __builtin_amdgcn_readfirstlane(strip * WH_BK * KT);
    const int y0 = __builtin_amdgcn_readfirstlane(chunk * P.rch);
    const int y1 = __builtin_amdgcn_readfirstlane(min(H, y0 + P.rch));
    // prologue: source rows y0 - 1 and y0 into their ring slots, A(y0) and row y0 + 1; the registers
    // then hold tile y0 + 1's staging
    if (is_b) {
      load_b(rv0, y0 - 1, ox0);
      store_b(rv0, (y0 + 3) & 3);
      load_b(rv0, y0, ox0);
      store_b(rv0, y0 & 3);
    }
    load_stage(rv0, y0, y0 + 1, ox0);
    store_stage(rv0, y0 & 1, (y0 + 1) & 3);
    if (y0 + 1 < y1) load_stage(rv0, y0 + 1, y0 + 2, ox0);
    __syncthreads();
    // step y: LDS holds A(y) and source rows y - 1 .. y + 1; the registers hold tile y + 1 (loaded
    // during step y - 1), stored into the A buffer and ring slot tile y does not read.
    // Single products: store first, then issue tile y + 2's loads into the same registers and run tile
    // y's MFMAs over them (the store's wait is exact: no younger load pending).  bf16x6: tile y + 2's
    // loads go into a second register set before the MFMAs and the store (the VALU-heavy three-way
    // split) follows them, beside the other waves' MFMAs.  Measured on the residual / decoder shapes
    // (tools/wgrad_bench.py, one box each): bf16x6 store-first 1.08 / 0.74 of the row-tiled kernel's
    // time, this order 1.01 / 0.69; fp16 store-first 0.63 / 0.59, the bf16x6 order 0.70 / 0.72.
    if constexpr (PREC != 3) {
      for (int y = y0; y < y1; ++y) {
        if (y + 1 < y1) store_stage(rv0, (y + 1) & 1, (y + 2) & 3);
        if (y + 2 < y1) load_stage(rv0, y + 2, y + 3, ox0);
        compute(y, y & 1);
        __syncthreads();
      }
    } else {
      auto step = [&](int y, float (&cur)[NRV], float (&nxt)[NRV]) {
        if (y + 2 < y1) load_stage(nxt, y + 2, y + 3, ox0);
        compute(y, y & 1);
        if (y + 1 < y1) store_stage(cur, (y + 1) & 1, (y + 2) & 3);
        __syncthreads();
      };
      for (int y = y0; y < y1; y += 2) {
        step(y, rv0, rv1);
        if (y + 1 < y1) step(y + 1, rv1, rv0);
      }
    }
  }

  // raw sums of this block's segments: slab[bz][m][(kh*3 + kw)*Cs + c0 + lo] (each tile pair's block
  // bz writes its own region of slab bz, so the NB slabs together cover every (m, j))
  float* slab = P.slab + (long)bz * P.Mpad * P.J;
#pragma unroll
  for (int kw = 0; kw < 3; ++kw) {
    const int j = (kh * 3 + kw) * P.Cs + c0 + lo;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * hi;
      if (m < P.M) slab[(long)m * P.J + j] = acc[kw][r];
    }
  }
}

template <int PREC, int GMODE>
void launch_wm(int wm, dim3 g, hipStream_t st, const WhParams& P) {
  if (wm == 4) wgrad_halo_kernel<4, PREC, GMODE><<<g, 768, 0, st>>>(P);
  else wgrad_halo_kernel<2, PREC, GMODE><<<g, 384, 0, st>>>(P);
}

template <int PREC>
void launch_prec(int wm, int gmode, dim3 g, hipStream_t st, const WhParams& P) {
  if (gmode == 0) launch_wm<PREC, 0>(wm, g, st, P);
  else launch_wm<PREC, 1>(wm, g, st, P);
}

}  // namespace

// block rows (32 x WM) for M weight rows: 64 (the 192- and 64-row layers), 128 for 128-multiples
static int wgrad_halo_bm(int M) { return (M % 128 == 0) ? 128 : 64; }

// Feasibility only (3x3 stride-1 pad-1, 32-channel blocks, 16-column strips); which layers use it is
// the caller's choice (VST_GEMM_PERTAP in the mode selects the row-tiled kernel: vst/ops.py keeps
// ReCoNet's bf16x6 residual layers there, where the halo form only ties it and overlaps the
// data-gradient GEMMs worse on the side stream).
bool wgrad_halo_ok(int M, int Cs, int H, int W, int KH, int KW, int stride, int pad, int up, int gmode, int mode) {
  const int am = vst_mode_arith(mode);
  return KH == 3 && KW == 3 && stride == 1 && pad == 1 && up == 1 && (gmode == 0 || gmode == 1) &&
         Cs % WH_CB == 0 && W % (WH_BK * wh_kt(am, wgrad_halo_bm(M) / 32)) == 0 && H >= 2 && W >= 2 &&
         (am == VST_GEMM_BF16X6 || am == VST_GEMM_BF16 || am == VST_GEMM_F16);
}

// Split plan: one resident round of blocks (two 6-wave blocks or one 12-wave block per CU), NB
// blocks per (channel block, M tile) pair, each summing a contiguous share of the pair's
// (image, strip, row chunk) segments into its own slab -- NB slabs of Mpad x 9 Cs whatever the batch
// and image size.  Row chunks halve (down to 16 rows; each costs a two-row ring prologue) until
// every block has >= 4 segments, so the shares differ by at most a quarter.
WhPlan wgrad_halo_plan(int N, int M, int Cs, int H, int W, int mode) {
  WhPlan p;
  const int bm = wgrad_halo_bm(M);
  p.Mpad = (M + bm - 1) / bm * bm;
  const int nstrip = W / (WH_BK * wh_kt(vst_mode_arith(mode), bm / 32));
  const int pairs = (Cs / WH_CB) * (p.Mpad / bm);
  const int slots = 256 * (4 * WH_WAVES / (3 * (bm / 32)));
  p.NB = slots / pairs > 1 ? slots / pairs : 1;
  p.nchunk = 1;
  while ((long)N * nstrip * p.nchunk < 4L * p.NB && (H + 2 * p.nchunk - 1) / (2 * p.nchunk) >= 16) p.nchunk *= 2;
  p.rch = (H + p.nchunk - 1) / p.nchunk;
  p.nchunk = (H + p.rch - 1) / p.rch;
  const long T = (long)N * nstrip * p.nchunk;
  if (p.NB > T) p.NB = (int)T;
  return p;
}

long wgrad_halo_slab_floats(int N, int Cs, const WhPlan& p) {
  (void)N;
  return (long)p.NB * p.Mpad * 9L * Cs;
}

int wgrad_halo_launch(const WhPlan& p, const float* dy, const float* x, float* slab, int N, int M, int Cs, int H,
                      int W, int gmode, int mode, hipStream_t st) {
  WhParams P;
  P.a = dy;
  P.x = x;
  P.slab = slab;
  P.M = M;
  P.Mpad = p.Mpad;
  P.J = 9 * Cs;
  P.Cs = Cs;
  P.H = H;
  P.W = W;
  P.nchunk = p.nchunk;
  P.rch = p.rch;
  P.NB = p.NB;
  P.N = N;
  const int bm = wgrad_halo_bm(M);
  dim3 g(Cs / WH_CB, P.Mpad / bm, P.NB);
  const int wm = bm / 32;
  switch (vst_mode_arith(mode)) {
    case VST_GEMM_BF16X6: launch_prec<3>(wm, gmode, g, st, P); break;
    case VST_GEMM_F16: launch_prec<4>(wm, gmode, g, st, P); break;
    default: launch_prec<2>(wm, gmode, g, st, P); break;
  }
  return vst_launch_status();
}
