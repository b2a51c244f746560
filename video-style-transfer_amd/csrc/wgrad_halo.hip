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
// owns ALL nine taps of a 32-channel block (288 GEMM columns) and walks a 16-column strip of the
// output DOWN its rows, one k-tile (16 pixels of one output row y) per step:
//   * the source rows y - 1, y, y + 1 sit in a four-slot LDS ring, so each step loads and splits ONE
//     new source row (18 columns) per channel -- the other two were staged by the previous steps;
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

template <int WM, int PREC, int GMODE>
// (3 waves per SIMD: two 6-wave blocks, four 3-wave blocks or one 12-wave block per CU)
__global__ __launch_bounds__(WM * 3 * 64, 3) void wgrad_halo_kernel(WhParams P) {
  static_assert(PREC == 2 || PREC == 3 || PREC == 4, "halo wgrad: bf16x6, bf16 or fp16 products");
  constexpr int NTH = WM * 3 * 64;
  constexpr int BM = WM * 32;
  constexpr int NPC = PREC == 3 ? 3 : 1;   // bf16 pieces per value
  constexpr int LS = NPC * 8 + 4;          // LDS dwords per (row | channel) of a k-tile (+4: conflict-free)
  constexpr int R = NTH / 64;              // staging: one B task per R threads, A tasks on the rest
  constexpr int A_TASKS = 4 * BM;          // (row, 4-pixel quarter)
  constexpr int OOR = 0x7ffffff0;
  static_assert(64 * (R - 1) >= A_TASKS, "staging tasks");

  __shared__ __attribute__((aligned(16))) float As[2][BM][LS];
  __shared__ __attribute__((aligned(16))) float Bs[4][3][WH_CB][LS];  // [ring slot][kw copy][channel]

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
  const int n = __builtin_amdgcn_readfirstlane(bz / P.S);
  const int sidx = bz - n * P.S;
  const int H = P.H, W = P.W, HW = H * W;

  const float* a_n = P.a + (long)n * P.M * HW;
  const float* x_n = P.x + (long)n * P.Cs * HW;
  const __amdgpu_buffer_rsrc_t asrd = uniform_rsrc(a_n, (uint32_t)((long)P.M * HW * 4));
  const __amdgpu_buffer_rsrc_t xsrd = uniform_rsrc(x_n, (uint32_t)((long)P.Cs * HW * 4));

  // staging task of this thread
  const bool is_b = (tid % R) == 0;
  const int bt = tid / R;                                  // B task: channel bt % 32, half bt / 32
  const int at = (tid / R) * (R - 1) + (tid % R) - 1;      // A task: row at % BM, quarter at / BM
  const bool a_ok = !is_b && at < A_TASKS;
  const int a_row = a_ok ? at % BM : 0, a_q = a_ok ? at / BM : 0;
  const bool a_live = a_ok && m0 + a_row < P.M;
  const int a_voff = a_live ? ((m0 + a_row) * HW + 4 * a_q) * 4 : OOR;
  const int b_c = bt & 31, b_h = bt >> 5;
  const int b_cbase = (c0 + b_c) * HW;

  f32x16 acc[3];
#pragma unroll
  for (int j = 0; j < 3; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;

  float rv[10];  // staged values: A (4) or B (10)

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

  // global loads of one k-tile's staging: the dY quarter row (A task) of output row y, or the 10
  // source values x[c][row(yb)][ox0 + 8h - 1 .. ox0 + 8h + 8] (B task) of logical source row yb
  auto load_a = [&](int y, int ox0) {
    const int soff = __builtin_amdgcn_readfirstlane((y * W + ox0) * 4);
    const f32x4 v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(asrd, a_voff, soff, 0));
#pragma unroll
    for (int e = 0; e < 4; ++e) rv[e] = v[e];
  };
  auto load_b = [&](int yb, int ox0) {
    const int sy = src_row(yb);
    const int x0 = ox0 + 8 * b_h - 1;
    if (sy >= 0 && x0 >= 0 && x0 + 9 < W) {
      const int vo = (b_cbase + sy * W + x0) * 4;
      const f32x4 v0 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xsrd, vo, 0, 0));
      const f32x4 v1 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xsrd, vo + 16, 0, 0));
      const f32x2 v2 = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(xsrd, vo + 32, 0, 0));
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        rv[e] = v0[e];
        rv[4 + e] = v1[e];
      }
      rv[8] = v2[0];
      rv[9] = v2[1];
    } else {
#pragma unroll
      for (int e = 0; e < 10; ++e) {
        const int sx = src_col(x0 + e);
        const int vo = (sy >= 0 && sx >= 0) ? (b_cbase + sy * W + sx) * 4 : OOR;
        rv[e] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xsrd, vo, 0, 0));
      }
    }
  };
  auto load_stage = [&](int y, int yb, int ox0) {
    if (is_b) load_b(yb, ox0);
    else if (a_ok) load_a(y, ox0);
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
  auto store_a = [&](int buf) {
    if (!a_ok) return;
    uint32_t p0[3], p1[3];
    split_pair(rv[0], rv[1], p0);
    split_pair(rv[2], rv[3], p1);
    uint32_t* d = reinterpret_cast<uint32_t*>(&As[buf][a_row][0]) + 2 * a_q;
#pragma unroll
    for (int pc = 0; pc < NPC; ++pc) *reinterpret_cast<u32x2*>(d + 8 * pc) = u32x2{p0[pc], p1[pc]};
  };
  auto store_b = [&](int slot) {
    uint32_t p[5][3];
#pragma unroll
    for (int q = 0; q < 5; ++q) split_pair(rv[2 * q], rv[2 * q + 1], p[q]);
#pragma unroll
    for (int pc = 0; pc < NPC; ++pc) {
      uint32_t* d0 = reinterpret_cast<uint32_t*>(&Bs[slot][0][b_c][0]) + 8 * pc + 4 * b_h;
      uint32_t* d1 = reinterpret_cast<uint32_t*>(&Bs[slot][1][b_c][0]) + 8 * pc + 4 * b_h;
      uint32_t* d2 = reinterpret_cast<uint32_t*>(&Bs[slot][2][b_c][0]) + 8 * pc + 4 * b_h;
      *reinterpret_cast<u32x4*>(d0) = u32x4{p[0][pc], p[1][pc], p[2][pc], p[3][pc]};
      *reinterpret_cast<u32x4*>(d2) = u32x4{p[1][pc], p[2][pc], p[3][pc], p[4][pc]};
      // kw = 1: values 1..8 = the odd shift, re-paired from neighbouring dwords
      *reinterpret_cast<u32x4*>(d1) =
          u32x4{__builtin_amdgcn_alignbit(p[1][pc], p[0][pc], 16), __builtin_amdgcn_alignbit(p[2][pc], p[1][pc], 16),
                __builtin_amdgcn_alignbit(p[3][pc], p[2][pc], 16), __builtin_amdgcn_alignbit(p[4][pc], p[3][pc], 16)};
    }
  };
  auto store_stage = [&](int buf, int slot) {
    if (is_b) store_b(slot);
    else store_a(buf);
  };

  // the three taps (kh, kw = 0..2) of this wave for k-tile y (A buffer buf)
  auto compute = [&](int y, int buf) {
    const int slot = (y + kh + 3) & 3;  // logical source row y + kh - 1
    const float* ap = &As[buf][wm * 32 + lo][4 * hi];
    bf16x8_t af[3];
#pragma unroll
    for (int pc = 0; pc < NPC; ++pc) af[pc] = *reinterpret_cast<const bf16x8_t*>(ap + 8 * pc);
    bf16x8_t bfr[3][3];
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const float* bp = &Bs[slot][kw][lo][4 * hi];
#pragma unroll
      for (int pc = 0; pc < NPC; ++pc) bfr[kw][pc] = *reinterpret_cast<const bf16x8_t*>(bp + 8 * pc);
    }
    __builtin_amdgcn_sched_barrier(0);
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
  };

  // this block's segments: seg = sidx * G + i over (strip, row chunk), strip-major
  const int nstrip = W / WH_BK;
  const int nseg = nstrip * P.nchunk;
  const int g0 = sidx * P.G, g1 = min(nseg, g0 + P.G);
  for (int g = g0; g < g1; ++g) {
    const int strip = g / P.nchunk, chunk = g - strip * P.nchunk;
    const int ox0 = __builtin_amdgcn_readfirstlane(strip * WH_BK);
    const int y0 = __builtin_amdgcn_readfirstlane(chunk * P.rch);
    const int y1 = __builtin_amdgcn_readfirstlane(min(H, y0 + P.rch));
    // prologue: source rows y0 - 1 and y0 into their ring slots, then A(y0) and row y0 + 1
    if (is_b) {
      load_b(y0 - 1, ox0);
      store_b((y0 + 3) & 3);
      load_b(y0, ox0);
      store_b(y0 & 3);
    }
    load_stage(y0, y0 + 1, ox0);
    store_stage(y0 & 1, (y0 + 1) & 3);
    __syncthreads();
    for (int y = y0; y < y1; ++y) {
      const bool more = y + 1 < y1;
      if (more) load_stage(y + 1, y + 2, ox0);
      compute(y, y & 1);
      if (more) store_stage((y + 1) & 1, (y + 2) & 3);
      __syncthreads();
    }
  }

  // raw sums of this block's segments: slab[bz][m][(kh*3 + kw)*Cs + c0 + lo]
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
  if (wm == 1) wgrad_halo_kernel<1, PREC, GMODE><<<g, 192, 0, st>>>(P);
  else if (wm == 4) wgrad_halo_kernel<4, PREC, GMODE><<<g, 768, 0, st>>>(P);
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

bool wgrad_halo_ok(int Cs, int H, int W, int KH, int KW, int stride, int pad, int up, int gmode, int mode) {
  const int am = vst_mode_arith(mode);
  return VST_WGRAD_HALO && KH == 3 && KW == 3 && stride == 1 && pad == 1 && up == 1 && (gmode == 0 || gmode == 1) &&
         Cs % WH_CB == 0 && W % WH_BK == 0 && H >= 2 && W >= 2 &&
         (am == VST_GEMM_BF16X6 || am == VST_GEMM_BF16 || am == VST_GEMM_F16);
}

// Split plan: row chunks of >= 32 rows, S slabs per image each summing G consecutive (strip, chunk)
// segments.  Chosen like the row-tiled kernel's split count: minimise (waves of blocks at two per
// CU) x (k-tiles + ring prologue per block) plus the slab write / reduce traffic.
WhPlan wgrad_halo_plan(int N, int M, int Cs, int H, int W) {
  WhPlan p;
  const int bm = wgrad_halo_bm(M);
  p.Mpad = (M + bm - 1) / bm * bm;
  const int nstrip = W / WH_BK;
  const long tiles = (long)(Cs / WH_CB) * (p.Mpad / bm);
  const double slab_b = (double)p.Mpad * 9.0 * Cs * 4.0;
  const double t_kt = 0.8e-6;  // s per k-tile step of a resident block (18 bf16x6 MFMAs per wave, 3 waves / SIMD)
  double best = 1e30;
  p.nchunk = 1, p.G = nstrip, p.S = 1;
  for (int nchunk = 1; nchunk * 32 <= H || nchunk == 1; nchunk *= 2) {
    const int rch = (H + nchunk - 1) / nchunk, nseg = nstrip * nchunk;
    for (int G = 1; G <= nseg; ++G) {
      const int S = (nseg + G - 1) / G;
      if ((nseg + S - 1) / S != G) continue;  // (each distinct group size once)
      const long blocks = tiles * N * S;
      const long waves = (blocks + 511) / 512;
      const double t = waves * (double)G * (rch + 2) * t_kt + 2.0 * N * S * slab_b / 5e12;
      if (t < best * 0.995) {
        best = t;
        p.nchunk = nchunk;
        p.G = G;
        p.S = S;
      }
    }
  }
  p.rch = (H + p.nchunk - 1) / p.nchunk;
  return p;
}

long wgrad_halo_slab_floats(int N, int Cs, const WhPlan& p) { return (long)N * p.S * p.Mpad * 9L * Cs; }

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
  P.G = p.G;
  P.S = p.S;
  const int bm = wgrad_halo_bm(M);
  dim3 g(Cs / WH_CB, P.Mpad / bm, N * P.S);
  const int wm = bm / 32;
  switch (vst_mode_arith(mode)) {
    case VST_GEMM_BF16X6: launch_prec<3>(wm, gmode, g, st, P); break;
    case VST_GEMM_F16: launch_prec<4>(wm, gmode, g, st, P); break;
    default: launch_prec<2>(wm, gmode, g, st, P); break;
  }
  return vst_launch_status();
}
