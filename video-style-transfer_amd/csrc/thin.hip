// Convolutions with at most 4 output channels (the AdaAttN decoder's last conv 64 -> 3,
// AA/network.py:99): weight and data gradients in exact fp32 on the VALU.  As GEMMs their M (3, or 9
// row-split rows) fills a tenth of a 32-row MFMA tile while the operand gathers and the 2 GB-class
// activation read / write stay whole (config 5: 2.3 ms each); here each source / output row is moved
// once, with 16-byte accesses.
//
// Built with -fno-slp-vectorize (Makefile): the packed pairs below are written out explicitly
// (v_pk_fma_f32 over column pairs); the SLP vectorizer paired the scalar weight FMAs of the data
// gradient through lane moves and scalar-register spills (500 extra moves per four rows).
#include <type_traits>

#include "thin.h"
#include "vst_common.h"
#include "vst_hip.h"

namespace {

// ---------------------------------------------------------------------------------------------
// Weight gradient of a 3x3 stride-1 pad-1 conv with at most 4 output channels (the AdaAttN
// decoder's last conv 64 -> 3, AA/network.py:99), in exact fp32 on the VALU:
//   dW[co][ci][kh][kw] = sum_{n,y,x} dY[n][co][y][x] * X[n][ci][y + kh - 1][x + kw - 1]
// As a GEMM its M is 3 (or 9 row-split rows): a 32-row MFMA tile wastes 70-90 % of its products and
// the row-tiled kernel gathers every source element once per kw tap (2.3 ms at config 5, where the
// 2.1 GB source read alone takes ~0.35 ms).  Here a thread owns 4 consecutive columns of CI (2 or 4)
// input channels and walks a row range DOWN the image: each step loads ONE source row (16 B + two
// 4-byte neighbours per channel) and ONE dY row (16 B per output channel), keeps the three dY rows
// y-1, y, y+1 that meet the source row in registers, and does CO x CI x 9 x 4 FMAs (as packed pairs)
// into private sums; the next step's rows are loaded before this step's FMAs.  The block (256 threads)
// sums its threads' partials (a 64-lane reduce-scatter, then the four waves in order) into one slab
// [co][ci][kh][kw] per (image, row chunk, column block); thin_wgrad_reduce adds the slabs in a fixed
// order (deterministic, no atomics).  Blocks of the same rows and different channel groups are
// consecutive in the XCD-remapped order, so a dY row is fetched from HBM about once per XCD.
struct ThinWgParams {
  const float* dy;  // [N][CO][H][W]
  const float* x;   // [N][Cin][H][W]
  float* slab;      // [N * nchunk * ncolb][CO][Cin][9]
  int Cin, H, W;
  int tcb, rpar, ncolb, nchunk, rch;
};
constexpr int THIN_CI = 4;  // channel multiple the path requires (the kernel's group: thin_ci)
// input channels per thread: 4 for one output channel, 1 for four, else 2 (CO x CI x 18 accumulator pairs, the
// four dY row slots and two source row sets within the two-waves-per-SIMD budget; 4 channels at CO 3
// spilled)
constexpr int thin_ci(int CO) { return CO == 1 ? 4 : CO == 4 ? 1 : 2; }

// one level of a 64-lane reduce-scatter: lanes with bit `off` set keep the upper half of the values
// (summed with the partner's upper half), the others the lower half
template <int NV>
__device__ __forceinline__ void rs_level(const float (&in)[NV], float (&out)[(NV + 1) / 2], int off, bool up) {
  constexpr int H = (NV + 1) / 2;
#pragma unroll
  for (int i = 0; i < H; ++i) {
    const float lo = in[i];
    const float hi = (H + i < NV) ? in[H + i] : 0.f;
    out[i] = (up ? hi : lo) + __shfl_xor(up ? lo : hi, off, 64);
  }
}

template <int CO, bool REFLECT>
__global__ __launch_bounds__(256, 2) void thin_wgrad_kernel(ThinWgParams P) {
  constexpr int CI = thin_ci(CO), NV = CO * CI * 9, OOR = 0x7ffffff0;
  const int CG = P.Cin / CI;
  const int wk = xcd_remap(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z),
                           gridDim.x * gridDim.y * gridDim.z);
  const int cg = __builtin_amdgcn_readfirstlane(wk % CG);
  int rest = __builtin_amdgcn_readfirstlane(wk / CG);
  const int chunk = __builtin_amdgcn_readfirstlane(rest % P.nchunk);
  rest = __builtin_amdgcn_readfirstlane(rest / P.nchunk);
  const int colb = __builtin_amdgcn_readfirstlane(rest % P.ncolb);
  const int n = __builtin_amdgcn_readfirstlane(rest / P.ncolb);
  const int H = P.H, W = P.W;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int rl = t / P.tcb, q = t - rl * P.tcb;
  const int px0 = 4 * (colb * P.tcb + q);
  const bool act = rl < P.rpar && px0 < W;
  // rows of this block, then of this thread's row lane (a uniform step count: rows past a lane's
  // range read zero dY and contribute nothing)
  const int cy0 = chunk * P.rch, cy1 = min(H, cy0 + P.rch);
  const int per = (cy1 - cy0 + P.rpar - 1) / P.rpar;
  const int ly0 = cy0 + rl * per, ly1 = min(cy1, ly0 + per);
  const int nsteps = per + 2;
  const long plane = (long)H * W;
  const __amdgpu_buffer_rsrc_t xr = uniform_rsrc(P.x + ((long)n * P.Cin + cg * CI) * plane, (uint32_t)(CI * plane * 4));
  const __amdgpu_buffer_rsrc_t dr = uniform_rsrc(P.dy + (long)n * CO * plane, (uint32_t)(CO * plane * 4));
  // column byte offsets of the 16-byte body and the two neighbours (-1: zero)
  int cl = px0 - 1, cr = px0 + 4;
  if (REFLECT) {
    cl = cl < 0 ? 1 : cl;
    cr = cr >= W ? W - 2 : cr;
  } else {
    cl = cl < 0 ? -1 : cl;
    cr = cr >= W ? -1 : cr;
  }
  const int pstride = (int)(plane * 4);

  // acc[co][ci][tap] = {sum over even columns j, sum over odd j}: the pixel pairs (j, j+1) of a quad
  // go through one packed FMA (v_pk_fma_f32) with the dY pair {d_j, d_j+1} (aligned halves of the
  // 16-byte load) and the source pair {x_j+kw, x_j+kw+1}
  f32x2 acc[CO][CI][9];
#pragma unroll
  for (int co = 0; co < CO; ++co)
#pragma unroll
    for (int ci = 0; ci < CI; ++ci)
#pragma unroll
      for (int k = 0; k < 9; ++k) acc[co][ci][k] = f32x2{0.f, 0.f};
  float X[2][CI][6];  // source row r (current set) and r + 1 (prefetched)
  float D[4][CO][4];  // dY rows r - 1, r, r + 1 and the prefetched r + 2 (slot = (row - ly0 + 2) & 3)
  auto load_x = [&](int r, float (&xv)[CI][6]) {
    int rr = r;
    bool ok = act;
    if (REFLECT) {
      ok = ok && r >= -1 && r <= H;
      rr = rr < 0 ? -rr : (rr >= H ? 2 * H - 2 - rr : rr);
    } else {
      ok = ok && r >= 0 && r < H;
    }
    const int rb = rr * W * 4;
    const int vm = ok ? rb + px0 * 4 : OOR, vl = ok && cl >= 0 ? rb + cl * 4 : OOR,
              vr = ok && cr >= 0 ? rb + cr * 4 : OOR;
#pragma unroll
    for (int ci = 0; ci < CI; ++ci) {
      const f32x4 m = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, vm, ci * pstride, 0));
      xv[ci][0] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, vl, ci * pstride, 0));
      xv[ci][1] = m[0];
      xv[ci][2] = m[1];
      xv[ci][3] = m[2];
      xv[ci][4] = m[3];
      xv[ci][5] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, vr, ci * pstride, 0));
    }
  };
  auto load_d = [&](int y, float (&dv)[CO][4]) {
    const bool ok = act && y >= ly0 && y < ly1;
    const int vo = ok ? (y * W + px0) * 4 : OOR;
#pragma unroll
    for (int co = 0; co < CO; ++co) {
      const f32x4 m = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(dr, vo, co * pstride, 0));
#pragma unroll
      for (int j = 0; j < 4; ++j) dv[co][j] = m[j];
    }
  };
  // step s: source row r = ly0 - 1 + s meets dY rows r + 1 (kh 0), r (kh 1), r - 1 (kh 2)
  auto step = [&](auto pc, int s) {
    constexpr int p = decltype(pc)::value;
    const int r = ly0 - 1 + s;
    if (s + 1 < nsteps) {
      load_x(r + 1, X[(p + 1) & 1]);
      load_d(r + 2, D[(p + 3) & 3]);
    }
    const float(&xv)[CI][6] = X[p & 1];
    f32x2 xp[CI][5];  // source pairs {x_c, x_c+1}, c = j + kw
#pragma unroll
    for (int ci = 0; ci < CI; ++ci)
#pragma unroll
      for (int c = 0; c < 5; ++c) xp[ci][c] = f32x2{xv[ci][c], xv[ci][c + 1]};
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const float(&dv)[CO][4] = D[(p + 2 - kh) & 3];
#pragma unroll
      for (int co = 0; co < CO; ++co) {
        const f32x2 d01 = {dv[co][0], dv[co][1]}, d23 = {dv[co][2], dv[co][3]};
#pragma unroll
        for (int ci = 0; ci < CI; ++ci)
#pragma unroll
          for (int kw = 0; kw < 3; ++kw) {
            f32x2& a = acc[co][ci][kh * 3 + kw];
            a = __builtin_elementwise_fma(d01, xp[ci][kw], a);
            a = __builtin_elementwise_fma(d23, xp[ci][kw + 2], a);
          }
      }
    }
  };
#pragma unroll
  for (int co = 0; co < CO; ++co)
#pragma unroll
    for (int j = 0; j < 4; ++j) D[0][co][j] = 0.f;  // dY row ly0 - 2: outside every range
  load_d(ly0 - 1, D[1]);
  load_d(ly0, D[2]);
  load_x(ly0 - 1, X[0]);
  for (int s = 0; s < nsteps; s += 4) {
    step(std::integral_constant<int, 0>{}, s);
    if (s + 1 < nsteps) step(std::integral_constant<int, 1>{}, s + 1);
    if (s + 2 < nsteps) step(std::integral_constant<int, 2>{}, s + 2);
    if (s + 3 < nsteps) step(std::integral_constant<int, 3>{}, s + 3);
  }

  // block sum: reduce-scatter over the 64 lanes (NV -> 2 values per lane), then the waves in order
  float v0[NV];
#pragma unroll
  for (int co = 0; co < CO; ++co)
#pragma unroll
    for (int ci = 0; ci < CI; ++ci)
#pragma unroll
      for (int k = 0; k < 9; ++k) v0[(co * CI + ci) * 9 + k] = acc[co][ci][k][0] + acc[co][ci][k][1];
  constexpr int N1 = (NV + 1) / 2, N2 = (N1 + 1) / 2, N3 = (N2 + 1) / 2, N4 = (N3 + 1) / 2, N5 = (N4 + 1) / 2,
                N6 = (N5 + 1) / 2;
  float v1[N1], v2[N2], v3[N3], v4[N4], v5[N5], v6[N6];
  rs_level<NV>(v0, v1, 32, lane & 32);
  rs_level<N1>(v1, v2, 16, lane & 16);
  rs_level<N2>(v2, v3, 8, lane & 8);
  rs_level<N3>(v3, v4, 4, lane & 4);
  rs_level<N4>(v4, v5, 2, lane & 2);
  rs_level<N5>(v5, v6, 1, lane & 1);
  __shared__ float red[4][NV];
  constexpr int sz[7] = {NV, N1, N2, N3, N4, N5, N6};
#pragma unroll
  for (int k = 0; k < N6; ++k) {
    int idx = k;
    bool ok = true;
#pragma unroll
    for (int lv = 6; lv >= 1; --lv) {
      idx += (lane & (64 >> lv)) ? sz[lv] : 0;
      ok = ok && idx < sz[lv - 1];
    }
    if (ok) red[wave][idx] = v6[k];
  }
  __syncthreads();
  float* slab = P.slab + ((long)(n * P.nchunk + chunk) * P.ncolb + colb) * CO * P.Cin * 9;
  for (int i = t; i < NV; i += 256) {
    const float s = ((red[0][i] + red[1][i]) + red[2][i]) + red[3][i];
    const int co = i / (CI * 9), rem = i - co * CI * 9, ci = rem / 9, k = rem - ci * 9;
    slab[((long)co * P.Cin + cg * CI + ci) * 9 + k] = s;
  }
}

// dw[co][ci][kh][kw] (+)= sum over the S slabs, in slab order
__global__ void thin_wgrad_reduce_kernel(const float* __restrict__ slab, float* __restrict__ dw, int S, int total,
                                         int accumulate) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  float s = 0.f;
  for (int k = 0; k < S; ++k) s += slab[(long)k * total + i];
  dw[i] = accumulate ? dw[i] + s : s;
}

struct ThinPlan {
  int tcb, rpar, ncolb, nchunk, rch;
};
// the thin path: Cout <= 4, 3x3 stride 1 pad 1 over the unpadded grid, 4-channel groups, 4-column quads
bool thin_wgrad_ok(int Cout, int Cin, int Hs, int Ws, int Ho, int Wo, int KH, int KW, int gmode, int stride,
                          int pad, int up, int mode) {
  return !(mode & VST_GEMM_PERTAP) && Cout <= 4 && KH == 3 && KW == 3 && stride == 1 && pad == 1 && up == 1 &&
         Ho == Hs && Wo == Ws && Cin % THIN_CI == 0 && Ws % 4 == 0 && Ws >= 8 && Hs >= 2 && (gmode == 0 || gmode == 1);
}
// a block row lane covers up to 256 column quads; row chunks until ~2048 blocks (>= 4 rows per lane)
static ThinPlan thin_plan(int N, int Cout, int Cin, int H, int W) {
  ThinPlan p;
  const int quads = W / 4;
  p.tcb = quads >= 256 ? 256 : quads;
  p.ncolb = (quads + 255) / 256;
  p.rpar = 256 / p.tcb;
  const long base = (long)(Cin / thin_ci(Cout)) * N * p.ncolb;
  long nc = (2048 + base - 1) / base;
  const long cap = H / (4 * p.rpar) > 1 ? H / (4 * p.rpar) : 1;
  nc = nc < 1 ? 1 : (nc > cap ? cap : nc);
  p.rch = (int)((H + nc - 1) / nc);
  p.nchunk = (H + p.rch - 1) / p.rch;
  return p;
}
static long thin_slab_floats(int N, int Cout, int Cin, const ThinPlan& p) {
  return (long)N * p.nchunk * p.ncolb * Cout * Cin * 9;
}
static int thin_wgrad_launch_impl(const float* dy, const float* x, float* dw, float* slab, int N, int Cin, int H, int W,
                             int Cout, int gmode, int accumulate, hipStream_t st) {
  const ThinPlan p = thin_plan(N, Cout, Cin, H, W);
  ThinWgParams P{dy, x, slab, Cin, H, W, p.tcb, p.rpar, p.ncolb, p.nchunk, p.rch};
  dim3 g(Cin / thin_ci(Cout), p.nchunk, N * p.ncolb);
  const bool refl = gmode == 0;
  switch (Cout) {
#define VST_THIN_CASE(C)                                                              \
  case C:                                                                             \
    if (refl) thin_wgrad_kernel<C, true><<<g, 256, 0, st>>>(P);                       \
    else thin_wgrad_kernel<C, false><<<g, 256, 0, st>>>(P);                           \
    break;
    VST_THIN_CASE(1)
    VST_THIN_CASE(2)
    VST_THIN_CASE(3)
    VST_THIN_CASE(4)
#undef VST_THIN_CASE
    default: return VST_EINVAL;
  }
  const int total = Cout * Cin * 9;
  thin_wgrad_reduce_kernel<<<ceil_div(total, 256), 256, 0, st>>>(slab, dw, N * p.nchunk * p.ncolb, total, accumulate);
  return vst_launch_status();
}


// ---------------------------------------------------------------------------------------------
// Data gradient of a 3x3 stride-1 pad-1 conv with at most 4 output channels (the AdaAttN decoder's
// last conv 64 -> 3 under its fused ReLU mask, AA/network.py:99), in exact fp32 on the VALU:
//   dXpad[ci][u][v] = sum_{co,kh,kw} W[co][ci][kh][kw] * dY[co][u - kh][v - kw]   (dY zero outside)
// over the padded grid; its interior (u, v) = (y + 1, x + 1) is dx (masked by mask > 0), its ring
// (reflect pad only) goes to the border buffer for vst_fold_border.  As the transposed GEMM this is
// M = Cin rows over K = 27 (or 48 kw-unfolded) products per output: 2.4 ms at config 5 for a 2.1 GB
// output.  Here a thread owns 4 consecutive columns of 2 input channels and walks a row range: each
// step loads ONE dY row (16 B + two neighbours per output channel; the rows y-1, y, y+1 stay in
// registers), the mask row, and writes one 16-byte dx row segment per channel; the weights of the
// block's channel pair sit in scalar registers.
struct ThinDgParams {
  const float* dy;    // [N][CO][H][W]
  const float* w;     // [CO][Cin][3][3]
  const float* mask;  // [N][Cin][H][W] or null
  float* dx;          // [N][Cin][H][W]
  int Cin, H, W;
  int tcb, rpar, ncolb, nchunk, rch;
};
constexpr int THIN_DG_CI = 2;

template <int CO, bool MASK>
__global__ __launch_bounds__(256) void thin_dgrad_kernel(ThinDgParams P) {
  constexpr int CI = THIN_DG_CI, OOR = 0x7ffffff0;
  const int CG = P.Cin / CI;
  const int wk = xcd_remap(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z),
                           gridDim.x * gridDim.y * gridDim.z);
  const int cg = __builtin_amdgcn_readfirstlane(wk % CG);
  int rest = __builtin_amdgcn_readfirstlane(wk / CG);
  const int chunk = __builtin_amdgcn_readfirstlane(rest % P.nchunk);
  rest = __builtin_amdgcn_readfirstlane(rest / P.nchunk);
  const int colb = __builtin_amdgcn_readfirstlane(rest % P.ncolb);
  const int n = __builtin_amdgcn_readfirstlane(rest / P.ncolb);
  const int H = P.H, W = P.W;
  const int t = threadIdx.x;
  const int rl = t / P.tcb, q = t - rl * P.tcb;
  const int px0 = 4 * (colb * P.tcb + q);
  const bool act = rl < P.rpar && px0 < W;
  const int cy0 = chunk * P.rch, cy1 = min(H, cy0 + P.rch);
  const int per = (cy1 - cy0 + P.rpar - 1) / P.rpar;
  const int ly0 = cy0 + rl * per, ly1 = min(cy1, ly0 + per);
  const long plane = (long)H * W;
  const int pstride = (int)(plane * 4);
  const __amdgpu_buffer_rsrc_t dr = uniform_rsrc(P.dy + (long)n * CO * plane, (uint32_t)(CO * plane * 4));
  const __amdgpu_buffer_rsrc_t mr =
      uniform_rsrc(MASK ? P.mask + ((long)n * P.Cin + cg * CI) * plane : P.dy, (uint32_t)(MASK ? CI * plane * 4 : 0));
  float* dxb = P.dx + ((long)n * P.Cin + cg * CI) * plane;
  // the block's weights W[co][cg*CI + c][tap] (uniform: scalar registers)
  float wt[CO][CI][9];
#pragma unroll
  for (int co = 0; co < CO; ++co)
#pragma unroll
    for (int c = 0; c < CI; ++c)
#pragma unroll
      for (int k = 0; k < 9; ++k)
        wt[co][c][k] = __int_as_float(
            __builtin_amdgcn_readfirstlane(__float_as_int(P.w[((long)co * P.Cin + cg * CI + c) * 9 + k])));
  // dY window columns px0 - 1 .. px0 + 4 (zero outside the image)
  const int cl = px0 - 1 >= 0 ? (px0 - 1) * 4 : -1, cr = px0 + 4 < W ? (px0 + 4) * 4 : -1;
  float D[4][CO][6];  // dY rows y - 1, y, y + 1 and the prefetched y + 2 (slot (row - ly0 + 1) & 3)
  f32x4 M[2][CI];     // mask rows y (current) and y + 1
  auto load_d = [&](int r, float (&dv)[CO][6]) {
    const bool ok = act && r >= 0 && r < H;
    const int rb = r * W * 4;
    const int vm = ok ? rb + px0 * 4 : OOR, vl = ok && cl >= 0 ? rb + cl : OOR, vr = ok && cr >= 0 ? rb + cr : OOR;
#pragma unroll
    for (int co = 0; co < CO; ++co) {
      const f32x4 m = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(dr, vm, co * pstride, 0));
      dv[co][0] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(dr, vl, co * pstride, 0));
      dv[co][1] = m[0];
      dv[co][2] = m[1];
      dv[co][3] = m[2];
      dv[co][4] = m[3];
      dv[co][5] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(dr, vr, co * pstride, 0));
    }
  };
  auto load_m = [&](int y, f32x4 (&mv)[CI]) {
    if constexpr (MASK) {
      const int vo = act && y < ly1 ? (y * W + px0) * 4 : OOR;
#pragma unroll
      for (int c = 0; c < CI; ++c)
        mv[c] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(mr, vo, c * pstride, 0));
    }
  };
  // step s: output row y = ly0 + s reads dY rows y + 1 (kh 0), y (kh 1), y - 1 (kh 2)
  auto step = [&](auto pc, int s) {
    constexpr int p = decltype(pc)::value;
    const int y = ly0 + s;
    if (s + 1 < per) {
      load_d(y + 2, D[(p + 3) & 3]);
      load_m(y + 1, M[(p + 1) & 1]);
    }
    float o[CI][4];
#pragma unroll
    for (int c = 0; c < CI; ++c)
#pragma unroll
      for (int j = 0; j < 4; ++j) o[c][j] = 0.f;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const float(&dv)[CO][6] = D[(p + 2 - kh) & 3];
#pragma unroll
      for (int co = 0; co < CO; ++co)
#pragma unroll
        for (int c = 0; c < CI; ++c)
#pragma unroll
          for (int kw = 0; kw < 3; ++kw)
#pragma unroll
            for (int j = 0; j < 4; ++j) o[c][j] = fmaf(wt[co][c][kh * 3 + kw], dv[co][j + 2 - kw], o[c][j]);
    }
    if (act && y < ly1) {
#pragma unroll
      for (int c = 0; c < CI; ++c) {
        f32x4 r = {o[c][0], o[c][1], o[c][2], o[c][3]};
        if constexpr (MASK) {
#pragma unroll
          for (int j = 0; j < 4; ++j) r[j] = M[p & 1][c][j] > 0.f ? r[j] : 0.f;
        }
        *reinterpret_cast<f32x4*>(dxb + c * plane + (long)y * W + px0) = r;
      }
    }
  };
  load_d(ly0 - 1, D[0]);
  load_d(ly0, D[1]);
  load_d(ly0 + 1, D[2]);
  load_m(ly0, M[0]);
  for (int s = 0; s < per; s += 4) {
    step(std::integral_constant<int, 0>{}, s);
    if (s + 1 < per) step(std::integral_constant<int, 1>{}, s + 1);
    if (s + 2 < per) step(std::integral_constant<int, 2>{}, s + 2);
    if (s + 3 < per) step(std::integral_constant<int, 3>{}, s + 3);
  }
}

// the padded grid's ring (u in {0, H+1} or v in {0, W+1}) of the same sum, into border [N][Cin][H+2][W+2]
__global__ void thin_dgrad_ring_kernel(const float* __restrict__ dy, const float* __restrict__ w,
                                       float* __restrict__ border, int N, int CO, int Cin, int H, int W) {
  const int Hp = H + 2, Wp = W + 2;
  const int per_plane = 2 * Wp + 2 * H;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)N * Cin * per_plane) return;
  const int nc = (int)(idx / per_plane), e = (int)(idx - (long)nc * per_plane);
  const int n = nc / Cin, ci = nc - n * Cin;
  int u, v;
  if (e < 2 * Wp) {
    u = e < Wp ? 0 : Hp - 1;
    v = e < Wp ? e : e - Wp;
  } else {
    const int f = e - 2 * Wp;
    u = 1 + (f >> 1);
    v = (f & 1) ? Wp - 1 : 0;
  }
  float s = 0.f;
  for (int co = 0; co < CO; ++co) {
    const float* dyp = dy + ((long)n * CO + co) * H * W;
    const float* wp = w + ((long)co * Cin + ci) * 9;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int yy = u - kh;
      if (yy < 0 || yy >= H) continue;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int xx = v - kw;
        if (xx >= 0 && xx < W) s = fmaf(wp[kh * 3 + kw], dyp[(long)yy * W + xx], s);
      }
    }
  }
  border[((long)nc * Hp + u) * Wp + v] = s;
}


}  // namespace

bool vst_thin_wgrad_ok(int Cout, int Cin, int Hs, int Ws, int Ho, int Wo, int KH, int KW, int gmode, int stride,
                       int pad, int up, int mode) {
  return thin_wgrad_ok(Cout, Cin, Hs, Ws, Ho, Wo, KH, KW, gmode, stride, pad, up, mode);
}
long vst_thin_wgrad_floats(int N, int Cout, int Cin, int Hs, int Ws) {
  return thin_slab_floats(N, Cout, Cin, thin_plan(N, Cout, Cin, Hs, Ws));
}
int vst_thin_wgrad_launch(const float* dy, const float* x, float* dw, float* slab, int N, int Cin, int H, int W,
                          int Cout, int gmode, int accumulate, hipStream_t st) {
  return thin_wgrad_launch_impl(dy, x, dw, slab, N, Cin, H, W, Cout, gmode, accumulate, st);
}

extern "C" {

int vst_conv_dgrad_thin(const float* dy, const float* w, const float* mask, float* dx, float* border, int N, int Cout,
                        int Cin, int H, int W, int reflect, void* stream) {
  VST_CHECK_ARG(dy && w && dx && N > 0 && Cout >= 1 && Cout <= 4 && Cin > 0 && Cin % THIN_DG_CI == 0 && H >= 2 &&
                W >= 8 && W % 4 == 0 && (!reflect || border));
  hipStream_t st = (hipStream_t)stream;
  // a row lane covers up to 256 column quads; row chunks until ~2048 blocks (>= 4 rows per lane)
  const int quads = W / 4;
  ThinDgParams P;
  P.dy = dy;
  P.w = w;
  P.mask = mask;
  P.dx = dx;
  P.Cin = Cin;
  P.H = H;
  P.W = W;
  P.tcb = quads >= 256 ? 256 : quads;
  P.ncolb = (quads + 255) / 256;
  P.rpar = 256 / P.tcb;
  const long base = (long)(Cin / THIN_DG_CI) * N * P.ncolb;
  long nc = (2048 + base - 1) / base;
  const long cap = H / (4 * P.rpar) > 1 ? H / (4 * P.rpar) : 1;
  nc = nc < 1 ? 1 : (nc > cap ? cap : nc);
  P.rch = (int)((H + nc - 1) / nc);
  P.nchunk = (H + P.rch - 1) / P.rch;
  dim3 g(Cin / THIN_DG_CI, P.nchunk, N * P.ncolb);
  switch (Cout) {
#define VST_THIN_DG(C)                                                       \
  case C:                                                                    \
    if (mask) thin_dgrad_kernel<C, true><<<g, 256, 0, st>>>(P);              \
    else thin_dgrad_kernel<C, false><<<g, 256, 0, st>>>(P);                  \
    break;
    VST_THIN_DG(1)
    VST_THIN_DG(2)
    VST_THIN_DG(3)
    VST_THIN_DG(4)
#undef VST_THIN_DG
  }
  if (reflect) {
    const long ring = (long)N * Cin * (2 * (W + 2) + 2 * H);
    thin_dgrad_ring_kernel<<<ceil_div(ring, 256), 256, 0, st>>>(dy, w, border, N, Cout, Cin, H, W);
    const int rc = vst_launch_status();
    if (rc) return rc;
    return vst_fold_border(border, mask, dx, (long)N * Cin, H, W, 1, stream);
  }
  return vst_launch_status();
}

}  // extern "C"
