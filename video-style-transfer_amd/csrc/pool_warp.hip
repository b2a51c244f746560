// Gather/scatter kernels of the ReCoNet step for gfx950:
//   * MaxPool2d(2, 2) forward / backward (VGG features "M" layers, RC/network.py:17-24),
//   * flow warp forward / backward (RC/utilities.py:39-57: bilinear grid_sample, zeros padding,
//     align_corners=False, grid normalised by (W-1)/(H-1) -> source x = ((2(x+u)/(W-1)-1)+1)W/2-0.5),
//   * forward-backward flow consistency mask (RC/utilities.py:60-90),
//   * bilinear resize with align_corners=False (F.interpolate, train_candy.py:91,97).
#include "vst_common.h"
#include "vst_hip.h"

namespace {

__global__ void maxpool_fwd_kernel(const float* __restrict__ x, float* __restrict__ y, long NC, int H, int W) {
  const int Ho = H / 2, Wo = W / 2;
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= NC * Ho * Wo) return;
  int ox = (int)(idx % Wo);
  long t = idx / Wo;
  int oy = (int)(t % Ho);
  long nc = t / Ho;
  const float* p = x + nc * H * W + (long)(2 * oy) * W + 2 * ox;
  float2 a = make_float2(p[0], p[1]);
  float2 b = make_float2(p[W], p[W + 1]);
  // first maximum in scan order wins (matches max_pool2d's `val > maxval` scan; NaN propagates)
  float m = a.x;
  if (a.y > m || isnan(a.y)) m = a.y;
  if (b.x > m || isnan(b.x)) m = b.x;
  if (b.y > m || isnan(b.y)) m = b.y;
  y[idx] = m;
}

// gx over the full input (zeros where no window routes a gradient)
__global__ void maxpool_bwd_kernel(const float* __restrict__ x, const float* __restrict__ gy, float* __restrict__ gx,
                                   long NC, int H, int W, int relu_mask) {
  const int Ho = H / 2, Wo = W / 2;
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= NC * H * W) return;
  int ix = (int)(idx % W);
  long t = idx / W;
  int iy = (int)(t % H);
  long nc = t / H;
  int oy = iy >> 1, ox = ix >> 1;
  float g = 0.f;
  if (oy < Ho && ox < Wo) {
    const float* p = x + nc * H * W + (long)(2 * oy) * W + 2 * ox;
    float v[4] = {p[0], p[1], p[W], p[W + 1]};
    int arg = 0;
    float m = v[0];
#pragma unroll
    for (int k = 1; k < 4; ++k)
      if (v[k] > m || isnan(v[k])) {
        m = v[k];
        arg = k;
      }
    // relu_mask: x is a ReLU output whose only consumer is this pool -> fold the ReLU backward in
    if (arg == (iy & 1) * 2 + (ix & 1) && (!relu_mask || m > 0.f)) g = gy[nc * Ho * Wo + (long)oy * Wo + ox];
  }
  gx[idx] = g;
}

// gx = relu_mask(pool_bwd(gy) + addend) for a ReLU output x that feeds both a MaxPool2d(2, 2) and
// another consumer (a VGG slice output used by the losses); gy / addend may be NULL.  One thread
// per 2x2 cell (trailing odd row/column: cells without a window, addend only).
__global__ void maxpool_bwd_add_kernel(const float* __restrict__ x, const float* __restrict__ gy,
                                       const float* __restrict__ addend, float* __restrict__ gx, long NC, int H, int W,
                                       int relu_mask) {
  const int Ho = H / 2, Wo = W / 2, Hc = (H + 1) / 2, Wc = (W + 1) / 2;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= NC * Hc * Wc) return;
  const int cx = (int)(idx % Wc);
  const long t = idx / Wc;
  const int cy = (int)(t % Hc);
  const long nc = t / Hc;
  const long base = nc * H * W + (long)(2 * cy) * W + 2 * cx;
  const bool has_r = 2 * cy + 1 < H, has_c = 2 * cx + 1 < W;
  float v[4];
  v[0] = x[base];
  v[1] = has_c ? x[base + 1] : 0.f;
  v[2] = has_r ? x[base + W] : 0.f;
  v[3] = has_r && has_c ? x[base + W + 1] : 0.f;
  float g[4] = {0.f, 0.f, 0.f, 0.f};
  if (gy && cy < Ho && cx < Wo) {  // a full pooling window: route to the first maximum
    int arg = 0;
    float m = v[0];
#pragma unroll
    for (int k = 1; k < 4; ++k)
      if (v[k] > m || isnan(v[k])) {
        m = v[k];
        arg = k;
      }
#pragma unroll
    for (int k = 0; k < 4; ++k) g[k] = k == arg ? gy[nc * Ho * Wo + (long)cy * Wo + cx] : 0.f;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if ((k & 1) && !has_c) continue;
    if ((k & 2) && !has_r) continue;
    const long o = base + (k >> 1) * (long)W + (k & 1);
    float s = g[k] + (addend ? addend[o] : 0.f);
    if (relu_mask && !(v[k] > 0.f)) s = 0.f;
    gx[o] = s;
  }
}

// Vector forms of the three pooling kernels above, for W % 4 == 0 and 16-byte aligned planes (every
// VGG layer of the training steps).  The per-element kernels decode (plane, row, column) with 64-bit
// division by runtime H / W per element, which made them VALU-bound at well under half the HBM rate
// (config-5 pool backward: 844 us per launch); here the plane is blockIdx.z, the row blockIdx.y*4 +
// threadIdx.y, and each thread owns two adjacent 2x2 windows: two float4 loads of x, one float2 of gy,
// two float4 stores of gx -- no division at all.  Same routing rule (first maximum in scan order,
// NaN wins) and the same trailing-row treatment for odd H.
__device__ __forceinline__ int pool_arg(float a, float b, float c, float d) {
  int arg = 0;
  float m = a;
  if (b > m || isnan(b)) m = b, arg = 1;
  if (c > m || isnan(c)) m = c, arg = 2;
  if (d > m || isnan(d)) m = d, arg = 3;
  return arg;
}

__global__ __launch_bounds__(256) void maxpool_fwd_vec_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                              int H, int W) {
  const int Ho = H >> 1, Wo = W >> 1, Wq = W >> 2;
  const int j = blockIdx.x * 64 + threadIdx.x, oy = blockIdx.y * 4 + threadIdx.y;
  if (j >= Wq || oy >= Ho) return;
  const float* p = x + (long)blockIdx.z * H * W + (long)(2 * oy) * W + 4 * j;
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + W);
  float m0 = a.x, m1 = a.z;
  if (a.y > m0 || isnan(a.y)) m0 = a.y;
  if (b.x > m0 || isnan(b.x)) m0 = b.x;
  if (b.y > m0 || isnan(b.y)) m0 = b.y;
  if (a.w > m1 || isnan(a.w)) m1 = a.w;
  if (b.z > m1 || isnan(b.z)) m1 = b.z;
  if (b.w > m1 || isnan(b.w)) m1 = b.w;
  *reinterpret_cast<float2*>(y + (long)blockIdx.z * Ho * Wo + (long)oy * Wo + 2 * j) = make_float2(m0, m1);
}

// gx = relu_mask(pool_bwd(gy) + addend) (gy / addend may be NULL): maxpool_bwd_kernel when addend is
// NULL, maxpool_bwd_add_kernel otherwise
__global__ __launch_bounds__(256) void maxpool_bwd_vec_kernel(const float* __restrict__ x, const float* __restrict__ gy,
                                                              const float* __restrict__ addend, float* __restrict__ gx,
                                                              int H, int W, int relu_mask) {
  const int Ho = H >> 1, Wo = W >> 1, Hc = (H + 1) >> 1, Wq = W >> 2;
  const int j = blockIdx.x * 64 + threadIdx.x, oy = blockIdx.y * 4 + threadIdx.y;
  if (j >= Wq || oy >= Hc) return;
  const bool full = oy < Ho;  // the window's second row exists (else: the trailing row of an odd H)
  const long o = (long)blockIdx.z * H * W + (long)(2 * oy) * W + 4 * j;
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  const float4 a = *reinterpret_cast<const float4*>(x + o);
  const float4 b = full ? *reinterpret_cast<const float4*>(x + o + W) : z4;
  float r0[4] = {0.f, 0.f, 0.f, 0.f}, r1[4] = {0.f, 0.f, 0.f, 0.f};
  if (gy && full) {
    const float2 g = *reinterpret_cast<const float2*>(gy + (long)blockIdx.z * Ho * Wo + (long)oy * Wo + 2 * j);
    const int a0 = pool_arg(a.x, a.y, b.x, b.y), a1 = pool_arg(a.z, a.w, b.z, b.w);
    r0[0] = a0 == 0 ? g.x : 0.f;
    r0[1] = a0 == 1 ? g.x : 0.f;
    r1[0] = a0 == 2 ? g.x : 0.f;
    r1[1] = a0 == 3 ? g.x : 0.f;
    r0[2] = a1 == 0 ? g.y : 0.f;
    r0[3] = a1 == 1 ? g.y : 0.f;
    r1[2] = a1 == 2 ? g.y : 0.f;
    r1[3] = a1 == 3 ? g.y : 0.f;
  }
  if (addend) {
    const float4 d0 = *reinterpret_cast<const float4*>(addend + o);
    const float4 d1 = full ? *reinterpret_cast<const float4*>(addend + o + W) : z4;
    r0[0] += d0.x, r0[1] += d0.y, r0[2] += d0.z, r0[3] += d0.w;
    r1[0] += d1.x, r1[1] += d1.y, r1[2] += d1.z, r1[3] += d1.w;
  }
  if (relu_mask) {
    const float xa[4] = {a.x, a.y, a.z, a.w}, xb[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (!(xa[k] > 0.f)) r0[k] = 0.f;
      if (!(xb[k] > 0.f)) r1[k] = 0.f;
    }
  }
  *reinterpret_cast<float4*>(gx + o) = make_float4(r0[0], r0[1], r0[2], r0[3]);
  if (full) *reinterpret_cast<float4*>(gx + o + W) = make_float4(r1[0], r1[1], r1[2], r1[3]);
}

// the vector forms apply: W % 4 == 0, 16-byte aligned x / gx / addend, 8-byte aligned y / gy, and a
// plane count that fits grid.z
inline bool pool_vec_ok(long NC, int W, const void* a16, const void* b16, const void* c16, const void* d8) {
  const uintptr_t m16 = (uintptr_t)a16 | (uintptr_t)b16 | (uintptr_t)c16;
  return (W & 3) == 0 && NC <= 65535 && (m16 & 15) == 0 && ((uintptr_t)d8 & 7) == 0;
}
inline dim3 pool_vec_grid(long NC, int rows, int W) {
  return dim3((unsigned)ceil_div((long)(W >> 2), 64), (unsigned)ceil_div((long)rows, 4), (unsigned)NC);
}

struct Bilin {
  int x0, y0;
  float w[4];  // nw, ne, sw, se
};

// grid_sample(align_corners=False) bilinear coordinates + weights, same fp32 op order as ATen
__device__ __forceinline__ Bilin warp_coords(int x, int y, float u, float v, int H, int W) {
  float gx = 2.0f * ((float)x + u) / (float)max(W - 1, 1) - 1.0f;
  float gy = 2.0f * ((float)y + v) / (float)max(H - 1, 1) - 1.0f;
  float ix = ((gx + 1.f) * W - 1.f) / 2.f;
  float iy = ((gy + 1.f) * H - 1.f) / 2.f;
  float fx = floorf(ix), fy = floorf(iy);
  Bilin b;
  b.x0 = (int)fx;
  b.y0 = (int)fy;
  float ix_se = fx + 1.f, iy_se = fy + 1.f;
  b.w[0] = (ix_se - ix) * (iy_se - iy);
  b.w[1] = (ix - fx) * (iy_se - iy);
  b.w[2] = (ix_se - ix) * (iy - fy);
  b.w[3] = (ix - fx) * (iy - fy);
  return b;
}

__global__ void warp_fwd_kernel(const float* __restrict__ x, const float* __restrict__ flo, float* __restrict__ out,
                                int B, int C, int H, int W) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long HW = (long)H * W;
  if (idx >= B * HW) return;
  const int b = (int)(idx / HW);
  const long p = idx - b * HW;
  const int y = (int)(p / W), xx = (int)(p % W);
  const float* f = flo + (long)b * 2 * HW;
  Bilin bl = warp_coords(xx, y, f[p], f[HW + p], H, W);
  long off[4];
  float wt[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    int cx = bl.x0 + (k & 1), cy = bl.y0 + (k >> 1);
    bool ok = cx >= 0 && cx < W && cy >= 0 && cy < H;
    off[k] = ok ? (long)cy * W + cx : 0;
    wt[k] = ok ? bl.w[k] : 0.f;
  }
  const float* xb = x + (long)b * C * HW;
  float* ob = out + (long)b * C * HW;
  for (int c = 0; c < C; ++c) {
    const float* xc = xb + c * HW;
    // ATen sums nw, ne, sw, se in this order; out-of-bounds corners contribute 0 (weight zeroed)
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) s += xc[off[k]] * wt[k];
    ob[c * HW + p] = s;
  }
}

// grid.y: groups of WB_CPT channels (the FTL feature warp has 192 channels on a 64x128 grid: one
// thread per pixel looping over all of them left the atomics latency-bound at 4 waves per CU)
constexpr int WB_CPT = 8;
__global__ void warp_bwd_kernel(const float* __restrict__ gout, const float* __restrict__ flo, float* __restrict__ gx,
                                int B, int C, int H, int W) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long HW = (long)H * W;
  if (idx >= B * HW) return;
  const int b = (int)(idx / HW);
  const long p = idx - b * HW;
  const int y = (int)(p / W), xx = (int)(p % W);
  const float* f = flo + (long)b * 2 * HW;
  Bilin bl = warp_coords(xx, y, f[p], f[HW + p], H, W);
  const int c0 = blockIdx.y * WB_CPT, c1 = min(C, c0 + WB_CPT);
  const float* gb = gout + ((long)b * C + c0) * HW;
  float* xb = gx + ((long)b * C + c0) * HW;
  float g[WB_CPT];
#pragma unroll
  for (int c = 0; c < WB_CPT; ++c) g[c] = c0 + c < c1 ? gb[c * HW + p] : 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    int cx = bl.x0 + (k & 1), cy = bl.y0 + (k >> 1);
    if (cx < 0 || cx >= W || cy < 0 || cy >= H) continue;
    long o = (long)cy * W + cx;
#pragma unroll
    for (int c = 0; c < WB_CPT; ++c)
      if (c0 + c < c1) atomicAdd(xb + c * HW + o, g[c] * bl.w[k]);
  }
}

// Gather form of the warp backward, deterministic (no float atomics on the gradient, a fixed
// summation order): the bilinear taps of every output pixel p are inverted once per image into
// per-source-pixel lists in CSR form (the flow is shared by all channels) -- a counting pass, an
// exclusive scan of the counts, a fill pass -- then each source pixel q sums its list for every
// channel in increasing p.  The fill pass takes list positions from integer atomics (their order
// varies run to run), so a sort pass orders each list by p first (once per call, not per channel
// group of the gather): an 8-input sorting network in registers, insertion sort in place for the
// rare longer lists (converging flow).
struct WgEntry {
  int p;
  float w;
};
constexpr int WG_REG = 8;     // lists up to this long are sorted in registers
constexpr int WS_BLOCK = 1024; // elements per block of the count scan

__device__ __forceinline__ void warp_taps(const float* __restrict__ flo, long idx, int H, int W, long q[4], float w[4]) {
  const long HW = (long)H * W;
  const int b = (int)(idx / HW);
  const long p = idx - b * HW;
  const int y = (int)(p / W), xx = (int)(p % W);
  const float* f = flo + (long)b * 2 * HW;
  const Bilin bl = warp_coords(xx, y, f[p], f[HW + p], H, W);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int cx = bl.x0 + (k & 1), cy = bl.y0 + (k >> 1);
    q[k] = (cx >= 0 && cx < W && cy >= 0 && cy < H) ? (long)b * HW + (long)cy * W + cx : -1;
    w[k] = bl.w[k];
  }
}

__global__ void warp_inv_count_kernel(const float* __restrict__ flo, int* __restrict__ cnt, int B, int H, int W) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)B * H * W) return;
  long q[4];
  float w[4];
  warp_taps(flo, idx, H, W, q, w);
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (q[k] >= 0) atomicAdd(cnt + q[k], 1);
}

// exclusive scan of cnt[0..n) into off[0..n], three passes: block-local scan (+ block totals),
// one-block scan of the totals, block offsets added
__global__ __launch_bounds__(256) void scan_blocks_kernel(const int* __restrict__ cnt, int* __restrict__ off,
                                                          int* __restrict__ bsum, long n) {
  __shared__ int sh[256];
  const long base = (long)blockIdx.x * WS_BLOCK + threadIdx.x * 4;
  int v[4], t = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[i] = base + i < n ? cnt[base + i] : 0;
    t += v[i];
  }
  sh[threadIdx.x] = t;
  __syncthreads();
  for (int d = 1; d < 256; d <<= 1) {  // Hillis-Steele inclusive scan of the thread totals
    const int a = threadIdx.x >= d ? sh[threadIdx.x - d] : 0;
    __syncthreads();
    sh[threadIdx.x] += a;
    __syncthreads();
  }
  int run = sh[threadIdx.x] - t;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (base + i < n) off[base + i] = run;
    run += v[i];
  }
  if (threadIdx.x == 255) bsum[blockIdx.x] = sh[255];
}

__global__ __launch_bounds__(1024) void scan_totals_kernel(int* __restrict__ bsum, int nb, int* __restrict__ total) {
  __shared__ int sh[1024];
  int carry = 0;
  for (int c0 = 0; c0 < nb; c0 += 1024) {
    const int i = c0 + threadIdx.x;
    const int v = i < nb ? bsum[i] : 0;
    sh[threadIdx.x] = v;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
      const int a = threadIdx.x >= d ? sh[threadIdx.x - d] : 0;
      __syncthreads();
      sh[threadIdx.x] += a;
      __syncthreads();
    }
    if (i < nb) bsum[i] = carry + sh[threadIdx.x] - v;  // exclusive
    carry += sh[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0) *total = carry;
}

__global__ __launch_bounds__(256) void scan_add_kernel(int* __restrict__ off, const int* __restrict__ bsum, long n) {
  const long base = (long)blockIdx.x * WS_BLOCK + threadIdx.x * 4;
  const int add = bsum[blockIdx.x];
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (base + i < n) off[base + i] += add;
}

// each tap's entry into its source pixel's list; cnt counts back down to 0 (ready for the next call)
__global__ void warp_inv_fill_kernel(const float* __restrict__ flo, int* __restrict__ cnt, const int* __restrict__ off,
                                     WgEntry* __restrict__ ent, int B, int H, int W) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long HW = (long)H * W;
  if (idx >= B * HW) return;
  long q[4];
  float w[4];
  warp_taps(flo, idx, H, W, q, w);
  int slot[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) slot[k] = q[k] >= 0 ? atomicSub(cnt + q[k], 1) - 1 : -1;  // all in flight
  const int p = (int)(idx % HW);
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (slot[k] >= 0) ent[off[q[k]] + slot[k]] = WgEntry{p, w[k]};
}

__device__ __forceinline__ void wg_cswap(WgEntry& a, WgEntry& b) {
  const bool sw = b.p < a.p;
  const WgEntry t = a;
  a = sw ? b : a;
  b = sw ? t : b;
}

// Batcher's odd-even merge sort network over N (a power of two) register entries, ascending p
template <int N>
__device__ __forceinline__ void wg_sort_net(WgEntry (&e)[N]) {
#pragma unroll
  for (int p = 1; p < N; p <<= 1)
#pragma unroll
    for (int k = p; k >= 1; k >>= 1)
#pragma unroll
      for (int j = k % p; j <= N - 1 - k; j += 2 * k)
#pragma unroll
        for (int i = 0; i <= (k - 1 < N - j - k - 1 ? k - 1 : N - j - k - 1); ++i)
          if ((i + j) / (2 * p) == (i + j + k) / (2 * p)) wg_cswap(e[i + j], e[i + j + k]);
}

template <int N>
__device__ __forceinline__ void wg_sort_list(WgEntry* __restrict__ L, int n) {
  WgEntry e[N];
#pragma unroll
  for (int j = 0; j < N; ++j) e[j] = j < n ? L[j] : WgEntry{0x7fffffff, 0.f};  // (empty slots sort last)
  wg_sort_net<N>(e);
#pragma unroll
  for (int j = 0; j < N; ++j)
    if (j < n) L[j] = e[j];
}

// sort each source pixel's list by output pixel p, once per call (the channel groups of the gather
// then read it in order): sorting networks in registers for lists of up to 8 / 16 entries; a longer
// list (strongly converging flow) is queued for warp_inv_sort_long_kernel, so no wave waits on one
// thread's long sort.  p is unique within a list, so the order is fully determined.
__global__ void warp_inv_sort_kernel(const int* __restrict__ off, WgEntry* __restrict__ ent, long n_src,
                                     int* __restrict__ long_count, int* __restrict__ long_queue) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n_src) return;
  const int s0 = off[idx], n = off[idx + 1] - s0;
  if (n <= 1) return;
  if (n <= 8) wg_sort_list<8>(ent + s0, n);
  else if (n <= 16) wg_sort_list<16>(ent + s0, n);
  else long_queue[atomicAdd(long_count, 1)] = (int)idx;  // (queue order is irrelevant)
}

// the queued long lists, one wave per list (grid-stride over the device-side count): the list is
// staged in the wave's LDS slice and every entry is written to its rank (the number of entries with
// a smaller p); a list beyond the slice (not seen on smooth flows) is insertion-sorted by one lane
constexpr int WG_LONG = 512;
__global__ __launch_bounds__(256) void warp_inv_sort_long_kernel(const int* __restrict__ off, WgEntry* __restrict__ ent,
                                                                 const int* __restrict__ long_count,
                                                                 const int* __restrict__ long_queue) {
  __shared__ WgEntry sh[4][WG_LONG];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int cnt = *long_count;
  for (int i = blockIdx.x * 4 + wv; i < cnt; i += gridDim.x * 4) {
    const int q = long_queue[i];
    const int s0 = off[q], n = off[q + 1] - s0;
    WgEntry* L = ent + s0;
    if (n > WG_LONG) {
      if (lane == 0)
        for (int a = 1; a < n; ++a) {
          const WgEntry v = L[a];
          int j = a - 1;
          while (j >= 0 && L[j].p > v.p) {
            L[j + 1] = L[j];
            --j;
          }
          L[j + 1] = v;
        }
      continue;
    }
    for (int j = lane; j < n; j += 64) sh[wv][j] = L[j];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    for (int j = lane; j < n; j += 64) {
      const int pj = sh[wv][j].p;
      int rank = 0;
      for (int k = 0; k < n; ++k) rank += sh[wv][k].p < pj;
      L[rank] = sh[wv][j];
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// gx[b][c][q] (+)= sum over q's (sorted) list of w * gout[b][c][p]; grid.y: channel groups of WB_CPT
__global__ void warp_inv_gather_kernel(const float* __restrict__ gout, const int* __restrict__ off,
                                       const WgEntry* __restrict__ ent, float* __restrict__ gx, int B, int C, int H,
                                       int W, int accumulate) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long HW = (long)H * W;
  if (idx >= B * HW) return;
  const int b = (int)(idx / HW);
  const long q = idx - b * HW;
  const int s0 = off[idx], n = off[idx + 1] - s0;
  const int c0 = blockIdx.y * WB_CPT, c1 = min(C, c0 + WB_CPT);
  const float* gb = gout + ((long)b * C + c0) * HW;
  float s[WB_CPT];
#pragma unroll
  for (int c = 0; c < WB_CPT; ++c) s[c] = 0.f;
  for (int j = 0; j < n; ++j) {
    const WgEntry e = ent[s0 + j];
#pragma unroll
    for (int c = 0; c < WB_CPT; ++c)
      if (c0 + c < c1) s[c] += e.w * gb[c * HW + e.p];
  }
  float* xb = gx + ((long)b * C + c0) * HW + q;
#pragma unroll
  for (int c = 0; c < WB_CPT; ++c)
    if (c0 + c < c1) xb[c * HW] = accumulate ? xb[c * HW] + s[c] : s[c];
}

// mask[y][x] = (|warp(grid+flo01, flo10) - grid|_1 < thr)
__global__ void flow_mask_kernel(const float* __restrict__ flo01, const float* __restrict__ flo10,
                                 float* __restrict__ mask, int B, int H, int W, float thr) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long HW = (long)H * W;
  if (idx >= B * HW) return;
  const int b = (int)(idx / HW);
  const long p = idx - b * HW;
  const int y = (int)(p / W), xx = (int)(p % W);
  const float* f10 = flo10 + (long)b * 2 * HW;
  const float* f01 = flo01 + (long)b * 2 * HW;
  Bilin bl = warp_coords(xx, y, f10[p], f10[HW + p], H, W);
  float s0 = 0.f, s1 = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    int cx = bl.x0 + (k & 1), cy = bl.y0 + (k >> 1);
    if (cx < 0 || cx >= W || cy < 0 || cy >= H) continue;
    long o = (long)cy * W + cx;
    s0 += ((float)cx + f01[o]) * bl.w[k];
    s1 += ((float)cy + f01[HW + o]) * bl.w[k];
  }
  float err = fabsf(s0 - (float)xx) + fabsf(s1 - (float)y);
  mask[idx] = err < thr ? 1.f : 0.f;
}

// scale: input pixels per output pixel along the axis -- n_in / n_out for a size-given resize, 1 / s for
// F.interpolate(scale_factor=s) (ATen's area_pixel_compute_scale; the two differ when n_in * s is not
// a whole number)
__device__ __forceinline__ void resize_axis(int d, int n_in, float scale, int& i0, int& i1, float& l1) {
  float src = ((float)d + 0.5f) * scale - 0.5f;
  src = src < 0.f ? 0.f : src;
  i0 = (int)src;
  i0 = i0 > n_in - 1 ? n_in - 1 : i0;
  i1 = i0 < n_in - 1 ? i0 + 1 : i0;
  l1 = src - (float)i0;
}

// the bilinear blend of the four taps (a b / c d), its fused multiply-adds spelled out so that every
// resize kernel rounds alike whatever the compiler would contract
__device__ __forceinline__ float bilerp(float a, float b, float c, float d, float lx, float ly) {
  const float top = fmaf(lx, b, (1.f - lx) * a), bot = fmaf(lx, d, (1.f - lx) * c);
  return fmaf(ly, bot, (1.f - ly) * top);
}

// out[n][c] = resize(x[nc]) * chscale[c] (+ addend[n][c]); binarize: out = out > 0
// out/addend images are out_bs floats apart (channel-concat targets, AA/utilities.py:98-109)
__global__ void resize_kernel(const float* __restrict__ x, float* __restrict__ out, long NC, int C, int H, int W, int Ho,
                              int Wo, float sy, float sx, const float* chscale, int binarize, long out_bs,
                              const float* __restrict__ addend) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= NC * Ho * Wo) return;
  int ox = (int)(idx % Wo);
  long t = idx / Wo;
  int oy = (int)(t % Ho);
  long nc = t / Ho;
  int y0, y1, x0, x1;
  float ly, lx;
  resize_axis(oy, H, sy, y0, y1, ly);
  resize_axis(ox, W, sx, x0, x1, lx);
  const float* p = x + nc * H * W;
  float v = bilerp(p[(long)y0 * W + x0], p[(long)y0 * W + x1], p[(long)y1 * W + x0], p[(long)y1 * W + x1], lx, ly);
  if (chscale) v *= chscale[nc % C];
  if (binarize) v = v > 0.f ? 1.f : 0.f;
  const long o = (nc / C) * out_bs + (nc % C) * (long)Ho * Wo + (long)oy * Wo + ox;
  if (addend) v += addend[o];
  out[o] = v;
}

// resize_kernel with the plane on blockIdx.z and the output row on blockIdx.y * 4 + threadIdx.y: the
// per-element 64-bit (plane, row, column) division of the flat form made it VALU-bound (config 5:
// 22 launches, 268 us each); same arithmetic per output element
__global__ __launch_bounds__(256) void resize_plane_kernel(const float* __restrict__ x, float* __restrict__ out, int C,
                                                           int H, int W, int Ho, int Wo, float sy, float sx,
                                                           const float* chscale, int binarize, long out_bs,
                                                           const float* __restrict__ addend) {
  const int ox = blockIdx.x * 64 + threadIdx.x, oy = blockIdx.y * 4 + threadIdx.y;
  if (ox >= Wo || oy >= Ho) return;
  const int nc = blockIdx.z, n = nc / C, c = nc - n * C;
  int y0, y1, x0, x1;
  float ly, lx;
  resize_axis(oy, H, sy, y0, y1, ly);
  resize_axis(ox, W, sx, x0, x1, lx);
  const float* p = x + (long)nc * H * W;
  float v = bilerp(p[(long)y0 * W + x0], p[(long)y0 * W + x1], p[(long)y1 * W + x0], p[(long)y1 * W + x1], lx, ly);
  if (chscale) v *= chscale[c];
  if (binarize) v = v > 0.f ? 1.f : 0.f;
  const long o = (long)n * out_bs + (long)c * Ho * Wo + (long)oy * Wo + ox;
  if (addend) v += addend[o];
  out[o] = v;
}

// resize_plane_kernel for an exact x2 upsample (Ho = 2H, Wo = 2W, both scales 0.5; W even, aligned
// rows): one thread writes output rows 2r, 2r + 1, columns 4q..4q+3 (two float4 stores) from the input
// values they read (per output row its two source rows, columns 2q-1..2q+2, clamped: 12 loads for 8
// outputs instead of 32, and no per-element index decode).  Each output takes resize_axis' indices and weights and the same
// bilerp, so the result is bitwise the per-element kernel's.
// the 4 taps of row `row` that output columns 4q..4q+3 read: column 2q-1 (clamped), 2q, 2q+1, 2q+2
// (clamped); (t[0], t[1]) / (t[1], t[2]) / (t[1], t[2]) / (t[2], t[3]) are resize_axis' (x0, x1)
// for the four columns, except at q = 0 where column 0 reads (x0, x1) = (0, 1) = (t[0], t[2])
__device__ __forceinline__ void up2_row(const float* row, int q, int W, float t[4]) {
  const float2 m = *reinterpret_cast<const float2*>(row + 2 * q);
  t[0] = row[q > 0 ? 2 * q - 1 : 0];
  t[1] = m.x;
  t[2] = m.y;
  t[3] = row[2 * q + 2 < W ? 2 * q + 2 : W - 1];
}
__device__ __forceinline__ void resize_up2_plane(const float* __restrict__ x, float* __restrict__ out, int nc, int C,
                                                 int H, int W, int r, int q, const float* chscale, int binarize,
                                                 long out_bs, const float* __restrict__ addend) {
  const int n = nc / C, c = nc - n * C;
  const float* p = x + (long)nc * H * W;
  float lx[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    int x0, x1;
    resize_axis(4 * q + b, W, 0.5f, x0, x1, lx[b]);
  }
  const float cs = chscale ? chscale[c] : 1.f;
  const int Wo = 2 * W;
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const int oy = 2 * r + a;
    int y0, y1;
    float ly;
    resize_axis(oy, H, 0.5f, y0, y1, ly);
    float t0[4], t1[4];
    up2_row(p + (long)y0 * W, q, W, t0);
    up2_row(p + (long)y1 * W, q, W, t1);
    // second tap of output column 4q: column 2q, or column 1 at q = 0
    const float t0b = q > 0 ? t0[1] : t0[2], t1b = q > 0 ? t1[1] : t1[2];
    float o4[4];
    o4[0] = bilerp(t0[0], t0b, t1[0], t1b, lx[0], ly);
    o4[1] = bilerp(t0[1], t0[2], t1[1], t1[2], lx[1], ly);
    o4[2] = bilerp(t0[1], t0[2], t1[1], t1[2], lx[2], ly);
    o4[3] = bilerp(t0[2], t0[3], t1[2], t1[3], lx[3], ly);
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      if (chscale) o4[b] *= cs;
      if (binarize) o4[b] = o4[b] > 0.f ? 1.f : 0.f;
    }
    const long o = (long)n * out_bs + (long)c * (2 * H) * Wo + (long)oy * Wo + 4 * q;
    if (addend) {
      const float4 d = *reinterpret_cast<const float4*>(addend + o);
      o4[0] += d.x, o4[1] += d.y, o4[2] += d.z, o4[3] += d.w;
    }
#pragma unroll
    for (int b = 0; b < 4; ++b) __builtin_nontemporal_store(o4[b], out + o + b);
  }
}

__global__ __launch_bounds__(256) void resize_up2_kernel(const float* __restrict__ x, float* __restrict__ out, int C,
                                                         int H, int W, const float* chscale, int binarize,
                                                         long out_bs, const float* __restrict__ addend) {
  // the plane's (row r, quad q) pairs in row-major order: a block writes whole output row pairs.
  // Consecutive blocks land on different XCDs (round robin): when the plane's block count allows, the
  // blocks of one XCD take one contiguous run of rows so that the rows a block shares with its
  // neighbours (r - 1, r + 1) hit that XCD's L2
  const int gx = gridDim.x, bx = (gx & 7) == 0 ? (blockIdx.x & 7) * (gx >> 3) + (blockIdx.x >> 3) : blockIdx.x;
  const int i = bx * 256 + threadIdx.x, Wq2 = W >> 1;
  if (i >= H * Wq2) return;
  const int r = i / Wq2, q = i - r * Wq2;
  resize_up2_plane(x, out, blockIdx.y, C, H, W, r, q, chscale, binarize, out_bs, addend);
}

// weight with which input index i enters output index d along one axis (0 if it does not)
__device__ __forceinline__ float resize_weight(int d, int i, int n_in, float scale) {
  int i0, i1;
  float l1;
  resize_axis(d, n_in, scale, i0, i1, l1);
  return (i0 == i ? 1.f - l1 : 0.f) + (i1 == i ? l1 : 0.f);
}

// output index range [lo, hi] that can read input index i (src(d) in [i-1, i+1], with slack)
__device__ __forceinline__ void resize_span(int i, int n_out, float scale, int& lo, int& hi) {
  const float inv = 1.f / scale;
  lo = (int)floorf(((float)i - 0.5f) * inv - 0.5f) - 1;
  hi = (int)ceilf(((float)i + 1.5f) * inv - 0.5f) + 1;
  lo = lo < 0 ? 0 : lo;
  hi = hi > n_out - 1 ? n_out - 1 : hi;
}

// adjoint of the bilinear resize as a gather: each input element sums the output gradients that
// read it, with the forward's own weights (deterministic, no atomics, every gx written once)
__global__ void resize_bwd_kernel(const float* __restrict__ gout, float* __restrict__ gx, long NC, int C, int H, int W,
                                  int Ho, int Wo, float sy, float sx, long gout_bs) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= NC * H * W) return;
  int ix = (int)(idx % W);
  long t = idx / W;
  int iy = (int)(t % H);
  long nc = t / H;
  int ylo, yhi, xlo, xhi;
  resize_span(iy, Ho, sy, ylo, yhi);
  resize_span(ix, Wo, sx, xlo, xhi);
  const float* g = gout + (nc / C) * gout_bs + (nc % C) * (long)Ho * Wo;
  float acc = 0.f;
  for (int oy = ylo; oy <= yhi; ++oy) {
    const float wy = resize_weight(oy, iy, H, sy);
    if (wy == 0.f) continue;
    float row = 0.f;
    for (int ox = xlo; ox <= xhi; ++ox) {
      const float wx = resize_weight(ox, ix, W, sx);
      if (wx != 0.f) row += wx * g[(long)oy * Wo + ox];
    }
    acc += wy * row;
  }
  gx[idx] = acc;
}

// Adjoint of the exact x2 bilinear upsample (align_corners=False, Ho = 2H, Wo = 2W), optionally
// times the ReLU mask of its input (the producer ConvReLU's backward, y > 0: ATen's
// threshold_backward on the ReLU result).  Along one axis input i is read by outputs 2i-1 .. 2i+2
// with the fixed weights 0.25, 0.75 (1 at i = 0: src clamps to 0), 0.75 (1 at i = n-1: i0 = i1),
// 0.25 -- the generic gather's per-candidate weight recomputation and +/-1 slack are gone.  Each
// thread produces two adjacent input columns (j = 2t, 2t+1) from one aligned float4 and two
// scalars per output row (W even; the launcher falls back to the generic gather otherwise).
__device__ __forceinline__ void up2_axis_w(int i, int n, float (&w)[4]) {
  w[0] = i >= 1 ? 0.25f : 0.f;
  w[1] = i == 0 ? 1.f : 0.75f;
  w[2] = i == n - 1 ? 1.f : 0.75f;
  w[3] = i <= n - 2 ? 0.25f : 0.f;
}

__global__ void up2_bwd_kernel(const float* __restrict__ gout, const float* __restrict__ ymask, float* __restrict__ gx,
                               long NC, int C, int H, int W, long gout_bs) {
  const int Wh = W >> 1;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= NC * H * Wh) return;
  const int t = (int)(idx % Wh);
  const long r = idx / Wh;
  const int iy = (int)(r % H);
  const long nc = r / H;
  const int Wo = 2 * W, Ho = 2 * H;
  const float* g = gout + (nc / C) * gout_bs + (nc % C) * (long)Ho * Wo;
  float wy[4], wa[4], wb[4];
  up2_axis_w(iy, H, wy);
  up2_axis_w(2 * t, W, wa);      // column j = 2t: outputs 4t-1 .. 4t+2
  up2_axis_w(2 * t + 1, W, wb);  // column j = 2t+1: outputs 4t+1 .. 4t+4
  float a0 = 0.f, a1 = 0.f;
#pragma unroll
  for (int dy = 0; dy < 4; ++dy) {
    const int oy = 2 * iy - 1 + dy;
    if (wy[dy] == 0.f) continue;  // out-of-range rows carry weight 0 (oy < 0 or oy >= Ho)
    const float* row = g + (long)oy * Wo;
    const f32x4 c = *reinterpret_cast<const f32x4*>(row + 4 * t);  // outputs 4t .. 4t+3
    const float l = t > 0 ? row[4 * t - 1] : 0.f;
    const float rr = 4 * t + 4 < Wo ? row[4 * t + 4] : 0.f;
    const float s0 = wa[0] * l + wa[1] * c[0] + wa[2] * c[1] + wa[3] * c[2];
    const float s1 = wb[0] * c[1] + wb[1] * c[2] + wb[2] * c[3] + wb[3] * rr;
    a0 += wy[dy] * s0;
    a1 += wy[dy] * s1;
  }
  const long o = (nc * H + iy) * (long)W + 2 * t;
  if (ymask) {
    const f32x2 m = *reinterpret_cast<const f32x2*>(ymask + o);
    a0 = m[0] > 0.f ? a0 : 0.f;
    a1 = m[1] > 0.f ? a1 : 0.f;
  }
  *reinterpret_cast<f32x2*>(gx + o) = f32x2{a0, a1};
}

}  // namespace

extern "C" {

int vst_upsample2x_bwd(const float* gout, const float* ymask, float* gx, long NC, int C, int H, int W, long gout_bs,
                       void* stream) {
  VST_CHECK_ARG(gout && gx && NC > 0 && C > 0 && H > 0 && W > 0 && NC % C == 0);
  const long Ho = 2L * H, Wo = 2L * W;
  if (gout_bs <= 0) gout_bs = (long)C * Ho * Wo;
  hipStream_t st = (hipStream_t)stream;
  const bool vec = (W % 2 == 0) && (gout_bs % 4 == 0) && (((uintptr_t)gout | (uintptr_t)gx | (uintptr_t)ymask) % 16 == 0);
  if (!vec) {
    if (ymask) return VST_EUNSUPPORTED;  // the generic gather has no mask epilogue
    resize_bwd_kernel<<<ceil_div(NC * H * W, 256), 256, 0, st>>>(gout, gx, NC, C, H, W, (int)Ho, (int)Wo, 0.5f, 0.5f,
                                                                  gout_bs);
    return vst_launch_status();
  }
  const long total = NC * H * (W / 2);
  up2_bwd_kernel<<<ceil_div(total, 256), 256, 0, st>>>(gout, ymask, gx, NC, C, H, W, gout_bs);
  return vst_launch_status();
}

int vst_maxpool2x2_fwd(const float* x, float* y, long NC, int H, int W, void* stream) {
  VST_CHECK_ARG(x && y && NC > 0 && H >= 2 && W >= 2);
  if (pool_vec_ok(NC, W, x, x, x, y)) {
    maxpool_fwd_vec_kernel<<<pool_vec_grid(NC, H / 2, W), dim3(64, 4), 0, (hipStream_t)stream>>>(x, y, H, W);
    return vst_launch_status();
  }
  long total = NC * (H / 2) * (W / 2);
  maxpool_fwd_kernel<<<ceil_div(total, 256), 256, 0, (hipStream_t)stream>>>(x, y, NC, H, W);
  return vst_launch_status();
}

int vst_maxpool2x2_bwd(const float* x, const float* gy, float* gx, long NC, int H, int W, int relu_mask, void* stream) {
  VST_CHECK_ARG(x && gy && gx && NC > 0 && H >= 2 && W >= 2);
  if (pool_vec_ok(NC, W, x, gx, gx, gy)) {
    maxpool_bwd_vec_kernel<<<pool_vec_grid(NC, (H + 1) / 2, W), dim3(64, 4), 0, (hipStream_t)stream>>>(
        x, gy, nullptr, gx, H, W, relu_mask);
    return vst_launch_status();
  }
  long total = NC * H * W;
  maxpool_bwd_kernel<<<ceil_div(total, 256), 256, 0, (hipStream_t)stream>>>(x, gy, gx, NC, H, W, relu_mask);
  return vst_launch_status();
}

int vst_maxpool2x2_bwd_add(const float* x, const float* gy, const float* addend, float* gx, long NC, int H, int W,
                           int relu_mask, void* stream) {
  VST_CHECK_ARG(x && gx && NC > 0 && H >= 2 && W >= 2);
  if (pool_vec_ok(NC, W, x, gx, addend, gy)) {
    maxpool_bwd_vec_kernel<<<pool_vec_grid(NC, (H + 1) / 2, W), dim3(64, 4), 0, (hipStream_t)stream>>>(
        x, gy, addend, gx, H, W, relu_mask);
    return vst_launch_status();
  }
  const long total = NC * ((H + 1) / 2) * ((W + 1) / 2);
  maxpool_bwd_add_kernel<<<ceil_div(total, 256), 256, 0, (hipStream_t)stream>>>(x, gy, addend, gx, NC, H, W,
                                                                                 relu_mask);
  return vst_launch_status();
}

int vst_warp_fwd(const float* x, const float* flo, float* out, int B, int C, int H, int W, void* stream) {
  VST_CHECK_ARG(x && flo && out && B > 0 && C > 0 && H > 0 && W > 0);
  long total = (long)B * H * W;
  warp_fwd_kernel<<<ceil_div(total, 256), 256, 0, (hipStream_t)stream>>>(x, flo, out, B, C, H, W);
  return vst_launch_status();
}

// gx must be zeroed (or hold a gradient to accumulate into): float atomics scatter into it
int vst_warp_bwd(const float* gout, const float* flo, float* gx, int B, int C, int H, int W, void* stream) {
  VST_CHECK_ARG(gout && flo && gx && B > 0 && C > 0 && H > 0 && W > 0);
  long total = (long)B * H * W;
  dim3 g(ceil_div(total, 256), (C + WB_CPT - 1) / WB_CPT);
  warp_bwd_kernel<<<g, 256, 0, (hipStream_t)stream>>>(gout, flo, gx, B, C, H, W);
  return vst_launch_status();
}

// workspace: [cnt: n ints + the long-list count][off: n + 1 ints][block totals][long-list queue: n ints]
// [entries: up to 4 per pixel], 16-B aligned
static long align16(long x) { return (x + 15) / 16 * 16; }
long vst_warp_bwd_workspace(int B, int H, int W) {
  const long n = (long)B * H * W, nb = (n + WS_BLOCK - 1) / WS_BLOCK;
  return align16((n + 1) * 4) + align16((n + 1) * 4) + align16((nb + 1) * 4) + align16(n * 4) +
         4 * n * (long)sizeof(WgEntry);
}

int vst_warp_bwd_gather(const float* gout, const float* flo, float* gx, void* workspace, int B, int C, int H, int W,
                        int accumulate, void* stream) {
  VST_CHECK_ARG(gout && flo && gx && workspace && B > 0 && C > 0 && H > 0 && W > 0);
  VST_CHECK_ARG(((uintptr_t)workspace & 15) == 0);
  const long n = (long)B * H * W, nb = (n + WS_BLOCK - 1) / WS_BLOCK;
  VST_CHECK_ARG(4 * n < (1L << 31));
  hipStream_t st = (hipStream_t)stream;
  char* base = static_cast<char*>(workspace);
  int* cnt = reinterpret_cast<int*>(base);  // (cnt[n]: the long-list count)
  int* off = reinterpret_cast<int*>(base + align16((n + 1) * 4));
  int* bsum = reinterpret_cast<int*>(base + 2 * align16((n + 1) * 4));
  int* lq = reinterpret_cast<int*>(base + 2 * align16((n + 1) * 4) + align16((nb + 1) * 4));
  WgEntry* ent = reinterpret_cast<WgEntry*>(base + 2 * align16((n + 1) * 4) + align16((nb + 1) * 4) + align16(n * 4));
  hipError_t e = hipMemsetAsync(cnt, 0, (n + 1) * 4, st);
  if (e != hipSuccess) return (int)e;
  warp_inv_count_kernel<<<ceil_div(n, 256), 256, 0, st>>>(flo, cnt, B, H, W);
  scan_blocks_kernel<<<nb, 256, 0, st>>>(cnt, off, bsum, n);
  scan_totals_kernel<<<1, 1024, 0, st>>>(bsum, (int)nb, off + n);
  scan_add_kernel<<<nb, 256, 0, st>>>(off, bsum, n);
  warp_inv_fill_kernel<<<ceil_div(n, 256), 256, 0, st>>>(flo, cnt, off, ent, B, H, W);
  warp_inv_sort_kernel<<<ceil_div(n, 256), 256, 0, st>>>(off, ent, n, cnt + n, lq);
  warp_inv_sort_long_kernel<<<256, 256, 0, st>>>(off, ent, cnt + n, lq);
  dim3 g(ceil_div(n, 256), (C + WB_CPT - 1) / WB_CPT);
  warp_inv_gather_kernel<<<g, 256, 0, st>>>(gout, off, ent, gx, B, C, H, W, accumulate);
  return vst_launch_status();
}

int vst_flow_warp_mask(const float* flo01, const float* flo10, float* mask, int B, int H, int W, float threshold,
                       void* stream) {
  VST_CHECK_ARG(flo01 && flo10 && mask && B > 0 && H > 0 && W > 0);
  long total = (long)B * H * W;
  flow_mask_kernel<<<ceil_div(total, 256), 256, 0, (hipStream_t)stream>>>(flo01, flo10, mask, B, H, W, threshold);
  return vst_launch_status();
}

int vst_resize_bilinear_scaled(const float* x, float* out, long NC, int C, int H, int W, int Ho, int Wo, float scale_y,
                               float scale_x, const float* chscale, int binarize, long out_bs, const float* addend,
                               void* stream) {
  VST_CHECK_ARG(x && out && NC > 0 && C > 0 && H > 0 && W > 0 && Ho > 0 && Wo > 0 && NC % C == 0);
  VST_CHECK_ARG(scale_y > 0.f && scale_x > 0.f);
  long total = NC * Ho * Wo;
  if (out_bs <= 0) out_bs = (long)C * Ho * Wo;
  if (NC <= 65535 && Ho == 2 * H && Wo == 2 * W && scale_y == 0.5f && scale_x == 0.5f && W % 2 == 0 &&
      (long)H * W < (1L << 31) && out_bs % 4 == 0 && ((uintptr_t)x & 7) == 0 && (((uintptr_t)out | (uintptr_t)addend) & 15) == 0) {
    const dim3 g((unsigned)ceil_div((long)H * (W / 2), 256), (unsigned)NC);
    resize_up2_kernel<<<g, 256, 0, (hipStream_t)stream>>>(x, out, C, H, W, chscale, binarize, out_bs, addend);
    return vst_launch_status();
  }
  if (NC <= 65535 && Ho <= 4 * 65535) {
    const dim3 g((unsigned)ceil_div(Wo, 64), (unsigned)ceil_div(Ho, 4), (unsigned)NC);
    resize_plane_kernel<<<g, dim3(64, 4), 0, (hipStream_t)stream>>>(x, out, C, H, W, Ho, Wo, scale_y, scale_x, chscale,
                                                                    binarize, out_bs, addend);
    return vst_launch_status();
  }
  resize_kernel<<<ceil_div(total, 256), 256, 0, (hipStream_t)stream>>>(x, out, NC, C, H, W, Ho, Wo, scale_y, scale_x,
                                                                       chscale, binarize, out_bs, addend);
  return vst_launch_status();
}

int vst_resize_bilinear(const float* x, float* out, long NC, int C, int H, int W, int Ho, int Wo,
                        const float* chscale, int binarize, long out_bs, const float* addend, void* stream) {
  VST_CHECK_ARG(Ho > 0 && Wo > 0);
  return vst_resize_bilinear_scaled(x, out, NC, C, H, W, Ho, Wo, (float)H / (float)Ho, (float)W / (float)Wo, chscale,
                                    binarize, out_bs, addend, stream);
}

int vst_resize_bilinear_scaled_bwd(const float* gout, float* gx, long NC, int C, int H, int W, int Ho, int Wo,
                                   float scale_y, float scale_x, long gout_bs, void* stream) {
  VST_CHECK_ARG(gout && gx && NC > 0 && C > 0 && H > 0 && W > 0 && Ho > 0 && Wo > 0 && NC % C == 0);
  VST_CHECK_ARG(scale_y > 0.f && scale_x > 0.f);
  long total = NC * H * W;
  if (gout_bs <= 0) gout_bs = (long)C * Ho * Wo;
  resize_bwd_kernel<<<ceil_div(total, 256), 256, 0, (hipStream_t)stream>>>(gout, gx, NC, C, H, W, Ho, Wo, scale_y,
                                                                           scale_x, gout_bs);
  return vst_launch_status();
}

int vst_resize_bilinear_bwd(const float* gout, float* gx, long NC, int C, int H, int W, int Ho, int Wo, long gout_bs,
                            void* stream) {
  VST_CHECK_ARG(Ho > 0 && Wo > 0);
  return vst_resize_bilinear_scaled_bwd(gout, gx, NC, C, H, W, Ho, Wo, (float)H / (float)Ho, (float)W / (float)Wo,
                                        gout_bs, stream);
}

}  // extern "C"
