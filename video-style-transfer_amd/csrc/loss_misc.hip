// Loss reductions, elementwise ops and the optimizer of the ReCoNet training step (gfx950).
//
// Every loss is a two-stage deterministic reduction: a grid-stride kernel writes per-block
// partials {sum, count}; a one-block finisher sums them in fixed order and writes
//   out[0] = weight * sum / denom,  out[1] = weight / denom
// (denom = the on-device non-zero count for the temporal losses, so the reference's
// `torch.nonzero(mask).shape[0]` host sync disappears; numel for MSE; 1 for TV).  Backward
// kernels read the upstream gradient and out[1] from device memory: no host round trip.
//
// Reference semantics: RC/train_single/train_candy.py:90-145 (FTL, OTL, content, style, TV),
// RC/utilities.py:101-106 (vgg_normalize), RC/network.py:83-85 (ConvTanh),
// torch.optim.Adam defaults (train_candy.py:44,152).
#include "vst_common.h"
#include "vst_hip.h"

namespace {

constexpr int RT = 256;
constexpr int MAXB = 1024;

__device__ __forceinline__ void block_partial(float s, float c, float* partial) {
  __shared__ float sh[2][RT / 64];
  s = wave_sum(s);
  c = wave_sum(c);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    sh[0][w] = s;
    sh[1][w] = c;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = 0.f, b = 0.f;
    for (int i = 0; i < RT / 64; ++i) {
      a += sh[0][i];
      b += sh[1][i];
    }
    partial[2 * blockIdx.x] = a;
    partial[2 * blockIdx.x + 1] = b;
  }
}

__global__ void finish_kernel(const float* __restrict__ partial, int nb, float* __restrict__ out, float weight,
                              double fixed_denom, int use_count) {
  __shared__ double sh[2][RT / 64];
  double s = 0.0, c = 0.0;
  for (int i = threadIdx.x; i < nb; i += RT) {
    s += partial[2 * i];
    c += partial[2 * i + 1];
  }
  s = wave_sum_d(s);
  c = wave_sum_d(c);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    sh[0][w] = s;
    sh[1][w] = c;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0, b = 0.0;
    for (int i = 0; i < RT / 64; ++i) {
      a += sh[0][i];
      b += sh[1][i];
    }
    double d = use_count ? b : fixed_denom;
    float inv = (float)(1.0 / (d > 0.0 ? d : 1.0));
    // reference: loss = sum * (1 / nnz) * LAMBDA   (train_candy.py:105-106) in fp32
    float sum = (float)a;
    out[0] = sum * inv * weight;
    out[1] = inv * weight;
    out[2] = (float)b;
  }
}

// FTL (mode 0): sum_{n,c,p} m(n,p) * (a - b)^2, m = (mask > 0), count = C * nnz(m)
// OTL (mode 1): ot = a - b, it = lum(c - d); sum_{n,c,p} m * (ot - it)^2, count = C * nnz(m != 0)
template <int MODE>
__global__ void masked_sqdiff_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                     const float* __restrict__ c, const float* __restrict__ d,
                                     const float* __restrict__ mask, int N, int C, long HW, float* partial) {
  float s = 0.f, cnt = 0.f;
  const long total = (long)N * HW;
  for (long idx = (long)blockIdx.x * RT + threadIdx.x; idx < total; idx += (long)gridDim.x * RT) {
    const long n = idx / HW, p = idx - n * HW;
    float m = mask[idx];
    if (MODE == 0) m = m > 0.f ? 1.f : 0.f;
    if (m == 0.f) continue;
    cnt += (float)C;
    const long base = n * C * HW + p;
    if (MODE == 0) {
      for (int ch = 0; ch < C; ++ch) {
        float df = a[base + ch * HW] - b[base + ch * HW];
        s += m * (df * df);
      }
    } else {
      float i0 = c[base] - d[base], i1 = c[base + HW] - d[base + HW], i2 = c[base + 2 * HW] - d[base + 2 * HW];
      float it = 0.2126f * i0 + 0.7152f * i1 + 0.0722f * i2;
      for (int ch = 0; ch < 3; ++ch) {
        float df = (a[base + ch * HW] - b[base + ch * HW]) - it;
        s += m * (df * df);
      }
    }
  }
  block_partial(s, cnt, partial);
}

template <int MODE>
__global__ void masked_sqdiff_bwd_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                         const float* __restrict__ c, const float* __restrict__ d,
                                         const float* __restrict__ mask, int N, int C, long HW,
                                         const float* __restrict__ gout, const float* __restrict__ scale,
                                         float* __restrict__ ga, float* __restrict__ gb) {
  const long total = (long)N * HW;
  const float k = 2.f * gout[0] * scale[1];
  for (long idx = (long)blockIdx.x * RT + threadIdx.x; idx < total; idx += (long)gridDim.x * RT) {
    const long n = idx / HW, p = idx - n * HW;
    float m = mask[idx];
    if (MODE == 0) m = m > 0.f ? 1.f : 0.f;
    const long base = n * C * HW + p;
    float it = 0.f;
    if (MODE == 1) {
      float i0 = c[base] - d[base], i1 = c[base + HW] - d[base + HW], i2 = c[base + 2 * HW] - d[base + 2 * HW];
      it = 0.2126f * i0 + 0.7152f * i1 + 0.0722f * i2;
    }
    for (int ch = 0; ch < C; ++ch) {
      const long o = base + ch * HW;
      float g = k * m * ((a[o] - b[o]) - it);
      if (ga) ga[o] = g;
      if (gb) gb[o] = -g;
    }
  }
}

// sum (a - b[i % nb])^2
__global__ void sqdiff_kernel(const float* __restrict__ a, const float* __restrict__ b, long n, long nb,
                              float* partial) {
  float s = 0.f;
  for (long i = (long)blockIdx.x * RT + threadIdx.x; i < n; i += (long)gridDim.x * RT) {
    float df = a[i] - b[i % nb];
    s += df * df;
  }
  block_partial(s, 0.f, partial);
}

__global__ void sqdiff_bwd_kernel(const float* __restrict__ a, const float* __restrict__ b, long n, long nb,
                                  const float* __restrict__ gout, const float* __restrict__ scale,
                                  float* __restrict__ ga, float* __restrict__ gb) {
  const float k = 2.f * gout[0] * scale[1];
  for (long i = (long)blockIdx.x * RT + threadIdx.x; i < n; i += (long)gridDim.x * RT) {
    float g = k * (a[i] - b[i % nb]);
    if (ga) ga[i] = g;
    if (gb) gb[i] = -g;
  }
}

// sum of a vector (for per-image partial losses)
__global__ void vsum_kernel(const float* __restrict__ x, long n, float* partial) {
  float s = 0.f;
  for (long i = (long)blockIdx.x * RT + threadIdx.x; i < n; i += (long)gridDim.x * RT) s += x[i];
  block_partial(s, 0.f, partial);
}

// TV: sum over y<H-1, x<W-1 of (s[y][x+1]-s[y][x])^2 + (s[y+1][x]-s[y][x])^2  (train_candy.py:141-145)
__global__ void tv_kernel(const float* __restrict__ s, long NC, int H, int W, float* partial) {
  float acc = 0.f;
  const long total = NC * (H - 1) * (W - 1);
  for (long i = (long)blockIdx.x * RT + threadIdx.x; i < total; i += (long)gridDim.x * RT) {
    int x = (int)(i % (W - 1));
    long t = i / (W - 1);
    int y = (int)(t % (H - 1));
    long nc = t / (H - 1);
    const float* p = s + nc * H * W + (long)y * W + x;
    float d1 = p[1] - p[0], d2 = p[W] - p[0];
    acc += d1 * d1 + d2 * d2;
  }
  block_partial(acc, 0.f, partial);
}

__global__ void tv_bwd_kernel(const float* __restrict__ s, long NC, int H, int W, const float* __restrict__ gout,
                              const float* __restrict__ scale, float* __restrict__ gs) {
  const float k = 2.f * gout[0] * scale[1];
  const long total = NC * H * W;
  for (long i = (long)blockIdx.x * RT + threadIdx.x; i < total; i += (long)gridDim.x * RT) {
    int x = (int)(i % W);
    long t = i / W;
    int y = (int)(t % H);
    const float* p = s + i;
    float g = 0.f;
    if (y < H - 1 && x < W - 1) g -= (p[1] - p[0]) + (p[W] - p[0]);
    if (x >= 1 && y < H - 1) g += p[0] - p[-1];
    if (y >= 1 && x < W - 1) g += p[0] - p[-W];
    gs[i] = k * g;
  }
}

// S[n](k, m) = scale * (g[n][k][m] + g[n][m][k]) for k, m < C, zero padded, in the packed A layout
// (bmm backward of F F^T: dF = (gG + gG^T) F / (C H W); S is symmetric so [k][m] is the packed A)
__global__ void symmetrize_kernel(const float* __restrict__ g, float* __restrict__ S, int N, int C, int Kpad, int Mpad,
                                  float scale, int bsplit) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)N * Kpad * Mpad) return;
  int m = (int)(idx % Mpad);
  long t = idx / Mpad;
  int k = (int)(t % Kpad);
  long n = t / Kpad;
  float v = 0.f;
  if (k < C && m < C) {
    const float* gn = g + n * C * C;
    v = (gn[k * C + m] + gn[m * C + k]) * scale;
  }
  apack_store(S + n * (long)Kpad * Mpad * ((bsplit & 3) == 2 ? 3 : 2) / 2, k, m, Mpad, v, bsplit);  // bf16x6 packs are 1.5x
}

// ReLU backward: gx = gy * (y > 0)
__global__ void relu_bwd_kernel(const float* __restrict__ gy, const float* __restrict__ y, float* __restrict__ gx,
                                long n) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  gx[i] = y[i] > 0.f ? gy[i] : 0.f;
}

// gx = (g1 + g2) * (y > 0); g2 may be NULL
__global__ void relu_bwd_add_kernel(const float* __restrict__ g1, const float* __restrict__ g2,
                                    const float* __restrict__ y, float* __restrict__ gx, long n) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  gx[i] = y[i] > 0.f ? g1[i] + (g2 ? g2[i] : 0.f) : 0.f;
}

__global__ __launch_bounds__(256) void relu_bwd_add_vec_kernel(const float4* __restrict__ g1,
                                                               const float4* __restrict__ g2,
                                                               const float4* __restrict__ y, float4* __restrict__ gx,
                                                               long n4) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  float4 g = g1[i];
  if (g2) {
    const float4 h = g2[i];
    g = make_float4(g.x + h.x, g.y + h.y, g.z + h.z, g.w + h.w);
  }
  const float4 v = y[i];
  gx[i] = make_float4(v.x > 0.f ? g.x : 0.f, v.y > 0.f ? g.y : 0.f, v.z > 0.f ? g.z : 0.f, v.w > 0.f ? g.w : 0.f);
}

// four elements per thread (n % 4 == 0, 16-byte aligned): one float4 per stream
__global__ __launch_bounds__(256) void relu_bwd_vec_kernel(const float4* __restrict__ gy, const float4* __restrict__ y,
                                                           float4* __restrict__ gx, long n4) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const float4 g = gy[i], v = y[i];
  gx[i] = make_float4(v.x > 0.f ? g.x : 0.f, v.y > 0.f ? g.y : 0.f, v.z > 0.f ? g.z : 0.f, v.w > 0.f ? g.w : 0.f);
}

__constant__ float kMean[3] = {0.485f, 0.456f, 0.406f};
__constant__ float kStd[3] = {0.229f, 0.224f, 0.225f};

// out = (x/255 - mean[c]) / std[c]; inplace_scale: x <- x/255 (RC/utilities.py:105 `batch.div_(255.0)`)
__global__ void vgg_norm_kernel(float* __restrict__ x, float* __restrict__ out, long total, long HW,
                                int inplace_scale) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  int c = (int)((i / HW) % 3);
  float v = x[i] / 255.0f;
  if (inplace_scale) x[i] = v;
  out[i] = (v - kMean[c]) / kStd[c];
}

// gx = (gout / std[c]) / 255 (+ g_scaled / 255 when the mutated input also carries a gradient)
__global__ void vgg_norm_bwd_kernel(const float* __restrict__ gout, const float* __restrict__ gscaled,
                                    float* __restrict__ gx, long total, long HW) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  int c = (int)((i / HW) % 3);
  float g = gout[i] / kStd[c];
  if (gscaled) g += gscaled[i];
  gx[i] = g / 255.0f;
}

// ConvTanh backward from the saved tanh value t: gv = ((gy * 150) * (1 - t^2)) / 255
// prenorm: gy = (gy / std[c]) / 255 first (fused vgg_normalize backward)
__global__ void tanh_out_bwd_kernel(const float* __restrict__ gy, const float* __restrict__ t, float* __restrict__ gv,
                                    long total, long HW, int prenorm) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  float g = gy[i];
  if (prenorm) {
    int c = (int)((i / HW) % 3);
    g = (g / kStd[c]) / 255.0f;
  }
  float tt = t[i];
  gv[i] = ((g * 150.0f) * (1.0f - tt * tt)) / 255.0f;
}

// torch.optim.Adam (no weight decay / amsgrad / maximize): exp_avg.lerp_(g, 1-b1);
// exp_avg_sq = exp_avg_sq*b2 + (1-b2) g^2; p -= step_size * exp_avg / (sqrt(exp_avg_sq)/bc2_sqrt + eps)
__global__ void adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, long n, float b1, float b2, float eps, float step_size,
                            float bc2_sqrt, float gscale) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float gi = g[i] * gscale;
  float mi = m[i];
  mi = mi + (1.0f - b1) * (gi - mi);
  float vi = v[i] * b2 + (1.0f - b2) * gi * gi;
  m[i] = mi;
  v[i] = vi;
  float denom = sqrtf(vi) / bc2_sqrt + eps;
  p[i] = p[i] + (-step_size) * (mi / denom);
}

// ---- dynamic loss scale (the fp16 training policy; torch.cuda.amp.GradScaler's rule, device-side)
// state (8 floats): [0] scale S (the next backward's seed), [1] clean steps since the last change,
// [2] Adam step count (advanced on clean steps only), [3] found-inf of the last step, [4] step_size
// and [5] bc2_sqrt of the last clean step, [6] the last step's gradient factor world_scale / S,
// [7] skipped steps in total.  Nothing is read back to the host.
__device__ __forceinline__ bool nonfinite(float x) { return (__float_as_uint(x) & 0x7f800000u) == 0x7f800000u; }

// partial[b] = 1 if block b saw an Inf / NaN gradient (float4 grid-stride; the tail per element)
__global__ void grad_nonfinite_kernel(const float* __restrict__ g, long n, float* __restrict__ partial) {
  __shared__ int any;
  if (threadIdx.x == 0) any = 0;
  __syncthreads();
  bool bad = false;
  const long n4 = n >> 2;
  const float4* g4 = reinterpret_cast<const float4*>(g);
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const float4 v = g4[i];
    bad = bad || nonfinite(v.x) || nonfinite(v.y) || nonfinite(v.z) || nonfinite(v.w);
  }
  if (blockIdx.x == 0)
    for (long i = (n4 << 2) + threadIdx.x; i < n; i += blockDim.x) bad = bad || nonfinite(g[i]);
  if (__any(bad) && (threadIdx.x & 63) == 0) any = 1;  // benign same-value LDS write
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = (float)any;
}

// one block: fold the partial flags, decide skip / clean, advance the scale and Adam's step count
__global__ void loss_scale_update_kernel(const float* __restrict__ partial, int nb, float* __restrict__ state,
                                         float lr, float b1, float b2, float world_scale, int growth_interval,
                                         float growth, float backoff) {
  __shared__ int any;
  if (threadIdx.x == 0) any = 0;
  __syncthreads();
  bool bad = false;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) bad |= partial[i] != 0.f;
  if (__any(bad) && (threadIdx.x & 63) == 0) any = 1;
  __syncthreads();
  if (threadIdx.x != 0) return;
  const float S = state[0];
  state[6] = world_scale / S;
  if (any) {  // skip: parameters and moments untouched, scale backed off
    state[3] = 1.f;
    state[0] = S * backoff;
    state[1] = 0.f;
    state[7] += 1.f;
    return;
  }
  const float step = state[2] + 1.f;
  state[2] = step;
  state[3] = 0.f;
  // the same double-precision bias corrections as the host path (vst_adam)
  const double bc1 = 1.0 - pow((double)b1, (double)step), bc2 = 1.0 - pow((double)b2, (double)step);
  state[4] = (float)(lr / bc1);
  state[5] = (float)sqrt(bc2);
  float good = state[1] + 1.f;
  if (good >= (float)growth_interval) {
    state[0] = S * growth;
    good = 0.f;
  }
  state[1] = good;
}

// adam_kernel with its step size, bias correction and gradient factor read from the state; a
// skipped step returns before touching anything
__global__ void adam_scaled_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                   float* __restrict__ v, long n, float b1, float b2, float eps,
                                   const float* __restrict__ state) {
  if (state[3] != 0.f) return;
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float step_size = state[4], bc2_sqrt = state[5], gscale = state[6];
  float gi = g[i] * gscale;
  float mi = m[i];
  mi = mi + (1.0f - b1) * (gi - mi);
  float vi = v[i] * b2 + (1.0f - b2) * gi * gi;
  m[i] = mi;
  v[i] = vi;
  float denom = sqrtf(vi) / bc2_sqrt + eps;
  p[i] = p[i] + (-step_size) * (mi / denom);
}

// RTNSTV regularisation (RT/train.py:57-61): mean over (n, c, y < H-1, x < W-1) of
// sqrt(clamp(d1^2 + d2^2, 1e-8)), d1 = s[y][x+1] - s[y][x], d2 = s[y+1][x] - s[y][x]
__device__ __forceinline__ float tv_sqrt_term(const float* p, int W) {
  float d1 = p[1] - p[0], d2 = p[W] - p[0];
  float q = d1 * d1 + d2 * d2;
  return sqrtf(q < 1e-8f ? 1e-8f : q);
}

__global__ void tv_sqrt_kernel(const float* __restrict__ s, long NC, int H, int W, float* partial) {
  float acc = 0.f;
  const long total = NC * (H - 1) * (W - 1);
  for (long i = (long)blockIdx.x * RT + threadIdx.x; i < total; i += (long)gridDim.x * RT) {
    int x = (int)(i % (W - 1));
    long t = i / (W - 1);
    int y = (int)(t % (H - 1));
    long nc = t / (H - 1);
    acc += tv_sqrt_term(s + nc * H * W + (long)y * W + x, W);
  }
  block_partial(acc, 0.f, partial);
}

// d term(y,x) / d d1 = d1 / r (0 where the clamp is active, as torch's clamp backward), same for d2;
// gather form: a pixel is p[0] of its own term, p[1] of term (y, x-1) and p[W] of term (y-1, x)
__device__ __forceinline__ void tv_sqrt_grads(const float* p, int W, float& g1, float& g2) {
  float d1 = p[1] - p[0], d2 = p[W] - p[0];
  float q = d1 * d1 + d2 * d2;
  if (q < 1e-8f) {
    g1 = g2 = 0.f;
  } else {
    float inv = 1.f / (2.f * sqrtf(q));
    g1 = inv * (2.f * d1);
    g2 = inv * (2.f * d2);
  }
}

__global__ void tv_sqrt_bwd_kernel(const float* __restrict__ s, long NC, int H, int W, const float* __restrict__ gout,
                                   const float* __restrict__ scale, float* __restrict__ gs) {
  const float k = gout[0] * scale[1];
  const long total = NC * H * W;
  for (long i = (long)blockIdx.x * RT + threadIdx.x; i < total; i += (long)gridDim.x * RT) {
    int x = (int)(i % W);
    long t = i / W;
    int y = (int)(t % H);
    const float* p = s + i;
    float g = 0.f, g1, g2;
    if (y < H - 1 && x < W - 1) {
      tv_sqrt_grads(p, W, g1, g2);
      g -= g1 + g2;
    }
    if (x >= 1 && y < H - 1) {
      tv_sqrt_grads(p - 1, W, g1, g2);
      g += g1;
    }
    if (y >= 1 && x < W - 1) {
      tv_sqrt_grads(p - W, W, g1, g2);
      g += g2;
    }
    gs[i] = k * g;
  }
}

// RTNSTV output (RT/network.py:40-44 with Tanh, :93): y = (tanh(v) + 1) / 2 * 255, t saved
// image = 0: plain nn.Tanh (y = t)
__global__ void tanh_image_kernel(const float* __restrict__ v, float* __restrict__ y, float* __restrict__ t, long n,
                                  int image) {
  long i = (long)blockIdx.x * RT + threadIdx.x;
  if (i >= n) return;
  float th = tanhf(v[i]);
  t[i] = th;
  y[i] = image ? ((th + 1.0f) / 2.0f) * 255.0f : th;
}

__global__ void tanh_image_bwd_kernel(const float* __restrict__ gy, const float* __restrict__ t, float* __restrict__ gv,
                                      long n, int image) {
  long i = (long)blockIdx.x * RT + threadIdx.x;
  if (i >= n) return;
  float th = t[i];
  float g = image ? (gy[i] * 255.0f) / 2.0f : gy[i];
  gv[i] = g * (1.0f - th * th);
}

static int nblocks(long work) {
  long b = (work + RT - 1) / RT;
  return (int)(b < 1 ? 1 : (b > MAXB ? MAXB : b));
}

}  // namespace

// Gradient sums of a tensor with several consumers (vst_sum4): out = ((a + b) + c) + d, absent
// addends skipped (out may be one of the addends: each element is read before it is written); four elements per thread when every pointer is 16-byte aligned and n % 4 == 0.
template <int K>
__global__ __launch_bounds__(256) void sum4_vec_kernel(const float4* a, const float4* b,
                                                       const float4* c, const float4* d,
                                                       float4* out, long n4) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  float4 s = a[i];
  if (K > 1) {
    const float4 t = b[i];
    s = make_float4(s.x + t.x, s.y + t.y, s.z + t.z, s.w + t.w);
  }
  if (K > 2) {
    const float4 t = c[i];
    s = make_float4(s.x + t.x, s.y + t.y, s.z + t.z, s.w + t.w);
  }
  if (K > 3) {
    const float4 t = d[i];
    s = make_float4(s.x + t.x, s.y + t.y, s.z + t.z, s.w + t.w);
  }
  out[i] = s;
}

template <int K>
__global__ __launch_bounds__(256) void sum4_kernel(const float* a, const float* b,
                                                   const float* c, const float* d,
                                                   float* out, long n) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float s = a[i];
  if (K > 1) s += b[i];
  if (K > 2) s += c[i];
  if (K > 3) s += d[i];
  out[i] = s;
}

__global__ __launch_bounds__(256) void fill_vec_kernel(float4* __restrict__ x, long n4, float v) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < n4) x[i] = make_float4(v, v, v, v);
}

__global__ __launch_bounds__(256) void fill_kernel(float* __restrict__ x, long n, float v) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) x[i] = v;
}

template <int K>
static void launch_sum4(const float* a, const float* b, const float* c, const float* d, float* out, long n,
                        bool vec, hipStream_t s) {
  if (vec)
    sum4_vec_kernel<K><<<ceil_div(n / 4, 256), 256, 0, s>>>((const float4*)a, (const float4*)b, (const float4*)c,
                                                           (const float4*)d, (float4*)out, n / 4);
  else
    sum4_kernel<K><<<ceil_div(n, 256), 256, 0, s>>>(a, b, c, d, out, n);
}

extern "C" {

// workspace: >= 2*1024 floats; out: 3 floats (loss, weight/denom, count)
int vst_masked_sqdiff_fwd(int mode, const float* a, const float* b, const float* c, const float* d,
                          const float* mask, int N, int C, long HW, float weight, float* ws, float* out,
                          void* stream) {
  VST_CHECK_ARG(a && b && mask && ws && out && N > 0 && C > 0 && HW > 0 && (mode == 0 || mode == 1));
  VST_CHECK_ARG(mode == 0 || (c && d && C == 3));
  hipStream_t st = (hipStream_t)stream;
  int nb = nblocks((long)N * HW);
  if (mode == 0)
    masked_sqdiff_kernel<0><<<nb, RT, 0, st>>>(a, b, c, d, mask, N, C, HW, ws);
  else
    masked_sqdiff_kernel<1><<<nb, RT, 0, st>>>(a, b, c, d, mask, N, C, HW, ws);
  finish_kernel<<<1, RT, 0, st>>>(ws, nb, out, weight, 1.0, 1);
  return vst_launch_status();
}

int vst_masked_sqdiff_bwd(int mode, const float* a, const float* b, const float* c, const float* d,
                          const float* mask, int N, int C, long HW, const float* gout, const float* out, float* ga,
                          float* gb, void* stream) {
  VST_CHECK_ARG(a && b && mask && gout && out && N > 0 && C > 0 && HW > 0 && (mode == 0 || mode == 1));
  hipStream_t st = (hipStream_t)stream;
  int nb = nblocks((long)N * HW);
  if (mode == 0)
    masked_sqdiff_bwd_kernel<0><<<nb, RT, 0, st>>>(a, b, c, d, mask, N, C, HW, gout, out, ga, gb);
  else
    masked_sqdiff_bwd_kernel<1><<<nb, RT, 0, st>>>(a, b, c, d, mask, N, C, HW, gout, out, ga, gb);
  return vst_launch_status();
}

// loss = weight * mean((a - b[i % nb])^2) over n elements
int vst_mse_fwd(const float* a, const float* b, long n, long nb, float weight, float* ws, float* out, void* stream) {
  VST_CHECK_ARG(a && b && ws && out && n > 0 && nb > 0);
  hipStream_t st = (hipStream_t)stream;
  int g = nblocks(n);
  sqdiff_kernel<<<g, RT, 0, st>>>(a, b, n, nb, ws);
  finish_kernel<<<1, RT, 0, st>>>(ws, g, out, weight, (double)n, 0);
  return vst_launch_status();
}

int vst_mse_bwd(const float* a, const float* b, long n, long nb, const float* gout, const float* out, float* ga,
                float* gb, void* stream) {
  VST_CHECK_ARG(a && b && gout && out && n > 0 && nb > 0 && (!gb || nb == n));
  sqdiff_bwd_kernel<<<nblocks(n), RT, 0, (hipStream_t)stream>>>(a, b, n, nb, gout, out, ga, gb);
  return vst_launch_status();
}

// out = {weight * sum(x), weight, 0}
int vst_sum_scaled(const float* x, long n, float weight, float* ws, float* out, void* stream) {
  VST_CHECK_ARG(x && ws && out && n > 0);
  hipStream_t st = (hipStream_t)stream;
  int g = nblocks(n);
  vsum_kernel<<<g, RT, 0, st>>>(x, n, ws);
  finish_kernel<<<1, RT, 0, st>>>(ws, g, out, weight, 1.0, 0);
  return vst_launch_status();
}

int vst_tv_fwd(const float* s, long NC, int H, int W, float weight, float* ws, float* out, void* stream) {
  VST_CHECK_ARG(s && ws && out && NC > 0 && H > 1 && W > 1);
  hipStream_t st = (hipStream_t)stream;
  int g = nblocks(NC * (H - 1) * (W - 1));
  tv_kernel<<<g, RT, 0, st>>>(s, NC, H, W, ws);
  finish_kernel<<<1, RT, 0, st>>>(ws, g, out, weight, 1.0, 0);
  return vst_launch_status();
}

int vst_tv_bwd(const float* s, long NC, int H, int W, const float* gout, const float* out, float* gs, void* stream) {
  VST_CHECK_ARG(s && gout && out && gs && NC > 0 && H > 1 && W > 1);
  tv_bwd_kernel<<<nblocks(NC * H * W), RT, 0, (hipStream_t)stream>>>(s, NC, H, W, gout, out, gs);
  return vst_launch_status();
}

int vst_tv_sqrt_fwd(const float* s, long NC, int H, int W, float weight, float* ws, float* out, void* stream) {
  VST_CHECK_ARG(s && ws && out && NC > 0 && H > 1 && W > 1);
  hipStream_t st = (hipStream_t)stream;
  long terms = NC * (H - 1) * (W - 1);
  int g = nblocks(terms);
  tv_sqrt_kernel<<<g, RT, 0, st>>>(s, NC, H, W, ws);
  finish_kernel<<<1, RT, 0, st>>>(ws, g, out, weight, (double)terms, 0);
  return vst_launch_status();
}

int vst_tv_sqrt_bwd(const float* s, long NC, int H, int W, const float* gout, const float* out, float* gs,
                    void* stream) {
  VST_CHECK_ARG(s && gout && out && gs && NC > 0 && H > 1 && W > 1);
  tv_sqrt_bwd_kernel<<<nblocks(NC * H * W), RT, 0, (hipStream_t)stream>>>(s, NC, H, W, gout, out, gs);
  return vst_launch_status();
}

int vst_tanh_image_fwd(const float* v, float* y, float* t, long n, int image, void* stream) {
  VST_CHECK_ARG(v && y && t && n > 0);
  tanh_image_kernel<<<ceil_div(n, RT), RT, 0, (hipStream_t)stream>>>(v, y, t, n, image);
  return vst_launch_status();
}

int vst_tanh_image_bwd(const float* gy, const float* t, float* gv, long n, int image, void* stream) {
  VST_CHECK_ARG(gy && t && gv && n > 0);
  tanh_image_bwd_kernel<<<ceil_div(n, RT), RT, 0, (hipStream_t)stream>>>(gy, t, gv, n, image);
  return vst_launch_status();
}

int vst_symmetrize(const float* g, float* S, int N, int C, int Kpad, int Mpad, float scale, int mode, void* stream) {
  VST_CHECK_ARG(vst_mode_ok(mode));
  VST_CHECK_ARG(g && S && N > 0 && C > 0 && Kpad >= C && Mpad >= C);
  long total = (long)N * Kpad * Mpad;
  symmetrize_kernel<<<ceil_div(total, 256), 256, 0, (hipStream_t)stream>>>(g, S, N, C, Kpad, Mpad, scale,
                                                                           apack_split(mode));
  return vst_launch_status();
}

int vst_relu_bwd_add(const float* g1, const float* g2, const float* y, float* gx, long n, void* stream) {
  VST_CHECK_ARG(g1 && y && gx && n > 0);
  if ((n & 3) == 0 && (((uintptr_t)g1 | (uintptr_t)g2 | (uintptr_t)y | (uintptr_t)gx) & 15) == 0) {
    relu_bwd_add_vec_kernel<<<ceil_div(n / 4, 256), 256, 0, (hipStream_t)stream>>>(
        (const float4*)g1, (const float4*)g2, (const float4*)y, (float4*)gx, n / 4);
    return vst_launch_status();
  }
  relu_bwd_add_kernel<<<ceil_div(n, 256), 256, 0, (hipStream_t)stream>>>(g1, g2, y, gx, n);
  return vst_launch_status();
}

int vst_relu_bwd(const float* gy, const float* y, float* gx, long n, void* stream) {
  VST_CHECK_ARG(gy && y && gx && n > 0);
  if ((n & 3) == 0 && (((uintptr_t)gy | (uintptr_t)y | (uintptr_t)gx) & 15) == 0) {
    relu_bwd_vec_kernel<<<ceil_div(n / 4, 256), 256, 0, (hipStream_t)stream>>>((const float4*)gy, (const float4*)y,
                                                                               (float4*)gx, n / 4);
    return vst_launch_status();
  }
  relu_bwd_kernel<<<ceil_div(n, 256), 256, 0, (hipStream_t)stream>>>(gy, y, gx, n);
  return vst_launch_status();
}

int vst_vgg_normalize(float* x, float* out, int N, int HW, int inplace_scale, void* stream) {
  VST_CHECK_ARG(x && out && N > 0 && HW > 0);
  long total = (long)N * 3 * HW;
  vgg_norm_kernel<<<ceil_div(total, 256), 256, 0, (hipStream_t)stream>>>(x, out, total, HW, inplace_scale);
  return vst_launch_status();
}

int vst_vgg_normalize_bwd(const float* gout, const float* gscaled, float* gx, int N, int HW, void* stream) {
  VST_CHECK_ARG(gout && gx && N > 0 && HW > 0);
  long total = (long)N * 3 * HW;
  vgg_norm_bwd_kernel<<<ceil_div(total, 256), 256, 0, (hipStream_t)stream>>>(gout, gscaled, gx, total, HW);
  return vst_launch_status();
}

int vst_tanh_out_bwd(const float* gy, const float* t, float* gv, long total, long HW, int prenorm, void* stream) {
  VST_CHECK_ARG(gy && t && gv && total > 0 && HW > 0);
  tanh_out_bwd_kernel<<<ceil_div(total, 256), 256, 0, (hipStream_t)stream>>>(gy, t, gv, total, HW, prenorm);
  return vst_launch_status();
}

int vst_adam(float* p, const float* g, float* m, float* v, long n, float lr, float b1, float b2, float eps,
             long step, float gscale, void* stream) {
  VST_CHECK_ARG(p && g && m && v && n > 0 && step > 0);
  double bc1 = 1.0 - pow((double)b1, (double)step);
  double bc2 = 1.0 - pow((double)b2, (double)step);
  float step_size = (float)(lr / bc1);
  float bc2_sqrt = (float)sqrt(bc2);
  adam_kernel<<<ceil_div(n, 256), 256, 0, (hipStream_t)stream>>>(p, g, m, v, n, b1, b2, eps, step_size, bc2_sqrt,
                                                                 gscale);
  return vst_launch_status();
}

int vst_adam_loss_scaled(float* p, const float* g, float* m, float* v, long n, float lr, float b1, float b2,
                         float eps, float world_scale, float* state, float* ws, int growth_interval, float growth,
                         float backoff, void* stream) {
  VST_CHECK_ARG(p && g && m && v && state && ws && n > 0 && growth_interval > 0 && growth >= 1.f && backoff > 0.f &&
                backoff <= 1.f);
  VST_CHECK_ARG((((uintptr_t)g) & 15) == 0);
  hipStream_t st = (hipStream_t)stream;
  const long n4 = n >> 2;
  long nbl = (n4 + 255) / 256;
  nbl = nbl < 1 ? 1 : (nbl > VST_SCALER_WS ? VST_SCALER_WS : nbl);
  const int nb = (int)nbl;
  grad_nonfinite_kernel<<<nb, 256, 0, st>>>(g, n, ws);
  loss_scale_update_kernel<<<1, 256, 0, st>>>(ws, nb, state, lr, b1, b2, world_scale, growth_interval, growth, backoff);
  adam_scaled_kernel<<<ceil_div(n, 256), 256, 0, st>>>(p, g, m, v, n, b1, b2, eps, state);
  return vst_launch_status();
}

int vst_sum4(const float* a, const float* b, const float* c, const float* d, float* out, long n, void* stream) {
  // compact the present addends to the front, keeping their order
  const float* src[4] = {a, b, c, d};
  const float* p[4] = {nullptr, nullptr, nullptr, nullptr};
  int k = 0;
  uintptr_t align = (uintptr_t)out;
  for (int i = 0; i < 4; ++i)
    if (src[i]) {
      p[k++] = src[i];
      align |= (uintptr_t)src[i];
    }
  VST_CHECK_ARG(out && n > 0 && k > 0);
  const bool vec = (n & 3) == 0 && (align & 15) == 0;
  hipStream_t s = (hipStream_t)stream;
  switch (k) {
    case 1: launch_sum4<1>(p[0], p[1], p[2], p[3], out, n, vec, s); break;
    case 2: launch_sum4<2>(p[0], p[1], p[2], p[3], out, n, vec, s); break;
    case 3: launch_sum4<3>(p[0], p[1], p[2], p[3], out, n, vec, s); break;
    default: launch_sum4<4>(p[0], p[1], p[2], p[3], out, n, vec, s); break;
  }
  return vst_launch_status();
}

int vst_fill(float* x, long n, float value, void* stream) {
  VST_CHECK_ARG(x && n > 0);
  hipStream_t s = (hipStream_t)stream;
  if ((n & 3) == 0 && ((uintptr_t)x & 15) == 0)
    fill_vec_kernel<<<ceil_div(n / 4, 256), 256, 0, s>>>((float4*)x, n / 4, value);
  else
    fill_kernel<<<ceil_div(n, 256), 256, 0, s>>>(x, n, value);
  return vst_launch_status();
}

}  // extern "C"
