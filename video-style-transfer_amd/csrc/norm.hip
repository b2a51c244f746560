// InstanceNorm2d(affine=True, eps, biased variance, no running stats) forward/backward for gfx950,
// with ReLU and the residual add of RC/network.py:94-98, 129-133, 145-150 fused in.
// One workgroup per (n, c) plane; fp64 accumulation of the per-plane moments, plain (non-atomic)
// per-plane partials for the affine/bias gradients summed over n by a second tiny kernel
// (deterministic).
#include "vst_common.h"
#include "vst_hip.h"

namespace {

constexpr int NTN = 512;
// threads of the two-pass (large-plane) kernels: 1024 measured 217 vs 231 us (512) for the config-3
// 48 x 256 x 512 forward, equal for the backward (tools/norm_bench.py); capping blocks per CU so the
// second pass could re-read from the MALL did not help either
constexpr int IN_BIG_NT = 1024;

template <typename T, int NB = NTN>
__device__ __forceinline__ T block_sum(T v, T* sh) {
  // sh: NB/64 entries
  v = (sizeof(T) == 8) ? (T)wave_sum_d((double)v) : (T)wave_sum((float)v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) sh[w] = v;
  __syncthreads();
  T s = 0;
#pragma unroll
  for (int i = 0; i < NB / 64; ++i) s += sh[i];
  return s;
}

// The pre-activation (x - mean) * rstd * w + b with fixed rounding (no contraction left to the
// compiler): the backward recomputes it from x to get the ReLU mask instead of reading y, and must
// reproduce the forward's sign bit for bit.
__device__ __forceinline__ float in_affine(float x, float mean, float rstd, float w, float b) {
  return __fmaf_rn(__fmul_rn(__fsub_rn(x, mean), rstd), w, b);
}

// y = [relu]( (x - mean) * rstd * w + b ) [+ res]
// Two passes over the plane (it does not fit one block's registers); NT threads, two float4 loads in
// flight per thread per iteration.
template <int NT>
__global__ __launch_bounds__(NT) void in_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                    const float* __restrict__ b, const float* __restrict__ res,
                                                    float* __restrict__ y, float* __restrict__ stats, int C, int HW,
                                                    float eps, int relu) {
  __shared__ double sh[2][NT / 64];
  const long plane = blockIdx.x;
  const int c = (int)(plane % C);
  const float* xp = x + plane * HW;
  const bool v4 = (HW & 3) == 0;
  const int n4 = HW / 4;
  double s1 = 0.0, s2 = 0.0;
  if (v4) {
    const float4* x4 = reinterpret_cast<const float4*>(xp);
    auto acc = [&](const float4& v) {
      s1 += ((double)v.x + v.y) + ((double)v.z + v.w);
      s2 += ((double)v.x * v.x + (double)v.y * v.y) + ((double)v.z * v.z + (double)v.w * v.w);
    };
    int i = threadIdx.x;
    for (; i + NT < n4; i += 2 * NT) {
      const float4 v = x4[i], u = x4[i + NT];
      acc(v);
      acc(u);
    }
    if (i < n4) acc(x4[i]);
  } else {
    for (int i = threadIdx.x; i < HW; i += NT) {
      double v = xp[i];
      s1 += v;
      s2 += v * v;
    }
  }
  s1 = block_sum<double, NT>(s1, sh[0]);
  s2 = block_sum<double, NT>(s2, sh[1]);
  const double mean_d = s1 / HW;
  double var_d = s2 / HW - mean_d * mean_d;
  var_d = var_d < 0.0 ? 0.0 : var_d;
  const float mean = (float)mean_d;
  const float rstd = (float)(1.0 / sqrt(var_d + (double)eps));
  if (threadIdx.x == 0) {
    stats[2 * plane] = mean;
    stats[2 * plane + 1] = rstd;
  }
  const float wc = w[c], bc = b[c];
  float* yp = y + plane * HW;
  const float* rp = res ? res + plane * HW : nullptr;
  if (v4) {
    const float4* x4 = reinterpret_cast<const float4*>(xp);
    const float4* r4 = reinterpret_cast<const float4*>(rp);
    float4* y4 = reinterpret_cast<float4*>(yp);
    auto out = [&](const float4& v, int i) {
      float o[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        o[k] = in_affine(o[k], mean, rstd, wc, bc);
        if (relu) o[k] = fmaxf(o[k], 0.f);
      }
      if (rp) {
        const float4 r = r4[i];
        o[0] += r.x;
        o[1] += r.y;
        o[2] += r.z;
        o[3] += r.w;
      }
      y4[i] = make_float4(o[0], o[1], o[2], o[3]);
    };
    int i = threadIdx.x;
    for (; i + NT < n4; i += 2 * NT) {
      const float4 v = x4[i], u = x4[i + NT];
      out(v, i);
      out(u, i + NT);
    }
    if (i < n4) out(x4[i], i);
  } else {
    for (int i = threadIdx.x; i < HW; i += NT) {
      float o = in_affine(xp[i], mean, rstd, wc, bc);
      if (relu) o = fmaxf(o, 0.f);
      if (rp) o += rp[i];
      yp[i] = o;
    }
  }
}

// g = gy * (relu ? y > 0 : 1); xhat = (x-mean)*rstd
// gx = rstd*w*(g - mean(g) - xhat*mean(g*xhat));  partial[plane] = {sum g*xhat, sum g, sum gx}
// y == nullptr with relu: the mask is in_affine(x, ...) > 0, one tensor less to read (y > 0 is the
// mask only when no residual was added after the ReLU).
// Two passes, NT threads, two float4 positions in flight per thread (as in_fwd_kernel).
template <int NT>
__global__ __launch_bounds__(NT) void in_bwd_kernel(const float* __restrict__ gy, const float* __restrict__ x,
                                                    const float* __restrict__ y, const float* __restrict__ bias,
                                                    const float* __restrict__ stats,
                                                    const float* __restrict__ w, float* __restrict__ gx,
                                                    float* __restrict__ partial, int C, int HW, int relu) {
  __shared__ double sh[3][NT / 64];
  const long plane = blockIdx.x;
  const int c = (int)(plane % C);
  const float* gp = gy + plane * HW;
  const float* xp = x + plane * HW;
  const float* yp = y + plane * HW;
  const float mean = stats[2 * plane], rstd = stats[2 * plane + 1];
  const bool v4 = (HW & 3) == 0;
  const int n4 = HW / 4;
  const bool ymask = relu && y, amask = relu && !y;
  const float wc = w[c], bc = amask ? bias[c] : 0.f;
  const float4* g4 = reinterpret_cast<const float4*>(gp);
  const float4* x4 = reinterpret_cast<const float4*>(xp);
  const float4* y4 = reinterpret_cast<const float4*>(yp);
  auto mask4 = [&](float4 g, const float4& xv, int i) -> float4 {  // masked gradient, 4 consecutive elements
    if (ymask) {
      const float4 yv = y4[i];
      g.x = yv.x > 0.f ? g.x : 0.f;
      g.y = yv.y > 0.f ? g.y : 0.f;
      g.z = yv.z > 0.f ? g.z : 0.f;
      g.w = yv.w > 0.f ? g.w : 0.f;
    } else if (amask) {
      g.x = in_affine(xv.x, mean, rstd, wc, bc) > 0.f ? g.x : 0.f;
      g.y = in_affine(xv.y, mean, rstd, wc, bc) > 0.f ? g.y : 0.f;
      g.z = in_affine(xv.z, mean, rstd, wc, bc) > 0.f ? g.z : 0.f;
      g.w = in_affine(xv.w, mean, rstd, wc, bc) > 0.f ? g.w : 0.f;
    }
    return g;
  };
  auto mask1 = [&](int i, float g, float xv) -> float {
    if (ymask) return yp[i] > 0.f ? g : 0.f;
    if (amask) return in_affine(xv, mean, rstd, wc, bc) > 0.f ? g : 0.f;
    return g;
  };
  double sg = 0.0, sgx = 0.0;
  if (v4) {
    auto acc = [&](const float4& g, const float4& xv) {
      sg += ((double)g.x + g.y) + ((double)g.z + g.w);
      sgx += ((double)g.x * ((xv.x - mean) * rstd) + (double)g.y * ((xv.y - mean) * rstd)) +
             ((double)g.z * ((xv.z - mean) * rstd) + (double)g.w * ((xv.w - mean) * rstd));
    };
    int i = threadIdx.x;
    for (; i + NT < n4; i += 2 * NT) {
      const float4 xa = x4[i], xb = x4[i + NT], ga = g4[i], gb = g4[i + NT];
      acc(mask4(ga, xa, i), xa);
      acc(mask4(gb, xb, i + NT), xb);
    }
    if (i < n4) {
      const float4 xa = x4[i];
      acc(mask4(g4[i], xa, i), xa);
    }
  } else {
    for (int i = threadIdx.x; i < HW; i += NT) {
      const float g = mask1(i, gp[i], xp[i]);
      float xh = (xp[i] - mean) * rstd;
      sg += g;
      sgx += (double)g * xh;
    }
  }
  sg = block_sum<double, NT>(sg, sh[0]);
  sgx = block_sum<double, NT>(sgx, sh[1]);
  const float mg = (float)(sg / HW), mgx = (float)(sgx / HW);
  const float k = rstd * wc;
  float* gxp = gx + plane * HW;
  double sgo = 0.0;
  if (v4) {
    float4* o4 = reinterpret_cast<float4*>(gxp);
    auto out = [&](const float4& g, const float4& xv, int i) {
      const float4 o = make_float4(k * (g.x - mg - (xv.x - mean) * rstd * mgx), k * (g.y - mg - (xv.y - mean) * rstd * mgx),
                                   k * (g.z - mg - (xv.z - mean) * rstd * mgx), k * (g.w - mg - (xv.w - mean) * rstd * mgx));
      o4[i] = o;
      sgo += ((double)o.x + o.y) + ((double)o.z + o.w);
    };
    int i = threadIdx.x;
    for (; i + NT < n4; i += 2 * NT) {
      const float4 xa = x4[i], xb = x4[i + NT], ga = g4[i], gb = g4[i + NT];
      out(mask4(ga, xa, i), xa, i);
      out(mask4(gb, xb, i + NT), xb, i + NT);
    }
    if (i < n4) {
      const float4 xa = x4[i];
      out(mask4(g4[i], xa, i), xa, i);
    }
  } else {
    for (int i = threadIdx.x; i < HW; i += NT) {
      const float g = mask1(i, gp[i], xp[i]);
      float xh = (xp[i] - mean) * rstd;
      float o = k * (g - mg - xh * mgx);
      gxp[i] = o;
      sgo += o;
    }
  }
  sgo = block_sum<double, NT>(sgo, sh[2]);
  if (threadIdx.x == 0) {
    partial[3 * plane] = (float)sgx;
    partial[3 * plane + 1] = (float)sg;
    partial[3 * plane + 2] = (float)sgo;
  }
}

// Register-resident variants for planes of HW <= NT*4*V4 (HW % 4 == 0): every element is read
// from HBM once (the two-pass kernels above read the plane twice).  Backward only for <= 8192
// (a 1024-thread, 32768-element backward spills).
template <int NT, int V4>
__global__ __launch_bounds__(NT) void in_fwd_reg_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                         const float* __restrict__ b, const float* __restrict__ res,
                                                         float* __restrict__ y, float* __restrict__ stats, int C,
                                                         int HW, float eps, int relu) {
  __shared__ double sh[2][NT / 64];
  const long plane = blockIdx.x;
  const int c = (int)(plane % C);
  const int n4 = HW >> 2;
  const float4* x4 = reinterpret_cast<const float4*>(x + plane * HW);
  float4 v[V4];
  double s1 = 0.0, s2 = 0.0;
#pragma unroll
  for (int j = 0; j < V4; ++j) {
    const int i = threadIdx.x + j * NT;
    v[j] = i < n4 ? x4[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    s1 += (double)v[j].x + (double)v[j].y + (double)v[j].z + (double)v[j].w;
    s2 += (double)v[j].x * v[j].x + (double)v[j].y * v[j].y + (double)v[j].z * v[j].z + (double)v[j].w * v[j].w;
  }
  s1 = block_sum<double, NT>(s1, sh[0]);
  s2 = block_sum<double, NT>(s2, sh[1]);
  const double mean_d = s1 / HW;
  double var_d = s2 / HW - mean_d * mean_d;
  var_d = var_d < 0.0 ? 0.0 : var_d;
  const float mean = (float)mean_d;
  const float rstd = (float)(1.0 / sqrt(var_d + (double)eps));
  if (threadIdx.x == 0) {
    stats[2 * plane] = mean;
    stats[2 * plane + 1] = rstd;
  }
  const float wc = w[c], bc = b[c];
  float4* y4 = reinterpret_cast<float4*>(y + plane * HW);
  const float4* r4 = res ? reinterpret_cast<const float4*>(res + plane * HW) : nullptr;
#pragma unroll
  for (int j = 0; j < V4; ++j) {
    const int i = threadIdx.x + j * NT;
    if (i >= n4) break;
    float o0 = in_affine(v[j].x, mean, rstd, wc, bc), o1 = in_affine(v[j].y, mean, rstd, wc, bc);
    float o2 = in_affine(v[j].z, mean, rstd, wc, bc), o3 = in_affine(v[j].w, mean, rstd, wc, bc);
    if (relu) {
      o0 = fmaxf(o0, 0.f);
      o1 = fmaxf(o1, 0.f);
      o2 = fmaxf(o2, 0.f);
      o3 = fmaxf(o3, 0.f);
    }
    if (r4) {
      const float4 r = r4[i];
      o0 += r.x;
      o1 += r.y;
      o2 += r.z;
      o3 += r.w;
    }
    y4[i] = make_float4(o0, o1, o2, o3);
  }
}

template <int NT, int V4, bool KEEPX>
__global__ __launch_bounds__(NT) void in_bwd_reg_kernel(const float* __restrict__ gy, const float* __restrict__ x,
                                                         const float* __restrict__ y, const float* __restrict__ bias,
                                                         const float* __restrict__ stats,
                                                         const float* __restrict__ w, float* __restrict__ gx,
                                                         float* __restrict__ partial, int C, int HW, int relu) {
  __shared__ double sh[3][NT / 64];
  const long plane = blockIdx.x;
  const int c = (int)(plane % C);
  const int n4 = HW >> 2;
  const float4* g4 = reinterpret_cast<const float4*>(gy + plane * HW);
  const float4* x4 = reinterpret_cast<const float4*>(x + plane * HW);
  const float4* y4 = reinterpret_cast<const float4*>(y + plane * HW);
  const float mean = stats[2 * plane], rstd = stats[2 * plane + 1];
  const bool ymask = relu && y, amask = relu && !y;
  const float wc = w[c], bc = amask ? bias[c] : 0.f;
  float4 g[V4], xh[KEEPX ? V4 : 1];
  double sg = 0.0, sgx = 0.0;
#pragma unroll
  for (int j = 0; j < V4; ++j) {
    const int i = threadIdx.x + j * NT;
    float4 gv = make_float4(0.f, 0.f, 0.f, 0.f), xv = gv;
    if (i < n4) {
      gv = g4[i];
      xv = x4[i];
      if (ymask) {
        const float4 yv = y4[i];
        gv.x = yv.x > 0.f ? gv.x : 0.f;
        gv.y = yv.y > 0.f ? gv.y : 0.f;
        gv.z = yv.z > 0.f ? gv.z : 0.f;
        gv.w = yv.w > 0.f ? gv.w : 0.f;
      } else if (amask) {
        gv.x = in_affine(xv.x, mean, rstd, wc, bc) > 0.f ? gv.x : 0.f;
        gv.y = in_affine(xv.y, mean, rstd, wc, bc) > 0.f ? gv.y : 0.f;
        gv.z = in_affine(xv.z, mean, rstd, wc, bc) > 0.f ? gv.z : 0.f;
        gv.w = in_affine(xv.w, mean, rstd, wc, bc) > 0.f ? gv.w : 0.f;
      }
      xv = make_float4((xv.x - mean) * rstd, (xv.y - mean) * rstd, (xv.z - mean) * rstd, (xv.w - mean) * rstd);
    }
    g[j] = gv;
    if (KEEPX) xh[KEEPX ? j : 0] = xv;
    sg += (double)gv.x + (double)gv.y + (double)gv.z + (double)gv.w;
    sgx += (double)gv.x * xv.x + (double)gv.y * xv.y + (double)gv.z * xv.z + (double)gv.w * xv.w;
  }
  sg = block_sum<double, NT>(sg, sh[0]);
  sgx = block_sum<double, NT>(sgx, sh[1]);
  const float mg = (float)(sg / HW), mgx = (float)(sgx / HW);
  const float k = rstd * wc;
  float4* o4 = reinterpret_cast<float4*>(gx + plane * HW);
  double sgo = 0.0;
#pragma unroll
  for (int j = 0; j < V4; ++j) {
    const int i = threadIdx.x + j * NT;
    if (i >= n4) break;
    float4 h;
    if (KEEPX) {
      h = xh[KEEPX ? j : 0];
    } else {
      const float4 xv = x4[i];
      h = make_float4((xv.x - mean) * rstd, (xv.y - mean) * rstd, (xv.z - mean) * rstd, (xv.w - mean) * rstd);
    }
    const float4 o = make_float4(k * (g[j].x - mg - h.x * mgx), k * (g[j].y - mg - h.y * mgx),
                                 k * (g[j].z - mg - h.z * mgx), k * (g[j].w - mg - h.w * mgx));
    o4[i] = o;
    sgo += (double)o.x + (double)o.y + (double)o.z + (double)o.w;
  }
  sgo = block_sum<double, NT>(sgo, sh[2]);
  if (threadIdx.x == 0) {
    partial[3 * plane] = (float)sgx;
    partial[3 * plane + 1] = (float)sg;
    partial[3 * plane + 2] = (float)sgo;
  }
}

// One-pass backward for planes of 8192 < HW <= 32768 (HW % 4 == 0): the masked gradient stays in
// registers and the plane of x in LDS (128 KB) between the two reductions, so gy and x are read from
// HBM once -- 3 plane-sized transfers instead of in_bwd_kernel's 5 (the register-only form of this
// size spills: in_bwd_reg_kernel<1024, 8, *> needs > 128 VGPRs).  Same element arithmetic as
// in_bwd_reg_kernel; the plane sums add fp32 sums of four in fp64.
constexpr int LDS_NT = 1024, LDS_V4 = 8;
__global__ __launch_bounds__(LDS_NT) void in_bwd_lds_kernel(const float* __restrict__ gy, const float* __restrict__ x,
                                                            const float* __restrict__ y, const float* __restrict__ bias,
                                                            const float* __restrict__ stats,
                                                            const float* __restrict__ w, float* __restrict__ gx,
                                                            float* __restrict__ partial, int C, int HW, int relu) {
  __shared__ float4 xs[LDS_V4 * LDS_NT];
  __shared__ double sh[3][LDS_NT / 64];
  const long plane = blockIdx.x;
  const int c = (int)(plane % C);
  const int n4 = HW >> 2;
  const float4* g4 = reinterpret_cast<const float4*>(gy + plane * HW);
  const float4* x4 = reinterpret_cast<const float4*>(x + plane * HW);
  const float4* y4 = reinterpret_cast<const float4*>(y + plane * HW);
  const float mean = stats[2 * plane], rstd = stats[2 * plane + 1];
  const bool ymask = relu && y, amask = relu && !y;
  const float wc = w[c], bc = amask ? bias[c] : 0.f;
  float4 g[LDS_V4];
  double sg = 0.0, sgx = 0.0;
#pragma unroll
  for (int j = 0; j < LDS_V4; ++j) {
    const int i = threadIdx.x + j * LDS_NT;
    float4 gv = make_float4(0.f, 0.f, 0.f, 0.f), xv = gv;
    if (i < n4) {
      gv = g4[i];
      xv = x4[i];
      if (ymask) {
        const float4 yv = y4[i];
        gv.x = yv.x > 0.f ? gv.x : 0.f;
        gv.y = yv.y > 0.f ? gv.y : 0.f;
        gv.z = yv.z > 0.f ? gv.z : 0.f;
        gv.w = yv.w > 0.f ? gv.w : 0.f;
      } else if (amask) {
        gv.x = in_affine(xv.x, mean, rstd, wc, bc) > 0.f ? gv.x : 0.f;
        gv.y = in_affine(xv.y, mean, rstd, wc, bc) > 0.f ? gv.y : 0.f;
        gv.z = in_affine(xv.z, mean, rstd, wc, bc) > 0.f ? gv.z : 0.f;
        gv.w = in_affine(xv.w, mean, rstd, wc, bc) > 0.f ? gv.w : 0.f;
      }
      xs[j * LDS_NT + threadIdx.x] = xv;
      xv = make_float4((xv.x - mean) * rstd, (xv.y - mean) * rstd, (xv.z - mean) * rstd, (xv.w - mean) * rstd);
    }
    g[j] = gv;
    // fp32 sums of 4, accumulated in fp64 (fp64 per element needs > 128 VGPRs here)
    sg += (double)((gv.x + gv.y) + (gv.z + gv.w));
    sgx += (double)((gv.x * xv.x + gv.y * xv.y) + (gv.z * xv.z + gv.w * xv.w));
  }
  sg = block_sum<double, LDS_NT>(sg, sh[0]);
  sgx = block_sum<double, LDS_NT>(sgx, sh[1]);
  const float mg = (float)(sg / HW), mgx = (float)(sgx / HW);
  const float k = rstd * wc;
  float4* o4 = reinterpret_cast<float4*>(gx + plane * HW);
  double sgo = 0.0;
#pragma unroll
  for (int j = 0; j < LDS_V4; ++j) {
    const int i = threadIdx.x + j * LDS_NT;
    if (i >= n4) break;
    const float4 xv = xs[j * LDS_NT + threadIdx.x];  // written by this thread: no barrier needed
    const float4 h = make_float4((xv.x - mean) * rstd, (xv.y - mean) * rstd, (xv.z - mean) * rstd, (xv.w - mean) * rstd);
    const float4 o = make_float4(k * (g[j].x - mg - h.x * mgx), k * (g[j].y - mg - h.y * mgx),
                                 k * (g[j].z - mg - h.z * mgx), k * (g[j].w - mg - h.w * mgx));
    o4[i] = o;
    sgo += (double)((o.x + o.y) + (o.z + o.w));
  }
  sgo = block_sum<double, LDS_NT>(sgo, sh[2]);
  if (threadIdx.x == 0) {
    partial[3 * plane] = (float)sgx;
    partial[3 * plane + 1] = (float)sg;
    partial[3 * plane + 2] = (float)sgo;
  }
}

// dst_k[c] (+)= sum_n partial[(n*C + c)*NP + k] for the non-null dst_k
__global__ void sum_over_n_kernel(const float* __restrict__ partial, int N, int C, int NP, float* d0, float* d1,
                                  float* d2, int accumulate) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float* dst[3] = {d0, d1, d2};
  for (int k = 0; k < NP && k < 3; ++k) {
    if (!dst[k]) continue;
    double s = 0.0;
    for (int n = 0; n < N; ++n) s += partial[((long)n * C + c) * NP + k];
    dst[k][c] = accumulate ? dst[k][c] + (float)s : (float)s;
  }
}

// per-plane sums: out[plane] = sum_i x[plane][i]
__global__ __launch_bounds__(NTN) void plane_sum_kernel(const float* __restrict__ x, float* __restrict__ out, int HW) {
  __shared__ double sh[NTN / 64];
  const long plane = blockIdx.x;
  const float* xp = x + plane * HW;
  double s = 0.0;
  for (int i = threadIdx.x; i < HW; i += NTN) s += xp[i];
  s = block_sum(s, sh);
  if (threadIdx.x == 0) out[plane] = (float)s;
}

// plane_sum_kernel over float4 (HW % 4 == 0, 16-byte aligned x): two float4 loads in flight per
// thread per iteration instead of one scalar (the config-5 bias gradients sum 512x1024 planes)
__global__ __launch_bounds__(NTN) void plane_sum_vec_kernel(const float4* __restrict__ x, float* __restrict__ out,
                                                            int HW4) {
  __shared__ double sh[NTN / 64];
  const float4* xp = x + (long)blockIdx.x * HW4;
  double s = 0.0;
  int i = threadIdx.x;
#pragma unroll 4
  for (; i + NTN < HW4; i += 2 * NTN) {
    const float4 a = xp[i], b = xp[i + NTN];
    s += (((double)a.x + a.y) + ((double)a.z + a.w)) + (((double)b.x + b.y) + ((double)b.z + b.w));
  }
  if (i < HW4) {
    const float4 a = xp[i];
    s += ((double)a.x + a.y) + ((double)a.z + a.w);
  }
  s = block_sum(s, sh);
  if (threadIdx.x == 0) out[blockIdx.x] = (float)s;
}

}  // namespace

extern "C" {

int vst_instnorm_fwd(const float* x, const float* w, const float* b, const float* res, float* y, float* stats, int N,
                     int C, int HW, float eps, int relu, void* stream) {
  VST_CHECK_ARG(x && w && b && y && stats && N > 0 && C > 0 && HW > 0);
  hipStream_t st = (hipStream_t)stream;
  if ((HW & 3) == 0 && HW <= NTN * 4 * 4)
    in_fwd_reg_kernel<512, 4><<<N * C, 512, 0, st>>>(x, w, b, res, y, stats, C, HW, eps, relu);
  else if ((HW & 3) == 0 && HW <= 1024 * 4 * 8)
    in_fwd_reg_kernel<1024, 8><<<N * C, 1024, 0, st>>>(x, w, b, res, y, stats, C, HW, eps, relu);
  else
    in_fwd_kernel<IN_BIG_NT><<<N * C, IN_BIG_NT, 0, st>>>(x, w, b, res, y, stats, C, HW, eps, relu);
  return vst_launch_status();
}

// partial: workspace of N*C*3 floats. gw/gb: [C] weight/bias grads (accumulated if accumulate);
// gbias_prev: optional [C] grad of the bias of the conv feeding this norm (sum of gx).
// relu: the mask comes from y when y is given, else from the recomputed pre-activation with b
// (valid when the forward had no residual add).
int vst_instnorm_bwd(const float* gy, const float* x, const float* y, const float* b, const float* stats,
                     const float* w, float* gx, float* gw, float* gb, float* gbias_prev, float* partial, int N, int C,
                     int HW, int relu, int accumulate, void* stream) {
  VST_CHECK_ARG(gy && x && stats && w && gx && partial && N > 0 && C > 0 && HW > 0);
  VST_CHECK_ARG(!relu || y || b);
  hipStream_t st = (hipStream_t)stream;
  if ((HW & 3) == 0 && HW <= NTN * 4 * 4)
    in_bwd_reg_kernel<512, 4, true><<<N * C, 512, 0, st>>>(gy, x, y, b, stats, w, gx, partial, C, HW, relu);
  else if ((HW & 3) == 0 && HW <= LDS_NT * 4 * LDS_V4)
    in_bwd_lds_kernel<<<N * C, LDS_NT, 0, st>>>(gy, x, y, b, stats, w, gx, partial, C, HW, relu);
  else
    in_bwd_kernel<IN_BIG_NT><<<N * C, IN_BIG_NT, 0, st>>>(gy, x, y, b, stats, w, gx, partial, C, HW, relu);
  sum_over_n_kernel<<<ceil_div(C, 256), 256, 0, st>>>(partial, N, C, 3, gw, gb, gbias_prev, accumulate);
  return vst_launch_status();
}

// out[c] (+)= sum_{n,i} x[n][c][i]   (conv bias gradient); partial: N*C floats workspace
int vst_channel_sum(const float* x, float* out, float* partial, int N, int C, int HW, int accumulate, void* stream) {
  VST_CHECK_ARG(x && out && partial && N > 0 && C > 0 && HW > 0);
  hipStream_t st = (hipStream_t)stream;
  if ((HW & 3) == 0 && ((uintptr_t)x & 15) == 0)
    plane_sum_vec_kernel<<<N * C, NTN, 0, st>>>(reinterpret_cast<const float4*>(x), partial, HW / 4);
  else
    plane_sum_kernel<<<N * C, NTN, 0, st>>>(x, partial, HW);
  sum_over_n_kernel<<<ceil_div(C, 256), 256, 0, st>>>(partial, N, C, 1, out, nullptr, nullptr, accumulate);
  return vst_launch_status();
}

}  // extern "C"
