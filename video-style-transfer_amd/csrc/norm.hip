// InstanceNorm2d(affine=True, eps, biased variance, no running stats) forward/backward for gfx950,
// with ReLU and the residual add of RC/network.py:94-98, 129-133, 145-150 fused in.
// One workgroup per (n, c) plane; fp64 accumulation of the per-plane moments, plain (non-atomic)
// per-plane partials for the affine/bias gradients summed over n by a second tiny kernel
// (deterministic).
#include "vst_common.h"
#include "vst_hip.h"

namespace {

constexpr int NTN = 512;

template <typename T>
__device__ __forceinline__ T block_sum(T v, T* sh) {
  // sh: NTN/64 entries
  v = (sizeof(T) == 8) ? (T)wave_sum_d((double)v) : (T)wave_sum((float)v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) sh[w] = v;
  __syncthreads();
  T s = 0;
#pragma unroll
  for (int i = 0; i < NTN / 64; ++i) s += sh[i];
  return s;
}

// y = [relu]( (x - mean) * rstd * w + b ) [+ res]
__global__ __launch_bounds__(NTN) void in_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                     const float* __restrict__ b, const float* __restrict__ res,
                                                     float* __restrict__ y, float* __restrict__ stats, int C, int HW,
                                                     float eps, int relu) {
  __shared__ double sh[2][NTN / 64];
  const long plane = blockIdx.x;
  const int c = (int)(plane % C);
  const float* xp = x + plane * HW;
  double s1 = 0.0, s2 = 0.0;
  if ((HW & 3) == 0) {
    const float4* x4 = reinterpret_cast<const float4*>(xp);
    for (int i = threadIdx.x; i < HW / 4; i += NTN) {
      float4 v = x4[i];
      s1 += (double)v.x + (double)v.y + (double)v.z + (double)v.w;
      s2 += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
    }
  } else {
    for (int i = threadIdx.x; i < HW; i += NTN) {
      double v = xp[i];
      s1 += v;
      s2 += v * v;
    }
  }
  s1 = block_sum(s1, sh[0]);
  s2 = block_sum(s2, sh[1]);
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
  if ((HW & 3) == 0) {
    const float4* x4 = reinterpret_cast<const float4*>(xp);
    float4* y4 = reinterpret_cast<float4*>(yp);
    for (int i = threadIdx.x; i < HW / 4; i += NTN) {
      float4 v = x4[i];
      float o[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        o[k] = (o[k] - mean) * rstd * wc + bc;
        if (relu) o[k] = fmaxf(o[k], 0.f);
      }
      if (rp) {
        float4 r = reinterpret_cast<const float4*>(rp)[i];
        o[0] += r.x;
        o[1] += r.y;
        o[2] += r.z;
        o[3] += r.w;
      }
      y4[i] = make_float4(o[0], o[1], o[2], o[3]);
    }
  } else {
    for (int i = threadIdx.x; i < HW; i += NTN) {
      float o = (xp[i] - mean) * rstd * wc + bc;
      if (relu) o = fmaxf(o, 0.f);
      if (rp) o += rp[i];
      yp[i] = o;
    }
  }
}

// g = gy * (relu ? y > 0 : 1); xhat = (x-mean)*rstd
// gx = rstd*w*(g - mean(g) - xhat*mean(g*xhat));  partial[plane] = {sum g*xhat, sum g, sum gx}
__global__ __launch_bounds__(NTN) void in_bwd_kernel(const float* __restrict__ gy, const float* __restrict__ x,
                                                     const float* __restrict__ y, const float* __restrict__ stats,
                                                     const float* __restrict__ w, float* __restrict__ gx,
                                                     float* __restrict__ partial, int C, int HW, int relu) {
  __shared__ double sh[3][NTN / 64];
  const long plane = blockIdx.x;
  const int c = (int)(plane % C);
  const float* gp = gy + plane * HW;
  const float* xp = x + plane * HW;
  const float* yp = y + plane * HW;
  const float mean = stats[2 * plane], rstd = stats[2 * plane + 1];
  double sg = 0.0, sgx = 0.0;
  for (int i = threadIdx.x; i < HW; i += NTN) {
    float g = gp[i];
    if (relu && !(yp[i] > 0.f)) g = 0.f;
    float xh = (xp[i] - mean) * rstd;
    sg += g;
    sgx += (double)g * xh;
  }
  sg = block_sum(sg, sh[0]);
  sgx = block_sum(sgx, sh[1]);
  const float mg = (float)(sg / HW), mgx = (float)(sgx / HW);
  const float k = rstd * w[c];
  float* gxp = gx + plane * HW;
  double sgo = 0.0;
  for (int i = threadIdx.x; i < HW; i += NTN) {
    float g = gp[i];
    if (relu && !(yp[i] > 0.f)) g = 0.f;
    float xh = (xp[i] - mean) * rstd;
    float o = k * (g - mg - xh * mgx);
    gxp[i] = o;
    sgo += o;
  }
  sgo = block_sum(sgo, sh[2]);
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

}  // namespace

extern "C" {

int vst_instnorm_fwd(const float* x, const float* w, const float* b, const float* res, float* y, float* stats, int N,
                     int C, int HW, float eps, int relu, void* stream) {
  VST_CHECK_ARG(x && w && b && y && stats && N > 0 && C > 0 && HW > 0);
  in_fwd_kernel<<<N * C, NTN, 0, (hipStream_t)stream>>>(x, w, b, res, y, stats, C, HW, eps, relu);
  return vst_launch_status();
}

// partial: workspace of N*C*3 floats. gw/gb: [C] weight/bias grads (accumulated if accumulate);
// gbias_prev: optional [C] grad of the bias of the conv feeding this norm (sum of gx).
int vst_instnorm_bwd(const float* gy, const float* x, const float* y, const float* stats, const float* w, float* gx,
                     float* gw, float* gb, float* gbias_prev, float* partial, int N, int C, int HW, int relu,
                     int accumulate, void* stream) {
  VST_CHECK_ARG(gy && x && stats && w && gx && partial && N > 0 && C > 0 && HW > 0);
  VST_CHECK_ARG(!relu || y);
  hipStream_t st = (hipStream_t)stream;
  in_bwd_kernel<<<N * C, NTN, 0, st>>>(gy, x, y, stats, w, gx, partial, C, HW, relu);
  sum_over_n_kernel<<<ceil_div(C, 256), 256, 0, st>>>(partial, N, C, 3, gw, gb, gbias_prev, accumulate);
  return vst_launch_status();
}

// out[c] (+)= sum_{n,i} x[n][c][i]   (conv bias gradient); partial: N*C floats workspace
int vst_channel_sum(const float* x, float* out, float* partial, int N, int C, int HW, int accumulate, void* stream) {
  VST_CHECK_ARG(x && out && partial && N > 0 && C > 0 && HW > 0);
  hipStream_t st = (hipStream_t)stream;
  plane_sum_kernel<<<N * C, NTN, 0, st>>>(x, partial, HW);
  sum_over_n_kernel<<<ceil_div(C, 256), 256, 0, st>>>(partial, N, C, 1, out, nullptr, nullptr, accumulate);
  return vst_launch_status();
}

}  // extern "C"
