// AdaAttN path kernels for gfx950 (AA/network.py:102-220, AA/lossfn.py:5-53, AA/utilities.py:98-109).
//
// The attention matrices are materialised (HBM is 288 GB): S = Q^T K and A = cosine-normalised S
// per image, with the four products (S = Q^T K, [M; E2] = A [V; V^2], and the backward
// dA = [dM; dE2]^T [V; V^2], d[V; V^2] = [dM; dE2] A, dQ = K dS^T, dK = Q dS) running on the
// fp32-MFMA GEMM kernels (conv_gemm_kernel with 1x1 "convs", wgrad_kernel as A B^T); this file
// holds the row/column/elementwise parts and the small C x C loss math.
#include "vst_common.h"
#include "vst_hip.h"

namespace {

constexpr int RT = 256;

__device__ __forceinline__ double block_sum_d(double v, double* sh) {
  v = wave_sum_d(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) sh[w] = v;
  __syncthreads();
  double s = 0.0;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += sh[i];
  return s;
}

// packed GEMM A operand from a row-major matrix per batch: X[k][m] (transpose=0) or X[m][k]
__global__ void pack_matrix_kernel(const float* __restrict__ x, float* __restrict__ out, int B, int M, int K,
                                   int transpose, int Mpad, int Kpad, long x_bs, int bsplit) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long per = (long)Mpad * Kpad;
  if (idx >= B * per) return;
  int b = (int)(idx / per);
  long t = idx - b * per;
  int m = (int)(t % Mpad), k = (int)(t / Mpad);
  float v = 0.f;
  if (m < M && k < K) v = transpose ? x[b * x_bs + (long)m * K + k] : x[b * x_bs + (long)k * M + m];
  apack_store(out + b * per * ((bsplit & 3) == 2 ? 3 : 2) / 2, k, m, Mpad, v, bsplit);  // bf16x6 packs are 1.5x
}

// pack_matrix_kernel with one thread per (batch, k-tile, row m): the 16 k of its packed block are
// gathered, split and written as whole 16-byte words (the per-element form decoded its position
// with 64-bit division and wrote each piece as a separate 2-byte store); same arithmetic per element
// (split_bf16x2 / split3_bf16x2 are apack_store's splits two elements at a time)
__global__ __launch_bounds__(64) void pack_matrix_rows_kernel(const float* __restrict__ x, float* __restrict__ out,
                                                              int M, int K, int transpose, int Mpad, int Kpad,
                                                              long x_bs, int split) {
  const int m = blockIdx.x * 64 + threadIdx.x;
  if (m >= Mpad) return;
  const int kt = blockIdx.y, b = blockIdx.z;
  split &= 3;
  const float* xb = x + b * x_bs;
  float v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int k = kt * 16 + i;
    v[i] = (m < M && k < K) ? (transpose ? xb[(long)m * K + k] : xb[(long)k * M + m]) : 0.f;
  }
  const long per = (long)Mpad * Kpad;
  float* ob = out + b * per * (split == 2 ? 3 : 2) / 2;
  const long row = (long)kt * Mpad + m;
  if (split == 0) {  // apack_index: even k in dwords 0..7, odd k in 8..15
    f32x4* d = reinterpret_cast<f32x4*>(ob + row * 16);
    d[0] = f32x4{v[0], v[2], v[4], v[6]};
    d[1] = f32x4{v[8], v[10], v[12], v[14]};
    d[2] = f32x4{v[1], v[3], v[5], v[7]};
    d[3] = f32x4{v[9], v[11], v[13], v[15]};
  } else if (split == 2) {  // bf16x6: [hi k0..15][mid][lo]
    uint32_t h[8], md[8], l[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) split3_bf16x2(v[2 * q], v[2 * q + 1], h[q], md[q], l[q]);
    u32x4* d = reinterpret_cast<u32x4*>(ob + row * 24);
    d[0] = u32x4{h[0], h[1], h[2], h[3]};
    d[1] = u32x4{h[4], h[5], h[6], h[7]};
    d[2] = u32x4{md[0], md[1], md[2], md[3]};
    d[3] = u32x4{md[4], md[5], md[6], md[7]};
    d[4] = u32x4{l[0], l[1], l[2], l[3]};
    d[5] = u32x4{l[4], l[5], l[6], l[7]};
  } else {  // bf16x3 / bf16: [hi k0..15][lo]; fp16: [f16 k0..15][zeros]
    uint32_t h[8], l[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      if (split == 3) {
        h[q] = pack_f16x2(v[2 * q], v[2 * q + 1]);
        l[q] = 0u;
      } else {
        split_bf16x2(v[2 * q], v[2 * q + 1], h[q], l[q]);
      }
    }
    u32x4* d = reinterpret_cast<u32x4*>(ob + row * 16);
    d[0] = u32x4{h[0], h[1], h[2], h[3]};
    d[1] = u32x4{h[4], h[5], h[6], h[7]};
    d[2] = u32x4{l[0], l[1], l[2], l[3]};
    d[3] = u32x4{l[4], l[5], l[6], l[7]};
  }
}

// out[n][p] = sqrt(sum_c x[n][c][p]^2)  (vector_norm over the channel axis)
// block = 64 consecutive pixels x 4 channel quarters; coalesced 256-B row reads, LDS combine
__global__ void channel_norm_kernel(const float* __restrict__ x, float* __restrict__ out, int N, int C, int P) {
  __shared__ float part[4][64];
  const int lane = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int tiles = (P + 63) / 64;
  const int n = blockIdx.x / tiles;
  const int p = (blockIdx.x % tiles) * 64 + lane;
  float s0 = 0.f, s1 = 0.f;
  if (p < P) {
    const float* xp = x + (long)n * C * P + p;
    int c = grp;
#pragma unroll 4
    for (; c + 4 < C; c += 8) {
      const float a = xp[(long)c * P], b = xp[(long)(c + 4) * P];
      s0 += a * a;
      s1 += b * b;
    }
    for (; c < C; c += 4) {
      const float a = xp[(long)c * P];
      s0 += a * a;
    }
  }
  part[grp][lane] = s0 + s1;
  __syncthreads();
  if (grp == 0 && p < P) out[(long)n * P + p] = sqrtf(part[0][lane] + part[1][lane] + part[2][lane] + part[3][lane]);
}

// cosine attention rows (AA/network.py:121-124): s = S/(qn_i kn_j) + 1, A = s / sum_j s
__global__ void cos_rows_fwd_kernel(const float* __restrict__ S, const float* __restrict__ qn,
                                    const float* __restrict__ kn, float* __restrict__ A, float* __restrict__ rowsum,
                                    int Nc, int Ns) {
  __shared__ double sh[RT / 64];
  const long row = blockIdx.x;  // n * Nc + i
  const int n = (int)(row / Nc);
  const float q = qn[row];
  const float* knn = kn + (long)n * Ns;
  const float* Sr = S + row * Ns;
  float* Ar = A + row * Ns;
  double acc = 0.0;
  for (int j = threadIdx.x; j < Ns; j += RT) acc += Sr[j] / (q * knn[j]) + 1.0f;
  const float tot = (float)block_sum_d(acc, sh);
  for (int j = threadIdx.x; j < Ns; j += RT) Ar[j] = (Sr[j] / (q * knn[j]) + 1.0f) / tot;
  if (threadIdx.x == 0) rowsum[row] = tot;
}

// backward through the row normalisation and the cosine scaling, per row i:
//   r = sum_j dA A;  dSraw = (dA - r) / (rowsum * qn_i * kn_j);  t = dSraw * S (written over S)
//   dqn_i = -(sum_j t) / qn_i
__global__ void cos_rows_bwd_kernel(const float* __restrict__ dA, const float* __restrict__ A,
                                    float* __restrict__ S_t, const float* __restrict__ qn,
                                    const float* __restrict__ kn, const float* __restrict__ rowsum,
                                    float* __restrict__ dS, float* __restrict__ dqn, int Nc, int Ns) {
  __shared__ double sh[RT / 64];
  const long row = blockIdx.x;
  const int n = (int)(row / Nc);
  const float* knn = kn + (long)n * Ns;
  const float* dAr = dA + row * Ns;
  const float* Ar = A + row * Ns;
  double r = 0.0;
  for (int j = threadIdx.x; j < Ns; j += RT) r += (double)dAr[j] * Ar[j];
  const float rr = (float)block_sum_d(r, sh);
  const float q = qn[row], inv = 1.0f / rowsum[row];
  float* Sr = S_t + row * Ns;
  float* dSr = dS + row * Ns;
  double tsum = 0.0;
  for (int j = threadIdx.x; j < Ns; j += RT) {
    float d = (dAr[j] - rr) * inv / (q * knn[j]);
    dSr[j] = d;
    float t = d * Sr[j];
    Sr[j] = t;
    tsum += t;
  }
  const float ts = (float)block_sum_d(tsum, sh);
  if (threadIdx.x == 0) dqn[row] = -ts / q;
}

// column sums of X [N][R][Cc] in row chunks: part[n][chunk][j]
__global__ void colsum_part_kernel(const float* __restrict__ X, float* __restrict__ part, int R, int Cc, int chunk) {
  const int j = blockIdx.x * RT + threadIdx.x;
  const int ch = blockIdx.y, n = blockIdx.z;
  if (j >= Cc) return;
  const int r0 = ch * chunk, r1 = min(R, r0 + chunk);
  const float* x = X + ((long)n * R) * Cc + j;
  float s = 0.f;
  for (int r = r0; r < r1; ++r) s += x[(long)r * Cc];
  part[((long)n * gridDim.y + ch) * Cc + j] = s;
}

// dkn_j = -(sum over chunks) / kn_j
__global__ void colsum_finish_kernel(const float* __restrict__ part, const float* __restrict__ kn,
                                     float* __restrict__ dkn, int N, int nch, int Cc) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)N * Cc) return;
  int n = (int)(idx / Cc), j = (int)(idx % Cc);
  double s = 0.0;
  for (int c = 0; c < nch; ++c) s += part[((long)n * nch + c) * Cc + j];
  dkn[idx] = -(float)s / kn[idx];
}

// X[n][c][p] += s[n][p] / nrm[n][p] * Y[n][c][p]   (gradient through a channel-axis norm)
__global__ void norm_grad_add_kernel(float* __restrict__ X, const float* __restrict__ s, const float* __restrict__ nrm,
                                     const float* __restrict__ Y, int N, int C, int P) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)N * C * P) return;
  int p = (int)(idx % P);
  long n = idx / ((long)C * P);
  long q = n * P + p;
  X[idx] += s[q] / nrm[q] * Y[idx];
}

// VV2[n] = [V[n]; V[n]^2]
__global__ void square_concat_kernel(const float* __restrict__ V, float* __restrict__ VV2, int N, long per) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)N * per) return;
  long n = idx / per, t = idx - n * per;
  float v = V[idx];
  VV2[n * 2 * per + t] = v;
  VV2[n * 2 * per + per + t] = v * v;
}

// dV = d[V] + 2 V d[V^2]
__global__ void square_concat_bwd_kernel(const float* __restrict__ dVV2, const float* __restrict__ V,
                                         float* __restrict__ dV, int N, long per) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)N * per) return;
  long n = idx / per, t = idx - n * per;
  dV[idx] = dVV2[n * 2 * per + t] + 2.0f * V[idx] * dVV2[n * 2 * per + per + t];
}

// out = sqrt(clamp(E2 - M^2, 1e-6)) * cn + M   with MV[n] = [M; E2]  (AA/network.py:209-220)
__global__ void adaattn_out_kernel(const float* __restrict__ MV, const float* __restrict__ cn, float* __restrict__ out,
                                   int N, long per) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)N * per) return;
  long n = idx / per, t = idx - n * per;
  const float m = MV[n * 2 * per + t], e2 = MV[n * 2 * per + per + t];
  const float var = e2 - m * m;
  out[idx] = sqrtf(fmaxf(var, 1e-6f)) * cn[idx] + m;
}

__global__ void adaattn_out_bwd_kernel(const float* __restrict__ dout, const float* __restrict__ MV,
                                       const float* __restrict__ cn, float* __restrict__ dMV, int N, long per) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)N * per) return;
  long n = idx / per, t = idx - n * per;
  const float m = MV[n * 2 * per + t], e2 = MV[n * 2 * per + per + t];
  const float var = e2 - m * m;
  const float g = dout[idx];
  // clamp(min) passes the gradient where var >= 1e-6 (torch clamp backward: x >= min)
  const float dvar = var >= 1e-6f ? g * cn[idx] * 0.5f / sqrtf(var) : 0.f;
  dMV[n * 2 * per + t] = g - 2.0f * m * dvar;
  dMV[n * 2 * per + per + t] = dvar;
}

// the same, with the result's both halves scaled per column (dMV * w[n][p], per = dv * P): the
// linear-form cosine attention's dRh = dMV / rs without a second pass over [M; E2]
__global__ void adaattn_out_bwd_scaled_kernel(const float* __restrict__ dout, const float* __restrict__ MV,
                                              const float* __restrict__ cn, const float* __restrict__ w,
                                              float* __restrict__ dMV, int N, long per, int P) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)N * per) return;
  long n = idx / per, t = idx - n * per;
  const float m = MV[n * 2 * per + t], e2 = MV[n * 2 * per + per + t];
  const float var = e2 - m * m;
  const float g = dout[idx];
  const float dvar = var >= 1e-6f ? g * cn[idx] * 0.5f / sqrtf(var) : 0.f;
  const float s = w[n * P + t % P];
  dMV[n * 2 * per + t] = (g - 2.0f * m * dvar) * s;
  dMV[n * 2 * per + per + t] = dvar * s;
}

// Division-free forms of the four kernels above (one float4 per thread, image n on blockIdx.y, the
// column-scaled backward's channel on blockIdx.z): the flat forms decode (n, t) with a 64-bit
// division per element (and t % P in 64 bits), which made them VALU-bound under the HBM rate.
// Used when per (and P) is a multiple of 4 and the pointers are 16-byte aligned.
__global__ void square_concat_vec_kernel(const float4* __restrict__ V, float4* __restrict__ VV2, long per4) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= per4) return;
  const long n = blockIdx.y;
  const float4 v = V[n * per4 + t];
  VV2[n * 2 * per4 + t] = v;
  VV2[n * 2 * per4 + per4 + t] = make_float4(v.x * v.x, v.y * v.y, v.z * v.z, v.w * v.w);
}

__global__ void adaattn_out_vec_kernel(const float4* __restrict__ MV, const float4* __restrict__ cn,
                                       float4* __restrict__ out, long per4) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= per4) return;
  const long n = blockIdx.y;
  const float4 m = MV[n * 2 * per4 + t], e2 = MV[n * 2 * per4 + per4 + t], c = cn[n * per4 + t];
  float4 o;
  o.x = sqrtf(fmaxf(e2.x - m.x * m.x, 1e-6f)) * c.x + m.x;
  o.y = sqrtf(fmaxf(e2.y - m.y * m.y, 1e-6f)) * c.y + m.y;
  o.z = sqrtf(fmaxf(e2.z - m.z * m.z, 1e-6f)) * c.z + m.z;
  o.w = sqrtf(fmaxf(e2.w - m.w * m.w, 1e-6f)) * c.w + m.w;
  out[n * per4 + t] = o;
}

// grid (ceil(P4 / 256), dv, N): element (n, channel c, column p) of the dv x P plane stack
__global__ void adaattn_out_bwd_scaled_vec_kernel(const float4* __restrict__ dout, const float4* __restrict__ MV,
                                                  const float4* __restrict__ cn, const float4* __restrict__ w,
                                                  float4* __restrict__ dMV, int P4, long per4) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P4) return;
  const long n = blockIdx.z, t = (long)blockIdx.y * P4 + p;
  const float4 m = MV[n * 2 * per4 + t], e2 = MV[n * 2 * per4 + per4 + t], g = dout[n * per4 + t];
  const float4 c = cn[n * per4 + t], sc = w[n * P4 + p];
  float4 d0, d1;
  auto one = [](float m_, float e2_, float g_, float c_, float s_, float& a, float& b) {
    const float var = e2_ - m_ * m_;
    const float dvar = var >= 1e-6f ? g_ * c_ * 0.5f / sqrtf(var) : 0.f;
    a = (g_ - 2.0f * m_ * dvar) * s_;
    b = dvar * s_;
  };
  one(m.x, e2.x, g.x, c.x, sc.x, d0.x, d1.x);
  one(m.y, e2.y, g.y, c.y, sc.y, d0.y, d1.y);
  one(m.z, e2.z, g.z, c.z, sc.z, d0.z, d1.z);
  one(m.w, e2.w, g.w, c.w, sc.w, d0.w, d1.w);
  dMV[n * 2 * per4 + t] = d0;
  dMV[n * 2 * per4 + per4 + t] = d1;
}

// per-plane L2 norm with two float4 loads in flight per thread (fp64 accumulation as the flat form)
__global__ void plane_norm_vec_kernel(const float4* __restrict__ x, float* __restrict__ out, int HW4) {
  __shared__ double sh[RT / 64];
  const float4* xp = x + (long)blockIdx.x * HW4;
  double s = 0.0;
  int i = threadIdx.x;
  for (; i + RT < HW4; i += 2 * RT) {
    const float4 a = xp[i], b = xp[i + RT];
    s += ((double)a.x * a.x + (double)a.y * a.y) + ((double)a.z * a.z + (double)a.w * a.w) +
         (((double)b.x * b.x + (double)b.y * b.y) + ((double)b.z * b.z + (double)b.w * b.w));
  }
  if (i < HW4) {
    const float4 a = xp[i];
    s += ((double)a.x * a.x + (double)a.y * a.y) + ((double)a.z * a.z + (double)a.w * a.w);
  }
  const double t = block_sum_d(s, sh);
  if (threadIdx.x == 0) out[blockIdx.x] = (float)sqrt(t);
}

static bool al16(const void* a, const void* b = nullptr, const void* c = nullptr, const void* d = nullptr,
                 const void* e = nullptr) {
  return ((((uintptr_t)a) | ((uintptr_t)b) | ((uintptr_t)c) | ((uintptr_t)d) | ((uintptr_t)e)) & 15) == 0;
}

// per-plane mean and unbiased std (torch .mean / .std over (H, W))
__global__ void plane_meanstd_kernel(const float* __restrict__ x, float* __restrict__ mean, float* __restrict__ std_,
                                     int HW) {
  __shared__ double sh[RT / 64];
  const long plane = blockIdx.x;
  const float* xp = x + plane * HW;
  double s = 0.0;
#pragma unroll 8
  for (int i = threadIdx.x; i < HW; i += RT) s += xp[i];
  const double mu = block_sum_d(s, sh) / HW;
  double q = 0.0;
#pragma unroll 8
  for (int i = threadIdx.x; i < HW; i += RT) {
    double d = xp[i] - mu;
    q += d * d;
  }
  const double var = block_sum_d(q, sh) / (HW - 1);
  if (threadIdx.x == 0) {
    mean[plane] = (float)mu;
    std_[plane] = (float)sqrt(var);
  }
}

__global__ void plane_meanstd_bwd_kernel(const float* __restrict__ x, const float* __restrict__ mean,
                                         const float* __restrict__ std_, const float* __restrict__ gmean,
                                         const float* __restrict__ gstd, float* __restrict__ gx, int HW) {
  const long plane = blockIdx.x;
  const float mu = mean[plane], sd = std_[plane];
  const float a = gmean ? gmean[plane] / HW : 0.f;
  const float b = (gstd && sd > 0.f) ? gstd[plane] / ((HW - 1) * sd) : 0.f;
  const float* xp = x + plane * HW;
  float* gp = gx + plane * HW;
#pragma unroll 8
  for (int i = threadIdx.x; i < HW; i += RT) gp[i] = a + b * (xp[i] - mu);
}

// per-plane L2 norms: out[plane] = sqrt(sum x^2)
__global__ void plane_norm_kernel(const float* __restrict__ x, float* __restrict__ out, int HW) {
  __shared__ double sh[RT / 64];
  const long plane = blockIdx.x;
  const float* xp = x + plane * HW;
  double s = 0.0;
  for (int i = threadIdx.x; i < HW; i += RT) s += (double)xp[i] * xp[i];
  const double t = block_sum_d(s, sh);
  if (threadIdx.x == 0) out[plane] = (float)sqrt(t);
}

// image_similarity_loss core (AA/lossfn.py:25-53), both cosine distances:
//   D = 1 - G / (un_i vn_j + 1e-6);  Dn = D / colsum_j(D);  loss_n = sum |Dn_c - Dn_cs| / hw
// pass 1: column sums.  Block = 64 consecutive columns x 4 row quarters (rows i = grp, grp+4, ...),
// coalesced 256-B row reads, the quarters combined in a fixed order through LDS (grid ceil(C/64) x N:
// a column per thread over all C rows left most of the chip idle at C = 4096)
__global__ __launch_bounds__(256) void simloss_colsum_kernel(const float* __restrict__ Gc, const float* __restrict__ unc,
                                                             const float* __restrict__ vnc, const float* __restrict__ Gs,
                                                             const float* __restrict__ uns, const float* __restrict__ vns,
                                                             float* __restrict__ colc, float* __restrict__ cols, int C) {
  __shared__ double pa[4][64], pb[4][64];
  const int lane = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int n = blockIdx.y, j = blockIdx.x * 64 + lane;
  double a = 0.0, b = 0.0;
  if (j < C) {
    const long o = (long)n * C * C;
    const float vc = vnc[n * C + j], vs = vns[n * C + j];
#pragma unroll 8
    for (int i = grp; i < C; i += 4) {
      a += 1.0f - Gc[o + (long)i * C + j] / (unc[n * C + i] * vc + 1e-6f);
      b += 1.0f - Gs[o + (long)i * C + j] / (uns[n * C + i] * vs + 1e-6f);
    }
  }
  pa[grp][lane] = a;
  pb[grp][lane] = b;
  __syncthreads();
  if (grp == 0 && j < C) {
    colc[n * C + j] = (float)(((pa[0][lane] + pa[1][lane]) + pa[2][lane]) + pa[3][lane]);
    cols[n * C + j] = (float)(((pb[0][lane] + pb[1][lane]) + pb[2][lane]) + pb[3][lane]);
  }
}

// pass 2: one block per row (i, n): rowpart[n][i] = sum_j |Dn_c - Dn_cs| / hw
__global__ void simloss_rows_kernel(const float* __restrict__ Gc, const float* __restrict__ unc,
                                    const float* __restrict__ vnc, const float* __restrict__ Gs,
                                    const float* __restrict__ uns, const float* __restrict__ vns,
                                    const float* __restrict__ colc, const float* __restrict__ cols,
                                    float* __restrict__ rowpart, int C, float inv_hw) {
  __shared__ double sh[RT / 64];
  const int i = blockIdx.x, n = blockIdx.y;
  const long o = (long)n * C * C + (long)i * C;
  const float uc = unc[n * C + i], us = uns[n * C + i];
  double acc = 0.0;
  for (int j = threadIdx.x; j < C; j += RT) {
    const float dc = (1.0f - Gc[o + j] / (uc * vnc[n * C + j] + 1e-6f)) / colc[n * C + j];
    const float ds = (1.0f - Gs[o + j] / (us * vns[n * C + j] + 1e-6f)) / cols[n * C + j];
    acc += fabsf(dc - ds);
  }
  const double tot = block_sum_d(acc, sh);
  if (threadIdx.x == 0) rowpart[(long)n * C + i] = (float)tot * inv_hw;
}

// backward w.r.t. the stylised side: dG (C x C) plus dun (rows) and dvn (cols), scaled by gscale
__global__ void simloss_bwd_kernel(const float* __restrict__ Gc, const float* __restrict__ unc,
                                   const float* __restrict__ vnc, const float* __restrict__ Gs,
                                   const float* __restrict__ uns, const float* __restrict__ vns,
                                   const float* __restrict__ colc, const float* __restrict__ cols,
                                   const float* __restrict__ gout, float weight, float* __restrict__ dG,
                                   float* __restrict__ dun, float* __restrict__ dvn, int C, float inv_hw) {
  // one block per (n, column j): dDn_ij = sign(Ds_n - Dc_n) * g / hw;  dD_ij = (dDn_ij - sum_i dDn Dn) / colsum_j
  __shared__ double sh[RT / 64];
  const int n = blockIdx.y, j = blockIdx.x;
  const long o = (long)n * C * C;
  const float g = gout[0] * weight * inv_hw;
  const float cs = cols[n * C + j], cc = colc[n * C + j];
  const float vj = vns[n * C + j];
  double r = 0.0;
  for (int i = threadIdx.x; i < C; i += RT) {
    const float den = uns[n * C + i] * vj + 1e-6f;
    const float ds = (1.0f - Gs[o + (long)i * C + j] / den) / cs;
    const float dc = (1.0f - Gc[o + (long)i * C + j] / (unc[n * C + i] * vnc[n * C + j] + 1e-6f)) / cc;
    const float sg = ds > dc ? g : (ds < dc ? -g : 0.f);
    r += (double)sg * ds;
  }
  const float rr = (float)block_sum_d(r, sh);
  double dvacc = 0.0;
  for (int i = threadIdx.x; i < C; i += RT) {
    const float den = uns[n * C + i] * vj + 1e-6f;
    const float G = Gs[o + (long)i * C + j];
    const float ds = (1.0f - G / den) / cs;
    const float dc = (1.0f - Gc[o + (long)i * C + j] / (unc[n * C + i] * vnc[n * C + j] + 1e-6f)) / cc;
    const float sg = ds > dc ? g : (ds < dc ? -g : 0.f);
    const float dD = (sg - rr) / cs;  // grad w.r.t. D_ij (un-normalised distance)
    // D = 1 - G/den: dG = -dD/den; d(den) = dD * G / den^2
    dG[o + (long)i * C + j] = -dD / den;
    const float dden = dD * G / (den * den);
    dvacc += (double)dden * uns[n * C + i];
  }
  const double dv = block_sum_d(dvacc, sh);
  if (threadIdx.x == 0) dvn[n * C + j] = (float)dv;
}

// the row half of the same adjoint, one block per row (i, n): dun_i = sum_j d(den_ij) v_j with
// d(den_ij) = dD_ij G_ij / den_ij^2 = -dG_ij G_ij / den_ij (dG from simloss_bwd_kernel), summed in a
// fixed order (was a float atomic per (i, j): run-to-run reproducible now)
__global__ void simloss_bwd_rows_kernel(const float* __restrict__ Gs, const float* __restrict__ uns,
                                        const float* __restrict__ vns, const float* __restrict__ dG,
                                        float* __restrict__ dun, int C) {
  __shared__ double sh[RT / 64];
  const int i = blockIdx.x, n = blockIdx.y;
  const long o = (long)n * C * C + (long)i * C;
  const float ui = uns[n * C + i];
  double acc = 0.0;
  for (int j = threadIdx.x; j < C; j += RT) {
    const float vj = vns[n * C + j];
    const float den = ui * vj + 1e-6f;
    const float dden = -dG[o + j] * Gs[o + j] / den;
    acc += (double)(dden * vj);
  }
  const double tot = block_sum_d(acc, sh);
  if (threadIdx.x == 0) dun[n * C + i] = (float)tot;
}

// x[plane][i] += s[plane] / nrm[plane] * y[plane][i]   (gradient through per-plane L2 norms)
__global__ void plane_norm_grad_kernel(float* __restrict__ x, const float* __restrict__ s,
                                       const float* __restrict__ nrm, const float* __restrict__ y, int HW) {
  const long plane = blockIdx.x;
  const float k = nrm[plane] > 0.f ? s[plane] / nrm[plane] : 0.f;
#pragma unroll 8
  for (int i = threadIdx.x; i < HW; i += RT) x[plane * HW + i] += k * y[plane * HW + i];
}

}  // namespace

extern "C" {

int vst_pack_matrix(const float* x, float* packed, int B, int M, int K, int transpose, int Mpad, int Kpad, long x_bs,
                    int mode, void* stream) {
  VST_CHECK_ARG(vst_mode_ok(mode));
  VST_CHECK_ARG(x && packed && B > 0 && M > 0 && K > 0 && Mpad >= M && Kpad >= K);
  if (Kpad % 16 == 0 && Kpad / 16 <= 65535 && B <= 65535 && ((uintptr_t)packed & 15) == 0) {
    const dim3 g((unsigned)ceil_div(Mpad, 64), (unsigned)(Kpad / 16), (unsigned)B);
    pack_matrix_rows_kernel<<<g, 64, 0, (hipStream_t)stream>>>(x, packed, M, K, transpose, Mpad, Kpad, x_bs,
                                                               apack_split(mode));
    return vst_launch_status();
  }
  long total = (long)B * Mpad * Kpad;
  pack_matrix_kernel<<<ceil_div(total, 256), 256, 0, (hipStream_t)stream>>>(
      x, packed, B, M, K, transpose, Mpad, Kpad, x_bs, apack_split(mode));
  return vst_launch_status();
}

int vst_channel_norm(const float* x, float* out, int N, int C, int P, void* stream) {
  VST_CHECK_ARG(x && out && N > 0 && C > 0 && P > 0);
  channel_norm_kernel<<<N * ceil_div(P, 64), 256, 0, (hipStream_t)stream>>>(x, out, N, C, P);
  return vst_launch_status();
}

int vst_cos_attn_rows(const float* S, const float* qn, const float* kn, float* A, float* rowsum, int N, int Nc, int Ns,
                      void* stream) {
  VST_CHECK_ARG(S && qn && kn && A && rowsum && N > 0 && Nc > 0 && Ns > 0);
  cos_rows_fwd_kernel<<<N * Nc, RT, 0, (hipStream_t)stream>>>(S, qn, kn, A, rowsum, Nc, Ns);
  return vst_launch_status();
}

// S_t: S on entry, overwritten with t = dS*S; part: N * ceil(Nc/64) * Ns floats
int vst_cos_attn_rows_bwd(const float* dA, const float* A, float* S_t, const float* qn, const float* kn,
                          const float* rowsum, float* dS, float* dqn, float* dkn, float* part, int N, int Nc, int Ns,
                          void* stream) {
  VST_CHECK_ARG(dA && A && S_t && qn && kn && rowsum && dS && dqn && dkn && part && N > 0 && Nc > 0 && Ns > 0);
  hipStream_t st = (hipStream_t)stream;
  cos_rows_bwd_kernel<<<N * Nc, RT, 0, st>>>(dA, A, S_t, qn, kn, rowsum, dS, dqn, Nc, Ns);
  const int chunk = 64, nch = ceil_div(Nc, chunk);
  dim3 g(ceil_div(Ns, RT), nch, N);
  colsum_part_kernel<<<g, RT, 0, st>>>(S_t, part, Nc, Ns, chunk);
  colsum_finish_kernel<<<ceil_div((long)N * Ns, 256), 256, 0, st>>>(part, kn, dkn, N, nch, Ns);
  return vst_launch_status();
}

int vst_norm_grad_add(float* x, const float* s, const float* nrm, const float* y, int N, int C, int P, void* stream) {
  VST_CHECK_ARG(x && s && nrm && y && N > 0 && C > 0 && P > 0);
  norm_grad_add_kernel<<<ceil_div((long)N * C * P, 256), 256, 0, (hipStream_t)stream>>>(x, s, nrm, y, N, C, P);
  return vst_launch_status();
}

int vst_square_concat(const float* V, float* VV2, int N, long per, void* stream) {
  VST_CHECK_ARG(V && VV2 && N > 0 && per > 0);
  if (per % 4 == 0 && N <= 65535 && al16(V, VV2)) {
    dim3 g(ceil_div(per / 4, 256), N);
    square_concat_vec_kernel<<<g, 256, 0, (hipStream_t)stream>>>((const float4*)V, (float4*)VV2, per / 4);
    return vst_launch_status();
  }
  square_concat_kernel<<<ceil_div((long)N * per, 256), 256, 0, (hipStream_t)stream>>>(V, VV2, N, per);
  return vst_launch_status();
}

int vst_square_concat_bwd(const float* dVV2, const float* V, float* dV, int N, long per, void* stream) {
  VST_CHECK_ARG(dVV2 && V && dV && N > 0 && per > 0);
  square_concat_bwd_kernel<<<ceil_div((long)N * per, 256), 256, 0, (hipStream_t)stream>>>(dVV2, V, dV, N, per);
  return vst_launch_status();
}

int vst_adaattn_out(const float* MV, const float* cn, float* out, int N, long per, void* stream) {
  VST_CHECK_ARG(MV && cn && out && N > 0 && per > 0);
  if (per % 4 == 0 && N <= 65535 && al16(MV, cn, out)) {
    dim3 g(ceil_div(per / 4, 256), N);
    adaattn_out_vec_kernel<<<g, 256, 0, (hipStream_t)stream>>>((const float4*)MV, (const float4*)cn, (float4*)out,
                                                               per / 4);
    return vst_launch_status();
  }
  adaattn_out_kernel<<<ceil_div((long)N * per, 256), 256, 0, (hipStream_t)stream>>>(MV, cn, out, N, per);
  return vst_launch_status();
}

int vst_adaattn_out_bwd(const float* dout, const float* MV, const float* cn, float* dMV, int N, long per,
                        void* stream) {
  VST_CHECK_ARG(dout && MV && cn && dMV && N > 0 && per > 0);
  adaattn_out_bwd_kernel<<<ceil_div((long)N * per, 256), 256, 0, (hipStream_t)stream>>>(dout, MV, cn, dMV, N, per);
  return vst_launch_status();
}

int vst_adaattn_out_bwd_scaled(const float* dout, const float* MV, const float* cn, const float* colscale, float* dMV,
                               int N, long per, int P, void* stream) {
  VST_CHECK_ARG(dout && MV && cn && colscale && dMV && N > 0 && per > 0 && P > 0 && per % P == 0);
  if (P % 4 == 0 && per / P <= 65535 && N <= 65535 && al16(dout, MV, cn, colscale, dMV)) {
    dim3 g(ceil_div(P / 4, 256), per / P, N);
    adaattn_out_bwd_scaled_vec_kernel<<<g, 256, 0, (hipStream_t)stream>>>(
        (const float4*)dout, (const float4*)MV, (const float4*)cn, (const float4*)colscale, (float4*)dMV, P / 4, per / 4);
    return vst_launch_status();
  }
  adaattn_out_bwd_scaled_kernel<<<ceil_div((long)N * per, 256), 256, 0, (hipStream_t)stream>>>(dout, MV, cn, colscale,
                                                                                            dMV, N, per, P);
  return vst_launch_status();
}

int vst_plane_meanstd(const float* x, float* mean, float* std_, long NC, int HW, void* stream) {
  VST_CHECK_ARG(x && mean && std_ && NC > 0 && HW > 1);
  plane_meanstd_kernel<<<NC, RT, 0, (hipStream_t)stream>>>(x, mean, std_, HW);
  return vst_launch_status();
}

int vst_plane_meanstd_bwd(const float* x, const float* mean, const float* std_, const float* gmean, const float* gstd,
                          float* gx, long NC, int HW, void* stream) {
  VST_CHECK_ARG(x && mean && std_ && gx && NC > 0 && HW > 1);
  plane_meanstd_bwd_kernel<<<NC, RT, 0, (hipStream_t)stream>>>(x, mean, std_, gmean, gstd, gx, HW);
  return vst_launch_status();
}

int vst_plane_norm(const float* x, float* out, long NC, int HW, void* stream) {
  VST_CHECK_ARG(x && out && NC > 0 && HW > 0);
  if (HW % 4 == 0 && al16(x)) {
    plane_norm_vec_kernel<<<NC, RT, 0, (hipStream_t)stream>>>((const float4*)x, out, HW / 4);
    return vst_launch_status();
  }
  plane_norm_kernel<<<NC, RT, 0, (hipStream_t)stream>>>(x, out, HW);
  return vst_launch_status();
}

int vst_plane_norm_grad(float* x, const float* s, const float* nrm, const float* y, long NC, int HW, void* stream) {
  VST_CHECK_ARG(x && s && nrm && y && NC > 0 && HW > 0);
  plane_norm_grad_kernel<<<NC, RT, 0, (hipStream_t)stream>>>(x, s, nrm, y, HW);
  return vst_launch_status();
}

// partial: N*C floats (per-row loss, already / hw); colc, cols: N*C
int vst_simloss(const float* Gc, const float* unc, const float* vnc, const float* Gs, const float* uns,
                const float* vns, float* colc, float* cols, float* partial, int N, int C, int HW, void* stream) {
  VST_CHECK_ARG(Gc && unc && vnc && Gs && uns && vns && colc && cols && partial && N > 0 && C > 0 && HW > 0);
  hipStream_t st = (hipStream_t)stream;
  simloss_colsum_kernel<<<dim3(ceil_div(C, 64), N), 256, 0, st>>>(Gc, unc, vnc, Gs, uns, vns, colc, cols, C);
  simloss_rows_kernel<<<dim3(C, N), RT, 0, st>>>(Gc, unc, vnc, Gs, uns, vns, colc, cols, partial, C, 1.0f / HW);
  return vst_launch_status();
}

// dG, dun, dvn fully written (deterministic: no atomics)
int vst_simloss_bwd(const float* Gc, const float* unc, const float* vnc, const float* Gs, const float* uns,
                    const float* vns, const float* colc, const float* cols, const float* gout, float weight, float* dG,
                    float* dun, float* dvn, int N, int C, int HW, void* stream) {
  VST_CHECK_ARG(Gc && unc && vnc && Gs && uns && vns && colc && cols && gout && dG && dun && dvn && N > 0 && C > 0);
  dim3 g(C, N);
  simloss_bwd_kernel<<<g, RT, 0, (hipStream_t)stream>>>(Gc, unc, vnc, Gs, uns, vns, colc, cols, gout, weight, dG, dun,
                                                        dvn, C, 1.0f / HW);
  simloss_bwd_rows_kernel<<<dim3(C, N), RT, 0, (hipStream_t)stream>>>(Gs, uns, vns, dG, dun, C);
  return vst_launch_status();
}

}  // extern "C"

namespace {
__global__ void copy_planes_kernel(const float* __restrict__ src, long src_bs, float* __restrict__ dst, long dst_bs,
                                   int N, long per) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)N * per) return;
  long n = idx / per, t = idx - n * per;
  dst[n * dst_bs + t] = src[n * src_bs + t];
}

// copy_planes_kernel with the image on blockIdx.y and four floats per thread (per, src_bs, dst_bs
// multiples of 4 and 16-byte aligned bases): no per-element 64-bit division
__global__ __launch_bounds__(256) void copy_planes_vec_kernel(const float4* __restrict__ src, long src_bs4,
                                                              float4* __restrict__ dst, long dst_bs4, long per4) {
  const long t = (long)blockIdx.x * 256 + threadIdx.x;
  if (t >= per4) return;
  dst[blockIdx.y * dst_bs4 + t] = src[blockIdx.y * src_bs4 + t];
}

// D = 1 - G / (un_i vn_j + 1e-6)  (cosine_distance, AA/lossfn.py:25-38)
__global__ void cosdist_kernel(const float* __restrict__ G, const float* __restrict__ un, const float* __restrict__ vn,
                               float* __restrict__ D, int N, int C) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)N * C * C) return;
  int j = (int)(idx % C);
  long t = idx / C;
  int i = (int)(t % C);
  long n = t / C;
  D[idx] = 1.0f - G[idx] / (un[n * C + i] * vn[n * C + j] + 1e-6f);
}
}  // namespace

extern "C" int vst_copy_planes(const float* src, long src_bs, float* dst, long dst_bs, int N, long per, void* stream) {
  VST_CHECK_ARG(src && dst && N > 0 && per > 0);
  if (N <= 65535 && ((per | src_bs | dst_bs) & 3) == 0 && (((uintptr_t)src | (uintptr_t)dst) & 15) == 0) {
    copy_planes_vec_kernel<<<dim3((unsigned)ceil_div(per / 4, 256), (unsigned)N), 256, 0, (hipStream_t)stream>>>(
        (const float4*)src, src_bs / 4, (float4*)dst, dst_bs / 4, per / 4);
    return vst_launch_status();
  }
  copy_planes_kernel<<<ceil_div((long)N * per, 256), 256, 0, (hipStream_t)stream>>>(src, src_bs, dst, dst_bs, N, per);
  return vst_launch_status();
}

extern "C" int vst_cosdist(const float* G, const float* un, const float* vn, float* D, int N, int C, void* stream) {
  VST_CHECK_ARG(G && un && vn && D && N > 0 && C > 0);
  cosdist_kernel<<<ceil_div((long)N * C * C, 256), 256, 0, (hipStream_t)stream>>>(G, un, vn, D, N, C);
  return vst_launch_status();
}

namespace {
// row softmax (nn.Softmax(dim=-1), AA/network.py:102-108): A = exp(S - max) / sum
__global__ void softmax_rows_kernel(const float* __restrict__ S, float* __restrict__ A, int Ns) {
  __shared__ float shm[RT / 64];
  __shared__ double sh[RT / 64];
  const long row = blockIdx.x;
  const float* Sr = S + row * Ns;
  float* Ar = A + row * Ns;
  float mx = -INFINITY;
  for (int j = threadIdx.x; j < Ns; j += RT) mx = fmaxf(mx, Sr[j]);
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
  if ((threadIdx.x & 63) == 0) shm[threadIdx.x >> 6] = mx;
  __syncthreads();
  mx = shm[0];
  for (int i = 1; i < RT / 64; ++i) mx = fmaxf(mx, shm[i]);
  double acc = 0.0;
  for (int j = threadIdx.x; j < Ns; j += RT) acc += expf(Sr[j] - mx);
  const float inv = (float)(1.0 / block_sum_d(acc, sh));
  for (int j = threadIdx.x; j < Ns; j += RT) Ar[j] = expf(Sr[j] - mx) * inv;
}

// dS = A * (dA - sum_j dA A)
__global__ void softmax_rows_bwd_kernel(const float* dA, const float* __restrict__ A, float* dS, int Ns) {
  __shared__ double sh[RT / 64];
  const long row = blockIdx.x;
  const float* dAr = dA + row * Ns;
  const float* Ar = A + row * Ns;
  double r = 0.0;
  for (int j = threadIdx.x; j < Ns; j += RT) r += (double)dAr[j] * Ar[j];
  const float rr = (float)block_sum_d(r, sh);
  for (int j = threadIdx.x; j < Ns; j += RT) dS[row * Ns + j] = Ar[j] * (dAr[j] - rr);
}
}  // namespace

extern "C" int vst_softmax_rows(const float* S, float* A, long rows, int Ns, void* stream) {
  VST_CHECK_ARG(S && A && rows > 0 && Ns > 0);
  softmax_rows_kernel<<<rows, RT, 0, (hipStream_t)stream>>>(S, A, Ns);
  return vst_launch_status();
}

extern "C" int vst_softmax_rows_bwd(const float* dA, const float* A, float* dS, long rows, int Ns, void* stream) {
  VST_CHECK_ARG(dA && A && dS && rows > 0 && Ns > 0);
  softmax_rows_bwd_kernel<<<rows, RT, 0, (hipStream_t)stream>>>(dA, A, dS, Ns);
  return vst_launch_status();
}

// ---------------------------------------------------------------------------------------------
// Analytic cosine-attention statistics (AA/network.py:115-125).  With s_ij = S_ij/(qn_i kn_j) + 1
// and A = s / rowsum, every row/column reduction of the reference's N^2 matrices has a closed
// form in O(d (Nc + Ns)):
//   rowsum_i = (Q_i . kbar)/qn_i + Ns,          kbar = sum_j K_j / kn_j
//   r_i  = sum_j dA_ij A_ij = sum_v dMV_vi MV_vi,   DA_i = sum_j dA_ij = sum_v dMV_vi vsum_v
//   dqn_i = -(DA... ) see vst_attn_bwd_rows;  dkn_j via Y = Z^T [V;V^2], Z = (c . dMV) Q^T
// so A (and dS) come straight out of the GEMM epilogues and S is never stored.
namespace {

// out[n][c] = sum_p x[n][c][p] * (w ? w[n][p] : 1)   (one block per (n, c) plane)
__global__ void plane_dot_kernel(const float* __restrict__ x, const float* __restrict__ w, float* __restrict__ out,
                                 int C, int P) {
  __shared__ double sh[RT / 64];
  const long plane = blockIdx.x;
  const int n = (int)(plane / C);
  const float* xp = x + plane * P;
  const float* wp = w ? w + (long)n * P : nullptr;
  double acc = 0.0;
  for (int i = threadIdx.x; i < P; i += RT) acc += (double)xp[i] * (wp ? wp[i] : 1.f);
  const double t = block_sum_d(acc, sh);
  if (threadIdx.x == 0) out[plane] = (float)t;
}

// plane_dot_kernel over float4 (P % 4 == 0, 16-byte aligned x / w)
__global__ __launch_bounds__(RT) void plane_dot_vec_kernel(const float4* __restrict__ x, const float4* __restrict__ w,
                                                           float* __restrict__ out, int C, int P4) {
  __shared__ double sh[RT / 64];
  const long plane = blockIdx.x;
  const float4* xp = x + plane * P4;
  const float4* wp = w ? w + (long)(plane / C) * P4 : nullptr;
  double acc = 0.0;
  int i = threadIdx.x;
#pragma unroll 4
  for (; i + RT < P4; i += 2 * RT) {
    float4 a = xp[i], b = xp[i + RT];
    if (wp) {
      const float4 u = wp[i], v = wp[i + RT];
      acc += (((double)a.x * u.x + (double)a.y * u.y) + ((double)a.z * u.z + (double)a.w * u.w)) +
             (((double)b.x * v.x + (double)b.y * v.y) + ((double)b.z * v.z + (double)b.w * v.w));
    } else {
      acc += (((double)a.x + a.y) + ((double)a.z + a.w)) + (((double)b.x + b.y) + ((double)b.z + b.w));
    }
  }
  if (i < P4) {
    const float4 a = xp[i];
    const float4 u = wp ? wp[i] : make_float4(1.f, 1.f, 1.f, 1.f);
    acc += ((double)a.x * u.x + (double)a.y * u.y) + ((double)a.z * u.z + (double)a.w * u.w);
  }
  const double t = block_sum_d(acc, sh);
  if (threadIdx.x == 0) out[plane] = (float)t;
}

// out[n][p] = sum_c x[n][c][p] * (v ? v[n][c] : y[n][c][p])   (64 pixels x 4 channel groups per block)
__global__ void channel_dot_kernel(const float* __restrict__ x, const float* __restrict__ v,
                                   const float* __restrict__ y, float* __restrict__ out, int N, int C, int P) {
  __shared__ double part[4][64];
  const int lane = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int tiles = (P + 63) / 64;
  const int n = blockIdx.x / tiles;
  const int p = (blockIdx.x % tiles) * 64 + lane;
  double s = 0.0;
  if (p < P) {
    const float* xp = x + (long)n * C * P + p;
    const float* yp = y ? y + (long)n * C * P + p : nullptr;
    const float* vp = v ? v + (long)n * C : nullptr;
    // (the same summation order either way; unrolled so that eight channels' loads are in flight)
    if (vp) {
#pragma unroll 8
      for (int c = grp; c < C; c += 4) s += (double)xp[(long)c * P] * vp[c];
    } else {
#pragma unroll 8
      for (int c = grp; c < C; c += 4) s += (double)xp[(long)c * P] * yp[(long)c * P];
    }
  }
  part[grp][lane] = s;
  __syncthreads();
  if (grp == 0 && p < P) out[(long)n * P + p] = (float)(part[0][lane] + part[1][lane] + part[2][lane] + part[3][lane]);
}

// forward row terms: rowsum = qkbar/qn + Ns; c = 1/(rowsum qn); e = 1/rowsum; (ks = 1/kn separately)
__global__ void attn_fwd_rows_kernel(const float* __restrict__ qkbar, const float* __restrict__ qn, float* __restrict__ c,
                                     float* __restrict__ e, long n, int Ns) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float rs = qkbar[i] / qn[i] + (float)Ns;
  c[i] = 1.0f / (rs * qn[i]);
  e[i] = 1.0f / rs;
}

__global__ void reciprocal_kernel(const float* __restrict__ x, float* __restrict__ y, long n) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = 1.0f / x[i];
}

// backward row terms from r = sum_v dMV MV and DA = sum_v dMV vsum:
//   dqn = -(e/qn)(r Ns - DA);  nr = -r (epilogue offset);  cr = c r (for qtilde)
__global__ void attn_bwd_rows_kernel(const float* __restrict__ r, const float* __restrict__ DA,
                                     const float* __restrict__ qn, const float* __restrict__ c,
                                     const float* __restrict__ e, float* __restrict__ dqn, float* __restrict__ nr,
                                     float* __restrict__ cr, long n, int Ns) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  dqn[i] = -(e[i] / qn[i]) * (r[i] * (float)Ns - DA[i]);
  nr[i] = -r[i];
  cr[i] = c[i] * r[i];
}

// X[n][v][i] = dMV[n][v][i] * c[n][i]
__global__ void scale_cols_kernel(const float* __restrict__ x, const float* __restrict__ c, float* __restrict__ y,
                                  int N, int R, int P) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)N * R * P) return;
  const int p = (int)(idx % P);
  const long n = idx / ((long)R * P);
  y[idx] = x[idx] * c[n * P + p];
}

// dkn[n][j] = -ks_j^2 * sum_c K[c][j] (Y[c][j] - qt[c])
__global__ void attn_dkn_kernel(const float* __restrict__ K, const float* __restrict__ Y, const float* __restrict__ qt,
                                const float* __restrict__ ks, float* __restrict__ dkn, int N, int d, int Ns) {
  __shared__ double part[4][64];
  const int lane = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int tiles = (Ns + 63) / 64;
  const int n = blockIdx.x / tiles;
  const int j = (blockIdx.x % tiles) * 64 + lane;
  double s = 0.0;
  if (j < Ns) {
    const float* kp = K + (long)n * d * Ns + j;
    const float* yp = Y + (long)n * d * Ns + j;
    const float* qp = qt + (long)n * d;
#pragma unroll 8
    for (int c = grp; c < d; c += 4) s += (double)kp[(long)c * Ns] * ((double)yp[(long)c * Ns] - qp[c]);
  }
  part[grp][lane] = s;
  __syncthreads();
  if (grp == 0 && j < Ns) {
    const float k = ks[(long)n * Ns + j];
    dkn[(long)n * Ns + j] = -(float)(part[0][lane] + part[1][lane] + part[2][lane] + part[3][lane]) * k * k;
  }
}

}  // namespace

extern "C" {

int vst_plane_dot(const float* x, const float* w, float* out, int N, int C, int P, void* stream) {
  VST_CHECK_ARG(x && out && N > 0 && C > 0 && P > 0);
  if ((P & 3) == 0 && (((uintptr_t)x | (uintptr_t)w) & 15) == 0) {
    plane_dot_vec_kernel<<<N * C, RT, 0, (hipStream_t)stream>>>(reinterpret_cast<const float4*>(x),
                                                                reinterpret_cast<const float4*>(w), out, C, P / 4);
    return vst_launch_status();
  }
  plane_dot_kernel<<<N * C, RT, 0, (hipStream_t)stream>>>(x, w, out, C, P);
  return vst_launch_status();
}

int vst_channel_dot(const float* x, const float* v, const float* y, float* out, int N, int C, int P, void* stream) {
  VST_CHECK_ARG(x && out && (v || y) && N > 0 && C > 0 && P > 0);
  channel_dot_kernel<<<N * ceil_div(P, 64), 256, 0, (hipStream_t)stream>>>(x, v, y, out, N, C, P);
  return vst_launch_status();
}

int vst_attn_fwd_rows(const float* qkbar, const float* qn, float* c, float* e, long n, int Ns, void* stream) {
  VST_CHECK_ARG(qkbar && qn && c && e && n > 0 && Ns > 0);
  attn_fwd_rows_kernel<<<ceil_div(n, 256), 256, 0, (hipStream_t)stream>>>(qkbar, qn, c, e, n, Ns);
  return vst_launch_status();
}

int vst_reciprocal(const float* x, float* y, long n, void* stream) {
  VST_CHECK_ARG(x && y && n > 0);
  reciprocal_kernel<<<ceil_div(n, 256), 256, 0, (hipStream_t)stream>>>(x, y, n);
  return vst_launch_status();
}

int vst_attn_bwd_rows(const float* r, const float* DA, const float* qn, const float* c, const float* e, float* dqn,
                      float* nr, float* cr, long n, int Ns, void* stream) {
  VST_CHECK_ARG(r && DA && qn && c && e && dqn && nr && cr && n > 0);
  attn_bwd_rows_kernel<<<ceil_div(n, 256), 256, 0, (hipStream_t)stream>>>(r, DA, qn, c, e, dqn, nr, cr, n, Ns);
  return vst_launch_status();
}

int vst_scale_cols(const float* x, const float* c, float* y, int N, int R, int P, void* stream) {
  VST_CHECK_ARG(x && c && y && N > 0 && R > 0 && P > 0);
  scale_cols_kernel<<<ceil_div((long)N * R * P, 256), 256, 0, (hipStream_t)stream>>>(x, c, y, N, R, P);
  return vst_launch_status();
}

int vst_attn_dkn(const float* K, const float* Y, const float* qt, const float* ks, float* dkn, int N, int d, int Ns,
                 void* stream) {
  VST_CHECK_ARG(K && Y && qt && ks && dkn && N > 0 && d > 0 && Ns > 0);
  attn_dkn_kernel<<<N * ceil_div(Ns, 64), 256, 0, (hipStream_t)stream>>>(K, Y, qt, ks, dkn, N, d, Ns);
  return vst_launch_status();
}

}  // extern "C"

// ---------------------------------------------------------------------------------------------
// Cosine attention in linear form (vst/adaattn/attention.py LinearCosineAttnFn): the rank-1
// column/row updates and the column-normalisation adjoint around its d x 2dv GEMMs.
namespace {
// out[n][m][p] = (x[n][m][p] + alpha * u[n][m] * (v ? v[n][p] : 1)) * (w ? w[n][p] : 1)
__global__ void outer_axpy_kernel(const float* __restrict__ x, const float* __restrict__ u,
                                  const float* __restrict__ v, const float* __restrict__ w, float alpha, float* out,
                                  int M, long P, long total) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const long p = idx % P, nm = idx / P;
  const long n = nm / M;
  float a = x[idx];
  if (u) a += alpha * u[nm] * (v ? v[n * P + p] : 1.0f);
  if (w) a *= w[n * P + p];
  out[idx] = a;
}

// outer_axpy_kernel with the (n, m) row on blockIdx.y (P on x): the flat form's two 64-bit divisions
// per element made it VALU-bound (config 5: 18 launches, 213 us each)
__global__ __launch_bounds__(256) void outer_axpy_rows_kernel(const float* __restrict__ x, const float* __restrict__ u,
                                                              const float* __restrict__ v, const float* __restrict__ w,
                                                              float alpha, float* out, int M, long P) {
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  if (p >= P) return;
  const int nm = blockIdx.y, n = nm / M;
  const long idx = (long)nm * P + p;
  float a = x[idx];
  if (u) a += alpha * u[nm] * (v ? v[n * P + p] : 1.0f);
  if (w) a *= w[n * P + p];
  out[idx] = a;
}

// outer_axpy_rows_kernel, four consecutive pixels per thread (P % 4 == 0, 16-byte aligned rows): one
// float4 load / store per operand instead of four scalar accesses (the scalar form ran config 5's 15
// launches a step at ~3.2 TB/s); the same arithmetic per element
__global__ __launch_bounds__(256) void outer_axpy_rows4_kernel(const float* __restrict__ x, const float* __restrict__ u,
                                                               const float* __restrict__ v, const float* __restrict__ w,
                                                               float alpha, float* out, int M, long P) {
  const long p = ((long)blockIdx.x * 256 + threadIdx.x) * 4;
  if (p >= P) return;
  const int nm = blockIdx.y, n = nm / M;
  const long idx = (long)nm * P + p;
  float4 a = *reinterpret_cast<const float4*>(x + idx);
  if (u) {
    const float4 vv = v ? *reinterpret_cast<const float4*>(v + n * P + p) : make_float4(1.f, 1.f, 1.f, 1.f);
    const float au = alpha * u[nm];
    a.x += au * vv.x;
    a.y += au * vv.y;
    a.z += au * vv.z;
    a.w += au * vv.w;
  }
  if (w) {
    const float4 ww = *reinterpret_cast<const float4*>(w + n * P + p);
    a.x *= ww.x;
    a.y *= ww.y;
    a.z *= ww.z;
    a.w *= ww.w;
  }
  *reinterpret_cast<float4*>(out + idx) = a;
}

// out[i] = sum_{r < R} x[r * per + i]  (gradients of operands broadcast over R repeats of a batch)
__global__ void sum_repeats_kernel(const float* __restrict__ x, float* __restrict__ out, int R, long per) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= per) return;
  float s = 0.f;
  for (int r = 0; r < R; ++r) s += x[r * per + i];
  out[i] = s;
}

// out[n][c][p] = (dxh[n][c][p] - xh[n][c][p] * t[n][p]) * s[n][p]
// (adjoint of xh = x / ||x||_col with t = sum_c xh dxh and s = 1 / ||x||_col)
__global__ void normalize_cols_bwd_kernel(const float* __restrict__ xh, const float* __restrict__ dxh,
                                          const float* __restrict__ t, const float* __restrict__ s,
                                          float* __restrict__ out, int C, long P, long total) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const long p = idx % P, n = idx / P / C;
  const long np = n * P + p;
  out[idx] = (dxh[idx] - xh[idx] * t[np]) * s[np];
}

// normalize_cols_bwd_kernel with the (n, c) row on blockIdx.y
__global__ __launch_bounds__(256) void normalize_cols_bwd_rows_kernel(const float* __restrict__ xh,
                                                                      const float* __restrict__ dxh,
                                                                      const float* __restrict__ t,
                                                                      const float* __restrict__ s,
                                                                      float* __restrict__ out, int C, long P) {
  const long p = (long)blockIdx.x * 256 + threadIdx.x;
  if (p >= P) return;
  const int nc = blockIdx.y, n = nc / C;
  const long idx = (long)nc * P + p, np = (long)n * P + p;
  out[idx] = (dxh[idx] - xh[idx] * t[np]) * s[np];
}
// normalize_cols_bwd_rows_kernel, four consecutive pixels per thread (P % 4 == 0, aligned rows)
__global__ __launch_bounds__(256) void normalize_cols_bwd_rows4_kernel(const float* __restrict__ xh,
                                                                       const float* __restrict__ dxh,
                                                                       const float* __restrict__ t,
                                                                       const float* __restrict__ s,
                                                                       float* __restrict__ out, int C, long P) {
  const long p = ((long)blockIdx.x * 256 + threadIdx.x) * 4;
  if (p >= P) return;
  const int nc = blockIdx.y, n = nc / C;
  const long idx = (long)nc * P + p, np = (long)n * P + p;
  const float4 d = *reinterpret_cast<const float4*>(dxh + idx), h = *reinterpret_cast<const float4*>(xh + idx);
  const float4 tt = *reinterpret_cast<const float4*>(t + np), ss = *reinterpret_cast<const float4*>(s + np);
  *reinterpret_cast<float4*>(out + idx) =
      make_float4((d.x - h.x * tt.x) * ss.x, (d.y - h.y * tt.y) * ss.y, (d.z - h.z * tt.z) * ss.z, (d.w - h.w * tt.w) * ss.w);
}
}  // namespace

extern "C" int vst_outer_axpy(const float* x, const float* u, const float* v, const float* w, float alpha, float* out,
                              int N, int M, long P, void* stream) {
  VST_CHECK_ARG(x && out && N > 0 && M > 0 && P > 0);
  const long total = (long)N * M * P;
  if ((long)N * M <= 65535 && P >= 64 && P % 4 == 0 && al16(x, out, u ? v : nullptr, w)) {
    outer_axpy_rows4_kernel<<<dim3((unsigned)ceil_div(P / 4, 256), (unsigned)(N * M)), 256, 0, (hipStream_t)stream>>>(
        x, u, v, w, alpha, out, M, P);
    return vst_launch_status();
  }
  if ((long)N * M <= 65535 && P >= 64) {  // (short rows, e.g. _neg's P = 1, keep the flat form)
    outer_axpy_rows_kernel<<<dim3((unsigned)ceil_div(P, 256), (unsigned)(N * M)), 256, 0, (hipStream_t)stream>>>(
        x, u, v, w, alpha, out, M, P);
    return vst_launch_status();
  }
  outer_axpy_kernel<<<ceil_div(total, RT), RT, 0, (hipStream_t)stream>>>(x, u, v, w, alpha, out, M, P, total);
  return vst_launch_status();
}

extern "C" int vst_sum_repeats(const float* x, float* out, int R, long per, void* stream) {
  VST_CHECK_ARG(x && out && R > 0 && per > 0);
  sum_repeats_kernel<<<ceil_div(per, RT), RT, 0, (hipStream_t)stream>>>(x, out, R, per);
  return vst_launch_status();
}

extern "C" int vst_normalize_cols_bwd(const float* xh, const float* dxh, const float* t, const float* s, float* out,
                                      int N, int C, long P, void* stream) {
  VST_CHECK_ARG(xh && dxh && t && s && out && N > 0 && C > 0 && P > 0);
  const long total = (long)N * C * P;
  if ((long)N * C <= 65535 && P >= 64 && P % 4 == 0 && al16(xh, dxh, t, s, out)) {
    normalize_cols_bwd_rows4_kernel<<<dim3((unsigned)ceil_div(P / 4, 256), (unsigned)(N * C)), 256, 0,
                                      (hipStream_t)stream>>>(xh, dxh, t, s, out, C, P);
    return vst_launch_status();
  }
  if ((long)N * C <= 65535 && P >= 64) {
    normalize_cols_bwd_rows_kernel<<<dim3((unsigned)ceil_div(P, 256), (unsigned)(N * C)), 256, 0,
                                     (hipStream_t)stream>>>(xh, dxh, t, s, out, C, P);
    return vst_launch_status();
  }
  normalize_cols_bwd_kernel<<<ceil_div(total, RT), RT, 0, (hipStream_t)stream>>>(xh, dxh, t, s, out, C, P, total);
  return vst_launch_status();
}
