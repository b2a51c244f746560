// On-device frame-pair preparation of the ReCoNet flow datasets:
// FlyingThings3D / Monkaa `__getitem__` (RC/datasets.py:114-155, 210-251) for a whole batch.
//
//   * frames and motion boundaries: `Image.open(..).resize(resolution, Image.BILINEAR)` is
//     Pillow's two-pass 8-bit resampler (horizontal then vertical, triangle filter widened by
//     the downscale factor, 22-bit fixed-point coefficients, uint8 rounding after each pass).
//     `pil_resize_kernel` reproduces it bit for bit, both passes fused per output pixel (the
//     intermediate row values are the same uint8s Pillow stores), with the epilogue of the
//     caller: toTensor255 (`b / 255 * 255` in fp32, RC/utilities.py:12-17) into planar fp32, or
//     the motion mask `1 - (toTensor(m) != 0)` multiplied into the flow mask (RC/datasets.py:138-144).
//     The coefficient tables are built once per (in, out) size on the host
//     (`vst_pil_bilinear_coeffs`, the same double arithmetic as Pillow's precompute_coeffs and
//     normalize_coeffs_8bpc) and cached on the device by the caller.
//   * flows: flowlib.readPFM (RC/flowlib.py:34-69) parses the header on the host
//     (`vst_pfm_read_header` / `vst_pfm_read`, raw bytes into a caller buffer); the flipud, the
//     big-endian byte swap, the `[:-1]` channel drop, `F.interpolate(bilinear,
//     align_corners=False)` and the per-channel rescale (RC/datasets.py:121-136, including the
//     reference's x-by-height / y-by-width factors, passed in as sx / sy) are one kernel.
// The mask itself is vst_flow_warp_mask (pool_warp.hip) between the two.
// Everything here is HBM-bound byte / fp32 streaming: one thread per output pixel, coalesced
// planar stores, the gathered source rows stay in L2 (a 960x540 RGB frame is 1.5 MB).
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "vst_common.h"
#include "vst_hip.h"

namespace {

constexpr int PT = 256;
constexpr int PIL_PRECISION_BITS = 32 - 8 - 2;  // Pillow Resample.c, 8 bits per channel

__device__ __forceinline__ int clip8(int v) {
  v >>= PIL_PRECISION_BITS;  // arithmetic shift, then Pillow's clip8 lookup (clamp to 0..255)
  return v < 0 ? 0 : (v > 255 ? 255 : v);
}

constexpr int HALF = 1 << (PIL_PRECISION_BITS - 1);

template <int C>
__device__ __forceinline__ void store_pixel(float* __restrict__ out, long n, long p, long HWo, const int (&acc)[C],
                                            int mode) {
  if (mode == 0) {
    float* o = out + n * C * HWo + p;
#pragma unroll
    for (int c = 0; c < C; ++c) o[c * HWo] = ((float)clip8(acc[c]) / 255.0f) * 255.0f;
  } else {
    if (clip8(acc[0]) != 0) out[n * HWo + p] = 0.f;
  }
}

// Output tile of one workgroup: TX columns x TY rows of one image (64x8 measured best of 64x{4,8,16,32}).  The source window it needs is
// staged in LDS (coalesced byte rows), the horizontal pass writes its uint8 rows to LDS, the
// vertical pass reads them: every source byte is read from HBM/L2 once per tile instead of once
// per tap of every output pixel.  Windows larger than the LDS budget (strong downscales) take
// the per-pixel path, block-uniformly.
constexpr int TX = 64, TY = 8;
constexpr int SRC_ROWS = 24, SRC_ROW_BYTES = 512;

// src: N x Hs x Ws x C uint8 (PIL's interleaved raster); hb/vb: {min, count} per output column /
// row (monotone in the output coordinate); hk/vk: fixed-point taps, hks/vks per output coordinate.
// mode 0: out = N x C x Ho x Wo fp32, (b / 255) * 255;
// mode 1 (C == 1): out = N x Ho x Wo flow mask, multiplied by the motion mask (b == 0).
template <int C, int KX, int KY>
__global__ __launch_bounds__(PT) void pil_resize_kernel(const uint8_t* __restrict__ src, float* __restrict__ out,
                                                        int Hs, int Ws, int Ho, int Wo, int tiles_x, int tiles_y,
                                                        const int* __restrict__ hb, const int* __restrict__ hk,
                                                        int hks, const int* __restrict__ vb,
                                                        const int* __restrict__ vk, int vks, int mode) {
  __shared__ __attribute__((aligned(16))) uint8_t s_src[SRC_ROWS * SRC_ROW_BYTES];
  __shared__ uint8_t s_h[SRC_ROWS * TX * C];
  static_assert(PT % TX == 0, "tile rows per pass");
  const int tiles = tiles_x * tiles_y;
  const long n = blockIdx.x / tiles;
  const int t = blockIdx.x - (int)n * tiles;
  const int ty0 = (t / tiles_x) * TY, tx0 = (t % tiles_x) * TX;
  const int txv = min(TX, Wo - tx0), tyv = min(TY, Ho - ty0);
  const long HWo = (long)Ho * Wo;
  const uint8_t* img = src + n * Hs * Ws * C;
  const int xs0 = hb[2 * tx0], xs1 = hb[2 * (tx0 + txv - 1)] + hb[2 * (tx0 + txv - 1) + 1];
  const int ys0 = vb[2 * ty0], ys1 = vb[2 * (ty0 + tyv - 1)] + vb[2 * (ty0 + tyv - 1) + 1];
  const int rw = (xs1 - xs0) * C, rh = ys1 - ys0;
  if (rw + 6 + KX * C > SRC_ROW_BYTES || rh + KY > SRC_ROWS) {  // per-pixel path (6: dword lead + tail)
    for (int i = threadIdx.x; i < txv * tyv; i += PT) {
      const int yy = ty0 + i / txv, xx = tx0 + i % txv;
      const int xmin = hb[2 * xx], xcnt = hb[2 * xx + 1], ymin = vb[2 * yy], ycnt = vb[2 * yy + 1];
      int acc[C];
#pragma unroll
      for (int c = 0; c < C; ++c) acc[c] = HALF;
      for (int y = 0; y < ycnt; ++y) {
        const uint8_t* row = img + ((long)(ymin + y) * Ws + xmin) * C;
        int h[C];
#pragma unroll
        for (int c = 0; c < C; ++c) h[c] = HALF;
        for (int x = 0; x < xcnt; ++x) {
          const int k = hk[(long)xx * hks + x];
#pragma unroll
          for (int c = 0; c < C; ++c) h[c] += (int)row[x * C + c] * k;
        }
        const int k = vk[(long)yy * vks + y];
#pragma unroll
        for (int c = 0; c < C; ++c) acc[c] += clip8(h[c]) * k;
      }
      store_pixel<C>(out, n, (long)yy * Wo + xx, HWo, acc, mode);
    }
    return;
  }
  // 1. source window -> LDS: aligned dword loads covering each window row (the row start is at
  //    any byte offset); the LDS row keeps that offset (lds_off) so the dwords land unchanged
  int lds_off = 0;
  {
    const long abs0 = (long)(img - (const uint8_t*)0);
    const int lead = (int)((abs0 + ((long)ys0 * Ws + xs0) * C) & 3);  // same for every row iff Ws*C % 4 == 0
    if (((Ws * C) & 3) == 0 && (abs0 & 3) == 0) {  // then no dword crosses a row end
      lds_off = lead;
      const int words = (lead + rw + 3) >> 2;
      for (int i = threadIdx.x; i < rh * words; i += PT) {
        const int r = i / words, w = i - r * words;
        const uint8_t* rowp = img + ((long)(ys0 + r) * Ws + xs0) * C - lead;
        reinterpret_cast<uint32_t*>(s_src + r * SRC_ROW_BYTES)[w] = reinterpret_cast<const uint32_t*>(rowp)[w];
      }
    } else {
      for (int i = threadIdx.x; i < rh * rw; i += PT) {
        const int r = i / rw, b = i - r * rw;
        s_src[r * SRC_ROW_BYTES + b] = img[((long)(ys0 + r) * Ws + xs0) * C + b];
      }
    }
  }
  __syncthreads();
  // 2. horizontal pass over every window row (Pillow's intermediate uint8 image).  With KX > 0
  //    the tap loop has a fixed trip count: taps past a column's count are zero in the table and
  //    read in-bounds LDS bytes (the fallback test keeps KX*C bytes of slack in each row).
  const int x = threadIdx.x % TX;
  if (x < txv) {
    const int xx = tx0 + x;
    const int xmin = hb[2 * xx] - xs0;
    const int nx = KX > 0 ? KX : hb[2 * xx + 1];
    const int* k = hk + (long)xx * hks;
    for (int r = threadIdx.x / TX; r < rh; r += PT / TX) {
      const uint8_t* row = s_src + r * SRC_ROW_BYTES + lds_off + xmin * C;
      int h[C];
#pragma unroll
      for (int c = 0; c < C; ++c) h[c] = HALF;
#pragma unroll 5
      for (int j = 0; j < nx; ++j) {
        const int kj = k[j];
#pragma unroll
        for (int c = 0; c < C; ++c) h[c] += (int)row[j * C + c] * kj;
      }
#pragma unroll
      for (int c = 0; c < C; ++c) s_h[(r * TX + x) * C + c] = (uint8_t)clip8(h[c]);
    }
  }
  __syncthreads();
  // 3. vertical pass, coalesced planar stores
  if (x < txv) {
    for (int y = threadIdx.x / TX; y < tyv; y += PT / TX) {
      const int yy = ty0 + y;
      const int ymin = vb[2 * yy] - ys0;
      const int ny = KY > 0 ? KY : vb[2 * yy + 1];
      const int* k = vk + (long)yy * vks;
      int acc[C];
#pragma unroll
      for (int c = 0; c < C; ++c) acc[c] = HALF;
#pragma unroll 5
      for (int j = 0; j < ny; ++j) {
        const int kj = k[j];
        const uint8_t* hv = s_h + ((ymin + j) * TX + x) * C;
#pragma unroll
        for (int c = 0; c < C; ++c) acc[c] += (int)hv[c] * kj;
      }
      store_pixel<C>(out, n, (long)yy * Wo + tx0 + x, HWo, acc, mode);
    }
  }
}

__device__ __forceinline__ float load_flow(const uint32_t* raw, long idx, int big_endian) {
  uint32_t u = raw[idx];
  if (big_endian) u = __builtin_bswap32(u);
  return __uint_as_float(u);
}

__device__ __forceinline__ void lin_axis(int d, int n_in, int n_out, int& i0, int& i1, float& l1) {
  // torch upsample_bilinear2d, align_corners=False: src = max((d + 0.5) * in / out - 0.5, 0)
  const float scale = (float)n_in / (float)n_out;
  float s = ((float)d + 0.5f) * scale - 0.5f;
  s = s < 0.f ? 0.f : s;
  i0 = (int)s;
  i0 = i0 > n_in - 1 ? n_in - 1 : i0;
  i1 = i0 < n_in - 1 ? i0 + 1 : i0;
  l1 = s - (float)i0;
}

// raw: N x Hs x Ws x Cr floats in file order (rows bottom-up: readPFM's flipud); out: N x 2 x Ho x Wo
__global__ void flow_prep_kernel(const uint32_t* __restrict__ raw, float* __restrict__ out, int N, int Hs, int Ws,
                                 int Cr, int big_endian, int Ho, int Wo, float sx, float sy) {
  const long HWo = (long)Ho * Wo;
  const long total = (long)N * HWo;
  for (long i = (long)blockIdx.x * PT + threadIdx.x; i < total; i += (long)gridDim.x * PT) {
    const long n = i / HWo;
    const long p = i - n * HWo;
    const int yy = (int)(p / Wo), xx = (int)(p - (long)yy * Wo);
    int y0, y1, x0, x1;
    float ly, lx;
    lin_axis(yy, Hs, Ho, y0, y1, ly);
    lin_axis(xx, Ws, Wo, x0, x1, lx);
    const long base = (long)n * Hs * Ws;
    const long r0 = base + (long)(Hs - 1 - y0) * Ws, r1 = base + (long)(Hs - 1 - y1) * Ws;
    float* o = out + n * 2 * HWo + p;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const float v00 = load_flow(raw, (r0 + x0) * Cr + c, big_endian);
      const float v01 = load_flow(raw, (r0 + x1) * Cr + c, big_endian);
      const float v10 = load_flow(raw, (r1 + x0) * Cr + c, big_endian);
      const float v11 = load_flow(raw, (r1 + x1) * Cr + c, big_endian);
      const float top = (1.f - lx) * v00 + lx * v01;
      const float bot = (1.f - lx) * v10 + lx * v11;
      o[c * HWo] = ((1.f - ly) * top + ly * bot) * (c == 0 ? sx : sy);
    }
  }
}

int grid_of(long work) {
  long b = (work + PT - 1) / PT;
  return (int)(b < 1 ? 1 : (b > 8192 ? 8192 : b));
}

// PFM header line reader (readline(): up to and including '\n')
int read_line(FILE* f, char* buf, int cap) {
  int n = 0;
  for (;;) {
    int ch = fgetc(f);
    if (ch == EOF) break;
    if (n < cap - 1) buf[n++] = (char)ch;
    if (ch == '\n') break;
  }
  buf[n] = 0;
  return n;
}

bool is_space(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\f' || c == '\v'; }

// readPFM's dimension line: re.match(r'^(\d+)\s(\d+)\s$', line)
bool parse_dims(const char* s, int* w, int* h) {
  const char* p = s;
  long a = 0, b = 0;
  if (*p < '0' || *p > '9') return false;
  while (*p >= '0' && *p <= '9') a = a * 10 + (*p++ - '0');
  if (!is_space(*p)) return false;
  ++p;
  if (*p < '0' || *p > '9') return false;
  while (*p >= '0' && *p <= '9') b = b * 10 + (*p++ - '0');
  if (!is_space(*p)) return false;
  ++p;
  if (!(*p == 0 || (p[0] == '\n' && p[1] == 0))) return false;  // `$` also matches before a final '\n'
  if (a > (1 << 30) || b > (1 << 30)) return false;
  *w = (int)a;
  *h = (int)b;
  return true;
}

}  // namespace

extern "C" {

int vst_pil_bilinear_coeffs(int in_size, int out_size, int* bounds, int* kk, int ksize_cap) {
#pragma clang fp contract(off)
  VST_CHECK_ARG(in_size > 0 && out_size > 0 && bounds && kk);
  const double in0 = 0.0, in1 = (double)(float)in_size;
  const double scale = (in1 - in0) / out_size;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 1.0 * filterscale;  // BILINEAR: support 1.0
  const int ksize = (int)ceil(support) * 2 + 1;
  if (ksize > ksize_cap) return ksize;  // caller re-allocates: a positive return is the needed ksize
  double* pre = (double*)malloc(sizeof(double) * (size_t)ksize);
  if (!pre) return VST_EINVAL;
  for (int xx = 0; xx < out_size; ++xx) {
    const double center = in0 + (xx + 0.5) * scale;
    const double ss = 1.0 / filterscale;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in_size) xmax = in_size;
    xmax -= xmin;
    double ww = 0.0;
    for (int x = 0; x < xmax; ++x) {
      double t = (x + xmin - center + 0.5) * ss;
      if (t < 0.0) t = -t;
      const double w = t < 1.0 ? 1.0 - t : 0.0;
      pre[x] = w;
      ww += w;
    }
    for (int x = 0; x < xmax; ++x)
      if (ww != 0.0) pre[x] /= ww;
    for (int x = xmax; x < ksize; ++x) pre[x] = 0.0;
    for (int x = 0; x < ksize; ++x) {
      const double v = pre[x] * (1 << PIL_PRECISION_BITS);
      kk[(long)xx * ksize + x] = v < 0 ? (int)(-0.5 + v) : (int)(0.5 + v);
    }
    bounds[2 * xx] = xmin;
    bounds[2 * xx + 1] = xmax;
  }
  free(pre);
  return VST_OK;
}

int vst_pil_resize_u8(const void* src, float* out, int N, int Hs, int Ws, int C, int Ho, int Wo, const void* hbounds,
                      const void* hk, int hks, const void* vbounds, const void* vk, int vks, int mode, void* stream) {
  VST_CHECK_ARG(src && out && hbounds && hk && vbounds && vk && N >= 0 && Hs > 0 && Ws > 0 && Ho > 0 && Wo > 0);
  VST_CHECK_ARG(C >= 1 && C <= 4 && hks > 0 && vks > 0 && (mode == 0 || (mode == 1 && C == 1)));
  if ((long)N * Ho * Wo == 0) return VST_OK;
  const int tiles_x = (Wo + TX - 1) / TX, tiles_y = (Ho + TY - 1) / TY;
  const long blocks = (long)N * tiles_x * tiles_y;
  VST_CHECK_ARG(blocks < (1L << 31));
  const int* hbi = (const int*)hbounds;
  const int* hki = (const int*)hk;
  const int* vbi = (const int*)vbounds;
  const int* vki = (const int*)vk;
  hipStream_t st = (hipStream_t)stream;
#define VST_PIL_LAUNCH(CC, KXX, KYY)                                                                            \
  pil_resize_kernel<CC, KXX, KYY><<<(unsigned)blocks, PT, 0, st>>>((const uint8_t*)src, out, Hs, Ws, Ho, Wo, tiles_x, \
                                                                   tiles_y, hbi, hki, hks, vbi, vki, vks, mode)
  const int kfix = (hks == 5 && vks == 5) ? 5 : ((hks == 3 && vks == 3) ? 3 : 0);
  if (C == 3) {
    if (kfix == 5) VST_PIL_LAUNCH(3, 5, 5);
    else if (kfix == 3) VST_PIL_LAUNCH(3, 3, 3);
    else VST_PIL_LAUNCH(3, 0, 0);
  } else if (C == 1) {
    if (kfix == 5) VST_PIL_LAUNCH(1, 5, 5);
    else if (kfix == 3) VST_PIL_LAUNCH(1, 3, 3);
    else VST_PIL_LAUNCH(1, 0, 0);
  } else {
    return VST_EUNSUPPORTED;
  }
  return vst_launch_status();
}

int vst_flow_prep(const void* raw, float* out, int N, int Hs, int Ws, int Cr, int big_endian, int Ho, int Wo,
                  float sx, float sy, void* stream) {
  VST_CHECK_ARG(raw && out && N >= 0 && Hs > 0 && Ws > 0 && Cr >= 2 && Ho > 0 && Wo > 0);
  const long total = (long)N * Ho * Wo;
  if (total == 0) return VST_OK;
  flow_prep_kernel<<<grid_of(total), PT, 0, (hipStream_t)stream>>>((const uint32_t*)raw, out, N, Hs, Ws, Cr,
                                                                    big_endian, Ho, Wo, sx, sy);
  return vst_launch_status();
}

int vst_pfm_read_header(const char* path, int* width, int* height, int* channels, int* big_endian, int* offset,
                        float* scale) {
  VST_CHECK_ARG(path && width && height && channels && big_endian && offset && scale);
  FILE* f = fopen(path, "rb");
  if (!f) return VST_EIO;
  char line[256];
  read_line(f, line, sizeof line);
  int n = (int)strlen(line);
  while (n > 0 && is_space(line[n - 1])) line[--n] = 0;  // .rstrip()
  int rc = VST_OK;
  if (strcmp(line, "PF") == 0) {
    *channels = 3;
  } else if (strcmp(line, "Pf") == 0) {
    *channels = 1;
  } else {
    rc = VST_EPFM_MAGIC;
  }
  if (rc == VST_OK) {
    read_line(f, line, sizeof line);
    if (!parse_dims(line, width, height)) rc = VST_EPFM_HEADER;
  }
  if (rc == VST_OK) {
    read_line(f, line, sizeof line);
    char* end = nullptr;
    double s = strtod(line, &end);
    while (end && *end && is_space(*end)) ++end;
    if (end == line || (end && *end)) {
      rc = VST_EPFM_HEADER;  // float() of the scale line raised in the reference
    } else {
      *big_endian = s < 0 ? 0 : 1;
      *scale = (float)(s < 0 ? -s : s);
      long pos = ftell(f);
      fseek(f, 0, SEEK_END);
      long end_pos = ftell(f);
      long want = (long)(*width) * (*height) * (*channels) * 4;
      if (end_pos - pos != want) rc = VST_EPFM_SIZE;  // np.reshape(data, shape) raised
      *offset = (int)pos;
    }
  }
  fclose(f);
  return rc;
}

int vst_pfm_read(const char* path, void* dst, long bytes, int offset) {
  VST_CHECK_ARG(path && dst && bytes >= 0 && offset >= 0);
  FILE* f = fopen(path, "rb");
  if (!f) return VST_EIO;
  int rc = VST_OK;
  if (fseek(f, offset, SEEK_SET) != 0 || (long)fread(dst, 1, (size_t)bytes, f) != bytes) rc = VST_EPFM_SIZE;
  fclose(f);
  return rc;
}

}  // extern "C"
