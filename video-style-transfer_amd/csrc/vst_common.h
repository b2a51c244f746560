// Shared helpers for the gfx950 (CDNA4) kernels of libvst_hip.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "vst_hip.h"

#define VST_OK 0
#define VST_EINVAL (-1)
#define VST_EUNSUPPORTED (-2)
#define VST_EIO (-3)
#define VST_EPFM_MAGIC (-4)
#define VST_EPFM_HEADER (-5)
#define VST_EPFM_SIZE (-6)

#define VST_CHECK_ARG(cond) \
  do {                      \
    if (!(cond)) return VST_EINVAL; \
  } while (0)

static inline int vst_launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? VST_OK : (int)e;
}

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// Unsigned division by a runtime constant (Granlund-Montgomery, 32-bit): n / d == umulhi(n, mul) >> shift
// valid for n < 2^31.
struct FastDiv {
  uint32_t d, mul, shift;
};

static inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t s = 0;
  while ((1ull << s) < d) ++s;
  f.shift = s;
  f.mul = (uint32_t)((((1ull << 32) * ((1ull << s) - d)) / d) + 1);
  return f;
}

__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  uint32_t t = __umulhi(n, f.mul);
  return (t + n) >> f.shift;
}

// 64-lane wave reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

static inline int ceil_div(long a, long b) { return (int)((a + b - 1) / b); }

// GEMM arithmetic mode: a per-call argument of every GEMM / pack entry (vst_hip.h VST_GEMM_*, plus
// the VST_GEMM_KBLOCK K-order flag); the library keeps no mode state
static inline int vst_mode_arith(int mode) { return mode & 7; }
static inline bool vst_mode_ok(int mode) {
  const int a = vst_mode_arith(mode);
  return (mode & ~(VST_GEMM_KBLOCK | VST_GEMM_PERTAP | VST_GEMM_NOSPLIT | 7)) == 0 &&
         (a == VST_GEMM_F32 || a == VST_GEMM_BF16X3 || a == VST_GEMM_BF16 || a == VST_GEMM_BF16X6 ||
          a == VST_GEMM_F16);
}
// packed-A layout of a mode: 0 fp32, 1 hi+lo bf16 (bf16x3, bf16), 2 hi+mid+lo bf16 (bf16x6), 3 fp16
// (hi slot only, same 64-B blocks as 1); bit 4: channel-blocked K order (kblocked)
static inline int apack_split(int mode) {
  const int a = vst_mode_arith(mode);
  const int s = a == VST_GEMM_F32 ? 0 : (a == VST_GEMM_BF16X6 ? 2 : (a == VST_GEMM_F16 ? 3 : 1));
  return s | ((mode & VST_GEMM_KBLOCK) ? 16 : 0);
}

// K order of a conv GEMM (the packed A rows and the kernel's B walk must agree).  With
// VST_GEMM_KBLOCK and a channel count inside k that is a multiple of 16, k runs channel-block
// major, tap minor -- k = (c/16)*(16*T) + tap*16 + c%16 -- so the T taps of one 16-channel block
// are consecutive k-tiles and their B gathers re-read the same few source rows back to back
// (L2-resident: ~3 rows x 16 channels per block) instead of one tap sweeping all channels before
// the next (a reuse distance of Cs x 3 rows per block, past the XCD's 4 MB L2 at 64 blocks per
// XCD).  Otherwise k is tap-major, k = tap*Ck + c.
__host__ __device__ inline bool kblocked(int Ck, int kb) { return kb && Ck % 16 == 0; }
__host__ __device__ inline void kdecode(int k, int Ck, int T, int& tap, int& c, int kb) {
  if (kblocked(Ck, kb)) {
    const int g = k / (16 * T), r = k - g * 16 * T;
    tap = r >> 4;
    c = g * 16 + (r & 15);
  } else {
    tap = k / Ck;
    c = k - tap * Ck;
  }
}

// Packed GEMM A operand ("weights"), k-tiles of 16: element (k, m) lives at
//   ((k/16) * Mpad + m) * 16 + (k%2) * 8 + (k%16)/2
// so one MFMA lane's 8 values of a k-tile (k = 2s + hi, s = 0..7, for v_mfma_f32_32x32x2_f32)
// are contiguous: two ds_read_b128 per 32-row fragment, and a k-tile of BM rows is one
// contiguous BM*16-float block in global memory.
__host__ __device__ inline long apack_index(int k, int m, int Mpad) {
  return ((long)(k >> 4) * Mpad + m) * 16 + (k & 1) * 8 + ((k & 15) >> 1);
}

// ---- bf16 MFMA arithmetic ------------------------------------------------------------------
// VST_GEMM_F32:    exact fp32 MFMA (v_mfma_f32_32x32x2_f32, 64 cycles per 32x32x2).
// VST_GEMM_BF16X3: fp32 operands split x = hi + lo into two round-to-nearest bf16 values and
//   multiplied as lo*hi + hi*lo + hi*hi on v_mfma_f32_32x32x16_bf16 (fp32 accumulate).  The
//   dropped lo*lo term and the rounding of lo bound the per-product error by ~2^-16 relative
//   (fp32 MFMA: 2^-24), at 3 x 32 cycles per 32x32x16 instead of 8 x 64: 5.3x the MFMA rate.
// VST_GEMM_BF16:   hi*hi only (one bf16 MFMA, ~2^-8 relative per product): the reduced-precision
//   MFMA path of BASELINE config 5 (bf16 keeps fp32's exponent range: no loss scaling).
// Every packed A operand is written in the layout of the mode passed to its pack call, so a pack
// is only valid for GEMM calls with that same mode.
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// two floats -> packed bf16 pair (round to nearest even), element 0 in the low half
__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  f32x2 v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}

// two floats -> packed fp16 pair (round to nearest even; |x| > 65504 -> inf), element 0 low
__device__ __forceinline__ uint32_t pack_f16x2(float a, float b) {
  f32x2 v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, f16x2_t));
}

// split (a, b) into packed hi and lo bf16 pairs: a = hi_a + lo_a (+ ~2^-17 relative)
__device__ __forceinline__ void split_bf16x2(float a, float b, uint32_t& hi, uint32_t& lo) {
  hi = pack_bf16x2(a, b);
  const float ha = __uint_as_float(hi << 16), hb = __uint_as_float(hi & 0xffff0000u);
  lo = pack_bf16x2(a - ha, b - hb);
}

// the two-slot operand pair of a GEMM precision: PREC 1 / 2 bf16 hi + lo (2 uses only hi), PREC 4
// the fp16 value in the hi slot (no lo term)
template <int PREC>
__device__ __forceinline__ void split2(float a, float b, uint32_t& hi, uint32_t& lo) {
  if constexpr (PREC == 4) {
    hi = pack_f16x2(a, b);
    lo = 0u;
  } else {
    split_bf16x2(a, b, hi, lo);
  }
}

// three-way split: a = hi + mid + lo, residual ~2^-25 relative (bf16x6 mode)
__device__ __forceinline__ void split3_bf16x2(float a, float b, uint32_t& hi, uint32_t& mid, uint32_t& lo) {
  hi = pack_bf16x2(a, b);
  const float ra = a - __uint_as_float(hi << 16), rb = b - __uint_as_float(hi & 0xffff0000u);
  mid = pack_bf16x2(ra, rb);
  lo = pack_bf16x2(ra - __uint_as_float(mid << 16), rb - __uint_as_float(mid & 0xffff0000u));
}

// Split packed A layout: the 16 k of one (k-tile, row m) block (64 bytes, the same footprint as
// the fp32 block) hold 16 hi bf16 in natural k order, then the 16 lo bf16: an MFMA lane (k =
// 8h + j) reads its hi and lo fragments with one ds_read_b128 each.  split == 2 (bf16x6): 96-byte
// blocks [hi][mid][lo] (the pack buffer is 1.5x the fp32 one).
__device__ __forceinline__ void apack_store(float* out, int k, int m, int Mpad, float v, int split) {
  split &= 3;
  if (!split) {
    out[apack_index(k, m, Mpad)] = v;
    return;
  }
  const int aw = split == 2 ? 24 : 16;
  unsigned short* u = reinterpret_cast<unsigned short*>(out + ((long)(k >> 4) * Mpad + m) * aw);
  if (split == 3) {  // fp16: [f16 k0..15][unused]
    u[k & 15] = (unsigned short)(pack_f16x2(v, 0.f) & 0xffffu);
    u[16 + (k & 15)] = 0;
    return;
  }
  const uint32_t h = pack_bf16x2(v, 0.f) & 0xffffu;
  const float r = v - __uint_as_float(h << 16);
  const uint32_t md = pack_bf16x2(r, 0.f) & 0xffffu;
  u[k & 15] = (unsigned short)h;
  if (split == 2) {
    u[16 + (k & 15)] = (unsigned short)md;
    u[32 + (k & 15)] = (unsigned short)(pack_bf16x2(r - __uint_as_float(md << 16), 0.f) & 0xffffu);
  } else {
    u[16 + (k & 15)] = (unsigned short)md;
  }
}

// One 16-deep k-tile of a wave's TM x TN block of 32x32 accumulators from bf16 LDS rows
// ([hi k0..15][lo k0..15][pad], 20 dwords): rows a0 + 32i + lane&31 of A, b0 + 32j + lane&31 of B.
template <int TM, int TN, int PREC, int LS>
__device__ __forceinline__ void mfma_bf16_ktile(f32x16 (&acc)[TM][TN], float (*A)[LS], float (*B)[LS], int a0,
                                                int b0, int lane) {
  const int r = lane & 31, h = lane >> 5;
  if constexpr (PREC == 4) {  // fp16 rows: [f16 k0..15][unused]
    f16x8_t af[TM], bf[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const f16x8_t*>(&A[a0 + i * 32 + r][4 * h]);
#pragma unroll
    for (int j = 0; j < TN; ++j) bf[j] = *reinterpret_cast<const f16x8_t*>(&B[b0 + j * 32 + r][4 * h]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
    return;
  }
  bf16x8_t ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const float* p = &A[a0 + i * 32 + r][4 * h];
    ah[i] = *reinterpret_cast<const bf16x8_t*>(p);
    if (PREC == 1) al[i] = *reinterpret_cast<const bf16x8_t*>(p + 8);
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const float* p = &B[b0 + j * 32 + r][4 * h];
    bh[j] = *reinterpret_cast<const bf16x8_t*>(p);
    if (PREC == 1) bl[j] = *reinterpret_cast<const bf16x8_t*>(p + 8);
  }
  // every fragment read is issued before the first MFMA: the chain then waits on counted
  // lgkmcnt instead of re-reading into one register between MFMAs
  __builtin_amdgcn_sched_barrier(0);
  if (PREC == 1) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
}

// bf16x6: six products lo*hi + mid*mid + hi*lo + mid*hi + hi*mid + hi*hi (smallest first) of
// three-way splits; the dropped terms are below 2^-24 of |a b| (fp32-like error)
template <int TM, int TN, int LS>
__device__ __forceinline__ void mfma_bf16x6_ktile(f32x16 (&acc)[TM][TN], float (*A)[LS], float (*B)[LS], int a0,
                                                  int b0, int lane) {
  const int r = lane & 31, h = lane >> 5;
  bf16x8_t ah[TM], am[TM], al[TM], bh[TN], bm[TN], bl[TN];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const float* p = &A[a0 + i * 32 + r][4 * h];
    ah[i] = *reinterpret_cast<const bf16x8_t*>(p);
    am[i] = *reinterpret_cast<const bf16x8_t*>(p + 8);
    al[i] = *reinterpret_cast<const bf16x8_t*>(p + 16);
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const float* p = &B[b0 + j * 32 + r][4 * h];
    bh[j] = *reinterpret_cast<const bf16x8_t*>(p);
    bm[j] = *reinterpret_cast<const bf16x8_t*>(p + 8);
    bl[j] = *reinterpret_cast<const bf16x8_t*>(p + 16);
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      f32x16 c = acc[i][j];
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[i], bm[j], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am[i], bh[j], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bm[j], c, 0, 0, 0);
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], c, 0, 0, 0);
    }
}

// bf16x6 k-tile with the A fragments already in registers (hi, mid, lo per 32-row fragment, loaded
// straight from the packed weights) and B from LDS
template <int TM, int TN, int LS>
__device__ __forceinline__ void mfma_bf16x6_ktile_ra(f32x16 (&acc)[TM][TN], const bf16x8_t (&ar)[TM][3],
                                                     float (*B)[LS], int b0, int lane, int jstride = 32) {
  const int r = lane & 31, h = lane >> 5;
  bf16x8_t bh[TN], bm[TN], bl[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const float* p = &B[b0 + j * jstride + r][4 * h];
    bh[j] = *reinterpret_cast<const bf16x8_t*>(p);
    bm[j] = *reinterpret_cast<const bf16x8_t*>(p + 8);
    bl[j] = *reinterpret_cast<const bf16x8_t*>(p + 16);
  }
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      f32x16 c = acc[i][j];
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ar[i][2], bh[j], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ar[i][1], bm[j], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ar[i][0], bl[j], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ar[i][1], bh[j], c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ar[i][0], bm[j], c, 0, 0, 0);
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ar[i][0], bh[j], c, 0, 0, 0);
    }
}

// single-product (bf16 hi*hi, or fp16) k-tile with the A fragments in registers (loaded straight
// from the packed weights: the hi piece of each 32-row fragment) and B from LDS
template <int TM, int TN, int PREC, int LS>
__device__ __forceinline__ void mfma_single_ktile_ra(f32x16 (&acc)[TM][TN], const bf16x8_t (&ar)[TM][3],
                                                     float (*B)[LS], int b0, int lane, int jstride = 32) {
  const int r = lane & 31, h = lane >> 5;
  bf16x8_t bh[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) bh[j] = *reinterpret_cast<const bf16x8_t*>(&B[b0 + j * jstride + r][4 * h]);
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      if constexpr (PREC == 4)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8_t, ar[i][0]),
                                                           __builtin_bit_cast(f16x8_t, bh[j]), acc[i][j], 0, 0, 0);
      else
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ar[i][0], bh[j], acc[i][j], 0, 0, 0);
    }
}

// A wave-uniform pointer forced into SGPRs: a buffer descriptor built from a pointer the compiler
// keeps in VGPRs (e.g. after a 64-bit VALU multiply) makes every buffer load a waterfall loop.
__device__ __forceinline__ void* uniform_ptr(const void* p) {
  const uint64_t v = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (void*)(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(base), (short)0, (int)__builtin_amdgcn_readfirstlane(bytes),
                                           0x00020000);
}

// Dispatch hands workgroups to the 8 XCDs round-robin (bid % 8, a speed assumption only):
// remap so each XCD gets one contiguous range of the work order, which keeps blocks that share
// operands (neighbouring pixel tiles, all tiles of one split-K chunk) on one L2.
__device__ __forceinline__ int xcd_remap(int bid, int G) {
  const int q = G >> 3, r = G & 7, xcd = bid & 7, loc = bid >> 3;
  return xcd < r ? xcd * (q + 1) + loc : r * (q + 1) + (xcd - r) * q + loc;
}
