// Shared helpers for the gfx950 (CDNA4) kernels of libvst_hip.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define VST_OK 0
#define VST_EINVAL (-1)
#define VST_EUNSUPPORTED (-2)

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

// Packed GEMM A operand ("weights"), k-tiles of 16: element (k, m) lives at
//   ((k/16) * Mpad + m) * 16 + (k%2) * 8 + (k%16)/2
// so one MFMA lane's 8 values of a k-tile (k = 2s + hi, s = 0..7, for v_mfma_f32_32x32x2_f32)
// are contiguous: two ds_read_b128 per 32-row fragment, and a k-tile of BM rows is one
// contiguous BM*16-float block in global memory.
__host__ __device__ inline long apack_index(int k, int m, int Mpad) {
  return ((long)(k >> 4) * Mpad + m) * 16 + (k & 1) * 8 + ((k & 15) >> 1);
}
