// Calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for the access widths the library's
// kernels use (MI355X_MICROARCH.md: "calibrate on a known byte count in your own access pattern").
// Each kernel streams exactly BYTES bytes once (1 GiB >> 256 MiB Infinity Cache).
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr long NF = 1L << 28;  // 268M floats = 1 GiB

__global__ void rd_dword(const float* __restrict__ x, float* out) {
  float s = 0.f;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < NF; i += (long)gridDim.x * blockDim.x) s += x[i];
  if (s == 12345.f) out[0] = s;
}
__global__ void rd_dwordx4(const float4* __restrict__ x, float* out) {
  float s = 0.f;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < NF / 4; i += (long)gridDim.x * blockDim.x) {
    float4 v = x[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 12345.f) out[0] = s;
}
__global__ void rd_buffer_dword(const float* __restrict__ x, float* out) {
  // 1 GiB in 4 chunks of 256 MiB per buffer resource (num_records is 32-bit)
  float s = 0.f;
  for (int c = 0; c < 4; ++c) {
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)(x + (long)c * (NF / 4)), 0, (int)(NF), 0x00020000);
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < NF / 4; i += (long)gridDim.x * blockDim.x)
      s += __builtin_amdgcn_raw_buffer_load_b32(r, (int)(i * 4), 0, 0);
  }
  if (s == 12345.f) out[0] = s;
}
__global__ void wr_dword(float* __restrict__ y) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < NF; i += (long)gridDim.x * blockDim.x) y[i] = 1.f;
}
__global__ void wr_dwordx4(float4* __restrict__ y) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < NF / 4; i += (long)gridDim.x * blockDim.x)
    y[i] = make_float4(1.f, 2.f, 3.f, 4.f);
}

int main() {
  float *x, *y, *o;
  if (hipMalloc(&x, NF * 4) || hipMalloc(&y, NF * 4) || hipMalloc(&o, 64)) return 1;
  (void)hipMemset(x, 0, NF * 4);
  const int G = 256 * 16, B = 256;
  for (int rep = 0; rep < 2; ++rep) {
    rd_dword<<<G, B>>>(x, o);
    rd_dwordx4<<<G, B>>>((const float4*)x, o);
    rd_buffer_dword<<<G, B>>>(x, o);
    wr_dword<<<G, B>>>(y);
    wr_dwordx4<<<G, B>>>((float4*)y);
  }
  if (hipDeviceSynchronize()) return 2;
  printf("calibration done: %ld bytes per kernel\n", NF * 4);
  return 0;
}
