// Host-side entry of the thin-output-channel weight gradient (thin.hip) for vst_conv_wgrad
// (wgrad_gemm.hip); the data gradient is the C ABI's vst_conv_dgrad_thin.
#pragma once
#include <hip/hip_runtime.h>

bool vst_thin_wgrad_ok(int Cout, int Cin, int Hs, int Ws, int Ho, int Wo, int KH, int KW, int gmode, int stride,
                       int pad, int up, int mode);
long vst_thin_wgrad_floats(int N, int Cout, int Cin, int Hs, int Ws);
int vst_thin_wgrad_launch(const float* dy, const float* x, float* dw, float* slab, int N, int Cin, int H, int W,
                          int Cout, int gmode, int accumulate, hipStream_t st);
