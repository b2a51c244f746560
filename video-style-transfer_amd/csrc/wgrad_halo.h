// Halo weight gradient of 3x3 stride-1 pad-1 convolutions (wgrad_halo.hip), used by vst_conv_wgrad.
#pragma once
#include <hip/hip_runtime.h>


struct WhParams {
  const float* a;  // dY [N][M][H][W]
  const float* x;  // X  [N][Cs][H][W]
  float* slab;     // [NB][Mpad][9*Cs]
  int M, Mpad, J, Cs, H, W, N;
  int nchunk, rch, NB;  // row chunks of rch rows; NB blocks (slabs) per (channel block, M tile) pair
};

struct WhPlan {
  int Mpad, nchunk, rch, NB;
};

bool wgrad_halo_ok(int M, int Cs, int H, int W, int KH, int KW, int stride, int pad, int up, int gmode, int mode);
WhPlan wgrad_halo_plan(int N, int M, int Cs, int H, int W, int mode);
long wgrad_halo_slab_floats(int N, int Cs, const WhPlan& p);
int wgrad_halo_launch(const WhPlan& p, const float* dy, const float* x, float* slab, int N, int M, int Cs, int H,
                      int W, int gmode, int mode, hipStream_t st);
