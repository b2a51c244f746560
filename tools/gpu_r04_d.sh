#!/bin/bash
# halo block shapes: default (M64 2x2, M128 4x1, M192 3x2) vs v1 (2x1, 4x1, 6x1) vs v2 (2x2 one
# buffer, 4x2, 3x2), bf16x6 and fp16, vs the per-tap kernel
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
L=video-style-transfer_amd/vst
BENCH_ONLY=vgg,res BENCH_GEMM_MODES=19,20 timeout -k 10 300 python tools/gemm_bench.py $L/libvst_hip.so $L/variants/libv1.so $L/variants/libv2.so > gpurun_out/r04d_gemm.txt 2>&1 || { cat gpurun_out/r04d_gemm.txt; exit 3; }
cat gpurun_out/r04d_gemm.txt
BENCH_ONLY=vgg,res BENCH_GEMM_MODES=51,52 timeout -k 10 300 python tools/gemm_bench.py $L/libvst_hip.so > gpurun_out/r04d_gemm_pertap.txt 2>&1 || exit 4
cat gpurun_out/r04d_gemm_pertap.txt
echo done
