#!/bin/bash
# single-product weight-gradient variants: base (KD 2, 128x128 blocks) / k4 (4 k-tiles per stage) /
# n (128x256 blocks) / nk4 (both), on the config-5 decoder shapes (fp16) and the residual shape
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
L=video-style-transfer_amd/vst
BENCH_ONLY=aadec,res BENCH_GEMM_MODE=4 timeout -k 10 400 python tools/wgrad_bench.py $L/libvst_hip.so $L/variants/libk4.so $L/variants/libn.so $L/variants/libnk4.so > gpurun_out/r04i_wgrad_f16.txt 2>&1 || { cat gpurun_out/r04i_wgrad_f16.txt; exit 3; }
cat gpurun_out/r04i_wgrad_f16.txt
BENCH_ONLY=aadec,res BENCH_GEMM_MODE=3 timeout -k 10 400 python tools/wgrad_bench.py $L/libvst_hip.so > gpurun_out/r04i_wgrad_bf16x6.txt 2>&1 || exit 4
cat gpurun_out/r04i_wgrad_bf16x6.txt
echo done
