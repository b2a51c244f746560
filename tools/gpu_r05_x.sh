#!/bin/bash
# 192-row halo tiles: 2x2 one-buffer (shipped) vs two weight-row fragments per wave (3x1, 3x2, 3x2 one buffer)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
L=video-style-transfer_amd/vst
BENCH_GEMM_MODES=19,20 BENCH_ONLY=res,deconv2,conv2 timeout -k 10 300 python tools/gemm_bench.py $L/libvst_hip.so $L/libvst_x13.so $L/libvst_x14.so $L/libvst_x15.so > gpurun_out/r05x_gb.log 2>&1 || { tail -20 gpurun_out/r05x_gb.log; exit 2; }
cat gpurun_out/r05x_gb.log
