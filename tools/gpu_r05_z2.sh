#!/bin/bash
# halo weight gradient strips for the single products: 16 (previous) / 32 / 64 columns
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
L=video-style-transfer_amd/vst
BENCH_MODES=4,2 BENCH_ONLY=aadec timeout -k 10 300 python tools/wgrad_bench.py $L/libvst_base.so $L/libvst_hip.so $L/libvst_k4.so > gpurun_out/r05z2_wb.log 2>&1 || { tail -20 gpurun_out/r05z2_wb.log; exit 3; }
cat gpurun_out/r05z2_wb.log
