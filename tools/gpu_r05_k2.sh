#!/bin/bash
# halo weight gradient under bf16x6: 16- vs 32-column strips (and the row-tiled kernel, mode | PERTAP)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
L=video-style-transfer_amd/vst
BENCH_MODES=3,35 BENCH_ONLY=aadec1,aadec3,aadec5,aadec7,res timeout -k 10 300 python tools/wgrad_bench.py $L/libvst_base.so $L/libvst_k2.so > gpurun_out/r05k2_wb.log 2>&1 || { tail -20 gpurun_out/r05k2_wb.log; exit 3; }
cat gpurun_out/r05k2_wb.log
