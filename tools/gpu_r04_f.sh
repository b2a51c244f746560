#!/bin/bash
# residual-layer (M = 192) halo block shapes vs the per-tap kernel, and the residual dgrad's
# padded-grid path vs core (halo) + ring
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
L=video-style-transfer_amd/vst
BENCH_ONLY=res BENCH_GEMM_MODES=19,20 timeout -k 10 300 python tools/gemm_bench.py $L/libvst_hip.so $L/variants/libr1.so $L/variants/libr2.so $L/variants/libr3.so $L/variants/libr4.so $L/variants/libr5.so > gpurun_out/r04f_res.txt 2>&1 || { cat gpurun_out/r04f_res.txt; exit 3; }
cat gpurun_out/r04f_res.txt
timeout -k 10 300 python tools/dgrad_bench.py > gpurun_out/r04f_dgrad.txt 2>&1 || { cat gpurun_out/r04f_dgrad.txt; exit 4; }
cat gpurun_out/r04f_dgrad.txt
echo done
