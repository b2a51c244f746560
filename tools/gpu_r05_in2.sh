#!/bin/bash
# large-plane InstanceNorm kernels: threads per block and blocks per CU (MALL reuse of the second pass)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/norm_bench.py variants/r5c/video-style-transfer_amd/vst/libvst_hip.so variants/in_n512.so variants/in_n1024.so variants/in_n1024p.so variants/in_n512p.so > gpurun_out/in2_bench.log 2>&1 || { tail -30 gpurun_out/in2_bench.log; exit 5; }
cat gpurun_out/in2_bench.log
