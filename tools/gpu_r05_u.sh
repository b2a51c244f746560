#!/bin/bash
# halo weight gradient: single-product occupancy 3 / 5 / 6 waves per SIMD (variant builds), config-5 decoder shapes
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
L=video-style-transfer_amd/vst
BENCH_MODES=4,2 BENCH_ONLY=aadec timeout -k 10 300 python tools/wgrad_bench.py $L/libvst_w3.so $L/libvst_w5.so $L/libvst_hip.so > gpurun_out/r05u_wb.log 2>&1 || { tail -20 gpurun_out/r05u_wb.log; exit 2; }
cat gpurun_out/r05u_wb.log
timeout -k 10 400 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 10 --prof-steps 2 --no-cpu-baseline --no-vgg19 > gpurun_out/r05u_aa5.json 2> gpurun_out/r05u_aa5.err || exit 9
python tools/show_bench.py gpurun_out/r05u_aa5.json | head -3
