#!/bin/bash
# halo weight gradient, 32-column strips for the single products: tests, A/B vs the previous build, config 5
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_wgrad_halo.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05z_wh.log 2>&1 || { tail -30 gpurun_out/r05z_wh.log; exit 2; }
tail -1 gpurun_out/r05z_wh.log
L=video-style-transfer_amd/vst
BENCH_MODES=4,2,3 BENCH_ONLY=aadec,res timeout -k 10 300 python tools/wgrad_bench.py $L/libvst_base.so $L/libvst_hip.so > gpurun_out/r05z_wb.log 2>&1 || { tail -20 gpurun_out/r05z_wb.log; exit 3; }
cat gpurun_out/r05z_wb.log
for i in 1 2; do
timeout -k 10 400 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 10 --prof-steps 2 --no-cpu-baseline --no-vgg19 > gpurun_out/r05z_aa5.json 2> gpurun_out/r05z_aa5.err || exit 9
python tools/show_bench.py gpurun_out/r05z_aa5.json | head -3
done
