#!/bin/bash
# usage: gpu_ab_lib.sh variant.so -- A/B of a library build against the in-tree one: weight-gradient
# microbench (both libraries in one process), the GPU suite on the in-tree build, then the headline
# step (no CPU baseline / VGG19 sub-metric) in the order main / variant / main / variant
cd $GRAFT_REPO_ROOT
V=$1
L=video-style-transfer_amd/vst/libvst_hip.so
cp $L /tmp/libvst_main.so || exit 2
timeout -k 10 300 python tools/wgrad_bench.py $L $V > gpurun_out/ab_wgrad.log 2>&1 || exit 3
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_tests.log 2>&1 || exit 4
i=0
for lib in /tmp/libvst_main.so $V /tmp/libvst_main.so $V; do
  i=$((i+1))
  cp $lib $L || exit 2
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-vgg19 --steps 100 > gpurun_out/ab_bench_$i.json 2>/dev/null || { cp /tmp/libvst_main.so $L; exit 5; }
done
cp /tmp/libvst_main.so $L
echo ok
