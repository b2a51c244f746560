#!/bin/bash
# usage: gpu_r03b_ab.sh variant.so -- the GPU suite on the in-tree build, then the headline step and
# the config-5 step in the order main / variant / main / variant (variant loaded with
# VST_ALLOW_STALE_BUILD=1: it is built from other sources on purpose); config 5 also with the in-tree
# build's VST_ADS=0 (LDS-A single-product conv tiles) and VST_WKD2=0 (one k-tile per wgrad stage)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
V=$1
L=video-style-transfer_amd/vst/libvst_hip.so
cp $L /tmp/libvst_main.so || exit 2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_tests.log 2>&1 || exit 4
B5="--model adaattn --batch 8 --height 512 --width 1024 --steps 10 --warmup 3 --prof-steps 0 --no-cpu-baseline --no-vgg19"
i=0
for lib in /tmp/libvst_main.so $V /tmp/libvst_main.so $V; do
  i=$((i+1))
  cp $lib $L || exit 2
  VST_ALLOW_STALE_BUILD=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-vgg19 --steps 100 --prof-steps 0 > gpurun_out/ab3_$i.json 2>gpurun_out/ab3_$i.err || { cp /tmp/libvst_main.so $L; exit 5; }
  VST_ALLOW_STALE_BUILD=1 timeout -k 10 300 python bench.py $B5 > gpurun_out/ab5_$i.json 2> gpurun_out/ab5_$i.err || { cp /tmp/libvst_main.so $L; exit 6; }
  if [ $lib = /tmp/libvst_main.so ]; then
    VST_ADS=0 timeout -k 10 300 python bench.py $B5 > gpurun_out/ab5n_$i.json 2> gpurun_out/ab5n_$i.err || { cp /tmp/libvst_main.so $L; exit 7; }
    VST_WKD2=0 timeout -k 10 300 python bench.py $B5 > gpurun_out/ab5w_$i.json 2> gpurun_out/ab5w_$i.err || { cp /tmp/libvst_main.so $L; exit 8; }
  fi
done
cp /tmp/libvst_main.so $L
echo ok
