#!/bin/bash
# usage: gpu_r03c_ab.sh old.so -- GPU suite on the in-tree build, then config 5 and config 3 steps
# A/B/A/B: old library (stale build id allowed) vs the in-tree one
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OLD=$1
L=video-style-transfer_amd/vst/libvst_hip.so
cp $L /tmp/libvst_new.so || exit 2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 4; }
tail -2 gpurun_out/ab_tests.log
for i in 1 2; do
  for v in old new; do
    if [ $v = old ]; then cp $OLD $L; else cp /tmp/libvst_new.so $L; fi
    VST_ALLOW_STALE_BUILD=1 timeout -k 10 300 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 10 --warmup 3 --prof-steps 1 --no-cpu-baseline --no-vgg19 > gpurun_out/ab5_${v}_$i.json 2>/dev/null || { cp /tmp/libvst_new.so $L; exit 5; }
    python -c "import json;d=json.load(open('gpurun_out/ab5_${v}_$i.json'));print('c5 $v', round(d['ms_per_step'],2))"
  done
done
for i in 1 2; do
  for v in old new; do
    if [ $v = old ]; then cp $OLD $L; else cp /tmp/libvst_new.so $L; fi
    VST_ALLOW_STALE_BUILD=1 timeout -k 10 300 python bench.py --steps 60 --prof-steps 1 --no-cpu-baseline --no-vgg19 > gpurun_out/ab3_${v}_$i.json 2>/dev/null || { cp /tmp/libvst_new.so $L; exit 6; }
    python -c "import json;d=json.load(open('gpurun_out/ab3_${v}_$i.json'));print('c3 $v', round(d['ms_per_step'],2), round(d['value'],1))"
  done
done
cp /tmp/libvst_new.so $L
echo done
