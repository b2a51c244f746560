#!/bin/bash
# GPU suite with VST_HALVES=1, then the config-5 step under VST_HALVES 1 / 0 (twice)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
VST_HALVES=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/val_tests.log 2>&1 || exit 4
B5="--model adaattn --batch 8 --height 512 --width 1024 --steps 10 --warmup 3 --prof-steps 0 --no-cpu-baseline --no-vgg19"
for r in 1 2; do
  for h in 1 0; do
    VST_HALVES=$h timeout -k 10 300 python bench.py $B5 > gpurun_out/val5_h${h}_$r.json 2> gpurun_out/val5_h${h}_$r.err || exit 5
  done
done
echo ok
