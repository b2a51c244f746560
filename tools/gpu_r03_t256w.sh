#!/bin/bash
# A/B of the 256x256 single-product conv tile (VST_T256W) on the config-5 step, one box
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for i in 1 2; do
for w in 0 1; do
  VST_T256W=$w timeout -k 10 300 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 10 --prof-steps 2 --no-cpu-baseline --no-vgg19 > gpurun_out/r03_t256w_${w}_$i.json 2>gpurun_out/r03_t256w_${w}_$i.err || exit 5
done; done
VST_T256W=1 timeout -k 10 600 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 5 --prof-steps 2 --cpu-steps 1 --cpu-warmup 0 --no-vgg19 > gpurun_out/r03_t256w_par.json 2>gpurun_out/r03_t256w_par.err || exit 6
echo done
