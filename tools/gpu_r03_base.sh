#!/bin/bash
# round-3 opening measurement of HEAD on one box: headline line and the config-5 shape line
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --no-cpu-baseline --no-vgg19 > gpurun_out/r03_base_c3.json 2> gpurun_out/r03_base_c3.err || exit 5
timeout -k 10 300 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 20 --prof-steps 3 --no-cpu-baseline --no-vgg19 > gpurun_out/r03_base_c5.json 2> gpurun_out/r03_base_c5.err || exit 6
echo done
