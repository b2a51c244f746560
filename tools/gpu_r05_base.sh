#!/bin/bash
# round-5 baseline on a fresh box: the headline line (short), config-5 line, no cpu baseline
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 60 --no-cpu-baseline --no-vgg19 > gpurun_out/r05_base_c3.json 2> gpurun_out/r05_base_c3.err || exit 6
python tools/show_bench.py gpurun_out/r05_base_c3.json | head -2
timeout -k 10 400 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 10 --prof-steps 2 --no-cpu-baseline --no-vgg19 > gpurun_out/r05_base_aa5.json 2> gpurun_out/r05_base_aa5.err || exit 9
python tools/show_bench.py gpurun_out/r05_base_aa5.json | head -1
echo done
