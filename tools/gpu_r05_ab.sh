#!/bin/bash
# config 3: the round-5 closing build (variants/r5c, beed821) vs HEAD on one box, A/B/A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  (cd variants/r5c && timeout -k 10 300 python bench.py --steps 60 --no-cpu-baseline --no-vgg19 > ../../gpurun_out/r05ab_c_$i.json 2>/dev/null) || exit 5
  python tools/show_bench.py gpurun_out/r05ab_c_$i.json | head -1
  timeout -k 10 300 python bench.py --steps 60 --no-cpu-baseline --no-vgg19 > gpurun_out/r05ab_h_$i.json 2>/dev/null || exit 6
  python tools/show_bench.py gpurun_out/r05ab_h_$i.json | head -1
done
