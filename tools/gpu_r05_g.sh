#!/bin/bash
# A/B/A/B on one box: the round-4 tree (variants/r4, its own library) vs HEAD, config 3 headline
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  (cd variants/r4 && timeout -k 10 300 python bench.py --steps 60 --no-cpu-baseline --no-vgg19 > ../../gpurun_out/r05g_r4_$i.json 2>/dev/null) || exit 5
  python tools/show_bench.py gpurun_out/r05g_r4_$i.json | head -1
  timeout -k 10 300 python bench.py --steps 60 --no-cpu-baseline --no-vgg19 > gpurun_out/r05g_head_$i.json 2> gpurun_out/r05g_head.err || exit 6
  python tools/show_bench.py gpurun_out/r05g_head_$i.json | head -1
done
