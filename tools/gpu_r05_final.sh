#!/bin/bash
# round-5 final build: config-3 A/B/A/B of the residual skip accumulation (VST_SKIP_ACCUM on / off),
# then the closing measurement (tools/gpu_r05_close.sh: GPU suite + smoke, bench lines, rocprofv3)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 60 --no-cpu-baseline --no-vgg19 > gpurun_out/skip_on_$i.json 2>/dev/null || exit 2
  python tools/show_bench.py gpurun_out/skip_on_$i.json 2>/dev/null | head -1
  VST_SKIP_ACCUM=0 timeout -k 10 300 python bench.py --steps 60 --no-cpu-baseline --no-vgg19 > gpurun_out/skip_off_$i.json 2>/dev/null || exit 3
  python tools/show_bench.py gpurun_out/skip_off_$i.json 2>/dev/null | head -1
done
bash tools/gpu_r05_close.sh
