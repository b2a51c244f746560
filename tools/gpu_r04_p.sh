#!/bin/bash
# content targets on the side stream (VST_CONTENT_SIDE=1, default) vs in line: GPU suite, then
# config-3 steps A/B/A/B on one box
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04p_tests.log 2>&1 || { tail -30 gpurun_out/r04p_tests.log; exit 3; }
tail -1 gpurun_out/r04p_tests.log
for i in 1 2; do
  for S in 0 1; do
    VST_CONTENT_SIDE=$S timeout -k 10 300 python bench.py --steps 60 --prof-steps 0 --no-cpu-baseline --no-vgg19 > gpurun_out/r04p_c3_${S}_${i}.json 2>/dev/null || exit 7
    echo "content_side=$S"; python tools/show_bench.py gpurun_out/r04p_c3_${S}_${i}.json | head -1
  done
done
echo done
