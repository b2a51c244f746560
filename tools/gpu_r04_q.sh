#!/bin/bash
# AdaAttN local-feature targets on the side stream (VST_CONTENT_SIDE=1) vs in line: AdaAttN GPU tests,
# then config-5 and config-4 steps A/B/A/B on one box
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_adaattn.py tests/test_gpu_ddp.py tests/test_gpu_adaattn_api.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04q_tests.log 2>&1 || { tail -30 gpurun_out/r04q_tests.log; exit 3; }
tail -1 gpurun_out/r04q_tests.log
for i in 1 2; do
  for S in 0 1; do
    VST_CONTENT_SIDE=$S timeout -k 10 300 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 10 --warmup 3 --prof-steps 0 --no-cpu-baseline --no-vgg19 > gpurun_out/r04q_c5_${S}_${i}.json 2>/dev/null || exit 6
    echo "c5 content_side=$S"; python tools/show_bench.py gpurun_out/r04q_c5_${S}_${i}.json | head -1
    VST_CONTENT_SIDE=$S timeout -k 10 300 python bench.py --model adaattn --steps 30 --prof-steps 0 --no-cpu-baseline --no-vgg19 > gpurun_out/r04q_c4_${S}_${i}.json 2>/dev/null || exit 7
    echo "c4 content_side=$S"; python tools/show_bench.py gpurun_out/r04q_c4_${S}_${i}.json | head -1
  done
done
echo done
