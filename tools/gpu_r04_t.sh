#!/bin/bash
# the first conv's weight gradient on the main stream, beside the previous layer's on the side stream
# (VST_FIRST_INLINE=1, default) vs on the side stream after it (0): parity + DP tests, config-3 steps
# A/B/A/B on one box
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ddp.py tests/test_gpu_scaler.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04t_tests.log 2>&1 || { tail -30 gpurun_out/r04t_tests.log; exit 3; }
tail -1 gpurun_out/r04t_tests.log
for i in 1 2; do
  for S in 0 1; do
    VST_FIRST_INLINE=$S timeout -k 10 300 python bench.py --steps 60 --prof-steps 0 --no-cpu-baseline --no-vgg19 > gpurun_out/r04t_c3_${S}_$i.json 2>/dev/null || exit 7
    echo "first_inline=$S"; python tools/show_bench.py gpurun_out/r04t_c3_${S}_$i.json | head -1
  done
done
echo done
