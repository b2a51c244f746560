#!/bin/bash
# round 4: halo-tiled 3x3 conv kernel -- bitwise vs the per-tap kernel, the GPU suite, smoke(), and
# the headline / config-5 step timings
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_halo.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04b_halo.log 2>&1 || { tail -40 gpurun_out/r04b_halo.log; exit 3; }
tail -2 gpurun_out/r04b_halo.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04b_tests.log 2>&1 || { tail -40 gpurun_out/r04b_tests.log; exit 4; }
tail -2 gpurun_out/r04b_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 5
timeout -k 10 300 python bench.py --steps 100 --prof-steps 1 --no-cpu-baseline --no-vgg19 > gpurun_out/r04b_c3.json 2>/dev/null || exit 7
python tools/show_bench.py gpurun_out/r04b_c3.json | head -1
timeout -k 10 300 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 10 --warmup 3 --prof-steps 1 --no-cpu-baseline --no-vgg19 > gpurun_out/r04b_c5.json 2>/dev/null || exit 6
python tools/show_bench.py gpurun_out/r04b_c5.json | head -1
echo done
