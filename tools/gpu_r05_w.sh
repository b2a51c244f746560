#!/bin/bash
# GPU suite after the scaled-resize ABI (ConvReluInterpolate, any scale) + config 3 / 4 lines
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05w_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05w_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r05w_tests.log | head -30; exit 2; }
timeout -k 10 300 python bench.py --steps 60 --no-cpu-baseline --no-vgg19 > gpurun_out/r05w_c3.json 2>/dev/null || exit 5
python tools/show_bench.py gpurun_out/r05w_c3.json | head -3
timeout -k 10 400 python bench.py --model adaattn --steps 40 --no-cpu-baseline --no-vgg19 > gpurun_out/r05w_aa4.json 2>/dev/null || exit 6
python tools/show_bench.py gpurun_out/r05w_aa4.json | head -3
