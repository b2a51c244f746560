#!/bin/bash
# the split-K build (bf16x6 / bf16 launches only): full GPU suite, config-4 and config-3 steps
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04o_tests.log 2>&1 || { tail -30 gpurun_out/r04o_tests.log; exit 3; }
tail -1 gpurun_out/r04o_tests.log
timeout -k 10 300 python bench.py --model adaattn --steps 30 --no-cpu-baseline --no-vgg19 > gpurun_out/r04o_c4.json 2>/dev/null || exit 6
python tools/show_bench.py gpurun_out/r04o_c4.json | head -1
timeout -k 10 300 python bench.py --steps 60 --no-cpu-baseline --no-vgg19 > gpurun_out/r04o_c3.json 2>/dev/null || exit 7
python tools/show_bench.py gpurun_out/r04o_c3.json | head -1
echo done
