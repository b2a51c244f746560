#!/bin/bash
# round 5: halo weight gradient -- its tests, the GPU suite, the wgrad microbench (halo vs row-tiled),
# and short headline / config-5 lines
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_wgrad_halo.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05b_wh.log 2>&1 || { tail -40 gpurun_out/r05b_wh.log; exit 3; }
tail -1 gpurun_out/r05b_wh.log
BENCH_MODES=3,35,4,36 timeout -k 10 300 python tools/wgrad_bench.py > gpurun_out/r05b_wbench.txt 2>&1 || { cat gpurun_out/r05b_wbench.txt; exit 7; }
cat gpurun_out/r05b_wbench.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05b_tests.log 2>&1 || { tail -60 gpurun_out/r05b_tests.log; exit 4; }
tail -2 gpurun_out/r05b_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 5
timeout -k 10 400 python bench.py --steps 60 --no-cpu-baseline --no-vgg19 > gpurun_out/r05b_c3.json 2> gpurun_out/r05b_c3.err || exit 6
python tools/show_bench.py gpurun_out/r05b_c3.json | head -3
timeout -k 10 400 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 10 --prof-steps 2 --no-cpu-baseline --no-vgg19 > gpurun_out/r05b_aa5.json 2> gpurun_out/r05b_aa5.err || exit 9
python tools/show_bench.py gpurun_out/r05b_aa5.json | head -3
echo done
