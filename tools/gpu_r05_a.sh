#!/bin/bash
# round 5: GPU suite (caller-owned split-K workspace, deterministic warp / similarity adjoints, side
# stream bitwise test) + smoke + short headline and config-5 lines
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05a_tests.log 2>&1 || { tail -60 gpurun_out/r05a_tests.log; exit 4; }
tail -2 gpurun_out/r05a_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 5
timeout -k 10 400 python bench.py --steps 60 --no-cpu-baseline --no-vgg19 > gpurun_out/r05a_c3.json 2> gpurun_out/r05a_c3.err || exit 6
python tools/show_bench.py gpurun_out/r05a_c3.json | head -2
timeout -k 10 400 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 10 --prof-steps 2 --no-cpu-baseline --no-vgg19 > gpurun_out/r05a_aa5.json 2> gpurun_out/r05a_aa5.err || exit 9
python tools/show_bench.py gpurun_out/r05a_aa5.json | head -1
echo done
