#!/bin/bash
# final build check: GPU suite + smoke(), and one config-5 / headline step timing
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/last_tests.log 2>&1 || { tail -40 gpurun_out/last_tests.log; exit 4; }
tail -2 gpurun_out/last_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 5
timeout -k 10 300 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 10 --warmup 3 --prof-steps 1 --no-cpu-baseline --no-vgg19 > gpurun_out/last_c5.json 2>/dev/null || exit 6
python tools/show_bench.py gpurun_out/last_c5.json | head -1
timeout -k 10 300 python bench.py --steps 100 --prof-steps 1 --no-cpu-baseline --no-vgg19 > gpurun_out/last_c3.json 2>/dev/null || exit 7
python tools/show_bench.py gpurun_out/last_c3.json | head -1
echo done
