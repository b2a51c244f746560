#!/bin/bash
# rocprofv3 of the config-3 step, round-4 tree vs HEAD on one box (side streams off), per-kernel diff
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_streams.py tests/test_gpu_parity.py -x -q -k "warp or bitwise" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05l_tests.log 2>&1 || { tail -30 gpurun_out/r05l_tests.log; exit 2; }
tail -1 gpurun_out/r05l_tests.log
export VST_WGRAD_SIDE=0 VST_CONTENT_SIDE=0
(cd variants/r4 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ../../gpurun_out/r05l_p4 -o run -- \
  python3 bench.py --steps 10 --warmup 2 --prof-steps 0 --no-cpu-baseline --no-vgg19 > ../../gpurun_out/r05l_p4.log 2>&1) || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05l_p5 -o run -- \
  python3 bench.py --steps 10 --warmup 2 --prof-steps 0 --no-cpu-baseline --no-vgg19 > gpurun_out/r05l_p5.log 2>&1 || exit 4
python tools/prof_diff.py gpurun_out/r05l_p4 gpurun_out/r05l_p5 12
unset VST_WGRAD_SIDE VST_CONTENT_SIDE
(cd variants/r4 && timeout -k 10 300 python bench.py --steps 60 --no-cpu-baseline --no-vgg19 > ../../gpurun_out/r05l_r4.json 2>/dev/null) || exit 5
python tools/show_bench.py gpurun_out/r05l_r4.json | head -1
timeout -k 10 300 python bench.py --steps 60 --no-cpu-baseline --no-vgg19 > gpurun_out/r05l_head.json 2>/dev/null || exit 6
python tools/show_bench.py gpurun_out/r05l_head.json | head -1
VST_WGRAD_SIDE=0 VST_CONTENT_SIDE=0 timeout -k 10 300 python bench.py --steps 60 --no-cpu-baseline --no-vgg19 > gpurun_out/r05l_head_noside.json 2>/dev/null || exit 6
python tools/show_bench.py gpurun_out/r05l_head_noside.json | head -1
(cd variants/r4 && VST_WGRAD_SIDE=0 VST_CONTENT_SIDE=0 timeout -k 10 300 python bench.py --steps 60 --no-cpu-baseline --no-vgg19 > ../../gpurun_out/r05l_r4_noside.json 2>/dev/null) || exit 5
python tools/show_bench.py gpurun_out/r05l_r4_noside.json | head -1
rm -rf gpurun_out/r05l_p4 gpurun_out/r05l_p5
