#!/bin/bash
# new elementwise tests + config-5 / config-3 rocprofv3 kernel summaries of the in-tree build
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_elementwise.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ew_tests.log 2>&1 || { tail -40 gpurun_out/ew_tests.log; exit 4; }
tail -2 gpurun_out/ew_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c_prof5 -o run -- \
  python3 bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 5 --prof-steps 2 --no-cpu-baseline --no-vgg19 > gpurun_out/c_prof5.log 2>&1 || exit 10
python tools/prof_summary.py gpurun_out/c_prof5 12 > gpurun_out/c_adaattn_c5_kernel_summary.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c_prof3 -o run -- \
  python3 bench.py --steps 20 --prof-steps 5 --no-cpu-baseline --no-vgg19 > gpurun_out/c_prof3.log 2>&1 || exit 9
python tools/prof_summary.py gpurun_out/c_prof3 30 > gpurun_out/c_kernel_summary.txt 2>&1
echo done
