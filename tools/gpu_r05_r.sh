#!/bin/bash
# round-5 kernel summaries (config 3 and config 5, side streams off as bench.py's instrumented steps)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05r_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r05r_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r05r_tests.log | head -30; exit 2; }
VST_WGRAD_SIDE=0 VST_CONTENT_SIDE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05_prof3 -o run -- \
  python3 bench.py --steps 10 --warmup 2 --prof-steps 0 --no-cpu-baseline --no-vgg19 > gpurun_out/r05_prof3.log 2>&1 || exit 10
python tools/prof_summary.py gpurun_out/r05_prof3 12 -shapes > gpurun_out/r05_kernel_summary.txt 2>&1
cp gpurun_out/r05_prof3/run_kernel_stats.csv gpurun_out/r05_kernel_stats.csv
VST_WGRAD_SIDE=0 VST_CONTENT_SIDE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05_prof5 -o run -- \
  python3 bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 5 --warmup 2 --prof-steps 0 --no-cpu-baseline --no-vgg19 > gpurun_out/r05_prof5.log 2>&1 || exit 11
python tools/prof_summary.py gpurun_out/r05_prof5 7 -shapes > gpurun_out/r05_adaattn_c5_kernel_summary.txt 2>&1
cp gpurun_out/r05_prof5/run_kernel_stats.csv gpurun_out/r05_adaattn_c5_kernel_stats.csv
rm -rf gpurun_out/r05_prof3 gpurun_out/r05_prof5
head -60 gpurun_out/r05_kernel_summary.txt
bash tools/gpu_r05_pmc.sh
