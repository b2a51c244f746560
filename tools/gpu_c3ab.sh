#!/bin/bash
# halo / parity GPU tests, the config-3 line twice, the config-3 kernel summary and the config-5 line
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-c3}
timeout -k 10 600 python -u -m pytest tests/test_gpu_halo.py tests/test_gpu_parity.py tests/test_gpu_wgrad_halo.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 4; }
tail -1 gpurun_out/${T}_tests.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 60 --no-cpu-baseline --no-vgg19 > gpurun_out/${T}_c3_$i.json 2>/dev/null || exit 6
  python tools/show_bench.py gpurun_out/${T}_c3_$i.json | head -1
done
VST_WGRAD_SIDE=0 VST_CONTENT_SIDE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof3 -o run -- \
  python3 bench.py --steps 10 --warmup 2 --prof-steps 0 --no-cpu-baseline --no-vgg19 > gpurun_out/${T}_prof3.log 2>&1 || exit 10
python tools/prof_summary.py gpurun_out/${T}_prof3 12 -shapes > gpurun_out/${T}_c3_kernel_summary.txt 2>&1
rm -rf gpurun_out/${T}_prof3
head -3 gpurun_out/${T}_c3_kernel_summary.txt; grep -E "in_fwd|in_bwd" gpurun_out/${T}_c3_kernel_summary.txt
timeout -k 10 600 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 20 --prof-steps 0 --no-cpu-baseline --no-vgg19 > gpurun_out/${T}_aa5.json 2> gpurun_out/${T}_aa5.err || exit 9
python tools/show_bench.py gpurun_out/${T}_aa5.json | head -1
