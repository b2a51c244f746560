#!/bin/bash
# AdaAttN GPU tests and the config-5 line twice with its kernel summary
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-aa}
timeout -k 10 900 python -u -m pytest tests/test_gpu_adaattn.py tests/test_gpu_adaattn_api.py tests/test_gpu_elementwise.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 4; }
tail -1 gpurun_out/${T}_tests.log
for i in 1 2; do
  timeout -k 10 600 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 20 --prof-steps 0 --no-cpu-baseline --no-vgg19 > gpurun_out/${T}_aa5_$i.json 2> gpurun_out/${T}_aa5_$i.err || exit 9
  python tools/show_bench.py gpurun_out/${T}_aa5_$i.json | head -1
done
VST_WGRAD_SIDE=0 VST_CONTENT_SIDE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof5 -o run -- \
  python3 bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 5 --warmup 2 --prof-steps 0 --no-cpu-baseline --no-vgg19 > gpurun_out/${T}_prof5.log 2>&1 || exit 11
python tools/prof_summary.py gpurun_out/${T}_prof5 7 > gpurun_out/${T}_c5_kernel_summary.txt 2>&1
rm -rf gpurun_out/${T}_prof5
grep -E "total|resize|up2|channel_dot|channel_norm|plane_|simloss" gpurun_out/${T}_c5_kernel_summary.txt
