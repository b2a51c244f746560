#!/bin/bash
# round-6 thin-channel kernels: their GPU tests, the config-5 / config-3 lines and the config-5 kernel summary
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-thin}
timeout -k 10 600 python -u -m pytest tests/test_gpu_wgrad_halo.py tests/test_gpu_halo.py tests/test_gpu_parity.py tests/test_gpu_adaattn.py tests/test_gpu_abi.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 4; }
tail -2 gpurun_out/${T}_tests.log
timeout -k 10 600 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 20 --prof-steps 0 --no-cpu-baseline --no-vgg19 > gpurun_out/${T}_aa5.json 2> gpurun_out/${T}_aa5.err || exit 9
python tools/show_bench.py gpurun_out/${T}_aa5.json | head -1
VST_WGRAD_SIDE=0 VST_CONTENT_SIDE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof5 -o run -- \
  python3 bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 5 --warmup 2 --prof-steps 0 --no-cpu-baseline --no-vgg19 > gpurun_out/${T}_prof5.log 2>&1 || exit 11
python tools/prof_summary.py gpurun_out/${T}_prof5 7 -shapes > gpurun_out/${T}_c5_kernel_summary.txt 2>&1
rm -rf gpurun_out/${T}_prof5
head -30 gpurun_out/${T}_c5_kernel_summary.txt
grep -E "thin|cin3|conv_gemm_kernel<2, 1, 1, 4|wgrad2_kernel<1, 1, 4" gpurun_out/${T}_c5_kernel_summary.txt
timeout -k 10 300 python bench.py --steps 60 --no-cpu-baseline --no-vgg19 > gpurun_out/${T}_c3.json 2>/dev/null || exit 6
python tools/show_bench.py gpurun_out/${T}_c3.json | head -1
