#!/bin/bash
# bf16x3 on the 128-row per-tap tile instead of the 256-row one (config 5's loss-network 1x1 GEMMs):
# AdaAttN GPU tests, the config-5 line and its rocprofv3 kernel summary
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_adaattn.py tests/test_gpu_parity.py > gpurun_out/t128_tests.log 2>&1 || { tail -30 gpurun_out/t128_tests.log; exit 4; }
tail -1 gpurun_out/t128_tests.log
timeout -k 10 400 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 20 --prof-steps 3 --no-cpu-baseline --no-vgg19 > gpurun_out/t128_aa5.json 2>/dev/null || exit 5
python tools/show_bench.py gpurun_out/t128_aa5.json 2>/dev/null | head -2
VST_WGRAD_SIDE=0 VST_CONTENT_SIDE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/t128_prof5 -o run -- \
  python3 bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 5 --warmup 2 --prof-steps 0 --no-cpu-baseline --no-vgg19 > gpurun_out/t128_prof5.log 2>&1 || exit 6
python tools/prof_summary.py gpurun_out/t128_prof5 7 -shapes > gpurun_out/t128_c5_summary.txt 2>&1
rm -rf gpurun_out/t128_prof5
head -1 gpurun_out/t128_c5_summary.txt
grep "conv_gemm_kernel<2, 2, 2, 2, true, false, 3, 1\|conv_gemm_kernel<2, 4, 2, 2, true, false, 2, 1\|family" gpurun_out/t128_c5_summary.txt
echo done
