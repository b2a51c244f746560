#!/bin/bash
# single-product halo stages: KC = 2 (default) vs 1 vs 4 channel blocks per stage (fp16, VGG / decoder
# shapes), the halo bitwise tests on the KC = 2 build; weight gradients on the side stream
# (VST_WGRAD_SIDE=1, default) vs in series: parity + DP tests, config-5 and config-3 steps both ways
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
L=video-style-transfer_amd/vst
timeout -k 10 900 python -u -m pytest tests/test_gpu_halo.py tests/test_gpu_elementwise.py tests/test_gpu_parity.py tests/test_gpu_ddp.py tests/test_gpu_scaler.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04k_tests.log 2>&1 || { tail -30 gpurun_out/r04k_tests.log; exit 3; }
tail -1 gpurun_out/r04k_tests.log
BENCH_ONLY=vgg,res BENCH_GEMM_MODES=20 timeout -k 10 300 python tools/gemm_bench.py $L/libvst_hip.so $L/variants/libkc1.so $L/variants/libkc4.so > gpurun_out/r04k_gemm.txt 2>&1 || { cat gpurun_out/r04k_gemm.txt; exit 4; }
cat gpurun_out/r04k_gemm.txt
for S in 1 0; do
  VST_WGRAD_SIDE=$S timeout -k 10 300 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 10 --warmup 3 --prof-steps 1 --no-cpu-baseline --no-vgg19 > gpurun_out/r04k_c5_side$S.json 2>/dev/null || exit 6
  echo "side=$S"; python tools/show_bench.py gpurun_out/r04k_c5_side$S.json | head -1
  VST_WGRAD_SIDE=$S timeout -k 10 300 python bench.py --steps 60 --prof-steps 1 --no-cpu-baseline --no-vgg19 > gpurun_out/r04k_c3_side$S.json 2>/dev/null || exit 7
  echo "side=$S"; python tools/show_bench.py gpurun_out/r04k_c3_side$S.json | head -1
done
echo done
