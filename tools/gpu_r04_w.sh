#!/bin/bash
# two patches in flight for the bf16x6 8-wave halo tiles too (libpdx6) vs the default: halo tests on
# the variant, bf16x6 layer shapes, config-3 steps A/B/A/B on one box
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
L=video-style-transfer_amd/vst
V=$L/variants
VST_LIB_PATH=$V/libpdx6.so timeout -k 10 600 python -u -m pytest tests/test_gpu_halo.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04w_tests.log 2>&1 || { tail -30 gpurun_out/r04w_tests.log; exit 3; }
tail -1 gpurun_out/r04w_tests.log
BENCH_ONLY=vgg,aa4 BENCH_GEMM_MODES=19 timeout -k 10 300 python tools/gemm_bench.py $L/libvst_hip.so $V/libpdx6.so > gpurun_out/r04w_gemm.txt 2>&1 || { cat gpurun_out/r04w_gemm.txt; exit 4; }
cat gpurun_out/r04w_gemm.txt
for i in 1 2; do
  for v in default pdx6; do
    if [ $v = default ]; then LP=""; else LP=$V/lib$v.so; fi
    VST_LIB_PATH=$LP timeout -k 10 300 python bench.py --steps 60 --prof-steps 0 --no-cpu-baseline --no-vgg19 > gpurun_out/r04w_c3_${v}_$i.json 2>/dev/null || exit 7
    echo "$v"; python tools/show_bench.py gpurun_out/r04w_c3_${v}_$i.json | head -1
  done
done
echo done
