#!/bin/bash
# fp16 halo: depth-2 patch prefetch on the double-buffered tiles (default) vs depth 1 (libpd1) vs
# default + 3 waves/SIMD for the one-buffer single-product tiles (libsminw3): halo + AdaAttN tests,
# fp16 layer shapes, config-5 steps (A/B/C/A on one box)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
L=video-style-transfer_amd/vst
V=$L/variants
timeout -k 10 900 python -u -m pytest tests/test_gpu_halo.py tests/test_gpu_adaattn.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04u_tests.log 2>&1 || { tail -30 gpurun_out/r04u_tests.log; exit 3; }
tail -1 gpurun_out/r04u_tests.log
BENCH_ONLY=vgg,res,aa4 BENCH_GEMM_MODES=20 timeout -k 10 300 python tools/gemm_bench.py $L/libvst_hip.so $V/libpd1.so $V/libsminw3.so > gpurun_out/r04u_gemm.txt 2>&1 || { cat gpurun_out/r04u_gemm.txt; exit 4; }
cat gpurun_out/r04u_gemm.txt
n=0
for v in default pd1 sminw3 default; do
  n=$((n+1))
  if [ $v = default ]; then LP=""; else LP=$V/lib$v.so; fi
  VST_LIB_PATH=$LP timeout -k 10 300 python bench.py --model adaattn --batch 8 --height 512 --width 1024 --steps 10 --warmup 3 --prof-steps 0 --no-cpu-baseline --no-vgg19 > gpurun_out/r04u_c5_${n}_$v.json 2>/dev/null || exit 6
  echo "$v"; python tools/show_bench.py gpurun_out/r04u_c5_${n}_$v.json | head -1
done
echo done
