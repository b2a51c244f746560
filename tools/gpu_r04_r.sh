#!/bin/bash
# 192-row halo block shape: 2x4 one-buffer (default) vs 2x2 one-buffer vs 3x1 one-buffer -- residual
# layer shapes, then config-3 steps on each library (A/B/C/A on one box)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
L=video-style-transfer_amd/vst
V=$L/variants
BENCH_ONLY=res BENCH_GEMM_MODES=19,20 timeout -k 10 300 python tools/gemm_bench.py $L/libvst_hip.so $V/lib192_2x2s.so $V/lib192_3x1s.so > gpurun_out/r04r_gemm.txt 2>&1 || { cat gpurun_out/r04r_gemm.txt; exit 4; }
cat gpurun_out/r04r_gemm.txt
for v in default 192_2x2s 192_3x1s default; do
  if [ $v = default ]; then LP=""; else LP=$V/lib$v.so; fi
  VST_LIB_PATH=$LP timeout -k 10 300 python bench.py --steps 60 --prof-steps 0 --no-cpu-baseline --no-vgg19 > gpurun_out/r04r_c3_$v.json 2>/dev/null || exit 7
  echo "$v"; python tools/show_bench.py gpurun_out/r04r_c3_$v.json | head -1
done
echo done
