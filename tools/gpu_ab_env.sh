#!/bin/bash
# usage: gpu_ab_env.sh VAR "v1 v2 ..." -- conv microbench (bf16x6 tap-major and channel-blocked) per
# value of an environment switch, then the GPU suite and the headline bench on the defaults
cd $GRAFT_REPO_ROOT
var=$1; vals=$2
for v in $vals; do
  env $var=$v BENCH_GEMM_MODES=3,19 timeout -k 10 200 python tools/gemm_bench.py video-style-transfer_amd/vst/libvst_hip.so > gpurun_out/ab_${var}_$v.log 2>&1 || exit 3
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_tests.log 2>&1 || exit 4
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ab_bench.log 2>&1 || exit 5
echo ok
