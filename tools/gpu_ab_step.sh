#!/bin/bash
# usage: gpu_ab_step.sh VAR "v1 v2 ..." -- in-step GEMM breakdown (bf16x6) per value of an environment
# switch, then the GPU suite
cd $GRAFT_REPO_ROOT
var=$1; vals=$2
for v in $vals; do
  env $var=$v VST_GEMM_POLICY=bf16x6 timeout -k 10 200 python tools/conv_breakdown.py reconet 3 > gpurun_out/abs_${var}_$v.log 2>&1 || exit 3
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/abs_tests.log 2>&1 || exit 4
echo ok
