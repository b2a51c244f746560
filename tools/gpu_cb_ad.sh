#!/bin/bash
cd $GRAFT_REPO_ROOT
export VST_GEMM_POLICY=bf16x6
for cfg in "1 1" "0 0" "2 1"; do
  set -- $cfg
  VST_AD192=$1 VST_AD64=$2 timeout -k 10 200 python tools/conv_breakdown.py reconet 3 > gpurun_out/cb_$1_$2.log 2>&1 || exit 3
done
echo ok
