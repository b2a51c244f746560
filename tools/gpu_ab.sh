#!/bin/bash
# A/B of an env switch on the per-layer GEMM timings: tools/gpu_ab.sh VAR "gemm_modes args"
cd $GRAFT_REPO_ROOT
var=$1; shift
for v in 0 1; do
  echo "$var=$v"
  env $var=$v timeout -k 10 150 python tools/gemm_modes.py "$@" 2>&1 | grep -v amdgpu || exit 2
done
